# Round-5: origin-list candidates' sphere records read one pass ahead, A/B against HEAD.
set -uo pipefail
out=gpurun_out/r05zd; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="main = rev (7a4fcce kernels) + the list walk's LDS sphere reads one pass ahead (scratch 152/232 -> 148/228 B): if the per-pass LDS latency is exposed, configs 3-4 -1..-4 %; depth 0 unchanged" \
  run ab 500 python tools/ab.py config2x64,config3,config3x7,config4 rev main
echo done
