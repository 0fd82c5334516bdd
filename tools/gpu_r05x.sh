# Round-5: wave votes on compare lane masks (ballot against exec) vs HEAD.
set -uo pipefail
out=gpurun_out/r05x; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_ALLOW_SPILL=1 AB_PREDICTION="(scratch +4 B only in the deep Monte-Carlo kernels, which no config times) main = rev (bb9402a) + votes by ballot and a one-compare range vote in inv_sqrt: static VALU 2082 -> 2059 (config-2 shape), deep scratch -8 B; expect -0.5..-2 %" \
  run ab 500 python tools/ab.py config2,config2x64,config5,config3,config4 rev main
echo done
