# Round-5 GPU session: origin/level packing in the deep kernels' frame loop (scratch 188/268 -> 184/264 B).
set -uo pipefail
out=gpurun_out/r05i; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_ALLOW_SPILL=1 AB_PREDICTION="pack/packdone: 4 B less scratch per lane in depth-2/4; expect config3/config4 within +-1 % (no gain predicted beyond noise)" \
  run ab 600 python tools/ab.py config3,config3x7,config4 main pack packdone
echo done
