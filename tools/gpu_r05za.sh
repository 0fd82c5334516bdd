# Round-5: the room as a scene-shape constant (kShapeRoom), A/B against HEAD and the GPU suite.
set -uo pipefail
out=gpurun_out/r05za; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="main = rev (960f588) with the one-box shapes narrowed to rooms and the room's shadow shortcut folded: the probe (r05z) measured config 2 -2.0/-2.3 %, config 5 -2.5 %, config 3 -1.2 %, config 4 -0.7 %" \
  run ab 500 python tools/ab.py config2,config2x64,config5,config3,config4 rev main
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
echo done
