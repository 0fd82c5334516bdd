# Round-5: depth-0 kernels compiled for the scene's shape (RT_OPT_SCENE_SHAPES), A/B and the GPU suite.
set -uo pipefail
out=gpurun_out/r05p; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="scene shapes on (main) vs off (main:8=0): depth-0 scratch 16 -> 0 B; the probes (r05o) say config 2 -10..-12 %, config 5 a few %" \
  run ab 500 python tools/ab.py config2,config2x64,config5 main main:8=0 narrow
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
echo done
