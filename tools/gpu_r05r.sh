# Round-5: the recursive kernels in the wide-mask scene shape (RT_OPT_SCENE_SHAPES), A/B and the GPU suite.
set -uo pipefail
out=gpurun_out/r05r; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="scene shapes on (main) vs off (main:8=0) for the deep kernels: scratch 184/264 -> 160/240 B; the probe (r05q) says config 3 -9.6 %, config 4 -6.2 %; config 2 as r05p" \
  run ab 600 python tools/ab.py config2x64,config3,config3x7,config4 main main:8=0 pdeep
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
echo done
