# Round-5 checkpoint: the GPU suite, then the bench lines of every workload (same build as r05j's PMC passes).
set -uo pipefail
out=gpurun_out/r05j; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
bash tools/final_session.sh r05j bench
