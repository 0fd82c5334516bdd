# Round-5 final tree: the GPU suite, then the same-build PMC passes (final_session prof).
set -uo pipefail
out=gpurun_out/r05zj; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
bash tools/final_session.sh r05zj prof
