# Round-5: depth-0 shapes with the sphere bound and 12-texel masks as constants, A/B against HEAD and the GPU suite.
set -uo pipefail
out=gpurun_out/r05u; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="main = rev (c865eb0) + at most 64 spheres and 12-texel masks as constants in the depth-0 shapes: pd0 (r05t) measured config 2 -3 % one frame, -5 % at 64 per launch, config 5 -3 %" \
  run ab 400 python tools/ab.py config2,config2x64,config5 rev main
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
echo done
