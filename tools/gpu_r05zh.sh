# Round-5: depth-0 light loop over the launch's live lights; batches of scenes take the room shape only if every scene is a room. A/B and the GPU suite.
set -uo pipefail
out=gpurun_out/r05zh; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
AB_ALLOW_SPILL=1 AB_PREDICTION="(the general depth-0 kernels +4 B scratch; the timed shapes unchanged at 0 B) main = rev + depth-0 shading over the live lights only (the reference's ambient-only light 0 skipped): config 2 / 5 -0.5..-1.5 %, deep unchanged" \
  run ab 400 python tools/ab.py config2,config2x64,config5,config4 rev main
echo done
