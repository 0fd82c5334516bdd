# Round-5 GPU session (run through gpurun): parity suite, same-process A/B of
# the round-4 library (_ab/rev, tools/ablate.sh rev 7038a0d) against this
# tree with and without origin lists (main:7=0), and the issue / NULL-stream probes.
set -uo pipefail
out=gpurun_out/r05d; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread
AB_ALLOW_SPILL=1 run ab 600 python tools/ab.py config2,config2x64,config5,config3,config3x7,config4 rev main main:7=0
run issue_probe 120 tools/probes/issue_probe 2.4
run null_stream_ab 300 python tools/null_stream_ab.py rev main 300
echo done
