set -uo pipefail
out=gpurun_out/r05d; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run parity 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread
AB_ALLOW_SPILL=1 run ab_olist 300 python tools/ab.py config3,config4,config3x7 rev main
run issue_probe 120 tools/probes/issue_probe 2.4
run null_stream_ab 300 python tools/null_stream_ab.py rev main 300
echo done
