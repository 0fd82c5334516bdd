# Round-5 GPU session: event counts and per-phase wave time after the origin lists.
set -uo pipefail
out=gpurun_out/r05g; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run stats 300 python tools/stats.py stats config2 config3 config4
run cycles 300 python tools/cycles.py cycles config2 config3 config4
echo done
