# Round-5: RT_STATS / RT_CYCLES of configs 2-4 on the scene-shape kernels (the mix ran in the first call).
set -uo pipefail
out=gpurun_out/r05y; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run stats 300 python tools/stats.py stats
run cycles 300 python tools/cycles.py cycles
echo done
