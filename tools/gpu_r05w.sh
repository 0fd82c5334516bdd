# Round-5: per-rank shard timings of the final kernels (bench.py --gpus N predictions read them).
set -uo pipefail
out=gpurun_out/r05w; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run shard_timing 900 python tools/shard_timing.py --out $out/shard_timing_latest.json
echo done
