# Round-5 final kernels: per-rank shard timings (bench.py --gpus N predictions) and random-scene soaks.
set -uo pipefail
out=gpurun_out/r05zg; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run shard_timing 700 python tools/shard_timing.py --out $out/shard_timing_latest.json
run soak 400 python -u tools/soak.py 11000 400
run soak_batch 300 python -u tools/soak_batch.py 11400 150
echo done
