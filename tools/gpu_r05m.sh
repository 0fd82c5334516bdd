# Round-5: random-scene soaks of the final kernels (origin-sphere lists included).
set -uo pipefail
out=gpurun_out/r05m; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run soak 540 python -u tools/soak.py 8000 600
run soak_batch 540 python -u tools/soak_batch.py 8600 300
AB_ALLOW_SPILL=1 AB_PREDICTION="occupancy of the deep kernels with the origin lists: wpe7 72 VGPRs + 36 B more scratch, wpe5 96 VGPRs + 68 B less; round 3 measured 7 waves +2 % and 5 waves +9 % on config 4; expect the same sign (6 stays)" \
  run ab_wpe 600 python tools/ab.py config3,config3x7,config4 main wpe7 wpe5
echo done-ab
