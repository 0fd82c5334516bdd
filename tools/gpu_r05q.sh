# Round-5 probe: configs 3-4's scene features as compile-time constants (timing only).
set -uo pipefail
out=gpurun_out/r05q; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_ALLOW_SPILL=1 AB_PREDICTION="pdeep (cull, wide masks + lists + origin lists present, no LDS masks / cones, one box; scratch -24 B) and pdeepnb (the same without the box count): a few % on configs 3-4 if their feature tests cost what depth 0's did" \
  run ab 600 python tools/ab.py config3,config3x7,config4 main pdeep pdeepnb
run mix 400 bash tools/pmc_mix.sh $out/mix config4 main pdeep
echo done
