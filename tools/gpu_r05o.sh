# Round-5 probe: which of config 2's compile-time scene features pays (timing only).
set -uo pipefail
out=gpurun_out/r05o; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_ALLOW_SPILL=1 AB_PREDICTION="pflags (cull, 2-B masks, no cones, no BVH as constants; scratch 16 -> 0): most of narrow's -11 %; pnl (3 lights): loop unrolled, a few %; pnb (1 box; scratch 16 -> 28): small" \
  run ab 500 python tools/ab.py config2,config2x64 main narrow pflags pnl pnb
run mix 400 bash tools/pmc_mix.sh $out/mix config2 main pflags pnl pnb
echo done
