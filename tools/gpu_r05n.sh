# Round-5 probe: config 2's scene features as compile-time constants (timing only).
set -uo pipefail
out=gpurun_out/r05n; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_ALLOW_SPILL=1 AB_PREDICTION="narrow: depth-0 scratch 16 -> 0 B, feature checks folded, light and box loops unrolled; expect config 2 -2..-5 % if the scalar unit binds" \
  run ab 400 python tools/ab.py config2,config2x64 main narrow
run mix 300 bash tools/pmc_mix.sh $out/mix config2 main narrow
echo done
