# Round-5: depth-0 shapes assume at most 64 spheres (main) vs HEAD (rev); + 12-texel masks as a constant (pn12).
set -uo pipefail
out=gpurun_out/r05t; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="main = rev + the sphere-count bound in the LDS-mask shapes; pn12 = main + 12-texel masks as a constant; pd0 (r05s) was both: config 2 -3 % one frame, -5 % at 64 per launch" \
  run ab 500 python tools/ab.py config2,config2x64,config5 rev main pn12 pd0
echo done
AB_ALLOW_SPILL=1 AB_PREDICTION="Monte-Carlo kernel in its scene shape at 7 / 8 waves per SIMD (scratch 0 -> 36 / 68 B): round 3 measured 8 waves +9.5 % with the then 84 B of spills; expect 6 to stay unless the spills sit outside the sample loop" \
  run ab_mc 400 python tools/ab.py config5 main mc7 mc8
echo done-mc
