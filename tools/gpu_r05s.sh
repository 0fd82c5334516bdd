# Round-5 probe: light count and depth-0 sphere bound / mask resolution as constants (timing only).
set -uo pipefail
out=gpurun_out/r05s; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="pl3 (3 lights as a constant in the shaped kernels): depth 0 ~-1.5 % (r05o), deep unknown; pd0 (depth 0: at most 64 spheres, 12-texel masks as constants): ~-1 %" \
  run ab 600 python tools/ab.py config2,config2x64,config3,config3x7,config4 main pl3 pd0
echo done
