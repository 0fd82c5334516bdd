# Round-5: cube-map texel lookup by the hardware's cube instructions (host layout in their coordinates), A/B and the GPU suite.
set -uo pipefail
out=gpurun_out/r05ze; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }

AB_ALLOW_SPILL=1 AB_PREDICTION="(gate: see the GATE lines; the timed kernels lose scratch) main = rev (7a4fcce kernels) + direction_texel by v_cubeid/sc/tc/ma (about 10 VALU fewer per lookup; deep scratch 152/232 -> 144/224 B): config 2 -1..-2 %, configs 3-4 -1..-2 %" \
  run ab 500 python tools/ab.py config2,config2x64,config5,config3,config4 rev main
echo done
