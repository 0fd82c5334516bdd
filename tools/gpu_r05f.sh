# Round-5 GPU session: shadow-walk variant (flags in vector registers) against main.
set -uo pipefail
out=gpurun_out/r05f; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_ALLOW_SPILL=1 run ab 600 python tools/ab.py config2,config2x64,config5,config3,config4 main shadowv
run mix_config2 600 bash tools/pmc_mix.sh $out/mix2 config2 main shadowv
echo done
