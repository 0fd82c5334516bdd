# Round-5 GPU session: instruction mix per wave (ablation builds, PMC), A/B of
# the round-4 library against this tree, NULL-stream cost.
set -uo pipefail
out=gpurun_out/r05e; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run mix_probe 300 bash tools/pmc_mix.sh $out/mixp config2 probe
run mix_config2 900 bash tools/pmc_mix.sh $out/mix2 config2 main noshadow nophong notrace noraygen
run mix_config4 600 bash tools/pmc_mix.sh $out/mix4 config4 main
AB_ALLOW_SPILL=1 run ab 600 python tools/ab.py config2,config2x64,config5,config3,config3x7,config4 rev main main:7=0
run null_stream_ab 300 python tools/null_stream_ab.py rev main 300
echo done
