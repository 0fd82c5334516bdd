# Round-5 probe: the room box (translate-only, holding every live light) as a shape constant (timing only).
set -uo pipefail
out=gpurun_out/r05z; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
AB_PREDICTION="proom vs pbase (= main): the shadow query's box shortcut test folded, about 7 SALU and 3 SMEM per query; expect -1..-2 % on config 2" \
  run ab 500 python tools/ab.py config2,config2x64,config5,config3,config4 pbase proom
run mix 300 bash tools/pmc_mix.sh $out/mix config2 pbase proom
echo done
