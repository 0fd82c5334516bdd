#!/bin/bash
# Instruction mix per wave of the render kernel for several builds (development
# probe, run via gpurun): VALU, SALU, SMEM, LDS and branch instructions per
# wave from one rocprofv3 PMC pass per build (tools/ablate_time.py renders the
# config with that build), so ablation builds (tools/ablate.sh) attribute the
# kernel's scalar work (round 5: the scalar unit, ~0.8 SALU per CU-cycle,
# profiles/r05d_issue_probe.log, is a co-bound of the depth-0 kernel).
#   tools/pmc_mix.sh OUTDIR CONFIG BUILD [BUILD ...]     (BUILD: main or a directory under _ab)
set -uo pipefail
out=${1:?outdir}; cfg=${2:?config}; shift 2
mkdir -p $out
export TMPDIR=/tmp
# two passes per build (at most 8 SQ counters each)
passes=("SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_LDS SQ_INSTS_BRANCH"
        "SQ_INSTS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VSKIPPED SQ_WAVES")
for v in "$@"; do
  for k in 0 1; do
    if [ "$v" = probe ]; then cmd="tools/probes/issue_probe 2.4"; else cmd="python3 tools/ablate_time.py $v $cfg"; fi
    timeout -s KILL 120 rocprofv3 --pmc ${passes[$k]} --output-format csv -d $out/$v/p$k -o mix -- $cmd \
        > $out/$v.p$k.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "pmc pass $k of $v failed rc=$rc"; tail -5 $out/$v.p$k.log; exit $rc; }
  done
done
python3 - "$out" "$@" <<'PY'
import csv, glob, sys, collections
out, builds = sys.argv[1], sys.argv[2:]
for v in builds:
    agg = collections.defaultdict(list)
    for f in glob.glob("%s/%s/**/*counter_collection.csv" % (out, v), recursive=True):
        for r in csv.DictReader(open(f)):
            if "render_kernel" in r["Kernel_Name"] or (v == "probe" and "probeILi8ELb0" in r["Kernel_Name"]):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(x) / len(x) for k, x in agg.items()}
    w = m.get("SQ_WAVES", 0) or 1
    print("%-12s per wave: " % v + "  ".join("%s %.1f" % (k.replace("SQ_INSTS_", ""), m[k] / w)
                                             for k in sorted(m) if k != "SQ_WAVES") + "  (waves %.0f)" % w)
PY
