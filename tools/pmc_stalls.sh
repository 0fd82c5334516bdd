#!/bin/bash
# Stall breakdown of the render kernel (development probe, run via gpurun):
#   tools/pmc_stalls.sh <ablate-variant> <config>
set -euo pipefail
v=${1:-short}; cfg=${2:-config2}
out=gpurun_out/stalls/$v-$cfg; mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $out -o p1 -- python3 tools/ablate_time.py $v $cfg > $out/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out -o p2 -- python3 tools/ablate_time.py $v $cfg > $out/p2.log 2>&1
python3 - "$out" <<'PY'
import csv, sys, collections, glob
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "render_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print("%-24s %16.1f  (n=%d)" % (k, sum(v) / len(v), len(v)))
PY
