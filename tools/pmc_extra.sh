#!/bin/bash
# Extra PMC passes (development probe): VALU lane utilisation, LDS and
# memory-latency counters of the render kernel for one bench workload.
# usage: tools/pmc_extra.sh TAG [bench args...]   -> gpurun_out/TAG/x_*.csv
set -euo pipefail
tag=${1:?tag}; shift
out=gpurun_out/$tag; mkdir -p "$out"
export TMPDIR=/tmp
args=("$@")
pmc() { local name=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out" -o "$name" -- python3 bench.py --no-cpu-baseline --no-single-frame --no-rgba8 --no-pipelined "${args[@]}" > "$out/bench_$name.log" 2>&1; }
pmc x_valu SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS
pmc x_mem TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY
ls "$out"
