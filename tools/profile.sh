#!/bin/bash
# Profile bench.py on the GPU box (run through gpurun):
#   kernel trace + stats, then separate PMC passes (HBM write bytes, HBM fetch
#   bytes, VALU instruction/wave counters, cycles, scratch/LDS traffic) —
#   never combined with tracing of other domains. Outputs under
#   gpurun_out/prof/<tag>/.
# usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
tag=${1:-r01}; shift || true
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 50 --warmup 5)
args+=(--no-single-frame --no-rgba8 --no-pipelined --no-general --no-verify)  # one launch shape per profile: no one-frame, RGBA8, pipelined, general-kernel or verification launches
run() { timeout -k 10 300 "$@"; }
pmc() { local name=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out" -o "$name" -- python3 bench.py --no-cpu-baseline "${args[@]}" > "$out/bench_$name.log" 2>&1; }
run rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o trace -- python3 bench.py --no-cpu-baseline "${args[@]}" > "$out/bench_trace.log" 2>&1
pmc pmc_write WRITE_SIZE
pmc pmc_fetch FETCH_SIZE
pmc pmc_sq SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM
pmc pmc_cyc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
pmc pmc_l2 TCC_HIT_sum TCC_MISS_sum
pmc pmc_lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES
find "$out" -type f | sort
