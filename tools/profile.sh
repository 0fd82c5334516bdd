#!/bin/bash
# Profile bench.py on the GPU box (run through gpurun):
#   kernel trace + stats, then separate PMC passes (HBM write bytes, HBM fetch
#   bytes, VALU instruction/wave counters) — never combined with tracing of
#   other domains. Outputs under gpurun_out/prof/<tag>/.
# usage: tools/profile.sh <tag> [bench args...]
set -euo pipefail
tag=${1:-r01}; shift || true
out=gpurun_out/prof/$tag
mkdir -p "$out"
export TMPDIR=/tmp
args=("$@")
[ ${#args[@]} -eq 0 ] && args=(--steps 50 --warmup 5)
run() { timeout -k 10 300 "$@"; }
run rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o trace -- python3 bench.py --no-cpu-baseline "${args[@]}" > "$out/bench_trace.log" 2>&1
run rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out" -o pmc_write -- python3 bench.py --no-cpu-baseline "${args[@]}" > "$out/bench_pmc_write.log" 2>&1
run rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out" -o pmc_fetch -- python3 bench.py --no-cpu-baseline "${args[@]}" > "$out/bench_pmc_fetch.log" 2>&1
run rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d "$out" -o pmc_sq -- python3 bench.py --no-cpu-baseline "${args[@]}" > "$out/bench_pmc_sq.log" 2>&1
run rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d "$out" -o pmc_cyc -- python3 bench.py --no-cpu-baseline "${args[@]}" > "$out/bench_pmc_cyc.log" 2>&1
find "$out" -type f | sort
