#!/bin/bash
# One GPU-box session (run through gpurun): tests, bench lines, profiles and
# development probes, each step under its own time limit; the session stops at
# the first failing step (a fault, an abort or a time limit ends it there).
#
# usage: tools/gpu_session.sh TAG STEP [STEP ...]
#
# steps (outputs under gpurun_out/TAG/):
#   tests        pytest -m gpu (SOFT_TESTS=1: a test failure, rc 1, does not stop the session)
#   smoke        __graft_entry__.smoke()
#   bench        the bench lines of every workload (config2-5, shipped)
#   prof         same-build PMC passes of every workload (tools/final_session.sh TAG prof)
#   final        prof then bench, as tools/final_session.sh TAG
#   ab           tools/ab.py $AB_ARGS (interleaved A/B of builds under _ab/; AB_PREDICTION
#                states the prediction, AB_ALLOW_SPILL=1 admits a scratch-growing variant)
#   ab2          tools/ab.py $AB_ARGS2
#   mix          tools/pmc_mix.sh gpurun_out/TAG/mix $MIX_ARGS (per-wave instruction mix of builds)
#   shards       tools/shard_timing.py (the N > 1 predictions), to gpurun_out/TAG/shard_timing_latest.json
#   soak         tools/soak.py $SOAK_SEED $SOAK_N and tools/soak_batch.py $SOAK_SEED2 $SOAK_N2
#   soakbox      tools/soak.py over many-box scenes (SOAK_KIND=boxes, $SOAK_SEED3 $SOAK_N3)
#   cycles/stats tools/cycles.py, tools/stats.py (RT_CYCLES / RT_STATS builds)
#   phase        tools/phase_trace.py (config 2 single-frame phase trace)
#   acc          tools/ab_accuracy.py $ACC_ARGS
#   probe        tools/probes/issue_probe (scalar issue rate)
#   list         rocprofv3 -L (the box's counters)
# (Round 5 ran 29 one-off scripts of exactly these steps; git history keeps them.)
set -uo pipefail
tag=${1:?tag}; shift
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
STEPS=("$@")
want() { for a in "${STEPS[@]}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
step() {  # name timeout cmd... ; stops the session on any failure
  local name=$1 t=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 $t "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -3 $out/$name.log
  if [ $rc -ne 0 ]; then
    if [ "${SOFT_TESTS:-0}" = 1 ] && [ "$name" = gpu_tests ] && [ $rc -eq 1 ]; then echo "   (tests failed; continuing)"; return 0; fi
    echo "STOP after $name (rc=$rc)"; exit $rc
  fi
}
if want list; then step counters 60 rocprofv3 -L; fi
if want tests; then step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread; fi
if want smoke; then step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; fi
if want prof || want final; then step final_prof 1500 bash tools/final_session.sh $tag prof; fi
if want bench || want final; then step final_bench 1200 bash tools/final_session.sh $tag bench; fi
if want ab; then step ab 900 python tools/ab.py ${AB_ARGS:-}; fi
if want ab2; then step ab2 900 python tools/ab.py ${AB_ARGS2:-}; fi
if want mix; then step mix 900 bash tools/pmc_mix.sh $out/mix ${MIX_ARGS:-config2 main}; fi
if want shards; then step shard_timing 900 python tools/shard_timing.py --out $out/shard_timing_latest.json; fi
if want soak; then
  step soak 540 python -u tools/soak.py ${SOAK_SEED:-12000} ${SOAK_N:-400}
  step soak_batch 400 python -u tools/soak_batch.py ${SOAK_SEED2:-12400} ${SOAK_N2:-150}
fi
if want soakbox; then step soak_boxes 540 env SOAK_KIND=boxes python -u tools/soak.py ${SOAK_SEED3:-20000} ${SOAK_N3:-300}; fi
if want cycles; then step cycles 300 python tools/cycles.py cycles ${CYC_ARGS:-config2 config3 config4}; fi
if want stats; then step stats 300 python tools/stats.py stats ${CYC_ARGS:-config2 config3 config4}; fi
if want phase; then step phase 300 env PHASE_DUMP=gpurun_out/$tag/phase.npz python tools/phase_trace.py config2 phase; fi
if want acc; then step accuracy 600 python tools/ab_accuracy.py ${ACC_ARGS:-main}; fi
if want probe; then step issue_probe 120 tools/probes/issue_probe 2.4; fi
echo done
