#!/bin/bash
# Same-build profile + bench session (run through gpurun, usually via
# tools/gpu_session.sh TAG prof|bench|final):
#   tools/final_session.sh TAG prof    PMC passes of every bench workload; their
#                                      summaries go to profiles/ on the box and
#                                      travel back under gpurun_out/TAG/profiles
#                                      (copy them into profiles/ before the bench
#                                      call, so its lines take traffic / valu from
#                                      the same sources)
#   tools/final_session.sh TAG bench   the bench lines of every workload, smoke,
#                                      a self-launched N = 2 and a torchrun N = 4
#                                      gloo rehearsal of config 2
#   tools/final_session.sh TAG         both, in one call
# Every summary keeps only the timed launch shape (tools/pmc_summary.py): the
# profiled runs skip their verification renders (profile.sh), and --skip drops
# the warm-up launches (warmup x launches per step).
set -uo pipefail
tag=${1:?tag}
what=${2:-all}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
if [ "$what" = prof ] || [ "$what" = all ]; then
  run prof_config4 900 tools/profile.sh $tag/c4 --workload config4 --steps 3 --warmup 1
  run prof_config3 900 tools/profile.sh $tag/c3 --workload config3 --steps 10 --warmup 2
  run prof_config2 900 tools/profile.sh $tag/c2 --steps 50 --warmup 5
  run prof_config5 900 tools/profile.sh $tag/c5 --workload config5 --steps 2 --warmup 1
  run prof_shipped 900 tools/profile.sh $tag/cs --workload shipped --steps 50 --warmup 5
  run sum2 60 python tools/pmc_summary.py $out/c2 profiles/${tag}_config2 256 config2 --skip 5
  # config 3's step is one queued launch of the views it holds (bench.py): its frame count
  f3=$(timeout -k 10 120 python -c "import openglraytracer_amd as rt; c = rt.Context(0); s = rt.Scene(c, rt.bench_objects(64, 0)); print(max(k for k in range(1, 65) if rt.batch_launches(c, s, k, 2) == 1))") || exit 1
  run sum3 60 python tools/pmc_summary.py $out/c3 profiles/${tag}_config3 $f3 config3 --skip 2
  run sum4 60 python tools/pmc_summary.py $out/c4 profiles/${tag}_config4 1 config4 --skip 1
  run sum5 60 python tools/pmc_summary.py $out/c5 profiles/${tag}_config5 1 config5 --skip 1
  run sums 60 python tools/pmc_summary.py $out/cs profiles/${tag}_shipped 256 shipped --skip 5
  mkdir -p $out/profiles && cp profiles/${tag}_* profiles/pmc_*latest.json $out/profiles/
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  run bench_config2 300 python bench.py
  run bench_config3 300 python bench.py --workload config3 --steps 20 --warmup 3 --no-cpu-baseline
  run bench_config4 300 python bench.py --workload config4 --steps 5 --warmup 1 --no-cpu-baseline
  run bench_config5 300 python bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline
  run bench_shipped 300 python bench.py --workload shipped
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  # several ranks share the one GPU here (gloo): the step structure and the
  # byte-exact assembly, not scaling figures
  run selflaunch_config2_n2 400 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --frames 64 \
      --no-cpu-baseline
  run gloo_config2_n4 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
      --master-port 29611 bench.py --gpus 4 --dist-backend gloo --steps 5 --warmup 2 --frames 64 --no-cpu-baseline
fi
echo done
