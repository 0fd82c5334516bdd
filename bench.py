"""Benchmark: primary rays/s of the MI355X ray tracer on BASELINE.json's configs.

Default workload (BASELINE.json configs[1]):
1920x1080, room box + 16 seeded spheres, the reference's 3 lights and 7
materials, max_depth 0 (primary ray + shadow rays, raytrace_compute.glsl:325-405).

config2 (default). A step is the animated frame loop (main.cpp:81-86): F
frames of 1920x1080 per GPU (--frames-per-gpu, default 8; frame k is the
reference orbit camera at time k/60 s), rendered up to 8 frames per launch
(rt_render_batch; SURVEY.md §8(f) row 3 — several frames per launch amortise
the launch ramp-up and tail). At N=1 the line also carries the one-frame-per-
launch rate (`single_frame`, the shape of the reference's draw()). On N GPUs
a step holds N*F frames; the frames of the animated loop are independent
units, so rank k renders frames [kF, (k+1)F) whole, with no data-path
collective. Weak scaling. --frame-exchange all_to_all instead row-tiles every
frame across the N ranks in interleaved 8-row blocks, each rank renders its
blocks of all N*F frames, and one RCCL all-to-all over xGMI hands frames
[kF, (k+1)F) to rank k (N gathers at once), which de-interleaves its rows;
the shards travel as packed float3 (the alpha channel is the constant 0), and
the exchange of step i runs on its own stream beside the render of step i+1
(double-buffered).

config3 / config4 (3840x2160 / 64 spheres / depth 2, and
7680x4320 / 256 spheres / depth 4 row-tiled across the GPUs with an RCCL
gather). A step is ONE frame. N=1 renders it whole (float4). N>1: the frame's
interleaved 8-row blocks are dealt round-robin to the ranks (rt_render_shard,
packed float3 shards), one RCCL gather brings the shards to rank 0 and rank 0
de-interleaves them into the frame (frame.gather_frame); the gather of step i
overlaps the render of step i+1. Strong scaling. The line reports every
rank's kernel time and the gather and assembly times separately.

config5 (a Monte-Carlo extension the reference does not have): one step =
the 1920x1080 frame at 1024 jittered samples per pixel, samples sharded over
the N ranks, partial sums combined with one RCCL all-reduce: strong scaling;
value = samples/s.

value = primary rays (samples) of the step / step time (max over ranks), Mrays/s.
roofline = the render kernel against the HBM-write roofline: bytes stored per
launch (16 B per pixel for a float4 frame, 12 for float3 shards) / average
kernel time from HIP events on the launch stream (config2 at N=1: one pair
around the K back-to-back launches of the timed region; otherwise a pair
around every step's launches).
cpu_baseline = the reference's own shader on Mesa llvmpipe (oracle/_ref) on the
host cores, median of 3 dispatches, plus a 1-thread sample and the other
configs' row subsets (oracle/cpu_baseline.py, child process, N=1 only).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2|config3|config4|config5]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    "config2": dict(width=1920, height=1080, spheres=16, depth=0,
                    text="config2: 1920x1080, room box + 16 spheres, max_depth 0 (primary + shadow rays)"),
    "config3": dict(width=3840, height=2160, spheres=64, depth=2,
                    text="config3: 3840x2160, room box + 64 spheres, max_depth 2 (2 reflection/refraction "
                         "bounces + shadow rays)"),
    "config4": dict(width=7680, height=4320, spheres=256, depth=4,
                    text="config4: 7680x4320, room box + 256 spheres, max_depth 4 (4 bounces + shadow rays)"),
    "config5": dict(width=1920, height=1080, spheres=16, depth=0, spp=1024,
                    text="config5: 1920x1080 x 1024 spp Monte-Carlo, room box + 16 spheres, max_depth 0"),
}
BLOCK_ROWS = 8
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "primary Mrays/s at 1920×1080; achieved HBM GB/s vs peak; 1/2/4/8-GPU scaling"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="config2")
    ap.add_argument("--frames-per-gpu", type=int, default=8,
                    help="config2: animated frames each GPU renders per step, up to 8 per launch "
                         "(rt_render_batch; SURVEY.md §8(f) row 3)")
    ap.add_argument("--frame-exchange", choices=["none", "all_to_all"], default="none",
                    help="config2 at N>1: none = every rank renders whole frames of its own; all_to_all = "
                         "every frame row-tiled over the ranks and exchanged (frame k gathered to rank k)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=25.0,
                    help="approximate budget of the llvmpipe baseline samples")
    ap.add_argument("--no-single-frame", action="store_true",
                    help="config2: skip the one-frame-per-launch measurement (profiling runs: one launch shape)")
    return ap.parse_args()


def frame_time(k):
    return k / 60.0


def cpu_baseline(workload, budget_s):
    """Time the reference shader on llvmpipe (child process) — §8(d)."""
    threads = min(16, os.cpu_count() or 1)
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--threads", str(threads),
           "--budget", str(budget_s), "--workload", workload]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=max(180, 8 * budget_s))
        if r.returncode == 0:
            return json.loads(r.stdout.strip().splitlines()[-1])
        sys.stderr.write("cpu baseline failed: %s\n" % r.stderr[-2000:])
    except Exception as e:  # the baseline is reported, never required
        sys.stderr.write("cpu baseline failed: %r\n" % (e,))
    return None


def pmc_latest(workload, frames_per_launch):
    """The committed PMC summary of the render kernel for this workload and
    launch shape at N=1 (profiles/pmc_<workload>_latest.json, written by
    tools/pmc_summary.py; config2 also profiles/pmc_latest.json), or {}."""
    for name in ("pmc_%s_latest.json" % workload, "pmc_latest.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
            if (d.get("workload") == workload and d.get("n_gpus", 1) == 1
                    and d.get("frames_per_launch", 1) == frames_per_launch):
                return d
        except (OSError, ValueError):
            pass
    return {}


def valu_bound(pmc, kernel_ms):
    """The bound the kernel actually sits against: VALU issue.
    Peak = one wave64 VALU instruction per 2 cycles per SIMD (SIMD-32),
    1024 SIMDs at 2.4 GHz (/opt/skills/guides/MI355X_MICROARCH.md)."""
    insts = pmc.get("sq_insts_valu_per_launch")
    if not insts or kernel_ms <= 0:
        return None
    peak = 1024 * 2.4e9 / 2 / 1e12  # T wave-instructions / s
    achieved = insts / (kernel_ms * 1e-3) / 1e12
    out = {"wave_insts_per_launch": insts, "achieved": round(achieved, 4), "peak": round(peak, 4),
           "unit": "T wave-instr/s", "frac": round(achieved / peak, 4),
           "source": "SQ_INSTS_VALU from profiles/pmc_*_latest.json (rocprofv3 --pmc pass of the build "
                     "committed before this run: %s)" % pmc.get("build", "?")}
    if pmc.get("scratch_bytes_per_lane") is not None:
        out["scratch_bytes_per_lane"] = pmc["scratch_bytes_per_lane"]
    return out


class Timer:
    """HIP event pairs on a stream; mean milliseconds per recorded pair."""

    def __init__(self, torch, n):
        self.ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]

    def start(self, i, stream):
        self.ev[i][0].record(stream)

    def stop(self, i, stream):
        self.ev[i][1].record(stream)

    def ms(self):
        return [a.elapsed_time(b) for a, b in self.ev]


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import openglraytracer_amd as rt
    from openglraytracer_amd import frame

    cfg = WORKLOADS[args.workload]
    W, H, DEPTH = cfg["width"], cfg["height"], cfg["depth"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    device = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    coll_dev = "cuda"
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.dist_backend)
            coll_dev = "cpu"

    ctx = rt.Context(device)
    scene = rt.Scene(ctx, rt.bench_objects(cfg["spheres"], 0))
    ctx.set_timing(False)  # no per-launch markers of the library's own
    # Streams of our own: renders are launched asynchronously on `render_s`
    # (the C-ABI treats a NULL stream — torch's default stream handle is 0 —
    # as "synchronous on the context's stream", like glFinish); the current
    # stream `comm_s` orders the collectives (RCCL runs on its own stream
    # behind it) and the frame assembly.
    render_s = torch.cuda.Stream()
    comm_s = torch.cuda.Stream()
    torch.cuda.set_stream(comm_s)
    sh = render_s.cuda_stream
    assert sh, "need a non-default HIP stream"
    wl = args.workload
    mc = wl == "config5"
    batched = wl == "config2"  # N*F frames per step in batched launches
    exchange = batched and world > 1 and args.frame_exchange == "all_to_all"
    sharded = world > 1 and not mc and (exchange or not batched)  # ranks render row-tiles of shared frames
    channels = 3 if sharded else 4
    bytes_per_pixel = 4 * channels  # the render's store per pixel (algorithmic HBM bytes)
    if channels == 3:
        ctx.set_output(rt.abi.RT_OUTPUT_RGB32F)
    extra = {}

    if batched and not exchange:
        # N*F frames in flight, frame k = the orbit camera at t = k/60 s;
        # rank r renders frames [rF, (r+1)F) whole, up to 8 per launch
        # (rt_render_batch), in place, launches back to back.
        fpg = args.frames_per_gpu
        n_frames = fpg
        views = [rt.make_view(None, frame_time(rank * fpg + k)) for k in range(fpg)]
        bufs = [torch.zeros(fpg * H * W * 4, dtype=torch.float32, device="cuda")]
        chunks = [(j, views[j:j + rt.abi.RT_MAX_BATCH]) for j in range(0, fpg, rt.abi.RT_MAX_BATCH)]
        frame_elems = H * W * 4
        launches_per_step = len(chunks)
        px_per_launch = W * H * fpg // launches_per_step
        rays_per_step = world * fpg * W * H

        def render(buf):
            for j, vs in chunks:
                rt.render_batch(ctx, scene, buf.data_ptr() + 4 * j * frame_elems, W, H, DEPTH, vs, stream=sh)
    elif batched:
        # N frames in flight, frame k = the orbit camera at t = k/60 s; every
        # rank renders its interleaved 8-row blocks of all N frames in one
        # launch (rt_render_batch); one all-to-all hands frame k's rows to
        # rank k (N gathers at once), which de-interleaves its frame. Double
        # buffered: the exchange of step i overlaps the render of step i+1.
        fpg = args.frames_per_gpu
        n_frames = world * fpg
        views = [rt.make_view(None, frame_time(k)) for k in range(n_frames)]
        rows_mine = H if world == 1 else rt.shard_rows(H, BLOCK_ROWS, world, rank)
        bufs = [torch.zeros(n_frames * rows_mine * W * channels, dtype=torch.float32, device="cuda")
                for _ in range(2 if world > 1 else 1)]
        chunks = [(j, views[j:j + rt.abi.RT_MAX_BATCH]) for j in range(0, n_frames, rt.abi.RT_MAX_BATCH)]
        frame_elems = rows_mine * W * channels
        if world > 1:
            in_splits, out_splits = frame.exchange_splits(H, W, BLOCK_ROWS, world, rank, channels=channels,
                                                          frames_per_rank=fpg)
            recv = [torch.empty(sum(out_splits), dtype=torch.float32, device=coll_dev) for _ in bufs]
            idx = torch.as_tensor(frame.assembly_rows(H, BLOCK_ROWS, world, fpg), device=coll_dev)
        launches_per_step = len(chunks)
        px_per_launch = W * rows_mine * n_frames // launches_per_step
        rays_per_step = n_frames * W * H

        def render(buf):
            for j, vs in chunks:
                rt.render_batch(ctx, scene, buf.data_ptr() + 4 * j * frame_elems, W, H, DEPTH, vs,
                                BLOCK_ROWS, world, rank, stream=sh)
    elif mc:
        view = rt.make_view(None, 0.0)
        spp = cfg["spp"]
        spp_mine = spp // world + (1 if rank < spp % world else 0)
        sample0 = rank * (spp // world) + min(rank, spp % world)
        accum = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        px_per_launch = W * H
        rays_per_step = spp * W * H
        launches_per_step = 1
    else:
        # one frame per step: whole at N=1, row-tiled + gathered at N>1
        view = rt.make_view(None, 0.0)
        rows_mine = H if world == 1 else rt.shard_rows(H, BLOCK_ROWS, world, rank)
        shard_elems = frame.flat_shard_elems(1, H, W, BLOCK_ROWS, world, channels) if world > 1 else H * W * 4
        bufs = [torch.zeros(shard_elems, dtype=torch.float32, device="cuda") for _ in range(2 if world > 1 else 1)]
        if world > 1 and rank == 0:
            glists = [[torch.empty(shard_elems, dtype=torch.float32, device=coll_dev) for _ in range(world)]
                      for _ in bufs]
            perm = torch.as_tensor(frame.assembly_permutation(H, BLOCK_ROWS, world), device=coll_dev)
        launches_per_step = 1
        px_per_launch = W * rows_mine
        rays_per_step = W * H

        def render(buf):
            if world == 1:
                rt.render_device(ctx, scene, buf.data_ptr(), W, H, DEPTH, view=view, stream=sh)
            else:
                rt.render_shard(ctx, scene, buf.data_ptr(), W, H, DEPTH, BLOCK_ROWS, world, rank, view=view,
                                stream=sh)

    # Kernel time from HIP events on the render stream. config2 without an
    # exchange: a step is its render launches alone, one event pair brackets
    # the back-to-back launches of the whole timed region (no markers between
    # frames); otherwise a pair brackets every step's render launches.
    per_launch = not (batched and not exchange)
    kt = Timer(torch, args.steps if per_launch else 1)
    ct = Timer(torch, args.steps)  # collective (exchange / gather / all-reduce) on comm_s
    at = Timer(torch, args.steps)  # frame assembly on comm_s (rank 0 / every rank for the exchange)
    rendered = [torch.cuda.Event() for _ in range(2)]
    freed = [None, None]  # event: the collective has finished reading bufs[slot]
    state = {"collective": False}

    def step(timed, it=0):
        if mc:
            accum.zero_()  # on comm_s: after the previous step's all-reduce read it
            render_s.wait_stream(comm_s)
            if timed:
                kt.start(it, render_s)
            rt.render_accumulate(ctx, scene, accum.data_ptr(), W, H, DEPTH, spp_mine, sample0, seed=0, view=view,
                                 stream=sh)
            if timed:
                kt.stop(it, render_s)
            comm_s.wait_stream(render_s)
            if timed:
                ct.start(it, comm_s)
            if world > 1:
                total = accum if coll_dev == "cuda" else accum.cpu()
                dist.all_reduce(total)  # RCCL: the partial sums of all ranks' samples
                state["collective"] = True
            else:
                total = accum
            if timed:
                ct.stop(it, comm_s)
                at.start(it, comm_s)
            if rank == 0:
                total.mul_(1.0 / spp)  # the estimate: mean over all samples
            if timed:
                at.stop(it, comm_s)
            return
        if not per_launch:  # config2 without exchange: frames rendered in place, launches back to back
            render(bufs[0])
            return
        slot = it % 2 if world > 1 else 0
        if freed[slot] is not None:
            render_s.wait_event(freed[slot])  # the collective of step it-2 has read bufs[slot]
        if timed:
            kt.start(it, render_s)
        render(bufs[slot])
        if timed:
            kt.stop(it, render_s)
        if world == 1:
            return
        rendered[slot].record(render_s)
        comm_s.wait_event(rendered[slot])
        src = bufs[slot] if coll_dev == "cuda" else bufs[slot].cpu()
        if timed:
            ct.start(it, comm_s)
        if exchange:
            dist.all_to_all_single(recv[slot], src, out_splits, in_splits)  # frames [kF, (k+1)F) -> rank k
            if timed:
                ct.stop(it, comm_s)
                at.start(it, comm_s)
            frame.assemble_frames(recv[slot], fpg, H, W, BLOCK_ROWS, world, channels=channels, idx=idx)
        else:
            if rank == 0:
                dist.gather(src, glists[slot], dst=0)  # RCCL: every shard to rank 0
            else:
                dist.gather(src, None, dst=0)
            if timed:
                ct.stop(it, comm_s)
                at.start(it, comm_s)
            if rank == 0:  # de-interleave the row blocks into the frame
                frame.assemble(glists[slot], 1, H, W, BLOCK_ROWS, channels=channels, perm=perm)
        if timed:
            at.stop(it, comm_s)
        state["collective"] = True
        e = torch.cuda.Event()
        e.record(comm_s)
        freed[slot] = e

    for i in range(args.warmup):
        step(False, i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if not per_launch:
        kt.start(0, render_s)
    for it in range(args.steps):
        step(True, it)
    if not per_launch:
        kt.stop(0, render_s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = ([m / launches_per_step for m in kt.ms()] if per_launch else
                 [kt.ms()[0] / (args.steps * launches_per_step)])
    avg_kernel_ms = float(np.mean(kernel_ms))
    coll_ms = float(np.mean(ct.ms())) if (sharded or mc) else 0.0
    asm_ms = float(np.mean(at.ms())) if (sharded or mc) else 0.0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        mine = torch.tensor([avg_kernel_ms, coll_ms, asm_ms], dtype=torch.float64, device=coll_dev)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        per_rank = [[round(float(v), 5) for v in e.cpu().tolist()] for e in every]
    else:
        per_rank = [[round(avg_kernel_ms, 5), coll_ms, asm_ms]]
    if batched and world == 1 and rank == 0 and not args.no_single_frame:
        # one frame per launch (the shape of the reference's draw(),
        # main.cpp:210-238): K launches back to back, one event pair
        n1 = max(20, args.steps)
        one = torch.empty(H * W * 4, dtype=torch.float32, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for k in range(3):
            rt.render_batch(ctx, scene, one.data_ptr(), W, H, DEPTH, [views[k % len(views)]], stream=sh)
        e0.record(render_s)
        for k in range(n1):
            rt.render_batch(ctx, scene, one.data_ptr(), W, H, DEPTH, [views[k % len(views)]], stream=sh)
        e1.record(render_s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n1 * 1e3
        extra["single_frame"] = {"frames_per_launch": 1, "us_per_frame": round(us, 3),
                                 "value": round(W * H / us, 3), "unit": "Mrays/s",
                                 "roofline_frac": round(W * H * 16 / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5)}
    ms_per_step = elapsed / args.steps * 1e3
    value = rays_per_step * args.steps / elapsed / 1e6
    achieved = px_per_launch * bytes_per_pixel / (avg_kernel_ms * 1e-3) / 1e9
    fpl = 1 if not batched else n_frames // launches_per_step
    pmc = pmc_latest(wl, fpl) if world == 1 else {}
    traffic = pmc.get("hbm_bytes_per_launch")
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(wl, args.cpu_seconds)
        workload = {"workload": cfg["text"], "width": W, "height": H, "spheres": cfg["spheres"], "max_depth": DEPTH}
        if batched and not exchange:
            workload.update({"frames_per_step": world * fpg, "frames_per_gpu": fpg, "frames_per_launch": fpl,
                             "output": "float4 frames",
                             "parallelism": ("whole frames x%d (rank r renders frames [rF, (r+1)F) of the "
                                             "animated loop), no collective" % world) if world > 1
                                            else "single GPU"})
        elif batched:
            workload.update({"frames_per_step": n_frames, "frames_per_gpu": fpg,
                             "frames_per_launch": fpl, "row_block": BLOCK_ROWS,
                             "output": "float3 shards (alpha 0 dropped) exchanged",
                             "parallelism": ("row-tiles x%d + RCCL all-to-all frame exchange (frame k gathered to "
                                             "rank k), overlapped with the next render" % world)
                                            if world > 1 else "single GPU"})
        elif mc:
            workload.update({"spp": cfg["spp"],
                             "parallelism": ("samples x%d + RCCL all-reduce" % world) if world > 1 else "single GPU"})
        else:
            workload.update({"frames_per_step": 1, "row_block": BLOCK_ROWS,
                             "output": "float4 frame" if world == 1 else
                             "float3 shards (alpha 0 dropped) gathered to rank 0, de-interleaved there",
                             "parallelism": ("interleaved 8-row blocks x%d + RCCL gather to rank 0, overlapped "
                                             "with the next render" % world) if world > 1 else "single GPU"})
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak" if batched else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene, SURVEY.md §8(d) %s)" % wl,
            "config": workload,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "kernel_ms": round(avg_kernel_ms, 5),
                         "bytes_per_launch": px_per_launch * bytes_per_pixel,
                         "valu": valu_bound(pmc, avg_kernel_ms)},
            "timing": {"per_rank": [{"rank": r, "kernel_ms": v[0], "collective_ms": v[1], "assembly_ms": v[2]}
                                    for r, v in enumerate(per_rank)],
                       "collective": {"config2": "all_to_all_single (N frame gathers at once)",
                                      "config5": "all_reduce of the sample sums"}.get(
                                          wl, "gather to rank 0") if (sharded or mc) and world > 1 else "none",
                       "note": "HIP events: kernel on the render stream, collective and assembly on the "
                               "collective stream, means over the timed steps"},
            "cpu_baseline": cpu,
            "build": rt.lib().rt_version().decode(),
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    scene.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
