"""Benchmark: primary rays/s of the MI355X ray tracer on BASELINE.json's config.

Default workload (BASELINE.json configs[1]):
1920x1080, room box + 16 seeded spheres, the reference's 3 lights and 7
materials, max_depth 0 (primary ray + shadow rays, raytrace_compute.glsl:325-405).

A step is the animated frame loop (main.cpp:81-86): F frames of 1920x1080
per GPU (--frames-per-gpu, default 8; frame k is the reference orbit camera at
time k/60 s), rendered up to 8 frames per launch (rt_render_batch; SURVEY.md
§8(f) row 3 — several frames per launch amortise the launch ramp-up and
tail). On N GPUs a step holds N*F frames: every frame is row-tiled across the
N ranks in interleaved 8-row blocks, each rank renders its blocks of all N*F
frames, and one RCCL all-to-all over xGMI hands frames [kF, (k+1)F) to rank k
(N gathers at once, every link carrying 1/N of the frame traffic), which
de-interleaves its rows into the assembled frames. The shards travel as
packed float3 (the alpha channel is the constant 0). The exchange of step i
runs on its own stream beside the render of step i+1 (double-buffered).
Per-GPU work is F frames per step at every N: weak scaling. At N=1 the frames
are rendered in place (float4, no collective). --frames-per-gpu 1 gives the
single-frame launch.

--workload config5 (a Monte-Carlo extension the
reference does not have): one step = the 1920x1080 frame at 1024 jittered
samples per pixel, samples sharded over the N ranks, partial sums combined
with one RCCL all-reduce: strong scaling; value = samples/s.

value = primary rays (samples) of the step / step time (max over ranks), Mrays/s.
roofline = the render kernel against the HBM-write roofline: 16 B per pixel
(one float4 store) / average kernel time from HIP events on the launch stream
(N=1: one pair around the K back-to-back launches of the timed region; N>1:
a pair around every launch).
cpu_baseline = the reference's own shader on Mesa llvmpipe (oracle/_ref) over a
bounded band of the same frame, in a child process on the host cores.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2|config5]
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

WIDTH, HEIGHT, N_SPHERES, MAX_DEPTH = 1920, 1080, 16, 0
BLOCK_ROWS = 8
MC_SPP = 1024
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "primary Mrays/s at 1920×1080; achieved HBM GB/s vs peak; 1/2/4/8-GPU scaling"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["config2", "config5"], default="config2")
    ap.add_argument("--frames-per-gpu", type=int, default=8,
                    help="config2: animated frames each GPU renders per step, up to 8 per launch "
                         "(rt_render_batch; SURVEY.md §8(f) row 3)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="approximate budget of the llvmpipe baseline sample")
    return ap.parse_args()


def frame_time(k):
    return k / 60.0


def cpu_baseline(budget_s):
    """Time the reference shader on llvmpipe (child process) on a band of rows."""
    threads = min(16, os.cpu_count() or 1)
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--threads", str(threads),
           "--budget", str(budget_s)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=max(120, 6 * budget_s))
        if r.returncode == 0:
            return json.loads(r.stdout.strip().splitlines()[-1])
        sys.stderr.write("cpu baseline failed: %s\n" % r.stderr[-2000:])
    except Exception as e:  # the baseline is reported, never required
        sys.stderr.write("cpu baseline failed: %r\n" % (e,))
    return None


def pmc_latest(workload, frames_per_launch):
    """The committed PMC summary of the render kernel (profiles/pmc_latest.json,
    written by tools/pmc_summary.py) for this workload and launch shape at
    N=1, or {}."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
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
    return {"wave_insts_per_launch": insts, "achieved": round(achieved, 4), "peak": round(peak, 4),
            "unit": "T wave-instr/s", "frac": round(achieved / peak, 4),
            "source": "SQ_INSTS_VALU from profiles/pmc_latest.json (same build's rocprofv3 --pmc pass)"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import openglraytracer_amd as rt
    from openglraytracer_amd import frame

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
    scene = rt.Scene(ctx, rt.bench_objects(N_SPHERES, 0))
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
    mc = args.workload == "config5"
    channels = 3 if (world > 1 and not mc) else 4
    bytes_per_pixel = 4 * channels  # the render's store per pixel (algorithmic HBM bytes)

    if not mc:
        # N frames in flight, frame k = the orbit camera at t = k/60 s; every
        # rank renders its interleaved 8-row blocks of all N frames in one
        # launch (rt_render_batch); one all-to-all hands frame k's rows to
        # rank k (N gathers at once), which de-interleaves its frame. Double
        # buffered: the exchange of step i overlaps the render of step i+1.
        # The shard buffers that travel are packed float3 (RT_OUTPUT_RGB32F:
        # the alpha channel is the constant 0.0, raytrace_compute.glsl:404),
        # 3/4 of the float4 bytes over xGMI; N=1 renders float4 frames.
        # A step is the animated frame loop (main.cpp:81-86) F frames per
        # GPU: N*F frames at t = k/60 s, rank k's frames [kF, (k+1)F).
        fpg = args.frames_per_gpu
        n_frames = world * fpg
        views = [rt.make_view(None, frame_time(k)) for k in range(n_frames)]
        rows_mine = HEIGHT if world == 1 else rt.shard_rows(HEIGHT, BLOCK_ROWS, world, rank)
        if world > 1:
            ctx.set_output(rt.abi.RT_OUTPUT_RGB32F)
        bufs = [torch.zeros(n_frames * rows_mine * WIDTH * channels, dtype=torch.float32, device="cuda")
                for _ in range(2 if world > 1 else 1)]
        # launches of up to RT_MAX_BATCH views: (first frame, views) each
        chunks = [(j, views[j:j + rt.abi.RT_MAX_BATCH]) for j in range(0, n_frames, rt.abi.RT_MAX_BATCH)]
        frame_elems = rows_mine * WIDTH * channels
        if world > 1:
            in_splits, out_splits = frame.exchange_splits(HEIGHT, WIDTH, BLOCK_ROWS, world, rank, channels=channels,
                                                          frames_per_rank=fpg)
            recv = [torch.empty(sum(out_splits), dtype=torch.float32, device=coll_dev) for _ in bufs]
            idx = torch.as_tensor(frame.assembly_rows(HEIGHT, BLOCK_ROWS, world, fpg), device=coll_dev)
            frames_out = [None, None]
        launches_per_step = len(chunks)
        px_per_launch = WIDTH * rows_mine * n_frames // launches_per_step
        rays_per_step = n_frames * WIDTH * HEIGHT

        def render_frames(buf):
            for j, vs in chunks:
                rt.render_batch(ctx, scene, buf.data_ptr() + 4 * j * frame_elems, WIDTH, HEIGHT, MAX_DEPTH, vs,
                                BLOCK_ROWS, world, rank, stream=sh)
    else:
        view = rt.make_view(None, 0.0)
        spp_mine = MC_SPP // world + (1 if rank < MC_SPP % world else 0)
        sample0 = rank * (MC_SPP // world) + min(rank, MC_SPP % world)
        accum = torch.zeros((HEIGHT, WIDTH, 4), dtype=torch.float32, device="cuda")
        px_per_launch = WIDTH * HEIGHT
        rays_per_step = MC_SPP * WIDTH * HEIGHT
        launches_per_step = 1

    # Kernel time from HIP events on the render stream. At N=1 (config 2) a
    # step is its render launches alone: one event pair brackets the
    # back-to-back launches of the whole timed region (no markers between
    # frames); otherwise a pair brackets every step's render launches.
    per_launch = world > 1 or mc
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps if per_launch else 1)]
    rendered = [torch.cuda.Event() for _ in range(2)]
    freed = [None, None]  # event: the exchange has finished reading bufs[slot]

    def step(timed, it=0):
        if mc:
            accum.zero_()  # on comm_s: after the previous step's all-reduce read it
            render_s.wait_stream(comm_s)
            if timed:
                ev[it][0].record(render_s)
            rt.render_accumulate(ctx, scene, accum.data_ptr(), WIDTH, HEIGHT, MAX_DEPTH, spp_mine, sample0,
                                 seed=0, view=view, stream=sh)
            if timed:
                ev[it][1].record(render_s)
            comm_s.wait_stream(render_s)
            if world > 1:
                total = accum if coll_dev == "cuda" else accum.cpu()
                dist.all_reduce(total)  # RCCL: the partial sums of all ranks' samples
            else:
                total = accum
            if rank == 0:
                total.mul_(1.0 / MC_SPP)  # the estimate: mean over all samples
            return
        if world == 1:  # the frames rendered in place, launches back to back
            render_frames(bufs[0])
            return
        slot = it % 2
        if freed[slot] is not None:
            render_s.wait_event(freed[slot])  # the exchange of step it-2 has read bufs[slot]
        if timed:
            ev[it][0].record(render_s)
        render_frames(bufs[slot])
        if timed:
            ev[it][1].record(render_s)
        rendered[slot].record(render_s)
        comm_s.wait_event(rendered[slot])
        src = bufs[slot] if coll_dev == "cuda" else bufs[slot].cpu()
        dist.all_to_all_single(recv[slot], src, out_splits, in_splits)  # frames [kF, (k+1)F) -> rank k
        frames_out[slot] = frame.assemble_frames(recv[slot], fpg, HEIGHT, WIDTH, BLOCK_ROWS, world,
                                                 channels=channels, idx=idx)
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
        ev[0][0].record(render_s)
    for it in range(args.steps):
        step(True, it)
    if not per_launch:
        ev[0][1].record(render_s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    kernel_ms = ([a.elapsed_time(b) / launches_per_step for a, b in ev] if per_launch else
                 [ev[0][0].elapsed_time(ev[0][1]) / (args.steps * launches_per_step)])
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = rays_per_step * args.steps / elapsed / 1e6
    avg_kernel_ms = float(np.mean(kernel_ms))
    achieved = px_per_launch * bytes_per_pixel / (avg_kernel_ms * 1e-3) / 1e9
    pmc = pmc_latest(args.workload, 1 if mc else n_frames // launches_per_step) if world == 1 else {}
    traffic = pmc.get("hbm_bytes_per_launch")
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not mc:
            cpu = cpu_baseline(args.cpu_seconds)
        if not mc:
            workload = {"workload": "config2: 1920x1080, room box + 16 spheres, max_depth 0 "
                                    "(primary + shadow rays)",
                        "width": WIDTH, "height": HEIGHT, "spheres": N_SPHERES, "max_depth": MAX_DEPTH,
                        "frames_per_step": n_frames, "frames_per_gpu": fpg,
                        "frames_per_launch": n_frames // launches_per_step, "row_block": BLOCK_ROWS,
                        "output": "float4 frame" if world == 1 else "float3 shards (alpha 0 dropped) exchanged",
                        "parallelism": ("row-tiles x%d + RCCL all-to-all frame exchange (frame k gathered to "
                                        "rank k), overlapped with the next render" % world)
                                       if world > 1 else "single GPU"}
        else:
            workload = {"workload": "config5: 1920x1080 x 1024 spp Monte-Carlo, room box + 16 spheres, "
                                    "max_depth 0", "width": WIDTH, "height": HEIGHT, "spheres": N_SPHERES,
                        "spp": MC_SPP, "max_depth": MAX_DEPTH,
                        "parallelism": ("samples x%d + RCCL all-reduce" % world) if world > 1 else "single GPU"}
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "strong" if mc else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene, SURVEY.md §8(d) %s)" % args.workload,
            "config": workload,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "kernel_ms": round(avg_kernel_ms, 5),
                         "bytes_per_launch": px_per_launch * bytes_per_pixel,
                         "valu": valu_bound(pmc, avg_kernel_ms)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    scene.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
