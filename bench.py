"""Benchmark: primary rays/s of the MI355X ray tracer on BASELINE.json's configs.

Default workload (BASELINE.json configs[1]):
1920x1080, room box + 16 seeded spheres, the reference's 3 lights and 7
materials, max_depth 0 (primary ray + shadow rays, raytrace_compute.glsl:325-405).

config2 (default). A step is F frames of the animated frame loop
(main.cpp:81-86; --frames, default 256, about four seconds of the loop; frame k is
the reference orbit camera at time k/60 s), rendered in one launch
(rt_render_batch, up to 256 views; SURVEY.md §8(f) row 3 — several frames per
launch amortise the launch's ramp-up, tail and dispatch gap, about 22 us per
launch). The total work of a step is fixed: strong scaling.
  * N=1: every frame whole, float4 per pixel (16 B: the HBM-write roofline's
    bytes). The line also carries the one-frame-per-launch rate
    (`single_frame`, the shape of the reference's draw(), main.cpp:228-238),
    and `rgba8_surface`: the same frames into the GL_RGBA8 surface that the
    N>1 steps write, so the N=1 and N>1 points share a surface; every line's
    roofline also carries `frac_float4_equivalent` (the pixels at 16 B).
  * N>1 (north_star: "image row-tiles shard across the GPUs with an RCCL
    gather over xGMI to assemble the frame"): every frame of the step is
    row-tiled over the N ranks in interleaved 8-row blocks; each rank renders
    its blocks of all F frames (rt_render_batch with shards) into the shipped
    app's GL_RGBA8 surface format (main.cpp:152-159, :223; RT_OUTPUT_RGBA8,
    byte-exact vs the reference's GL render), and the shards travel without
    its alpha byte, which is always 0 (:404): 3 B per pixel. The default
    exchange (--frame-exchange spread) assembles frame k on rank k % N with
    one RCCL all-to-all per step: each frame is still gathered from all N
    row-tiles, but the step's bytes enter through every rank's xGMI links
    instead of rank 0's alone (xGMI is point-to-point; DESIGN.md §6 predicts
    the gather-to-rank-0 shape link-bound at every N). --frame-exchange
    gather brings every frame to rank 0 (one contiguous buffer, one
    index_select); all_to_all keeps F frames per rank in flight (weak
    scaling); none = independent whole frames. A step runs as four stages on
    four streams — render, RGB8 packing, collective, de-interleave — so the
    exchange of step i overlaps the render of step i+1 and the packing and
    assembly of its neighbours (double-buffered), and a step costs its
    longest stage rather than their sum. The line also carries
    `independent_frames` (every rank renders F whole frames of its own, no
    collective) and `verified`: the assembled frames of the last step equal
    the assembling rank's own whole-frame render byte for byte.

config3 at N=1 (3840x2160 / 64 spheres / depth 2): a step is
F frames of the animated loop (--frames, default: the views one queued
launch holds for this scene, every view's frame constants beside the scene
in LDS: 7),
rendered in one rt_render_batch launch whose wave tiles are taken
view after view from the queues, so the launch's tail is paid once per F
frames; `single_frame` is the same frames one per launch.

config3 at N>1 and config4 (7680x4320 / 256 spheres / depth 4 row-tiled across
the GPUs with an RCCL gather): a step is ONE frame. N=1 renders it whole
(float4; config 4's scene leaves LDS for one view per launch). N>1: the frame's
interleaved 8-row blocks are dealt round-robin to the ranks (rt_render_shard,
packed float3 shards), one RCCL gather brings the shards to rank 0 and rank 0
de-interleaves them into the frame (frame.gather_frame); the gather of step i
overlaps the render of step i+1. Strong scaling, verified like config2.

config5 (a Monte-Carlo extension the reference does not have): one step =
the 1920x1080 frame at 1024 jittered samples per pixel, samples sharded over
the N ranks, partial sums combined with one RCCL all-reduce: strong scaling;
value = samples/s.

At N>1 consecutive steps alternate between two render streams and two output
buffers (--streams 2), so a launch's last waves overlap the next step's
launch, as consecutive frames of a pipelined frame loop; every frame is still
rendered in full. At N=1 the line's value and roofline are one stream's
(each launch alone on the GPU); the two-stream rate is the `pipelined` field.

value = primary rays (samples) of the step / step time (max over ranks), Mrays/s.
roofline = the render kernel against the HBM-write roofline: bytes stored per
launch (16 B per pixel for a float4 frame, 12 for float3 shards, 4 for RGBA8)
/ average kernel time from HIP events on the launch stream (one pair around
the back-to-back launches of the timed region at N=1; at N>1 a pair around
every step's launches on its stream, which includes any overlap with the
neighbouring step's launch). Its `traffic` and `valu`
come from the committed rocprofv3 PMC summary of the same sources
(profiles/pmc_<workload>_latest.json), else they say which build they belong to.
cpu_baseline = the reference's own shader on Mesa llvmpipe (oracle/_ref) on the
host cores, median of 3 dispatches, plus a 1-thread sample and the other
configs' row subsets (oracle/cpu_baseline.py, child process, N=1 only).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2|config3|config4|config5|shipped]

--gpus N > 1 runs under torch.distributed.run (one rank per GPU, as the driver
launches it) or on its own: with WORLD_SIZE unset, this process starts the N
ranks itself (launch_ranks) before anything touches the GPU.

shipped (the reference app's own workload, main.cpp:17-19, raytrace_compute.glsl:
22, :261-321): 1280x720, the shipped scene moving with time, depth 0; a step
is F = 256 frames of the animated loop, frame k with its own scene, in one
rt_render_batch_scenes launch; `draw_loop` is the draw() shape with the
scene update on the host (rt_scene_update + one synchronous render per frame).
"""
import argparse
import datetime
import json
import os
import re
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
    # the reference app's own workload: its window (main.cpp:17-19), its
    # shipped scene (4 oriented boxes + 1 sphere, moving with `time`,
    # raytrace_compute.glsl:261-321) and MAX_RAYTRACE_DEPTH 0 (:22); every
    # frame of the animated loop has its own scene (rt_render_batch_scenes)
    "shipped": dict(width=1280, height=720, spheres=1, boxes=4, depth=0,
                    text="shipped: 1280x720, the reference's own animated scene (4 oriented boxes + 1 sphere, "
                         "every frame its own scene at t = k/60 s), max_depth 0 (main.cpp:17-19, "
                         "raytrace_compute.glsl:22, :261-321)"),
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
    ap.add_argument("--frames", type=int, default=None,
                    help="config2 (default 256) and config3 at N=1 (default: the views one queued launch holds, 7): "
                         "animated frames per step, up to "
                         "256 per rt_render_batch call (SURVEY.md §8(f) row 3); with all_to_all / none: frames per GPU")
    ap.add_argument("--frame-exchange", choices=["spread", "gather", "all_to_all", "none"], default="spread",
                    help="config2 at N>1: spread (default) = every frame of the step row-tiled over the ranks, "
                         "frame k assembled on rank k %% N by one all-to-all (rank 0's xGMI ingress 1/N of the "
                         "step); gather = every frame gathered to rank 0; all_to_all = F frames per rank in "
                         "flight, frame k gathered to rank k (weak scaling); none = every rank renders whole "
                         "frames of its own")
    ap.add_argument("--surface", choices=["auto", "rgba32f", "rgba8"], default="auto",
                    help="config2 surface: auto = float4 at N=1, the GL_RGBA8 surface for row-tiled frames at N>1")
    ap.add_argument("--no-independent", action="store_true",
                    help="config2 at N>1: skip the secondary independent-frames measurement")
    ap.add_argument("--no-verify", action="store_true",
                    help="N>1: skip checking the assembled frames against rank 0's whole-frame render")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--collective-timeout", type=float, default=300.0,
                    help="N>1: seconds after which a collective that cannot complete fails the rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=25.0,
                    help="approximate budget of the llvmpipe baseline samples")
    ap.add_argument("--streams", type=int, choices=[1, 2], default=None,
                    help="render streams the steps alternate between (with as many output buffers): 2 lets a "
                         "launch's last waves overlap the next step's launch; default 1 at N=1 (each launch alone "
                         "on the GPU, so its HIP-event duration is the kernel's, as rocprofv3 reports it; the "
                         "two-stream rate is the secondary `pipelined` field) and 2 at N>1")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="N=1: skip the secondary two-stream (`pipelined`) measurement")
    ap.add_argument("--no-rgba8", action="store_true",
                    help="config2 at N=1: skip the same-surface (GL_RGBA8) measurement")
    ap.add_argument("--no-general", action="store_true",
                    help="config2, shipped at N=1: skip the general-kernel (scene shapes off) measurement")
    ap.add_argument("--no-single-frame", action="store_true",
                    help="config2, config3 at N=1: skip the one-frame-per-launch measurement (profiling runs: one launch shape)")
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


def source_id(build):
    """The source hash of a build string (rt_version(): '... (gfx950, src
    <hash>, git <rev>)'), or the whole string for older builds."""
    m = re.search(r"src ([0-9a-f]+)", build or "")
    return m.group(1) if m else (build or "")


def pmc_latest(workload, frames_per_launch, build):
    """The committed PMC summary of the render kernel for this workload and
    launch shape at N=1 (profiles/pmc_<workload>_latest.json, written by
    tools/pmc_summary.py; config2 also profiles/pmc_latest.json), or {}.
    A summary profiled on a build with other sources is returned only as
    {"stale_build": ...}: its counters are not this kernel's."""
    for name in ("pmc_%s_latest.json" % workload, "pmc_latest.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if (d.get("workload") == workload and d.get("n_gpus", 1) == 1
                and d.get("frames_per_launch", 1) == frames_per_launch):
            if source_id(d.get("build")) != source_id(build):
                return {"stale_build": d.get("build"), "profile": name}
            return d
    return {}


def valu_bound(pmc, kernel_ms):
    """The bound the kernel actually sits against: VALU issue.
    Peak = one wave64 VALU instruction per 2 cycles per SIMD (SIMD-32),
    1024 SIMDs at 2.4 GHz (/opt/skills/guides/MI355X_MICROARCH.md)."""
    if "stale_build" in pmc:
        return {"stale_build": pmc["stale_build"], "note": "profiles/%s was measured on other sources; "
                "no VALU figure for this build" % pmc["profile"]}
    insts = pmc.get("sq_insts_valu_per_launch")
    if not insts or kernel_ms <= 0:
        return None
    peak = 1024 * 2.4e9 / 2 / 1e12  # T wave-instructions / s
    achieved = insts / (kernel_ms * 1e-3) / 1e12
    out = {"wave_insts_per_launch": insts, "achieved": round(achieved, 4), "peak": round(peak, 4),
           "unit": "T wave-instr/s", "frac": round(achieved / peak, 4),
           "source": "SQ_INSTS_VALU from profiles/pmc_*_latest.json (rocprofv3 --pmc pass of this build: %s)"
                     % pmc.get("build", "?")}
    if pmc.get("scratch_bytes_per_lane") is not None:
        out["scratch_bytes_per_lane"] = pmc["scratch_bytes_per_lane"]
    if pmc.get("effective_clock_ghz"):
        clk = pmc["effective_clock_ghz"]
        out["frac_at_measured_clock"] = round(insts * 2 / (1024 * clk * 1e9 * kernel_ms * 1e-3), 4)
        out["measured_clock_ghz"] = round(clk, 3)
    return out


def check_traffic(pmc, stored):
    """A launch stores every pixel once, so a PMC summary whose WRITE_SIZE is
    below the launch's stored bytes belongs to another launch shape (round
    5's mixed-shape averages): returns (pmc or {}, the check record or None)."""
    if pmc.get("write_bytes_per_launch") is None:
        return pmc, None
    rec = {"write_bytes_per_launch": pmc["write_bytes_per_launch"], "stored_bytes_per_launch": stored,
           "ok": pmc["write_bytes_per_launch"] >= 0.99 * stored}
    return (pmc if rec["ok"] else {}), rec


LINK_GBPS = (50.0, 100.0)  # per-direction rate RCCL may reach on one xGMI link (nominal ≈150 GB/s)


def shard_timing():
    """The committed per-rank timings of the N-GPU steps, measured on one GPU
    (tools/shard_timing.py --out profiles/shard_timing_latest.json), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "shard_timing_latest.json")) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def predict_step_ms(wl, world, mode, frames, rows_max, height, link_bytes_max, assembled_frames, spp_share=1.0):
    """DESIGN.md §6's model of an N>1 step: render, RGB8 packing, collective
    and de-interleave run on four streams, so a step takes its longest stage:
    max(render, pack, busiest link bytes / B, assembly), for B in LINK_GBPS.
    Render, packing and assembly times come from the committed one-GPU shard
    timings (scaled to this step's frames; an N absent from them scales the
    N=1 render by the shard's rows). Returns a dict, or None without data."""
    st = shard_timing()
    if st is None:
        return None
    recs = {r["n"]: r for r in st["records"] if r["workload"] == ("config2" if wl == "config2" else wl)}
    if wl == "config5":
        recs = {r["n"]: r for r in st["records"] if r["workload"] == "config2"}
    if 1 not in recs:
        return None
    base = recs.get(world)
    scale_f = frames / recs[1]["frames_per_step"]
    if base is not None:
        render = base.get("shard0_two_streams_ms", base["kernel_ms_max"]) * scale_f
        src = "shard timing at N=%d" % world
    else:
        render = recs[1]["kernel_ms_max"] * scale_f * rows_max / height
        src = "N=1 render x rows share (no shard timing at N=%d)" % world
    if wl == "config5":
        # the sample frames of config 2's scene: samples / frames of the N=1 step
        render = recs[1]["kernel_ms_max"] / recs[1]["frames_per_step"] * spp_share
        src = "config-2 frame time x samples of this rank"
    near = base or recs[max(recs)]
    pack = near.get("pack_rgb8_ms", 0.0) * scale_f * (near["n"] / world) if (wl == "config2" and mode in (
        "spread", "gather")) else 0.0
    asm = near.get("assembly_ms", 0.0) * assembled_frames / near["frames_per_step"] if near.get("assembly_ms") else 0.0
    out = {"stages_ms": {"render": round(render, 4), "pack": round(pack, 4), "assembly": round(asm, 4)},
           "busiest_link_bytes": int(link_bytes_max), "render_source": src,
           "model": "max(render, pack, busiest link / B, assembly): four stages on four streams (DESIGN.md §6)",
           "timings": "profiles/shard_timing_latest.json (%s)" % st.get("build", "?")}
    for b in LINK_GBPS:
        link = link_bytes_max / (b * 1e9) * 1e3
        out["ms_per_step_B%d" % int(b)] = round(max(render, pack, link, asm), 4)
        out["bound_B%d" % int(b)] = max([("render", render), ("pack", pack), ("link", link), ("assembly", asm)],
                                        key=lambda kv: kv[1])[0]
    return out


def link_rate(v):
    """A rank's achieved collective rates from [kernel, collective, assembly,
    pack ms, busiest-link bytes, collective bytes]: bytes / the collective's
    HIP-event time (which includes waiting for the slowest peer, so a lower
    bound on what the links carry)."""
    if len(v) < 6 or not v[4] or v[1] <= 0:
        return {}
    return {"link_bytes": int(v[4]), "collective_bytes": int(v[5]),
            "link_GBps": round(v[4] / (v[1] * 1e-3) / 1e9, 3),
            "collective_GBps": round(v[5] / (v[1] * 1e-3) / 1e9, 3)}


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


class Plan:
    """One measured step shape: what a step renders (on the render stream),
    how the shards are packed (pack stream), exchanged (collective stream) and
    assembled (assembly stream): four stages on four streams, so step i's
    exchange overlaps step i+1's render, step i+1's packing and step i-1's
    assembly, and the step takes the longest stage, not their sum."""

    def __init__(self, bufs, render, rays_per_step, px_per_launch, bytes_per_pixel, launches_per_step=1,
                 collective=None, assemble=None, per_launch=True, prepare=None):
        self.bufs = bufs
        self.render = render            # render(buf), asynchronous on the render stream
        self.prepare = prepare          # prepare(slot, src): pack the shards to send (pack stream), or None
        self.collective = collective    # collective(slot, src): on the collective stream after slot's packing
        self.assemble = assemble        # assemble(slot): on the assembly stream after the collective
        self.rays_per_step = rays_per_step
        self.px_per_launch = px_per_launch
        self.bytes_per_pixel = bytes_per_pixel
        self.launches_per_step = launches_per_step
        # one kernel event pair per step (else one pair around the timed region)
        self.per_launch = per_launch or collective is not None
        self.last = None                # assembled output of the last step (assemble's return value)
        # this rank's collective bytes per step: over its busiest peer link
        # (sent or received) and in total (sent + received, other ranks only)
        self.link_bytes = 0
        self.coll_bytes = 0

    def set_link(self, sent, received):
        """sent[p] / received[p]: bytes to / from rank p this step (own rank 0)."""
        self.link_bytes = max([max(a, b) for a, b in zip(sent, received)] + [0])
        self.coll_bytes = sum(sent) + sum(received)


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
    if args.workload == "shipped" and world > 1:
        raise SystemExit("--workload shipped is the reference app's one-GPU frame loop (main.cpp:81-86); "
                         "the multi-GPU shapes are config2-5's")
    device = local % max(1, torch.cuda.device_count())  # (counting devices does not initialise the GPU)
    coll_dev = "cuda"
    if world > 1:
        # a collective that cannot complete (a peer gone, RCCL failing) raises
        # within --collective-timeout; guarded() turns it into a nonzero exit
        # of this rank (an RCCL error aborts the frame)
        timeout = datetime.timedelta(seconds=args.collective_timeout)
        if args.dist_backend == "nccl":
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", device), timeout=timeout)
        else:
            dist.init_process_group(args.dist_backend, timeout=timeout)
            coll_dev = "cpu"
        inject_fault(rank, "init")
        dist.barrier()  # every rank is up before any GPU work
    torch.cuda.set_device(device)

    ctx = rt.Context(device)
    wl = args.workload
    # (config3 at N = 1: F = the views one queued launch holds beside the
    # scene in LDS, found below once the scene exists)
    F = args.frames or (0 if wl == "config3" and world == 1 else 7 if wl == "config3" else 256)
    scenes = None  # shipped: frame k's own scene (the reference's objects at t = k/60 s)
    if wl == "shipped":
        scenes = [rt.Scene(ctx, rt.reference_objects(frame_time(k))) for k in range(F)]
        scene = scenes[0]
    else:
        scene = rt.Scene(ctx, rt.bench_objects(cfg["spheres"], 0))
    if F == 0:  # config3 at N = 1: one queued launch per step
        F = max(k for k in range(1, 65) if rt.batch_launches(ctx, scene, k, DEPTH) == 1)
    ctx.set_timing(False)  # no per-launch markers of the library's own
    # Streams of our own: renders are launched asynchronously on `render_s`
    # (the C-ABI treats a NULL stream — torch's default stream handle is 0 —
    # as "synchronous on the context's stream", like glFinish); the current
    # stream `comm_s` orders the collectives (RCCL runs on its own stream
    # behind it) and the frame assembly.
    render_s = torch.cuda.Stream()
    # N>1 steps render on two streams in turn (step i on render_streams[i % 2],
    # into buffer slot i % 2): step i+1's launch may start while step i's
    # drains (its last waves), as consecutive frames of a pipelined frame
    # loop; the slot's previous exchange must have read the buffer first (the
    # `freed` events). Measured on one MI355X (tools/shard_timing.py,
    # profiles/r04c_shard_timing.log): rank 0's config-2 step at N = 8
    # 56.2 -> 46.0 us, N = 2 185.5 -> 174.9 us.
    render_streams = [render_s, torch.cuda.Stream()]
    cur = {"s": render_s}
    n_streams = {"n": args.streams or (1 if world == 1 else 2)}  # read by the plan builders
    comm_s = torch.cuda.Stream()
    pack_s = torch.cuda.Stream()  # N>1: the shards' RGB8 packing
    asm_s = torch.cuda.Stream()  # N>1: the received frames' de-interleave
    torch.cuda.set_stream(comm_s)
    sh = render_s.cuda_stream
    assert sh, "need a non-default HIP stream"
    mc = wl == "config5"
    batched = wl in ("config2", "shipped") or (wl == "config3" and world == 1)
    extra = {}
    surfaces = {"rgba32f": (rt.abi.RT_OUTPUT_RGBA32F, 4, torch.float32, "float4"),
                "rgb32f": (rt.abi.RT_OUTPUT_RGB32F, 3, torch.float32, "packed float3 (alpha 0 dropped)"),
                "rgba8": (rt.abi.RT_OUTPUT_RGBA8, 1, torch.int32, "GL_RGBA8 surface (4 B per pixel)")}

    def surface(name):
        fmt, ch, dt, text = surfaces[name]
        ctx.set_output(fmt)
        return ch, dt, text

    def render_frames(ptr, j, vs, stream, n_shards=1, shard=0):
        """Frames j, j+1, ... of the step (views vs) in one rt_render_batch
        call; `shipped`: each frame with its own scene (rt_render_batch_scenes)."""
        if scenes is not None:
            rt.render_batch_scenes(ctx, scenes[j:j + len(vs)], ptr, W, H, DEPTH, vs, BLOCK_ROWS, n_shards, shard,
                                   stream=stream)
        else:
            rt.render_batch(ctx, scene, ptr, W, H, DEPTH, vs, BLOCK_ROWS, n_shards, shard, stream=stream)

    def batch_plan(mode, surf):
        """config2: F frames per step (per rank for `none`, all_to_all),
        rendered up to 8 per launch; see the module docstring."""
        ch, dt, _ = surface(surf)
        esize = 4  # bytes per element (float32 / int32)
        if mode == "none" or world == 1:
            # frames [rF, (r+1)F) whole on rank r, launches back to back (with
            # two streams: the steps alternating between two streams and two
            # buffers, step i+1's launch under step i's last waves)
            views = [rt.make_view(None, frame_time(rank * F + k)) for k in range(F)]
            bufs = [torch.zeros(F * H * W * ch, dtype=dt, device="cuda") for _ in range(n_streams["n"])]
            chunks = [(j, views[j:j + rt.abi.RT_MAX_BATCH]) for j in range(0, F, rt.abi.RT_MAX_BATCH)]

            def render(buf):
                for j, vs in chunks:
                    render_frames(buf.data_ptr() + esize * j * H * W * ch, j, vs, cur["s"].cuda_stream)
            # (two streams: an event pair around every step's launches on its
            # stream, so kernel_ms is each launch's own duration, overlap
            # included, as rocprofv3 reports it; the step time is shorter)
            # kernel launches per step: the library splits a deep batch into
            # queued launches of as many views as fit beside the scene in LDS
            launches = sum(rt.batch_launches(ctx, scene, len(vs), DEPTH) for _, vs in chunks)
            return Plan(bufs, render, world * F * W * H, W * H * F // launches, esize * ch, launches,
                        per_launch=n_streams["n"] == 2)
        if mode == "spread":
            return spread_plan()
        n_frames = F if mode == "gather" else world * F
        views = [rt.make_view(None, frame_time(k)) for k in range(n_frames)]
        rows_mine = rt.shard_rows(H, BLOCK_ROWS, world, rank)
        if mode == "gather":
            elems = frame.flat_shard_elems(n_frames, H, W, BLOCK_ROWS, world, ch)
        else:
            elems = n_frames * rows_mine * W * ch
        bufs = [torch.zeros(elems, dtype=dt, device="cuda") for _ in range(2)]
        chunks = [(j, views[j:j + rt.abi.RT_MAX_BATCH]) for j in range(0, n_frames, rt.abi.RT_MAX_BATCH)]
        frame_elems = rows_mine * W * ch

        def render(buf):
            for j, vs in chunks:
                rt.render_batch(ctx, scene, buf.data_ptr() + esize * j * frame_elems, W, H, DEPTH, vs,
                                BLOCK_ROWS, world, rank, stream=cur["s"].cuda_stream)
        if mode == "gather" and surf == "rgba8":
            # GL_RGBA8 shards sent without their alpha byte (always 0, :404):
            # 3 B per pixel through rank 0's xGMI ingress instead of 4; the
            # gather lands in one contiguous buffer per slot, and one
            # index_select de-interleaves all F frames (packed RGB8, alpha 0)
            px = frame.flat_shard_elems(n_frames, H, W, BLOCK_ROWS, world, 1)
            sends = [torch.empty(px * 3, dtype=torch.uint8, device=coll_dev) for _ in bufs]
            bigs = ([torch.empty(world * px * 3, dtype=torch.uint8, device=coll_dev) for _ in bufs]
                    if rank == 0 else None)
            idx = torch.as_tensor(frame.contiguous_assembly_rows(n_frames, H, BLOCK_ROWS, world), device=coll_dev)

            def prepare(slot, src):
                frame.pack_rgb8(src, sends[slot])

            def collective(slot, src):
                dist.gather(sends[slot], [bigs[slot][r * px * 3:(r + 1) * px * 3] for r in range(world)]
                            if rank == 0 else None, dst=0)  # RCCL: every shard to rank 0

            def assemble(slot):
                if rank == 0:
                    return frame.assemble_contiguous(bigs[slot], n_frames, H, W, 3, idx)
                return None
        elif mode == "gather":
            prepare = None
            glists = ([[torch.empty(elems, dtype=dt, device=coll_dev) for _ in range(world)] for _ in bufs]
                      if rank == 0 else None)
            perm = torch.as_tensor(frame.assembly_permutation(H, BLOCK_ROWS, world), device=coll_dev)

            def collective(slot, src):
                dist.gather(src, glists[slot] if rank == 0 else None, dst=0)  # RCCL: every shard to rank 0

            def assemble(slot):
                if rank == 0:  # de-interleave the row blocks into the F frames
                    return frame.assemble(glists[slot], n_frames, H, W, BLOCK_ROWS, channels=ch, perm=perm)
                return None
        else:
            prepare = None
            in_splits, out_splits = frame.exchange_splits(H, W, BLOCK_ROWS, world, rank, channels=ch,
                                                          frames_per_rank=F)
            recv = [torch.empty(sum(out_splits), dtype=dt, device=coll_dev) for _ in bufs]
            idx = torch.as_tensor(frame.assembly_rows(H, BLOCK_ROWS, world, F), device=coll_dev)

            def collective(slot, src):
                dist.all_to_all_single(recv[slot], src, out_splits, in_splits)  # frames [kF, (k+1)F) -> rank k

            def assemble(slot):
                return frame.assemble_frames(recv[slot], F, H, W, BLOCK_ROWS, world, channels=ch, idx=idx)
        plan = Plan(bufs, render, n_frames * W * H, W * rows_mine * n_frames // len(chunks), esize * ch,
                    len(chunks), collective, assemble, prepare=prepare)
        if mode == "gather":
            # every rank's equal-size flat shard buffer to rank 0 (RGB8: 3 B
            # per pixel; else the surface's elements)
            per = 3 * frame.flat_shard_elems(n_frames, H, W, BLOCK_ROWS, world, 1) if surf == "rgba8" else esize * elems
            plan.set_link([per if (rank != 0 and p == 0) else 0 for p in range(world)],
                          [per if (rank == 0 and p != 0) else 0 for p in range(world)])
        else:
            plan.set_link([esize * v if p != rank else 0 for p, v in enumerate(in_splits)],
                          [esize * v if p != rank else 0 for p, v in enumerate(out_splits)])
        return plan

    def spread_plan():
        """config2 at N>1, --frame-exchange spread (the default): the step's F
        frames row-tiled over all ranks, frame k assembled on rank k % N by
        one all-to-all of RGB8 shards; rank r renders its row blocks of all F
        frames, grouped by destination (frame.spread_plan)."""
        surface("rgba8")
        order, ins, outs, mine = frame.spread_plan(H, W, BLOCK_ROWS, world, rank, F, channels=3)
        views = [rt.make_view(None, frame_time(k)) for k in order]
        rows_mine = rt.shard_rows(H, BLOCK_ROWS, world, rank)
        frame_elems = rows_mine * W
        bufs = [torch.zeros(F * frame_elems, dtype=torch.int32, device="cuda") for _ in range(2)]
        sends = [torch.empty(F * frame_elems * 3, dtype=torch.uint8, device=coll_dev) for _ in bufs]
        recvs = [torch.empty(sum(outs), dtype=torch.uint8, device=coll_dev) for _ in bufs]
        idx = torch.as_tensor(frame.assembly_rows(H, BLOCK_ROWS, world, len(mine)), device=coll_dev)
        chunks = [(j, views[j:j + rt.abi.RT_MAX_BATCH]) for j in range(0, F, rt.abi.RT_MAX_BATCH)]

        def render(buf):
            for j, vs in chunks:
                rt.render_batch(ctx, scene, buf.data_ptr() + 4 * j * frame_elems, W, H, DEPTH, vs,
                                BLOCK_ROWS, world, rank, stream=cur["s"].cuda_stream)

        def prepare(slot, src):
            frame.pack_rgb8(src, sends[slot])

        def collective(slot, src):
            dist.all_to_all_single(recvs[slot], sends[slot], outs, ins)  # RCCL: frame k -> rank k % N

        def assemble(slot):
            if not mine:
                return None
            return frame.assemble_frames(recvs[slot], len(mine), H, W, BLOCK_ROWS, world, channels=3, idx=idx)
        plan = Plan(bufs, render, F * W * H, frame_elems * F // len(chunks), 4, len(chunks), collective, assemble,
                    prepare=prepare)
        plan.mine = mine
        plan.set_link([v if p != rank else 0 for p, v in enumerate(ins)],
                      [v if p != rank else 0 for p, v in enumerate(outs)])
        return plan

    def frame_plan():
        """config3 / config4: one frame per step, whole at N=1, row-tiled +
        gathered at N>1."""
        ch, dt, _ = surface("rgba32f" if world == 1 else "rgb32f")
        view = rt.make_view(None, 0.0)
        if world == 1:
            # (with two streams: consecutive steps on two streams and buffers,
            # the next frame's launch under this one's last wave tiles)
            bufs = [torch.zeros(H * W * 4, dtype=dt, device="cuda") for _ in range(n_streams["n"])]
            return Plan(bufs, lambda buf: rt.render_device(ctx, scene, buf.data_ptr(), W, H, DEPTH, view=view,
                                                           stream=cur["s"].cuda_stream), W * H, W * H, 16)
        rows_mine = rt.shard_rows(H, BLOCK_ROWS, world, rank)
        elems = frame.flat_shard_elems(1, H, W, BLOCK_ROWS, world, ch)
        bufs = [torch.zeros(elems, dtype=dt, device="cuda") for _ in range(2)]
        # the gather lands in one contiguous buffer per slot; one index_select
        # de-interleaves the frame
        bigs = ([torch.empty(world * elems, dtype=dt, device=coll_dev) for _ in bufs] if rank == 0 else None)
        idx = torch.as_tensor(frame.contiguous_assembly_rows(1, H, BLOCK_ROWS, world), device=coll_dev)

        def collective(slot, src):
            dist.gather(src, [bigs[slot][r * elems:(r + 1) * elems] for r in range(world)] if rank == 0 else None,
                        dst=0)  # RCCL: every shard to rank 0

        def assemble(slot):
            if rank == 0:
                return frame.assemble_contiguous(bigs[slot], 1, H, W, ch, idx)
            return None
        plan = Plan(bufs, lambda buf: rt.render_shard(ctx, scene, buf.data_ptr(), W, H, DEPTH, BLOCK_ROWS, world,
                                                      rank, view=view, stream=cur["s"].cuda_stream),
                    W * H, W * rows_mine, 4 * ch, 1, collective, assemble)
        per = 4 * elems  # every rank's flat float3 shard buffer to rank 0
        plan.set_link([per if (rank != 0 and p == 0) else 0 for p in range(world)],
                      [per if (rank == 0 and p != 0) else 0 for p in range(world)])
        return plan

    def measure(plan, steps, warmup):
        """Warm-up, then `steps` timed steps between barriers; returns the
        elapsed seconds (max over ranks) and mean kernel / collective /
        assembly ms of every rank."""
        kt = Timer(torch, steps if plan.per_launch else 1)
        pt = Timer(torch, steps)  # packing on pack_s
        ct = Timer(torch, steps)  # collective on comm_s
        at = Timer(torch, steps)  # assembly on asm_s (Monte-Carlo: the scaling, on comm_s)
        rendered = [torch.cuda.Event() for _ in plan.bufs]
        freed = [None] * len(plan.bufs)  # event: bufs[slot] has been read (by the packing or the collective)
        sent = [None] * len(plan.bufs)  # event: the collective has read the slot's send buffer
        assembled = [None] * len(plan.bufs)  # event: the assembly has read the slot's receive buffer

        # one-stream plans launch on render_s, where their event pair is
        # recorded (a previous two-stream measurement may have left cur["s"]
        # on the other render stream)
        cur["s"] = render_s

        def step(timed, it):
            if not plan.per_launch:  # frames rendered in place, launches back to back (one stream)
                plan.render(plan.bufs[0])
                return
            slot = it % len(plan.bufs)
            # (--streams 1 at N>1: both buffer slots on render_s)
            rs = render_streams[slot % n_streams["n"]]
            cur["s"] = rs
            if freed[slot] is not None:
                rs.wait_event(freed[slot])  # step it-2's packing (or collective) has read bufs[slot]
            if timed:
                kt.start(it, rs)
            plan.render(plan.bufs[slot])
            if timed:
                kt.stop(it, rs)
            if plan.collective is None:
                return
            rendered[slot].record(rs)
            if plan.prepare is not None:
                # packing on its own stream: the render buffer is free again
                # once packed, and the collective stream carries only the
                # transfer
                pack_s.wait_event(rendered[slot])
                if sent[slot] is not None:
                    pack_s.wait_event(sent[slot])  # step it-2's collective has read the send buffer
                with torch.cuda.stream(pack_s):
                    src = plan.bufs[slot] if coll_dev == "cuda" else plan.bufs[slot].cpu()
                    if timed:
                        pt.start(it, pack_s)
                    plan.prepare(slot, src)
                    if timed:
                        pt.stop(it, pack_s)
                packed = torch.cuda.Event()
                packed.record(pack_s)
                freed[slot] = packed
                comm_s.wait_event(packed)
            else:
                comm_s.wait_event(rendered[slot])
                src = plan.bufs[slot] if coll_dev == "cuda" else plan.bufs[slot].cpu()
            if assembled[slot] is not None:
                comm_s.wait_event(assembled[slot])  # step it-2's assembly has read the receive buffer
            if timed and it == 0:
                inject_fault(rank, "step")
            if timed:
                ct.start(it, comm_s)
            plan.collective(slot, src)
            if timed:
                ct.stop(it, comm_s)
            done = torch.cuda.Event()
            done.record(comm_s)
            sent[slot] = done
            if plan.prepare is None:
                freed[slot] = done
            # assembly on its own stream, beside the next step's transfer
            asm_s.wait_event(done)
            with torch.cuda.stream(asm_s):
                if timed:
                    at.start(it, asm_s)
                plan.last = plan.assemble(slot)
                if timed:
                    at.stop(it, asm_s)
            read = torch.cuda.Event()
            read.record(asm_s)
            assembled[slot] = read

        def mc_step(timed, it):
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
            else:
                total = accum
            if timed:
                ct.stop(it, comm_s)
                at.start(it, comm_s)
            if rank == 0:
                total.mul_(1.0 / spp)  # the estimate: mean over all samples
            if timed:
                at.stop(it, comm_s)

        run = mc_step if mc else step
        for i in range(warmup):
            run(False, i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if not plan.per_launch:
            kt.start(0, cur["s"])
        for it in range(steps):
            run(True, it)
        if not plan.per_launch:
            kt.stop(0, cur["s"])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kernel_ms = ([m / plan.launches_per_step for m in kt.ms()] if plan.per_launch else
                     [kt.ms()[0] / (steps * plan.launches_per_step)])
        kms = float(np.mean(kernel_ms))
        exchanged = mc or plan.collective is not None
        cms = float(np.mean(ct.ms())) if exchanged else 0.0
        ams = float(np.mean(at.ms())) if exchanged else 0.0
        pms = float(np.mean(pt.ms())) if plan.prepare is not None else 0.0
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            mine = torch.tensor([kms, cms, ams, pms, plan.link_bytes, plan.coll_bytes], dtype=torch.float64,
                                device=coll_dev)
            every = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(every, mine)
            per_rank = [[round(float(v), 5) for v in e.cpu().tolist()] for e in every]
        else:
            per_rank = [[round(kms, 5), round(cms, 5), round(ams, 5), round(pms, 5), 0, 0]]
        return elapsed, kms, per_rank

    def verify(plan, n_frames, times, ch, dt, frames_of_rank=None):
        """The assembled frames of the last step against this rank's own
        whole-frame renders in the same surface format, byte for byte; the
        mismatch count is summed over the ranks that assemble."""
        bad, px = 0, 0
        if plan.last is not None:
            # (empty: the render overwrites every pixel; torch's allocation
            # and any fill would be queued on comm_s, which nothing orders
            # before the synchronous render on the context's own stream)
            ref = torch.empty((n_frames, H, W, ch), dtype=dt, device="cuda")
            torch.cuda.synchronize()
            views = [rt.make_view(None, t) for t in times]
            for j in range(0, n_frames, rt.abi.RT_MAX_BATCH):
                rt.render_batch(ctx, scene, ref[j].data_ptr(), W, H, DEPTH, views[j:j + rt.abi.RT_MAX_BATCH])
            torch.cuda.synchronize()
            if plan.last.dtype == torch.uint8:  # RGB8 frames (the alpha byte dropped): against the RGBA8 texels
                texels = ref.view(torch.uint8).reshape(n_frames, H, W, 4)
                got = plan.last.reshape(n_frames, H, W, 3).to(ref.device)
                diff = (got != texels[..., :3]).any(-1) | (texels[..., 3] != 0)
            else:
                got = plan.last.reshape(n_frames, H, W, ch)
                diff = (got.to(ref.device) != ref).reshape(n_frames * H * W, ch).any(-1)
            bad, px = int(diff.reshape(-1).sum().item()), n_frames * H * W
        if world > 1:
            t = torch.tensor([bad, px], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t)
            bad, px = int(t[0].item()), int(t[1].item())
        return {"frames_checked": px // (H * W), "pixels": px, "mismatched_pixels": bad, "bit_exact": bad == 0,
                "against": "the assembling rank's own whole-frame render of the same frames, same surface"}

    def verify_n1(buf, frames, ch, dt):
        torch.cuda.synchronize()
        one = torch.empty((H, W, ch), dtype=dt, device="cuda")
        got_all = buf.view(dt).reshape(-1, H, W, ch)
        bad = 0
        for k in frames:
            render_frames(one.data_ptr(), k, [rt.make_view(None, frame_time(k))], None)  # synchronous
            diff = got_all[k].view(torch.int32) != one.view(torch.int32)
            bad += int(diff.reshape(H * W, -1).any(-1).sum().item())
        return {"frames_checked": frames, "pixels": len(frames) * H * W, "mismatched_pixels": bad,
                "bit_exact": bad == 0,
                "against": "single-frame renders of the same views (one view per launch, the draw() shape), "
                           "compared as bytes"}

    def verify_bands(buf, bands, accumulate=False):
        """N=1, one frame per step (configs 4 and 5): rows of the last timed
        step's frame — config 5: of its accumulator, after the 1/spp scaling
        — against a render of those rows alone (a launch of its own shape: a
        tiled launch of the band instead of the frame's queued one; the
        band's pixels accumulated by a call of their own), compared as bytes
        (raytrace_compute.glsl:404)."""
        torch.cuda.synchronize()
        got = buf.view(torch.int32).reshape(H, W, 4)
        v0 = rt.make_view(None, 0.0)
        bad = 0
        for r0, r1 in bands:
            band = torch.zeros((r1 - r0, W, 4), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            if accumulate:
                rt.render_accumulate(ctx, scene, band.data_ptr(), W, H, DEPTH, spp_mine, sample0, seed=0, view=v0,
                                     rows=(r0, r1))  # synchronous
                band.mul_(1.0 / spp)
            else:
                rt.render_device(ctx, scene, band.data_ptr(), W, H, DEPTH, view=v0, rows=(r0, r1))  # synchronous
            torch.cuda.synchronize()
            bad += int((got[r0:r1] != band.view(torch.int32)).any(-1).sum().item())
        px = sum(r1 - r0 for r0, r1 in bands) * W
        return {"rows": [list(b) for b in bands], "pixels": px, "mismatched_pixels": bad, "bit_exact": bad == 0,
                "against": ("the same rows' samples accumulated by a call of their own (rows only), scaled by "
                            "1/spp" if accumulate else "a render of the same rows alone (rt_render rows, a tiled "
                            "launch of the band)") + ", compared as bytes"}

    view = None
    if batched:
        mode = args.frame_exchange if world > 1 else "none"
        surf = args.surface if args.surface != "auto" else ("rgba8" if world > 1 and mode != "none" else "rgba32f")
        if mode == "spread":
            surf = "rgba8"  # (the exchange packs GL_RGBA8 texels to RGB8)
        plan = batch_plan(mode, surf)
    elif mc:
        view = rt.make_view(None, 0.0)
        spp = cfg["spp"]
        spp_mine = spp // world + (1 if rank < spp % world else 0)
        sample0 = rank * (spp // world) + min(rank, spp % world)
        accum = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        plan = Plan([accum], None, spp * W * H, W * H, 16)
        if world > 1:
            # a ring all-reduce moves 2 (N-1)/N of the buffer over each link
            # in each direction (RCCL's choice of algorithm may differ)
            ring = int(2 * (world - 1) / world * H * W * 16)
            nxt, prv = (rank + 1) % world, (rank - 1) % world
            plan.set_link([ring if p == nxt else 0 for p in range(world)],
                          [ring if p == prv else 0 for p in range(world)])
    else:
        plan = frame_plan()

    elapsed, avg_kernel_ms, per_rank = measure(plan, args.steps, args.warmup)
    verified = None
    if batched and world == 1 and not args.no_verify:
        # N=1: frames of the last timed step (the first, middle and last of
        # the F) against single renders of the same views — one view per
        # launch, the draw() shape (main.cpp:228-238), a kernel instance of
        # its own — byte for byte (raytrace_compute.glsl:404)
        last = plan.bufs[(args.steps - 1) % len(plan.bufs) if plan.per_launch else 0]
        verified = verify_n1(last, sorted({0, (F - 1) // 2, F - 1}), surfaces[surf][1], surfaces[surf][2])
    elif world == 1 and not args.no_verify and not mc:
        # config 4 (config 3 at N=1 is batched): two 8-row bands of the last timed frame
        verified = verify_bands(plan.bufs[(args.steps - 1) % len(plan.bufs)],
                                [(H // 2, H // 2 + BLOCK_ROWS), (3 * H // 4, 3 * H // 4 + BLOCK_ROWS)])
    elif world == 1 and not args.no_verify and mc:
        # config 5: two 2-row bands of the last timed step's estimate
        verified = verify_bands(accum, [(H // 2 - 2, H // 2), (1000 * H // 1080, 1000 * H // 1080 + 2)],
                                accumulate=True)
    if world > 1 and not args.no_verify and not mc:
        if batched and mode == "gather":
            verified = verify(plan, F, [frame_time(k) for k in range(F)], surfaces[surf][1], surfaces[surf][2])
        elif batched and mode == "spread":
            verified = verify(plan, len(plan.mine), [frame_time(k) for k in plan.mine], surfaces["rgba8"][1],
                              surfaces["rgba8"][2])
        elif batched and mode == "all_to_all":
            verified = verify(plan, F, [frame_time(rank * F + k) for k in range(F)], surfaces[surf][1],
                              surfaces[surf][2])
        elif not batched:
            ch, dt, _ = surfaces["rgb32f"][1:]
            ctx.set_output(rt.abi.RT_OUTPUT_RGB32F)
            verified = verify(plan, 1, [0.0], ch, dt)
    if batched and world > 1 and mode != "none" and not args.no_independent:
        # secondary: every rank renders F whole frames of its own, no collective
        ind = batch_plan("none", "rgba32f")
        e2, k2, r2 = measure(ind, args.steps, args.warmup)
        extra["independent_frames"] = {
            "value": round(ind.rays_per_step * args.steps / e2 / 1e6, 3), "unit": "Mrays/s",
            "ms_per_step": round(e2 / args.steps * 1e3, 5), "frames_per_step": world * F, "frames_per_gpu": F,
            "scaling": "weak", "output": "float4 frames",
            "parallelism": "whole frames x%d (rank r renders frames [rF, (r+1)F) of the animated loop), "
                           "no collective" % world,
            "kernel_ms_per_rank": [v[0] for v in r2]}
        del ind
    if batched and world == 1 and rank == 0 and not args.no_single_frame:
        # one frame per launch (the shape of the reference's draw(),
        # main.cpp:210-238): K launches back to back, one event pair
        n1 = max(20, args.steps)
        one = torch.empty(H * W * 4, dtype=torch.float32, device="cuda")
        two = [one, torch.empty_like(one)]
        views1 = [rt.make_view(None, frame_time(k)) for k in range(F)]
        s2 = [render_s, render_streams[1]]

        def one_stream():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(render_s)
            for k in range(n1):
                render_frames(one.data_ptr(), k % F, [views1[k % F]], sh)
            e1.record(render_s)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / n1 * 1e3

        def two_streams():
            # the same launches alternating between two streams and two
            # output buffers (a draw loop whose output image is
            # double-buffered): frame k+1's launch may fill the CUs that
            # frame k's last waves leave idle
            e2, e3 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e2.record(render_s)
            s2[1].wait_event(e2)
            for k in range(n1):
                render_frames(two[k % 2].data_ptr(), k % F, [views1[k % F]], s2[k % 2].cuda_stream)
            render_s.wait_stream(s2[1])
            e3.record(render_s)
            torch.cuda.synchronize()
            return e2.elapsed_time(e3) / n1 * 1e3
        # both shapes warmed on both streams, then 3 interleaved repeats each
        # (the chip's clock drifts with load): medians and spreads
        for k in range(4):
            render_frames(two[k % 2].data_ptr(), k % F, [views1[k % F]], s2[k % 2].cuda_stream)
        torch.cuda.synchronize()
        ones, twos = [], []
        for _ in range(3):
            ones.append(one_stream())
            twos.append(two_streams())
        us, us2 = float(np.median(ones)), float(np.median(twos))
        extra["single_frame"] = {"frames_per_launch": 1, "us_per_frame": round(us, 3), "frames": "the step's F",
                                 "value": round(W * H / us, 3), "unit": "Mrays/s",
                                 "repeats_us": [round(v, 3) for v in ones],
                                 "roofline_frac": round(W * H * 16 / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
                                 "two_streams": {"us_per_frame": round(us2, 3), "value": round(W * H / us2, 3),
                                                 "repeats_us": [round(v, 3) for v in twos],
                                                 "note": "the same launches alternating between two streams "
                                                         "and two output buffers; median of 3 repeats "
                                                         "interleaved with the one-stream ones"}}
        del two
    if wl == "shipped" and rank == 0 and not args.no_single_frame:
        # the reference's draw() as a drop-in caller runs it (main.cpp:210-238,
        # INTEGRATION.md): per frame, the scene moved to the frame's time on
        # the host (rt_scene_update: objects, transforms, shadow masks, upload)
        # and one synchronous render (NULL stream, the glFinish of :238); wall
        # clock per frame, host work included
        live = rt.Scene(ctx, rt.reference_objects(0.0))
        one_d = torch.empty(H * W * 4, dtype=torch.float32, device="cuda")
        n_d = max(20, args.steps)
        torch.cuda.synchronize()

        def draw(k):
            t = frame_time(k)
            live.update(rt.reference_objects(t))
            rt.render_batch(ctx, live, one_d.data_ptr(), W, H, DEPTH, [rt.make_view(None, t)])  # synchronous
        for k in range(3):
            draw(k)
        loops, hosts = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            for k in range(n_d):
                draw(k)
            loops.append((time.perf_counter() - t0) / n_d * 1e6)
            t0 = time.perf_counter()
            for k in range(n_d):
                live.update(rt.reference_objects(frame_time(k)))
            hosts.append((time.perf_counter() - t0) / n_d * 1e6)
        us = float(np.median(loops))
        extra["draw_loop"] = {"us_per_frame": round(us, 3), "value": round(W * H / us, 3), "unit": "Mrays/s",
                              "scene_update_us": round(float(np.median(hosts)), 3),
                              "repeats_us": [round(v, 3) for v in loops],
                              "note": "per frame: Scene.update(rt_reference_objects(t)) + one synchronous "
                                      "render (NULL stream), wall clock, median of 3 repeats; scene_update_us "
                                      "is the update alone (host build + upload)"}
        live.close()
        del one_d
    if world == 1 and not mc and n_streams["n"] == 1 and not args.no_pipelined:
        # the same steps alternating between two render streams and buffers:
        # a launch's last waves overlap the next step's launch (consecutive
        # frames of a pipelined frame loop; every frame rendered in full).
        # Its per-launch event spans include that overlap, so this rate
        # carries no roofline of its own.
        n_streams["n"] = 2
        pp = batch_plan("none", "rgba32f") if batched else frame_plan()
        ep, _, _ = measure(pp, args.steps, args.warmup)
        extra["pipelined"] = {"value": round(pp.rays_per_step * args.steps / ep / 1e6, 3), "unit": "Mrays/s",
                              "ms_per_step": round(ep / args.steps * 1e3, 5), "render_streams": 2,
                              "note": "consecutive steps on two alternating streams and buffers"}
        n_streams["n"] = 1
        del pp
    if batched and wl in ("config2", "shipped") and world == 1 and rank == 0 and not args.no_rgba8:
        # the same F frames into the GL_RGBA8 surface the row-tiled N>1
        # steps write (main.cpp:223): the same-surface point of the 1..8-GPU
        # curve, with its 4-B and its float4-equivalent roofline
        r8 = batch_plan("none", "rgba8")
        e8, k8, _ = measure(r8, args.steps, args.warmup)
        px8 = r8.px_per_launch
        extra["rgba8_surface"] = {
            "value": round(r8.rays_per_step * args.steps / e8 / 1e6, 3), "unit": "Mrays/s",
            "ms_per_step": round(e8 / args.steps * 1e3, 5), "kernel_ms": round(k8, 5),
            "frames_per_launch": px8 // (W * H), "output": "GL_RGBA8 surface (4 B per pixel), whole frames",
            "roofline_frac": round(px8 * 4 / (k8 * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "roofline_frac_float4_equivalent": round(px8 * 16 / (k8 * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
        surface("rgba32f")
        del r8
    if batched and wl in ("config2", "shipped") and world == 1 and rank == 0 and not args.no_general:
        # the same F frames through the general depth-0 kernel (the scene's
        # features read at run time, RT_OPT_SCENE_SHAPES off): what a scene
        # outside the compiled shapes pays per primary ray (DESIGN.md §3,
        # "Scene shapes"); frame 0 compared with the shaped kernel's frame 0
        gp = batch_plan("none", "rgba32f")
        ctx.set_scene_shapes(False)
        try:
            eg, kg, _ = measure(gp, args.steps, args.warmup)
            torch.cuda.synchronize()
            gen0 = gp.bufs[0][: W * H * 4].clone()
        finally:
            ctx.set_scene_shapes(True)
        gp.render(gp.bufs[0])
        torch.cuda.synchronize()
        same0 = bool(torch.equal(gen0, gp.bufs[0][: W * H * 4]))
        fr = gp.px_per_launch // (W * H)
        extra["general_kernel"] = {
            "value": round(gp.rays_per_step * args.steps / eg / 1e6, 3), "unit": "Mrays/s",
            "kernel_ms": round(kg, 5), "us_per_frame": round(kg / fr * 1e3, 3), "frames_per_launch": fr,
            "vs_shaped": round(kg / avg_kernel_ms, 4), "frame0_identical_to_shaped": same0,
            "note": "RT_OPT_SCENE_SHAPES off: the general depth-0 kernel on the same frames"}
        if not same0:
            raise SystemExit("general kernel: frame 0 differs from the shaped kernel's")
        del gp, gen0
    ms_per_step = elapsed / args.steps * 1e3
    value = plan.rays_per_step * args.steps / elapsed / 1e6
    # time basis of the roofline: the kernel's own launch duration when each
    # launch has the GPU alone (one render stream); with two overlapping
    # render streams a launch's event span includes its neighbour's run, so
    # the basis is the step: this GPU's stored bytes per step / step time
    # (a lower bound on the kernel's rate; at one stream the two agree)
    overlapped = n_streams["n"] == 2 and not mc
    basis_ms = ms_per_step / plan.launches_per_step if overlapped else avg_kernel_ms
    achieved = plan.px_per_launch * plan.bytes_per_pixel / (basis_ms * 1e-3) / 1e9
    # the same pixels at 16 B each (the float4 frame of the N=1 line): one
    # roofline scale for every point of a 1..8-GPU curve whatever its surface
    achieved_f4 = plan.px_per_launch * 16 / (basis_ms * 1e-3) / 1e9
    fpl = plan.px_per_launch // (W * H) if batched and world == 1 else 1
    build = rt.lib().rt_version().decode()
    pmc = pmc_latest(wl, fpl, build) if world == 1 else {}
    # a launch stores every pixel once: a PMC summary that writes fewer
    # bytes than the launch stores belongs to another launch shape (round 5's
    # mixed-shape average), so none of its figures is this launch's
    stored = plan.px_per_launch * plan.bytes_per_pixel
    pmc, traffic_check = check_traffic(pmc, stored)
    if traffic_check is not None and not traffic_check["ok"]:
        sys.stderr.write("bench.py: profiles/pmc_%s_latest.json writes %.4g B per launch, below the %.4g B the "
                         "launch stores: not this launch shape's counters; traffic and valu left out\n"
                         % (wl, traffic_check["write_bytes_per_launch"], stored))
    traffic = pmc.get("hbm_bytes_per_launch")
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(wl, args.cpu_seconds)
        workload = {"workload": cfg["text"], "width": W, "height": H, "spheres": cfg["spheres"], "max_depth": DEPTH}
        collective = "none"
        if batched and (world == 1 or mode == "none"):
            workload.update({"frames_per_step": world * F, "frames_per_gpu": F, "frames_per_launch": fpl,
                             "output": "float4 frames",
                             "parallelism": ("whole frames x%d (rank r renders frames [rF, (r+1)F) of the "
                                             "animated loop), no collective" % world) if world > 1
                                            else "single GPU"})
        elif batched and mode == "spread":
            collective = "all_to_all_single (frame k of the step to rank k % N; RGB8 shards)"
            workload.update({"frames_per_step": F, "frames_per_launch": min(F, rt.abi.RT_MAX_BATCH),
                             "row_block": BLOCK_ROWS,
                             "output": "GL_RGBA8 surface (4 B per pixel) shards, sent as RGB8 (the constant "
                                       "alpha byte dropped); frame k assembled on rank k % N",
                             "parallelism": "every frame row-tiled x%d in interleaved %d-row blocks + one RCCL "
                                            "all-to-all per step assembling frame k on rank k %% %d, overlapped "
                                            "with the next render" % (world, BLOCK_ROWS, world)})
        elif batched and mode == "gather":
            collective = "gather to rank 0 (one per step: the shards of all F frames)"
            workload.update({"frames_per_step": F, "frames_per_launch": min(F, rt.abi.RT_MAX_BATCH),
                             "row_block": BLOCK_ROWS,
                             "output": (surfaces[surf][3] + (" shards, sent as RGB8 (the constant alpha byte dropped), "
                                                             "gathered to rank 0" if surf == "rgba8" else
                                                             " shards gathered to rank 0")),
                             "parallelism": "every frame row-tiled x%d in interleaved %d-row blocks + RCCL gather "
                                            "to rank 0, de-interleaved there, overlapped with the next render"
                                            % (world, BLOCK_ROWS)})
        elif batched:
            collective = "all_to_all_single (N frame gathers at once)"
            workload.update({"frames_per_step": world * F, "frames_per_gpu": F,
                             "frames_per_launch": min(world * F, rt.abi.RT_MAX_BATCH), "row_block": BLOCK_ROWS,
                             "output": surfaces[surf][3] + " shards exchanged",
                             "parallelism": "row-tiles x%d + RCCL all-to-all frame exchange (frame k gathered "
                                            "to rank k), overlapped with the next render" % world})
        elif mc:
            collective = "all_reduce of the sample sums" if world > 1 else "none"
            workload.update({"spp": cfg["spp"],
                             "parallelism": ("samples x%d + RCCL all-reduce" % world) if world > 1 else "single GPU"})
        else:
            collective = "gather to rank 0" if world > 1 else "none"
            workload.update({"frames_per_step": 1, "row_block": BLOCK_ROWS,
                             "output": "float4 frame" if world == 1 else
                             "float3 shards (alpha 0 dropped) gathered to rank 0, de-interleaved there",
                             "parallelism": ("interleaved 8-row blocks x%d + RCCL gather to rank 0, overlapped "
                                             "with the next render" % world) if world > 1 else "single GPU"})
        strong = not (batched and world > 1 and mode in ("none", "all_to_all"))  # (spread, gather: F frames per step)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene, SURVEY.md §8(d) %s)" % wl,
            "config": workload,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "frac_float4_equivalent": round(achieved_f4 / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "kernel_ms": round(avg_kernel_ms, 5),
                         "time_basis": ("step time per launch (two overlapping render streams: a launch's own "
                                        "event span includes its neighbour's run)" if overlapped else
                                        "kernel launch duration (HIP events, one render stream)"),
                         "bytes_per_launch": stored,
                         "traffic_check": traffic_check,
                         "valu": valu_bound(pmc, avg_kernel_ms)},
            "timing": {"per_rank": [dict({"rank": r, "kernel_ms": v[0], "collective_ms": v[1], "assembly_ms": v[2],
                                          "pack_ms": v[3]}, **link_rate(v)) for r, v in enumerate(per_rank)],
                       "collective": collective,
                       "render_streams": n_streams["n"],
                       "note": "HIP events, means over the timed steps: kernel on the render stream, packing, "
                               "collective and assembly each on a stream of its own (the Monte-Carlo "
                               "all-reduce and scaling on the collective stream)"},
            "cpu_baseline": cpu,
            "build": build,
        }
        if "stale_build" in pmc:
            line["roofline"]["traffic_note"] = "profiles/%s is of other sources (%s)" % (pmc["profile"],
                                                                                      pmc["stale_build"])
        if verified is not None:
            line["verified"] = verified
        if world > 1:
            # DESIGN.md §6's prediction of this step from the committed
            # one-GPU shard timings, beside the measured ms_per_step
            if batched:
                m = mode
                assembled = {"spread": -(-F // world), "gather": F, "all_to_all": F}.get(mode, 0)
                frames_step = F if mode in ("spread", "gather") else world * F
                # frames whose shards (whole frames for `none`) a rank renders per step
                frames_rank = world * F if mode == "all_to_all" else F
            else:
                m, assembled, frames_step, frames_rank = ("allreduce" if mc else "gather"), (0 if mc else 1), 1, 1
            pred = predict_step_ms(wl, world, m, frames_rank, rt.shard_rows(H, BLOCK_ROWS, world, 0), H,
                                   max(v[4] for v in per_rank), assembled,
                                   spp_share=(-(-cfg.get("spp", 1) // world)) if mc else 1.0)
            if pred is not None and not (batched and mode == "none"):
                pred["measured_ms_per_step"] = round(ms_per_step, 5)
                pred["frames_per_step"] = frames_step
                line["predicted_ms_per_step"] = pred
        line.update(extra)
        print(json.dumps(line), flush=True)
    for sc in scenes or [scene]:
        sc.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if verified is not None and not verified["bit_exact"]:
        raise SystemExit("assembled frames differ from the whole-frame render on %d pixels"
                         % verified["mismatched_pixels"])

EXIT_RANK_FAILED = 17  # this rank's step failed (a collective, a render, a check)
EXIT_FAULT_INJECTED = 3


def inject_fault(rank, stage):
    """Test hook (tests/test_bench.py): RT_BENCH_FAULT='<rank>:<stage>' makes
    that rank exit at once, without a word to its peers, at `stage` ('init':
    after joining the group; 'step': before its first timed collective) — a
    rank that dies mid-frame."""
    spec = os.environ.get("RT_BENCH_FAULT", "")
    if spec and spec == "%d:%s" % (rank, stage):
        sys.stderr.write("bench.py rank %d: injected fault at %s, exiting\n" % (rank, stage))
        sys.stderr.flush()
        os._exit(EXIT_FAULT_INJECTED)


def guarded(fn):
    """Run the bench; at N>1 any failure (a collective that errors or times
    out because a peer is gone, an RCCL error, a failed render) aborts this
    rank's frame with a message and a nonzero exit, without the process
    group's teardown, which would wait for the missing peer."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return fn()
    try:
        return fn()
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 — every failure ends the rank
        sys.stderr.write("bench.py rank %s: step failed, aborting the frame: %s: %s\n"
                         % (os.environ.get("RANK", "?"), type(e).__name__, str(e)[:500]))
        sys.stderr.flush()
        os._exit(EXIT_RANK_FAILED)


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None, grace_s=30.0):
    """`bench.py --gpus N` with no launcher (WORLD_SIZE unset): start N fresh
    worker processes of this script, one per GPU, with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as torch.distributed.run sets
    them — before anything touches the GPU (this parent never imports torch
    and never re-execs itself) — and relay their output (they share this
    process's stdout and stderr; rank 0 alone prints the JSON line). Returns
    0 when every rank exits 0, else the first failing rank's exit status
    (1 for a signal); once a rank has failed, the others (left waiting in a
    collective for the missing peer) get `grace_s` seconds and are then
    killed. A SIGTERM to this parent is passed on to the ranks."""
    import signal
    script = script or os.path.abspath(__file__)
    port = free_port()
    procs = []

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        raise SystemExit(143)
    old = signal.signal(signal.SIGTERM, stop)
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL (the host driver's only kind)
            procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
        rc = [None] * n
        deadline = None
        while any(c is None for c in rc):
            for i, p in enumerate(procs):
                if rc[i] is None:
                    rc[i] = p.poll()
            if deadline is None and any(c not in (None, 0) for c in rc):
                deadline = time.monotonic() + grace_s
            if deadline is not None and time.monotonic() > deadline:
                for i, p in enumerate(procs):
                    if rc[i] is None:
                        p.kill()
                        rc[i] = p.wait()
                break
            time.sleep(0.05)
    finally:
        for p in procs:  # (only after an exception here: every rank has exited otherwise)
            if p.poll() is None:
                p.kill()
                p.wait()
        signal.signal(signal.SIGTERM, old)
    bad = [(r, c) for r, c in enumerate(rc) if c != 0]
    if bad:
        sys.stderr.write("bench.py: %d of %d ranks failed (rank, exit status): %s\n" % (len(bad), n, bad))
        first = bad[0][1]
        return first if first > 0 else 1
    return 0


if __name__ == "__main__":
    if "WORLD_SIZE" not in os.environ:
        _n = parse().gpus
        if _n > 1:  # no launcher: this process starts the N ranks itself
            sys.exit(launch_ranks(_n, sys.argv[1:]))
    guarded(main)
