"""Interleaved A/B timing of several builds in ONE process (development probe).

    python tools/ab.py CONFIG[,CONFIG...] BUILD [BUILD ...]

BUILD is a directory under _ab (tools/ablate.sh) or "main" for the
in-tree library, optionally with context options (main:1=0 = RT_OPT_CULLING
off). CONFIG is config1..config4, "shipped" (the reference's own scene at
1280x720, depth 0), "config2x8" (8 animated frames per launch,
rt_render_batch) or "config5" (Monte-Carlo, 16 jittered samples per launch).
Every build gets its own context and scene; each round times every build once
— REPS/2 untimed launches, then one event pair around REPS back-to-back
launches on a non-default stream, about 60 ms of GPU work, so the clock is the
sustained one the bench sees rather than a short burst's — rounds interleaved
so clock drift hits all builds alike. Prints the median and min per-frame
(per-sample) kernel time and a hash of the frame.
"""
import ctypes as C
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import openglraytracer_amd as rt
from oracle import scenes

cfgs = sys.argv[1].split(",")
builds = sys.argv[2:]
ROUNDS = 7


def load(spec):
    # BUILD[:OPTION=VALUE...]: context options (rt_context_set) after the
    # build name, e.g. main:1=0 (RT_OPT_CULLING off)
    name, *opts = spec.split(":")
    path = rt.LIB_PATH if name == "main" else os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so")
    L = C.CDLL(path)
    vp, i = C.c_void_p, C.c_int
    L.rt_create.argtypes = [i, vp]
    L.rt_scene_create.argtypes = [vp, vp, i, vp, i, vp, i, vp]
    L.rt_scene_destroy.argtypes = [vp]
    L.rt_context_set.argtypes = [vp, i, i]
    L.rt_render_view.argtypes = [vp, vp, vp, i, i, i, i, i, vp, i, vp]
    L.rt_render_batch.argtypes = [vp, vp, vp, i, i, i, i, i, i, i, vp, vp]
    L.rt_render_accumulate.argtypes = [vp, vp, vp, i, i, i, i, i, C.c_uint32, i, i, i, vp, vp]
    ctx = C.c_void_p()
    assert L.rt_create(0, C.byref(ctx)) == 0
    L.rt_context_set(ctx, rt.abi.RT_OPT_TIMING, 0)
    for o in opts:
        k, v = o.split("=")
        assert L.rt_context_set(ctx, int(k), int(v)) == 0, spec
    return L, ctx


libs = {b: load(b) for b in builds}
# the register / spill gate (tools/resources.py): every build's registers and
# scratch head the log; a variant whose scratch grows (or occupancy drops) at
# any render kernel against the first build is not timed unless
# AB_ALLOW_SPILL=1 says its prediction accounts for it
sys.path.insert(0, os.path.join(ROOT, "tools"))
import resources  # noqa: E402
if os.environ.get("AB_PREDICTION"):
    # the change each variant is expected to make, stated before it is timed
    print("# prediction: %s" % os.environ["AB_PREDICTION"], flush=True)
for b in builds:
    print(resources.report(b.split(":")[0])[1], flush=True)
for b in builds[1:]:
    bad = resources.gate(builds[0].split(":")[0], b.split(":")[0])
    for k, x, y in bad:
        print("# GATE %s vs %s, %s: scratch %d -> %d B/lane, %d -> %d waves/SIMD" % (
            b, builds[0], k, x["scratch"], y["scratch"], x["waves_per_simd"], y["waves_per_simd"]), flush=True)
    if bad and os.environ.get("AB_ALLOW_SPILL") != "1":
        sys.exit("register gate: %s spills more than %s (AB_ALLOW_SPILL=1 to time it anyway)" % (b, builds[0]))
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
mats = rt.reference_materials()
lights = rt.reference_lights()
view = rt.make_view(None, 0.0)
for cfg in cfgs:
    # "<config>x<K>": K animated frames (t = k / 60) per launch (rt_render_batch);
    # "config5": Monte-Carlo, 16 jittered samples per launch (rt_render_accumulate)
    batch = int(cfg.split("x")[1]) if "x" in cfg.replace("config", "") else 0
    mc_spp = 16 if cfg == "config5" else 0
    build, w, h, depth = scenes.CONFIGS[cfg.split("x")[0]]
    views = (rt.View * max(batch, 1))(*[rt.make_view(None, k / 60.0) for k in range(max(batch, 1))])
    objs = build()
    if objs is None:  # "shipped": the reference's own scene (at t = 0 for every view)
        objs = rt.reference_objects(0.0)
    oa = (rt.Object * len(objs))(*objs)
    ma = (rt.Material * len(mats))(*mats)
    la = (rt.Light * len(lights))(*lights)
    out = torch.empty((max(batch, 1), h, w, 4), dtype=torch.float32, device="cuda")
    # sustained timing: each timed block is about 60 ms of GPU work (short
    # bursts run at a higher clock than the bench's back-to-back launches)
    est_ms = {"config1": 0.03, "config2": 0.045, "config3": 1.0, "config4": 15.0, "config5": 0.045 * 16,
              "shipped": 0.045}.get(
        cfg.split("x")[0], 1.0) * max(batch, 1)
    reps = max(2, int(round(60.0 / est_ms)))
    state = {}
    for b, (L, ctx) in libs.items():
        sc = C.c_void_p()
        assert L.rt_scene_create(ctx, oa, len(objs), ma, len(mats), la, len(lights), C.byref(sc)) == 0
        state[b] = sc
    times = {b: [] for b in builds}
    digests = {}

    def launch(b):
        L, ctx = libs[b]
        if mc_spp:
            rc = L.rt_render_accumulate(ctx, state[b], C.byref(view), w, h, depth, mc_spp, 0, 0, 1, 0, h,
                                        C.c_void_p(out.data_ptr()), C.c_void_p(stream.cuda_stream))
        elif batch:
            rc = L.rt_render_batch(ctx, state[b], views, batch, w, h, depth, 8, 1, 0, C.c_void_p(out.data_ptr()),
                                   C.c_void_p(stream.cuda_stream))
        else:
            rc = L.rt_render_view(ctx, state[b], C.byref(view), w, h, depth, 0, h, C.c_void_p(out.data_ptr()), 1,
                                  C.c_void_p(stream.cuda_stream))
        assert rc == 0, rc

    for b in builds:  # warm-up + frame hash
        if mc_spp:
            out.zero_()
        launch(b)
        torch.cuda.synchronize()
        digests[b] = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
    for _ in range(ROUNDS):
        for b in builds:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(reps // 2):  # warm to the sustained clock
                launch(b)
            e0.record(stream)
            for _ in range(reps):
                launch(b)
            e1.record(stream)
            torch.cuda.synchronize()
            times[b].append(e0.elapsed_time(e1) / reps)
    for b in builds:
        t = np.array(times[b]) / max(batch, 1, mc_spp)  # per frame (per sample)
        print("%-8s %-10s median %.4f ms  min %.4f ms  frame %s" % (cfg, b, np.median(t), t.min(), digests[b]),
              flush=True)
    for b, (L, ctx) in libs.items():
        L.rt_scene_destroy(state[b])
