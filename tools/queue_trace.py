"""Per-wave timeline of one queued (depth >= 2) launch (development probe).

    python tools/queue_trace.py [CONFIG] [N_VIEWS] [BUILD]

BUILD (default "phase") is an _ab build made with
`tools/ablate.sh flags phase "-DRT_PHASE_TRACE"`. Lane 0 of every resident
wave of the queued grid records the 100 MHz real-time clock at kernel entry
(phase 0), after the prologue barrier (13), when its first wave tile starts
(1) and when it leaves the tile loop (7). Prints where the launch's time
goes: the start ramp, the prologue, the tail (wave ends) and the wave-time
lost to each, i.e. what a neighbouring launch on a second stream can fill.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import openglraytracer_amd as rt  # noqa: E402
from oracle import scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
n_views = int(sys.argv[2]) if len(sys.argv) > 2 else 1
name = sys.argv[3] if len(sys.argv) > 3 else "phase"
L = C.CDLL(os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so"))
vp, i = C.c_void_p, C.c_int
L.rt_create.argtypes = [i, vp]
L.rt_scene_create.argtypes = [vp, vp, i, vp, i, vp, i, vp]
L.rt_render_batch.argtypes = [vp, vp, vp, i, i, i, i, i, i, i, vp, vp]
L.rt_debug_phase_read.argtypes = [vp, C.c_size_t]
ctx = C.c_void_p()
assert L.rt_create(0, C.byref(ctx)) == 0
build, w, h, depth = scenes.CONFIGS[cfg]
assert depth >= 2, "the probe reads the queued (depth >= 2) grid"
objs, mats, lights = build(), rt.reference_materials(), rt.reference_lights()
sc = C.c_void_p()
assert L.rt_scene_create(ctx, (rt.Object * len(objs))(*objs), len(objs), (rt.Material * len(mats))(*mats), len(mats),
                         (rt.Light * len(lights))(*lights), len(lights), C.byref(sc)) == 0
views = (rt.View * n_views)(*[rt.make_view(None, k / 60.0) for k in range(n_views)])
out = torch.empty((n_views, h, w, 4), dtype=torch.float32, device="cuda")
stream = torch.cuda.Stream()
slots = 6 * 4 * 256  # resident waves of the queued grid at 6 waves per SIMD (upper bound)
for _ in range(3):  # warm; the last launch's record is read
    assert L.rt_debug_phase_clear() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    assert L.rt_render_batch(ctx, sc, views, n_views, w, h, depth, 0, 0, 0, C.c_void_p(out.data_ptr()),
                             C.c_void_p(stream.cuda_stream)) == 0
    e1.record(stream)
    torch.cuda.synchronize()
buf = np.zeros(slots * 16, dtype=np.uint64)
assert L.rt_debug_phase_read(buf.ctypes.data, buf.nbytes) == 0
R = buf.reshape(slots, 16).astype(np.int64)
live = R[:, 0] > 0
R = R[live]
us = 0.01  # 100 MHz ticks
t0 = R[:, 0].min()
T = (R[:, :16] - t0) * us
start, after_barrier, first_tile, end = T[:, 0], T[:, 13], T[:, 1], T[:, 7]
span = end.max()
print(f"{cfg}, {n_views} view(s) in one launch: {live.sum()} waves; HIP events {e0.elapsed_time(e1) * 1e3:.1f} us, "
      f"first start -> last end {span:.1f} us")
for q in (0, 1, 10, 50, 90, 99, 100):
    print(f"  p{q:<3d} start {np.percentile(start, q):8.2f}  prologue done {np.percentile(after_barrier, q):8.2f}  "
          f"end {np.percentile(end, q):8.2f} us")
ramp = first_tile.mean()
tail = (span - end).mean()
print(f"mean wave-time before its first tile {ramp:.2f} us (start {start.mean():.2f}, prologue "
      f"{(after_barrier - start).mean():.2f}); mean idle after its last tile {tail:.2f} us; "
      f"both as a share of the span: {(ramp + tail) / span:.3f}")
print(f"per frame: span / views {span / n_views:.1f} us, lost wave-time per frame {(ramp + tail) / n_views:.1f} us")
# per queue (global wave g serves queue g % 32): when its last wave ends —
# the spread between queues is what sharing the queues' work at the end
# (stealing) could recover; the spread inside a queue is tile granularity
g = np.nonzero(live)[0]
q = g % 32
qend = np.array([end[q == k].max() for k in range(32)])
qmean = np.array([end[q == k].mean() for k in range(32)])
print("queue last end (us): min %.1f median %.1f max %.1f; queue mean wave end: min %.1f max %.1f"
      % (qend.min(), np.median(qend), qend.max(), qmean.min(), qmean.max()))
busy = (end - first_tile).sum()
print("busy wave-time / waves = %.1f us (the span if every wave ended together); span %.1f us"
      % (busy / len(end) + first_tile.mean(), span))
