"""Per-wave timeline of one depth-0 launch (development probe).

    python tools/phase_trace.py [CONFIG] [BUILD]

BUILD (default "phase") is an _ab build made with
`tools/ablate.sh flags phase "-DRT_PHASE_TRACE -DRT_WPE0=8"` (the probe
costs two VGPRs; RT_WPE0=8 keeps the product build's 8 waves/SIMD): lane 0 of every wave records
the 100 MHz real-time clock at kernel entry (0), after the prologue barrier
(1), before and after the closest-hit scan (2, 3), after the collision record
(4), at light 1's shadow query (5), after the light loop (6) and after the
store (7). Prints where a frame's time goes: wave start (ramp) and end (tail)
spreads, mean phase durations, and how wave durations grow with start time.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import openglraytracer_amd as rt
from oracle import scenes

cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
name = sys.argv[2] if len(sys.argv) > 2 else "phase"
L = C.CDLL(os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so"))
vp, i = C.c_void_p, C.c_int
L.rt_create.argtypes = [i, vp]
L.rt_scene_create.argtypes = [vp, vp, i, vp, i, vp, i, vp]
L.rt_render_view.argtypes = [vp, vp, vp, i, i, i, i, i, vp, i, vp]
L.rt_debug_phase_read.argtypes = [vp, C.c_size_t]
L.rt_debug_occupancy.argtypes = [C.c_size_t]
for lds in (0, 4096, 8192, 16384, 20480, 24576):
    print("occupancy query (work-groups/CU) at %6d B LDS: %d" % (lds, L.rt_debug_occupancy(lds)))
ctx = C.c_void_p()
assert L.rt_create(0, C.byref(ctx)) == 0
build, w, h, depth = scenes.CONFIGS[cfg]
assert depth == 0, "the probe instruments the depth-0 tiled path"
objs, mats, lights = build(), rt.reference_materials(), rt.reference_lights()
sc = C.c_void_p()
assert L.rt_scene_create(ctx, (rt.Object * len(objs))(*objs), len(objs), (rt.Material * len(mats))(*mats), len(mats),
                         (rt.Light * len(lights))(*lights), len(lights), C.byref(sc)) == 0
view = rt.make_view(None, 0.0)
out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
stream = torch.cuda.Stream()
waves = ((w + 15) // 16) * ((h + 15) // 16) * 4
for _ in range(5):  # warm; the last launch's record is read
    assert L.rt_debug_phase_clear() == 0
    torch.cuda.synchronize()
    assert L.rt_render_view(ctx, sc, C.byref(view), w, h, 0, 0, h, C.c_void_p(out.data_ptr()), 1,
                            C.c_void_p(stream.cuda_stream)) == 0
    torch.cuda.synchronize()
buf = np.zeros(waves * 16, dtype=np.uint64)
assert L.rt_debug_phase_read(buf.ctypes.data, buf.nbytes) == 0
R = buf.reshape(waves, 16).astype(np.int64)
T = R[:, :8].copy()
hw, xcc = R[:, 8], R[:, 9]
print('waves with phase 2 unset:', int((T[:, 2] == 0).sum()), ' phase 7 unset:', int((T[:, 7] == 0).sum()))
us = 0.01  # 100 MHz ticks
t0 = T[:, 0].min()
T = (T - t0) * us
start, end = T[:, 0], T[:, 7]
span = end.max()
print(f"{cfg}: {waves} waves, first start 0, last end {span:.2f} us")
for q in (0, 10, 25, 50, 75, 90, 99, 100):
    print(f"  start p{q:<3d} {np.percentile(start, q):7.2f} us   end p{q:<3d} {np.percentile(end, q):7.2f} us")
names = ["prologue", "raygen/tile", "closest", "resolve", "phong to light1 shadow", "light1 shadow..loop end",
         "combine+store"]
has5 = T[:, 5] > 0
d = np.diff(T, axis=1)
print("mean phase durations (us):")
for k, nm in enumerate(names):
    col = d[:, k]
    if k in (4, 5):
        col = col[has5]
    if col.size == 0:
        continue
    print(f"  {k}->{k + 1} {nm:26s} {col.mean():7.2f}  p90 {np.percentile(col, 90):7.2f}")
dur = end - start
print(f"wave duration mean {dur.mean():.2f} us, p10 {np.percentile(dur, 10):.2f}, p90 {np.percentile(dur, 90):.2f}")
for lo in range(0, int(span) + 5, 5):
    m = (start >= lo) & (start < lo + 5)
    if m.any():
        live = ((start <= lo + 2.5) & (end > lo + 2.5)).sum()
        print(f"  start in [{lo:3d},{lo + 5:3d}) us: {m.sum():6d} waves, mean duration {dur[m].mean():6.2f} us, "
              f"waves live at {lo + 2.5:.1f} us: {live}")
# per-XCD finishing (work-group id round-robins over the 8 XCDs)
wgid = np.arange(waves) // 4
xcd_end = [end[wgid % 8 == x].max() for x in range(8)]
print("last end per XCD (us):", " ".join(f"{e:.1f}" for e in xcd_end))

cu = (hw >> 8) & 0xF
sh = (hw >> 12) & 1
se = (hw >> 13) & 0x7
simd = (hw >> 4) & 0x3
xc = xcc & 0xF
print("distinct XCCs", np.unique(xc).size, "SEs", np.unique(se).size, "SH", np.unique(sh).size, "CU ids", np.unique(cu).size)
key = (xc * 8 + se) * 32 + sh * 16 + cu
ucu = np.unique(key)
print("distinct CUs used:", ucu.size)
# peak concurrent waves per CU: sweep over the first 5 us
first = start < 5.0
cnt = np.bincount(key[first], minlength=key.max() + 1)
cnt = cnt[cnt > 0]
print("waves started in the first 5 us per CU: min %d max %d mean %.2f" % (cnt.min(), cnt.max(), cnt.mean()))

P = (R[:, 10:14] - t0) * us
print("prologue split (us): entry->raygen %.2f, raygen->blob in LDS %.2f, ->frame_setup done %.2f, barrier wait %.2f"
      % tuple(np.diff(np.concatenate([T[:, :1], P], axis=1), axis=1).mean(axis=0)))
Q = (R[:, 14:16] - t0) * us
print("entry split (us): entry->own pixel (kernargs) %.2f, ->camera ray done %.2f, ->phase 10 %.2f"
      % ((Q[:, 0] - T[:, 0]).mean(), (Q[:, 1] - Q[:, 0]).mean(), (P[:, 0] - Q[:, 1]).mean()))
w = np.arange(waves) % 4
for k in range(4):
    m = w == k
    print("  wave %d of its group: setup done %.2f, barrier left %.2f (from entry)" % (k, (P[m, 2] - T[m, 0]).mean(), (P[m, 3] - T[m, 0]).mean()))

# ---- work-group order and the launch's tail (round 4) -------------------
# Per work-group duration (first wave start to last wave end) by tile, and a
# list-scheduling replay of the 8 x 256 work-group slots (8 resident per CU)
# with the measured durations in three dispatch orders: the hardware's
# (blockIdx: row-major tiles), a static centre-out order, and longest first
# (the bound a perfect cost predictor would reach). A permuted order only
# pays if the measured durations are predictable from the tile position.
import heapq  # noqa: E402

_, W0, H0, _ = scenes.CONFIGS[cfg]
gx, gy = (W0 + 15) // 16, (H0 + 15) // 16
wg_start = start.reshape(-1, 4).min(1)
wg_end = end.reshape(-1, 4).max(1)
wg_dur = wg_end - wg_start
slots = 8 * 256


def replay(order):
    heap = [0.0] * slots
    last = 0.0
    for k in order:
        t = heapq.heappop(heap) + wg_dur[k]
        last = max(last, t)
        heapq.heappush(heap, t)
    return last


ty, tx = np.divmod(np.arange(gx * gy), gx)
centre = np.argsort(np.hypot((tx + 0.5) / gx - 0.5, ((ty + 0.5) / gy - 0.5) * gy / gx), kind="stable")
print("work-groups %d, duration mean %.2f us p10 %.2f p90 %.2f; measured last end %.2f us" %
      (gx * gy, wg_dur.mean(), np.percentile(wg_dur, 10), np.percentile(wg_dur, 90), span))
print("replay (us): ideal %.2f  blockIdx order %.2f  centre-out %.2f  longest-first %.2f" %
      (wg_dur.sum() / slots, replay(np.arange(gx * gy)), replay(centre), replay(np.argsort(-wg_dur, kind="stable"))))
rows = wg_dur.reshape(gy, gx)
print("mean work-group duration by tile-row band (top to bottom, 8 bands):",
      " ".join("%.2f" % b.mean() for b in np.array_split(rows, 8, axis=0)))
print("mean work-group duration by tile-column band (8 bands):",
      " ".join("%.2f" % b.mean() for b in np.array_split(rows, 8, axis=1)))
dump = os.environ.get("PHASE_DUMP")
if dump:
    np.savez_compressed(dump, start=start, end=end, gx=gx, gy=gy)
