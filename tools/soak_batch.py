"""Batch parity soak (development probe, run on the GPU box): seeded random
scenes (tests/test_gpu_parity.py random_scene) at depth >= 2, rendered as
multi-view batches large enough for the queued distribution (every view's
frame constants beside the scene in LDS, even launches when a batch exceeds
what one launch holds), whole frames and row-tiled shards, with host and
device frame constants — every frame against its own single render, bit
for bit. The single renders are pinned to the oracle by tools/soak.py and
the GPU tests, so this extends the oracle's parity to the batched launches.

    python tools/soak_batch.py FIRST_SEED N [W H VIEWS]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402  (HIP runtime first)
import openglraytracer_amd as rt  # noqa: E402
from openglraytracer_amd import frame  # noqa: E402
from test_gpu_parity import random_scene  # noqa: E402

first, n = int(sys.argv[1]), int(sys.argv[2])
W, H, V = (int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (800, 456, 5)
ctx = rt.Context(0)
bad, frames, depths = [], 0, {}
for seed in range(first, first + n):
    objs, mats, lights, t, depth, _, _ = random_scene(seed)
    depth = max(depth, 2)
    n_views = 2 + seed % (V - 1)  # 2..V views
    n_shards = 1 + seed % 3
    views = [rt.make_view(None, t + 0.15 * k) for k in range(n_views)]
    sc = rt.Scene(ctx, objs, materials=mats, lights=lights)
    try:
        singles = [rt.render(ctx, sc, W, H, depth, view=v) for v in views]
        for consts in (True, False):
            ctx.set_host_frame_consts(consts)
            for shard in range(n_shards):
                rows = frame.shard_row_ids(H, 8, n_shards, shard)
                out = torch.empty((n_views, len(rows), W, 4), dtype=torch.float32, device="cuda")
                torch.cuda.synchronize()
                rt.render_batch(ctx, sc, out.data_ptr(), W, H, depth, views, 8, n_shards, shard)
                got = out.cpu().numpy()
                for k in range(n_views):
                    frames += 1
                    ref = singles[k][rows]
                    if not np.array_equal(got[k], ref, equal_nan=True):
                        diff = int((~((got[k] == ref) | (np.isnan(got[k]) & np.isnan(ref)))).any(-1).sum())
                        bad.append((seed, len(objs), depth, n_views, n_shards, shard, consts, k, diff))
                        print("MISMATCH seed %d: %d objects, depth %d, %d views, %d shards (shard %d), host "
                              "consts %s, view %d: %d pixels differ" % bad[-1], flush=True)
    finally:
        ctx.set_host_frame_consts(True)
        sc.close()
    depths[depth] = depths.get(depth, 0) + 1
    if (seed - first + 1) % 25 == 0:
        print("%d scenes, %d frames compared, %d mismatching" % (seed - first + 1, frames, len(bad)), flush=True)
print("batch soak: %d random scenes (seeds %d..%d) at %dx%d, 2..%d views per batch, 1..3 shards, depths %s: "
      "%d frames (or shards) compared, %d mismatching"
      % (n, first, first + n - 1, W, H, V, dict(sorted(depths.items())), frames, len(bad)), flush=True)
sys.exit(1 if bad else 0)
