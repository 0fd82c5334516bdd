"""Wave-round quantisation of the Monte-Carlo launch (development probe).

    python tools/mc_rounds.py [SPP]

Every wave of rt_render_accumulate renders its 64 pixels' SPP samples in
order, so all waves of a launch last about as long and the launch runs in
rounds of the resident waves. Times the config-5 frame (1920 wide) at heights
whose wave count is a whole number of rounds of the 6 x 1024 resident waves
(1024 rows: 5 rounds) and at 1080 rows (5.31 rounds): if the rounds quantise,
1080 rows cost 6/5 of 1024 rows, not 1080/1024.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import openglraytracer_amd as rt  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
ctx = rt.Context(0)
ctx.set_timing(False)
scene = rt.Scene(ctx, rt.bench_objects(16, 0))
s = torch.cuda.Stream()
W = 1920
res = {}
for H in (1024, 1080, 1088, 1216, 1232):
    acc = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(2):
        rt.render_accumulate(ctx, scene, acc.data_ptr(), W, H, 0, spp, stream=s.cuda_stream)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(3):
            rt.render_accumulate(ctx, scene, acc.data_ptr(), W, H, 0, spp, stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 3)
    t = float(np.median(ts))
    waves = (W // 16) * ((H + 15) // 16) * 4
    res[H] = t
    print("%dx%d, %d spp: %d waves = %.2f rounds of 6144: %.3f ms per launch, %.3f us per sample-frame-row-pixel-M"
          % (W, H, spp, waves, waves / 6144, t, t * 1e3 / spp / (W * H) * 1e6), flush=True)
print("time ratio 1080/1024 rows %.3f (pixels 1.055, rounds 6/5 = 1.2)" % (res[1080] / res[1024]))
