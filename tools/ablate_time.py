"""Time one build from tools/ablate.sh (timing only):
    python tools/ablate_time.py NAME [config2 config3 ...]
Prints the median per-launch kernel time (HIP events on the context stream)
and the back-to-back rate (one event pair around REPS launches), plus a hash
of the frame so variants that must be bit-identical can be compared."""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401  (HIP runtime first)
import openglraytracer_amd as rt
from oracle import scenes

name = sys.argv[1]
cfgs = sys.argv[2:] or ["config2"]
if name != "main":  # "main": the in-tree library
    rt.LIB_PATH = os.path.join(ROOT, "_ab", name, "libopenglraytracer_amd.so")
ctx = rt.Context(0)
view = rt.make_view(None, 0.0)
stream = torch.cuda.Stream()  # non-default: the C-ABI runs NULL-stream calls synchronously
torch.cuda.set_stream(stream)
for cfg in cfgs:
    build, w, h, depth = scenes.CONFIGS[cfg]
    sc = rt.Scene(ctx, build())
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    reps = 30 if cfg in ("config1", "config2") else 5
    ms = []
    for i in range(reps + 3):
        rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view)
        if i >= 3:
            ms.append(ctx.last_kernel_ms())
    digest = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for i in range(reps):
        rt.render_device(ctx, sc, out.data_ptr(), w, h, depth, view=view, stream=stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    b2b = e0.elapsed_time(e1) / reps
    print("%-10s %s kernel ms median %.4f min %.4f | back-to-back %.4f | frame %s" % (
        name, cfg, np.median(ms), np.min(ms), b2b, digest), flush=True)
    sc.close()
