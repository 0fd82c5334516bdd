"""Per-launch time of config-2 shard launches (development probe).

    RT_LIB=path/to/libopenglraytracer_amd.so python tools/shard_probe.py

rt_render_batch of 64 animated 1080p frames into the GL_RGBA8 surface:
whole frames, then shard 0 (and 1) of N = 1, 2, 4, 8 interleaved row-block
shards at several block sizes; prints ms per launch and ms x N (the work of
all shards), so the cost of the shard path itself shows (whole frames = the
floor). RT_LIB selects a library build (A/B against tools/ablate.sh rev).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import openglraytracer_amd as rt  # noqa: E402

rt.LIB_PATH = os.environ.get("RT_LIB", rt.LIB_PATH)
ctx = rt.Context(0)
ctx.set_timing(False)
ctx.set_output(rt.abi.RT_OUTPUT_RGBA8)
s = torch.cuda.Stream()
torch.cuda.set_stream(s)
W, H, F = 1920, 1080, 64
views = [rt.make_view(None, k / 60.0) for k in range(F)]
sc = rt.Scene(ctx, rt.bench_objects(16, 0))
buf = torch.empty(F * H * W, dtype=torch.int32, device="cuda")


def t(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


print(rt.lib().rt_version().decode())
print("whole frames: %.4f ms" % t(lambda: rt.render_batch(ctx, sc, buf.data_ptr(), W, H, 0, views, stream=s.cuda_stream)))
for n, blk in [(2, 8), (2, 16), (2, 12), (4, 8), (8, 8)]:
    ms = max(t(lambda sh=sh: rt.render_batch(ctx, sc, buf.data_ptr(), W, H, 0, views, blk, n, sh,
                                             stream=s.cuda_stream)) for sh in range(min(n, 2)))
    print("n %d block %2d: %.4f ms per launch, x n %.4f" % (n, blk, ms, ms * n))
