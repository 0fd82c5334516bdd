"""Per-rank work of the N-GPU bench steps, timed on ONE GPU (development probe).

    python tools/shard_timing.py [--ns 1,2,4,8] [--reps R]

The driver's 1/2/4/8-GPU scaling run (bench.py --gpus N, one rank per GPU,
RCCL) cannot run on the one-GPU boxes of this pool. What a rank does per step
can: for every N this renders each shard s of N exactly as rank s would —
config 2: rt_render_batch of the step's F animated frames restricted to the
shard's interleaved 8-row blocks, into the GL_RGBA8 surface; config 4:
rt_render_shard of the 7680x4320 frame into packed float3 — and times it with
HIP events in sustained blocks (the max over shards is the step's critical
path). It also times what happens around the render: the RGB8 packing of a
config-2 shard (frame.pack_rgb8) and rank 0's de-interleave of the gathered
buffer (frame.assemble_contiguous, one index_select), and prints the bytes
each rank sends to rank 0 (the gather). DESIGN.md §6 turns these into a
predicted step time per N (reference: main.cpp:228-238 renders one frame per
dispatch; the row-tiled split is this repo's).

Prints one JSON line per (workload, N).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import openglraytracer_amd as rt  # noqa: E402
from openglraytracer_amd import frame  # noqa: E402

BLOCK = 8


def timed(fn, reps, stream, rounds=5):
    """Median ms per call of `fn` over `rounds` blocks of `reps` back-to-back
    calls on `stream` (each block preceded by reps // 2 untimed calls)."""
    out = []
    for _ in range(rounds):
        for _ in range(max(1, reps // 2)):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps)
    return float(np.median(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--workloads", default="config2,config4")
    ap.add_argument("--frames", type=int, default=256, help="config 2: frames per step (bench.py --frames)")
    ap.add_argument("--out", default=None,
                    help="also write every record to this JSON file (profiles/shard_timing_latest.json: "
                         "what bench.py --gpus N predicts its step time from)")
    args = ap.parse_args()
    records = []
    ns = [int(v) for v in args.ns.split(",")]
    ctx = rt.Context(0)
    ctx.set_timing(False)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sh = stream.cuda_stream
    for wl in args.workloads.split(","):
        if wl == "config2":
            W, H, depth, nsph, F = 1920, 1080, 0, 16, args.frames
            ctx.set_output(rt.abi.RT_OUTPUT_RGBA8)
            ch, dt, bpp_send = 1, torch.int32, 3
            views = [rt.make_view(None, k / 60.0) for k in range(F)]
            reps = max(10, 800 // F)
        else:
            W, H, depth, nsph, F = 7680, 4320, 4, 256, 1
            ctx.set_output(rt.abi.RT_OUTPUT_RGB32F)
            ch, dt, bpp_send = 3, torch.float32, 12
            view = rt.make_view(None, 0.0)
            reps = 4
        scene = rt.Scene(ctx, rt.bench_objects(nsph, 0))
        for n in ns:
            rows_max = rt.shard_rows(H, BLOCK, n, 0)
            buf = torch.empty(F * rows_max * W * ch, dtype=dt, device="cuda")
            per_shard = []
            for s in range(n):
                if wl == "config2":
                    def fn(s=s):
                        rt.render_batch(ctx, scene, buf.data_ptr(), W, H, depth, views, BLOCK, n, s, stream=sh)
                else:
                    def fn(s=s):
                        if n == 1:
                            rt.render_device(ctx, scene, buf.data_ptr(), W, H, depth, view=view, stream=sh)
                        else:
                            rt.render_shard(ctx, scene, buf.data_ptr(), W, H, depth, BLOCK, n, s, view=view,
                                            stream=sh)
                per_shard.append(timed(fn, reps, stream))
            if True:
                # the same launches alternating between two streams and two
                # output buffers (consecutive steps' launches free to overlap:
                # step i+1's ramp under step i's tail)
                s2 = torch.cuda.Stream()
                buf2 = torch.empty_like(buf)
                flip = [0]

                def alt():
                    k = flip[0]
                    flip[0] ^= 1
                    st, bb = (stream, buf) if k == 0 else (s2, buf2)
                    if wl == "config2":
                        rt.render_batch(ctx, scene, bb.data_ptr(), W, H, depth, views, BLOCK, n, 0,
                                        stream=st.cuda_stream)
                    elif n == 1:
                        rt.render_device(ctx, scene, bb.data_ptr(), W, H, depth, view=view, stream=st.cuda_stream)
                    else:
                        rt.render_shard(ctx, scene, bb.data_ptr(), W, H, depth, BLOCK, n, 0, view=view,
                                        stream=st.cuda_stream)

                def timed2(reps, rounds=5):
                    out = []
                    for _ in range(rounds):
                        for _ in range(reps // 2):
                            alt()
                        torch.cuda.synchronize()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record(stream)
                        s2.wait_stream(stream)
                        for _ in range(reps):
                            alt()
                        stream.wait_stream(s2)
                        e1.record(stream)
                        torch.cuda.synchronize()
                        out.append(e0.elapsed_time(e1) / reps)
                    return float(np.median(out))
                two_streams = timed2(reps)
            rec = {"workload": wl, "n": n, "frames_per_step": F, "kernel_ms_per_shard": [round(v, 5) for v in
                                                                                          per_shard],
                   "kernel_ms_max": round(max(per_shard), 5), "kernel_ms_mean": round(float(np.mean(per_shard)), 5)}
            px_shard = F * rows_max * W
            rec["shard0_two_streams_ms"] = round(two_streams, 5)
            rec["send_bytes_per_rank"] = px_shard * bpp_send
            rec["rank0_ingress_bytes"] = (n - 1) * px_shard * bpp_send
            if n > 1:
                padded = frame.flat_shard_elems(F, H, W, BLOCK, n, 1)
                if wl == "config2":
                    src = torch.empty(padded, dtype=torch.int32, device="cuda")
                    send = torch.empty(padded * 3, dtype=torch.uint8, device="cuda")
                    rec["pack_rgb8_ms"] = round(timed(lambda: frame.pack_rgb8(src, send), 50, stream), 5)
                    big = torch.empty(n * padded * 3, dtype=torch.uint8, device="cuda")
                    idx = torch.as_tensor(frame.contiguous_assembly_rows(F, H, BLOCK, n), device="cuda")
                    rec["assembly_ms"] = round(timed(lambda: frame.assemble_contiguous(big, F, H, W, 3, idx), 50,
                                                     stream), 5)
                else:
                    big = torch.empty(n * padded * 3, dtype=torch.float32, device="cuda")
                    idx = torch.as_tensor(frame.contiguous_assembly_rows(F, H, BLOCK, n), device="cuda")
                    rec["assembly_ms"] = round(timed(lambda: frame.assemble_contiguous(big, F, H, W, 3, idx), 10,
                                                     stream), 5)
            print(json.dumps(rec), flush=True)
            records.append(rec)
            del buf
        scene.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"tool": "tools/shard_timing.py",
                       "note": "every rank's per-step work timed on ONE MI355X (the render of each shard, the RGB8 "
                               "packing, the de-interleave); bench.py --gpus N predicts its step time from these "
                               "(DESIGN.md §6)",
                       "build": rt.lib().rt_version().decode(), "records": records}, f, indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
