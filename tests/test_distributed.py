"""Multi-rank frame assembly on CPU (gloo, world size 2 and 3).

The same row-tile layout and gather/assemble code bench.py runs over RCCL:
each rank renders its interleaved row blocks (here with the oracle on the
CPU — the checker stands in for the GPU kernel, which tests/test_gpu_parity.py
covers shard by shard), rank 0 gathers the padded shards and de-interleaves;
the result must equal the whole frame bit-for-bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

W, H, BLOCK, DEPTH = 64, 37, 4, 1
TIMES = [0.0, 0.5]
FRAMES = len(TIMES)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, result_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from openglraytracer_amd import frame
    from oracle import port as oracle_port, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    objs = scenes.bench_objects(16)
    ids = frame.shard_row_ids(H, BLOCK, world, rank)
    # the layout rt_render_batch writes: (frames, this shard's rows, W, 4)
    # at the start of an equal-size flat buffer
    buf = torch.zeros(frame.flat_shard_elems(FRAMES, H, W, BLOCK, world), dtype=torch.float32)
    data = np.stack([np.concatenate([oracle_port.render(objs, W, H, DEPTH, t, rows=(int(r), int(r) + 1))
                                     for r in ids]) for t in TIMES])
    buf[: data.size] = torch.from_numpy(data.reshape(-1))
    gathered = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    if rank == 0:
        np.save(result_path, frame.assemble(gathered, FRAMES, H, W, BLOCK).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_assembles_full_frame(tmp_path, world):
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "frame.npy")
    mp.start_processes(worker, args=(world, free_port(), out), nprocs=world, start_method="spawn")
    full = np.stack([oracle_port.render(scenes.bench_objects(16), W, H, DEPTH, t) for t in TIMES])
    assert np.array_equal(np.load(out), full)


def exchange_worker(rank, world, port, result_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from openglraytracer_amd import frame
    from oracle import port as oracle_port, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    objs = scenes.bench_objects(16)
    fpr = 2  # frames per rank in flight (bench.py --frames with --frame-exchange all_to_all)
    times = [k / 60.0 for k in range(world * fpr)]
    ids = frame.shard_row_ids(H, BLOCK, world, rank)
    # the batch buffer rt_render_batch writes in bench.py's exchange format
    # (RT_OUTPUT_RGB32F): (world * fpr frames, this shard's rows, W, 3)
    data = np.stack([np.concatenate([oracle_port.render(objs, W, H, DEPTH, t, rows=(int(r), int(r) + 1))
                                     for r in ids]) for t in times])[..., :3]
    send = torch.from_numpy(np.ascontiguousarray(data).reshape(-1))
    in_splits, out_splits = frame.exchange_splits(H, W, BLOCK, world, rank, channels=3, frames_per_rank=fpr)
    recv = torch.empty(sum(out_splits), dtype=torch.float32)
    dist.all_to_all_single(recv, send, out_splits, in_splits)  # frames [k fpr, (k+1) fpr) -> rank k
    np.save(result_path + ".%d.npy" % rank, frame.assemble_frames(recv, fpr, H, W, BLOCK, world, channels=3).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_assembles_one_frame_per_rank(tmp_path, world):
    """bench.py's N-GPU frame exchange: 2N frames in flight, every rank renders
    its row blocks of all of them, one all-to-all delivers frames 2k, 2k+1 to
    rank k, which de-interleaves them — bit-identical to the whole frame's rgb
    (the shards travel as packed float3; alpha is the constant 0)."""
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "frame")
    mp.start_processes(exchange_worker, args=(world, free_port(), out), nprocs=world, start_method="spawn")
    for k in range(world):
        got = np.load(out + ".%d.npy" % k)
        for f in range(2):
            full = oracle_port.render(scenes.bench_objects(16), W, H, DEPTH, (2 * k + f) / 60.0)
            assert (full[..., 3] == 0).all()
            assert np.array_equal(got[f], full[..., :3]), (k, f)


def mc_worker(rank, world, port, result_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import port as oracle_port, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spp_total, w, h = 8, 24, 14
    per = spp_total // world
    acc = oracle_port.render_accumulate(scenes.bench_objects(16), w, h, 0, per, rank * per, seed=3)
    t = torch.from_numpy(acc)
    dist.all_reduce(t)  # the RCCL all-reduce of config 5, here over gloo
    if rank == 0:
        np.save(result_path, (t / spp_total).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_monte_carlo_sample_sharding(tmp_path, world):
    """Config 5: samples sharded over ranks + all-reduce == one rank's
    estimate up to float re-association of the partial sums."""
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "mc.npy")
    mp.start_processes(mc_worker, args=(world, free_port(), out), nprocs=world, start_method="spawn")
    ref = oracle_port.render_accumulate(scenes.bench_objects(16), 24, 14, 0, 8, 0, seed=3) / 8
    got = np.load(out)
    assert np.allclose(got, ref, rtol=1e-6, atol=1e-6)


def gather_frame_worker(rank, world, port, result_path):
    """bench.py --workload config4 at N ranks: one frame, interleaved 8-row
    blocks per rank (packed float3 shards, RT_OUTPUT_RGB32F), one gather to
    rank 0 (frame.gather_frame), de-interleaved there."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from openglraytracer_amd import frame
    from oracle import port as oracle_port, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    objs = scenes.bench_objects(64)
    ids = frame.shard_row_ids(H, BLOCK, world, rank)
    shard = torch.zeros(frame.flat_shard_elems(1, H, W, BLOCK, world, channels=3), dtype=torch.float32)
    data = np.concatenate([oracle_port.render(objs, W, H, 2, 0.0, rows=(int(r), int(r) + 1)) for r in ids])[..., :3]
    shard[: data.size] = torch.from_numpy(np.ascontiguousarray(data).reshape(-1))
    out = frame.gather_frame(shard, H, W, BLOCK, world, rank, channels=3)
    if rank == 0:
        np.save(result_path, out.numpy())
    else:
        assert out is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_tiled_frame_gathers_to_rank0(tmp_path, world):
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "frame.npy")
    mp.start_processes(gather_frame_worker, args=(world, free_port(), out), nprocs=world, start_method="spawn")
    full = oracle_port.render(scenes.bench_objects(64), W, H, 2, 0.0)[..., :3]
    assert np.array_equal(np.load(out), full)


def rgba8_gather_worker(rank, world, port, result_path):
    """bench.py config2 at N ranks (the default --frame-exchange gather): F
    frames row-tiled in interleaved blocks, each rank's blocks of all F
    frames in the GL_RGBA8 surface format (RT_OUTPUT_RGBA8: one 4-byte texel
    per pixel, moved as int32), one gather to rank 0, de-interleaved there."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import openglraytracer_amd as rt
    from openglraytracer_amd import frame
    from oracle import port as oracle_port, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    objs = scenes.bench_objects(16)
    ids = frame.shard_row_ids(H, BLOCK, world, rank)
    buf = torch.zeros(frame.flat_shard_elems(FRAMES, H, W, BLOCK, world, channels=1), dtype=torch.int32)
    data = np.stack([rt.pack_rgba8(np.concatenate([oracle_port.render(objs, W, H, DEPTH, t, rows=(int(r), int(r) + 1))
                                                   for r in ids])) for t in TIMES])
    texels = np.ascontiguousarray(data).view(np.int32)  # (F, rows, W, 1)
    buf[: texels.size] = torch.from_numpy(texels.reshape(-1))
    gathered = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gathered, dst=0)
    if rank == 0:
        out = frame.assemble(gathered, FRAMES, H, W, BLOCK, channels=1).numpy()
        np.save(result_path, np.ascontiguousarray(out).view(np.uint8).reshape(FRAMES, H, W, 4))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rgba8_frames_gather_to_rank0(tmp_path, world):
    import openglraytracer_amd as rt
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "frames.npy")
    mp.start_processes(rgba8_gather_worker, args=(world, free_port(), out), nprocs=world, start_method="spawn")
    full = np.stack([rt.pack_rgba8(oracle_port.render(scenes.bench_objects(16), W, H, DEPTH, t)) for t in TIMES])
    assert np.array_equal(np.load(out), full)


def rgb8_contiguous_worker(rank, world, port, result_path):
    """bench.py config2's gather at N ranks: the GL_RGBA8 shards packed to
    RGB8 (frame.pack_rgb8: the constant alpha byte dropped), gathered into
    one contiguous buffer on rank 0 and de-interleaved by one index_select
    (frame.contiguous_assembly_rows / assemble_contiguous)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import openglraytracer_amd as rt
    from openglraytracer_amd import frame
    from oracle import port as oracle_port, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    objs = scenes.bench_objects(16)
    ids = frame.shard_row_ids(H, BLOCK, world, rank)
    px = frame.flat_shard_elems(FRAMES, H, W, BLOCK, world, channels=1)
    texels = torch.zeros(px, dtype=torch.int32)
    data = np.stack([rt.pack_rgba8(np.concatenate([oracle_port.render(objs, W, H, DEPTH, t, rows=(int(r), int(r) + 1))
                                                   for r in ids])) for t in TIMES])
    flat = np.ascontiguousarray(data).view(np.int32).reshape(-1)
    texels[: flat.size] = torch.from_numpy(flat)
    send = frame.pack_rgb8(texels, torch.empty(px * 3, dtype=torch.uint8))
    big = torch.empty(world * px * 3, dtype=torch.uint8) if rank == 0 else None
    dist.gather(send, [big[r * px * 3:(r + 1) * px * 3] for r in range(world)] if rank == 0 else None, dst=0)
    if rank == 0:
        idx = frame.contiguous_assembly_rows(FRAMES, H, BLOCK, world)
        np.save(result_path, frame.assemble_contiguous(big, FRAMES, H, W, 3, idx).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rgb8_shards_gather_contiguously_to_rank0(tmp_path, world):
    import openglraytracer_amd as rt
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "frames.npy")
    mp.start_processes(rgb8_contiguous_worker, args=(world, free_port(), out), nprocs=world, start_method="spawn")
    full = np.stack([rt.pack_rgba8(oracle_port.render(scenes.bench_objects(16), W, H, DEPTH, t)) for t in TIMES])
    assert np.all(full[..., 3] == 0)
    assert np.array_equal(np.load(out), full[..., :3])


def spread_worker(rank, world, port, result_path, n_frames):
    """bench.py config2 at N ranks, the default --frame-exchange spread: the
    step's F frames row-tiled over all ranks (rendered in spread_plan's
    order, grouped by destination), packed to RGB8, one all-to-all delivers
    frame k's shards to rank k % N, which de-interleaves them
    (frame.spread_plan / assemble_frames)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import openglraytracer_amd as rt
    from openglraytracer_amd import frame
    from oracle import port as oracle_port, scenes
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    objs = scenes.bench_objects(16)
    ids = frame.shard_row_ids(H, BLOCK, world, rank)
    order, ins, outs, mine = frame.spread_plan(H, W, BLOCK, world, rank, n_frames, channels=3)
    # rt_render_batch of the views in `order`, shard `rank`, RT_OUTPUT_RGBA8
    data = np.stack([rt.pack_rgba8(np.concatenate([oracle_port.render(objs, W, H, DEPTH, k / 60.0,
                                                                      rows=(int(r), int(r) + 1)) for r in ids]))
                     for k in order])
    texels = torch.from_numpy(np.ascontiguousarray(data).view(np.int32).reshape(-1))
    send = frame.pack_rgb8(texels, torch.empty(texels.numel() * 3, dtype=torch.uint8))
    assert send.numel() == sum(ins)
    recv = torch.empty(sum(outs), dtype=torch.uint8)
    dist.all_to_all_single(recv, send, outs, ins)  # frame k -> rank k % N
    got = frame.assemble_frames(recv, len(mine), H, W, BLOCK, world, channels=3).numpy() if mine else None
    np.save(result_path + ".%d.npy" % rank, np.array(mine))
    if mine:
        np.save(result_path + ".%d.frames.npy" % rank, got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_frames", [(2, 5), (3, 5), (4, 3)])
def test_spread_exchange_assembles_every_frame_once(tmp_path, world, n_frames):
    """Every frame of the step lands whole on exactly one rank (k % N), byte
    for byte the GL_RGBA8 texels of the whole-frame render without alpha;
    uneven counts (5 frames on 2 or 3 ranks) and idle ranks (3 frames on 4)."""
    import openglraytracer_amd as rt
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "spread")
    mp.start_processes(spread_worker, args=(world, free_port(), out, n_frames), nprocs=world, start_method="spawn")
    seen = []
    for r in range(world):
        mine = list(np.load(out + ".%d.npy" % r))
        assert all(k % world == r for k in mine)
        seen += mine
        if mine:
            got = np.load(out + ".%d.frames.npy" % r)
            for j, k in enumerate(mine):
                full = rt.pack_rgba8(oracle_port.render(scenes.bench_objects(16), W, H, DEPTH, k / 60.0))
                assert np.array_equal(got[j], full[..., :3]), (r, k)
    assert sorted(seen) == list(range(n_frames))
