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
    pad = frame.padded_shard_rows(H, BLOCK, world)
    shard = torch.zeros((pad, W, 4), dtype=torch.float32)
    for i, r in enumerate(ids):
        shard[i] = torch.from_numpy(oracle_port.render(objs, W, H, DEPTH, 0.0, rows=(int(r), int(r) + 1))[0])
    gathered = [torch.zeros_like(shard) for _ in range(world)] if rank == 0 else None
    dist.gather(shard, gathered, dst=0)
    if rank == 0:
        np.save(result_path, frame.assemble(gathered, H, BLOCK).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_assembles_full_frame(tmp_path, world):
    from oracle import port as oracle_port, scenes
    out = str(tmp_path / "frame.npy")
    mp.start_processes(worker, args=(world, free_port(), out), nprocs=world, start_method="spawn")
    full = oracle_port.render(scenes.bench_objects(16), W, H, DEPTH, 0.0)
    assert np.array_equal(np.load(out), full)
