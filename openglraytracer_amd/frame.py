"""Row-tiled multi-GPU frame layout.

A frame of H rows is cut into blocks of `block_rows` rows dealt round-robin to
N shards (rt_render_shard / rt_render_batch render shard s's blocks packed
densely, in order). Interleaved blocks balance the load: the cost of a row
depends on what it sees.

Two assemblies:
* gather: rank 0 assembles every frame after one gather of equal-size flat
  buffers (each shard's data first, then padding) — `assemble`;
* exchange: with N frames in flight (one per rank), frame k is gathered to
  rank k — N gathers at once, i.e. one all-to-all in which every rank sends
  frame k's rows to rank k — so each xGMI link carries 1/N of the traffic a
  single root would pull through its own links — `exchange_splits` +
  `assemble_frame`.

Pure index bookkeeping (numpy / torch tensors); no rendering here.
"""
import numpy as np


def shard_row_ids(height, block_rows, n_shards, shard):
    """Frame rows owned by `shard`, in packed order (matches rt_shard_rows)."""
    rows = np.arange(height)
    return rows[(rows // block_rows) % n_shards == shard]


def padded_shard_rows(height, block_rows, n_shards):
    return max(len(shard_row_ids(height, block_rows, n_shards, s)) for s in range(n_shards))


def flat_shard_elems(n_frames, height, width, block_rows, n_shards, channels=4):
    """Elements of the equal-size flat buffer every rank contributes."""
    return n_frames * padded_shard_rows(height, block_rows, n_shards) * width * channels


def assembly_permutation(height, block_rows, n_shards):
    """perm[r] = position of frame row r in the concatenation of the shards."""
    order = np.concatenate([shard_row_ids(height, block_rows, n_shards, s) for s in range(n_shards)])
    perm = np.empty(height, np.int64)
    perm[order] = np.arange(height)
    return perm


def assemble(flat, n_frames, height, width, block_rows, channels=4, perm=None):
    """flat: one flat buffer per shard (torch or numpy), shard s holding
    (n_frames, rows_s, width, channels) at its start. Returns the frames
    (n_frames, height, width, channels) in row order."""
    n = len(flat)
    if perm is None:
        perm = assembly_permutation(height, block_rows, n)
    parts = []
    for s, buf in enumerate(flat):
        rows = len(shard_row_ids(height, block_rows, n, s))
        parts.append(buf[: n_frames * rows * width * channels].reshape(n_frames, rows, width, channels))
    try:
        import torch
        if isinstance(flat[0], torch.Tensor):
            cat = torch.cat(parts, dim=1)
            idx = perm if isinstance(perm, torch.Tensor) else torch.as_tensor(perm, device=cat.device)
            return cat.index_select(1, idx)
    except ImportError:
        pass
    return np.concatenate(parts, axis=1)[:, perm]


def exchange_splits(height, width, block_rows, n_shards, rank, channels=4):
    """All-to-all split sizes (elements) for the frame exchange: this rank's
    batch buffer is (n_shards frames, rows_rank, width, channels), frame k's
    rows going to rank k; it receives its own frame's rows from every shard,
    concatenated in shard order. Returns (input_splits, output_splits)."""
    rows = [len(shard_row_ids(height, block_rows, n_shards, s)) for s in range(n_shards)]
    return [rows[rank] * width * channels] * n_shards, [r * width * channels for r in rows]


def assemble_frame(recv, height, width, block_rows, n_shards, channels=4, perm=None):
    """recv: one frame's shards concatenated in shard order (flat, torch or
    numpy). Returns the frame (height, width, channels) in row order."""
    if perm is None:
        perm = assembly_permutation(height, block_rows, n_shards)
    cat = recv.reshape(height, width, channels)
    try:
        import torch
        if isinstance(recv, torch.Tensor):
            idx = perm if isinstance(perm, torch.Tensor) else torch.as_tensor(perm, device=recv.device)
            return cat.index_select(0, idx)
    except ImportError:
        pass
    return cat[perm]
