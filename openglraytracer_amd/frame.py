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
  `assemble_frame`;
* spread: the same exchange for a fixed step of F frames (frame k assembled
  on rank k % N) — `spread_plan` + `assemble_frames`.

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


def contiguous_assembly_rows(n_frames, height, block_rows, n_shards):
    """For a gather into ONE contiguous buffer of n_shards equal chunks (chunk
    s = shard s's flat buffer, flat_shard_elems elements: (n_frames, rows_s,
    width, channels) at its start): idx[f * height + r] = the buffer row (of
    width * channels elements) holding frame f's row r. One index_select then
    assembles every frame (`assemble_contiguous`), without first
    concatenating the shards."""
    padded = padded_shard_rows(height, block_rows, n_shards)
    idx = np.empty((n_frames, height), np.int64)
    for s in range(n_shards):
        ids = shard_row_ids(height, block_rows, n_shards, s)
        for f in range(n_frames):
            idx[f, ids] = (s * n_frames * padded) + f * len(ids) + np.arange(len(ids))
    return idx.reshape(-1)


def assemble_contiguous(buf, n_frames, height, width, channels, idx):
    """buf: the contiguous gather buffer (torch or numpy, flat); idx:
    contiguous_assembly_rows. Returns (n_frames, height, width, channels)."""
    rows = buf.reshape(-1, width * channels)
    try:
        import torch
        if isinstance(buf, torch.Tensor):
            i = idx if isinstance(idx, torch.Tensor) else torch.as_tensor(idx, device=buf.device)
            return rows.index_select(0, i).reshape(n_frames, height, width, channels)
    except ImportError:
        pass
    return rows[idx].reshape(n_frames, height, width, channels)


def pack_rgb8(rgba8, out):
    """The GL_RGBA8 texels (RT_OUTPUT_RGBA8, one 4-byte texel per pixel, any
    integer dtype) without their alpha byte, which the reference stores as 0
    (imageStore of vec4(rgb, 0.0), raytrace_compute.glsl:404): 3 bytes per
    pixel into the uint8 tensor `out` (torch)."""
    import torch
    src = rgba8.view(torch.uint8).view(-1, 4)
    out.view(-1, 3)[: src.shape[0]].copy_(src[:, :3])
    return out


def exchange_splits(height, width, block_rows, n_shards, rank, channels=4, frames_per_rank=1):
    """All-to-all split sizes (elements) for the frame exchange: this rank's
    batch buffer is (n_shards * F frames, rows_rank, width, channels), frames
    [k F, (k+1) F) going to rank k (F = frames_per_rank); it receives its own
    frames' rows from every shard, concatenated in shard order (shard s's
    chunk: (F, rows_s, width, channels)). Returns (input_splits, output_splits)."""
    rows = [len(shard_row_ids(height, block_rows, n_shards, s)) for s in range(n_shards)]
    f = frames_per_rank
    return [f * rows[rank] * width * channels] * n_shards, [f * r * width * channels for r in rows]


def spread_plan(height, width, block_rows, n_shards, rank, n_frames, channels=3):
    """The "spread" exchange of a step of n_frames frames (strong scaling):
    every frame row-tiled over all ranks, frame k assembled on rank k % N, so
    rank 0's xGMI ingress is 1/N of the step's bytes instead of (N-1)/N and
    every rank's links carry their share (xGMI is point-to-point).
    Returns (order, input_splits, output_splits, mine):
    * order: the frames in the order each rank renders them (grouped by
      destination rank, so each destination's rows are contiguous in the
      send buffer (n_frames, rows_rank, width, channels));
    * input_splits / output_splits: all_to_all_single sizes (elements);
    * mine: the frames this rank assembles, in receive order (the receive
      buffer is, per source shard s, (len(mine), rows_s, width, channels) -
      assemble_frames with frames=len(mine))."""
    dest = [k % n_shards for k in range(n_frames)]
    order = [k for d in range(n_shards) for k in range(n_frames) if dest[k] == d]
    cnt = [dest.count(d) for d in range(n_shards)]
    rows = [len(shard_row_ids(height, block_rows, n_shards, s)) for s in range(n_shards)]
    ins = [cnt[d] * rows[rank] * width * channels for d in range(n_shards)]
    outs = [cnt[rank] * rows[s] * width * channels for s in range(n_shards)]
    mine = [k for k in order if dest[k] == rank]
    return order, ins, outs, mine


def assembly_rows(height, block_rows, n_shards, frames):
    """idx[f * height + r] = row of the received buffer (viewed as rows of
    width * channels elements: shard chunks (frames, rows_s) in shard order)
    holding frame f's row r."""
    base, local, size = np.empty(height, np.int64), np.empty(height, np.int64), []
    start = 0
    for s in range(n_shards):
        ids = shard_row_ids(height, block_rows, n_shards, s)
        base[ids] = start
        local[ids] = np.arange(len(ids))
        size.append(len(ids))
        start += frames * len(ids)
    rows_of = np.empty(height, np.int64)
    for s in range(n_shards):
        rows_of[shard_row_ids(height, block_rows, n_shards, s)] = size[s]
    f = np.arange(frames)[:, None]
    return (base[None, :] + f * rows_of[None, :] + local[None, :]).reshape(-1)


def assemble_frames(recv, frames, height, width, block_rows, n_shards, channels=4, idx=None):
    """recv: this rank's frames' shards as the exchange delivers them (flat;
    shard s's chunk (frames, rows_s, width, channels), shards in order).
    Returns (frames, height, width, channels) in row order — one gather."""
    if idx is None:
        idx = assembly_rows(height, block_rows, n_shards, frames)
    flat = recv.reshape(frames * height, width * channels)
    try:
        import torch
        if isinstance(recv, torch.Tensor):
            i = idx if isinstance(idx, torch.Tensor) else torch.as_tensor(idx, device=recv.device)
            return flat.index_select(0, i).reshape(frames, height, width, channels)
    except ImportError:
        pass
    return flat[idx].reshape(frames, height, width, channels)


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


def gather_frame(shard, height, width, block_rows, n_shards, rank, channels=4, gather_list=None, perm=None,
                 dst=0):
    """One frame row-tiled over the ranks of torch.distributed (SURVEY.md
    §8(e), config 4): `shard` is this rank's flat buffer of
    flat_shard_elems(1, ...) elements holding its packed rows (rt_render_shard)
    at the start. One gather (RCCL over xGMI with the nccl backend) brings
    every shard to rank `dst`, which de-interleaves them (one index_select)
    and returns the frame (height, width, channels); other ranks return None.
    `gather_list` (dst only): n_shards buffers like `shard` to receive into."""
    import torch.distributed as dist
    if rank == dst:
        if gather_list is None:
            gather_list = [shard.new_empty(shard.shape) for _ in range(n_shards)]
        dist.gather(shard, gather_list, dst=dst)
        return assemble(gather_list, 1, height, width, block_rows, channels=channels, perm=perm)[0]
    dist.gather(shard, None, dst=dst)
    return None
