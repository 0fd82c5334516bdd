"""Row-tiled multi-GPU frame layout.

A frame of H rows is cut into blocks of `block_rows` rows dealt round-robin to
N shards (rt_render_shard renders shard s's blocks packed densely, in order).
Interleaved blocks balance the load: the cost of a row depends on what it sees.
Rank 0 assembles the frame after a gather of equal-size (padded) shards.

Pure index bookkeeping (numpy / torch tensors); no rendering here.
"""
import numpy as np


def shard_row_ids(height, block_rows, n_shards, shard):
    """Frame rows owned by `shard`, in packed order (matches rt_shard_rows)."""
    rows = np.arange(height)
    return rows[(rows // block_rows) % n_shards == shard]


def padded_shard_rows(height, block_rows, n_shards):
    return max(len(shard_row_ids(height, block_rows, n_shards, s)) for s in range(n_shards))


def gather_index(height, block_rows, n_shards):
    """(src, dst): row src of the stacked padded shards -> frame row dst."""
    pad = padded_shard_rows(height, block_rows, n_shards)
    src, dst = [], []
    for s in range(n_shards):
        ids = shard_row_ids(height, block_rows, n_shards, s)
        src.append(s * pad + np.arange(len(ids)))
        dst.append(ids)
    return np.concatenate(src), np.concatenate(dst)


def assemble(gathered, height, block_rows):
    """gathered: list (one per shard) of tensors (..., pad_rows, W, C) with the
    row axis at -3. Returns the frame (..., H, W, C) (torch or numpy)."""
    n = len(gathered)
    src, dst = gather_index(height, block_rows, n)
    try:
        import torch
        if isinstance(gathered[0], torch.Tensor):
            stacked = torch.cat(list(gathered), dim=-3)
            out = torch.empty(stacked.shape[:-3] + (height,) + stacked.shape[-2:], dtype=stacked.dtype,
                              device=stacked.device)
            s_idx = torch.as_tensor(src, device=stacked.device)
            d_idx = torch.as_tensor(dst, device=stacked.device)
            out.index_copy_(out.dim() - 3, d_idx, stacked.index_select(stacked.dim() - 3, s_idx))
            return out
    except ImportError:
        pass
    stacked = np.concatenate(gathered, axis=-3)
    out = np.empty(stacked.shape[:-3] + (height,) + stacked.shape[-2:], stacked.dtype)
    out[..., dst, :, :] = stacked[..., src, :, :]
    return out
