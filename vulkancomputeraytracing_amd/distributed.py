"""Multi-GPU frame sharding: interleaved row stripes per rank + one framebuffer gather.

One process per GPU. Rank r renders the rows y with (y // stripe) % world == r (SURVEY.md 8(e):
interleaving balances cheap sky rows against expensive ground rows); the packed rank-local
framebuffers (padded to the largest rank's row count) are all-gathered over RCCL
(``torch.distributed`` backend "nccl") and rank 0 re-interleaves them with the vcrt_assemble
HIP kernel. The reference is single-GPU (Environment.cpp:157-165; "TODO: Cross-GPU sharing",
Frontend.cpp:107); the gather is the one exchange step of the path.
"""
from __future__ import annotations

import numpy as np

from .renderer import rows_for_rank


def rows_per_rank(height: int, stripe: int, world: int) -> int:
    """Rows of the largest rank: the padded per-rank slab of the gather."""
    return max(len(rows_for_rank(height, stripe, world, r)) for r in range(world))


def stripe_row_map(height: int, stripe: int, world: int) -> np.ndarray:
    """For each global row y: (owning rank, row index in that rank's packed framebuffer).
    The host-side statement of the index map vcrt_assemble applies on the GPU."""
    y = np.arange(height)
    s = y // stripe
    rank = s % world
    local = (s // world) * stripe + y % stripe
    return np.stack([rank, local], axis=1)


def gather_stripes(local, rows_pad: int, group=None):
    """All-gather the ranks' packed framebuffers. `local` is [rows_pad, W, 4] (rows past the
    rank's own count are padding). Returns [world * rows_pad, W, 4] (rank-major)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    assert local.shape[0] == rows_pad and local.is_contiguous()
    out = torch.empty((world * rows_pad,) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out


def assemble_frame(renderer, gathered, frame, rows_pad: int) -> None:
    """Re-interleave gathered stripes into `frame` [H, W, 4] on the GPU (vcrt_assemble)."""
    renderer.assemble_stripes(gathered.data_ptr(), frame.data_ptr(), rows_pad)
