"""Multi-GPU frame sharding: diagonally interleaved 8x8 tiles per rank + one framebuffer gather.

One process per GPU. The frame is cut into 8x8 tiles (tx, ty); rank r renders the tiles with
(tx + ty) % world == r, so every work item stays a coherent 8x8 tile and every rank gets the
same number of tiles (to one per row) spread over every row and column of the frame (sky and
ground, left and right alike: SURVEY.md 8(e)).
The product's gather is inside libvcrt.so: after vcrt_comm_init, vcrt_draw_next_frame sends the
packed rank framebuffers [tiles_per_rank][64] to rank 0 over RCCL (one grouped send/recv, on a
non-blocking communicator with a deadline) and rank 0 re-interleaves them with the vcrt_assemble
HIP kernel (capi.cpp gather_frame; bench.py drives it). This module keeps the tile helpers and a
torch.distributed rehearsal of the same exchange (gather_tiles / assemble_frame), used with the
"gloo" backend to run the N-rank flow on a box with fewer GPUs than ranks (RCCL needs one GPU per
rank) and by the CPU tests. The reference is single-GPU (Environment.cpp:157-165; "TODO:
Cross-GPU sharing", Frontend.cpp:107); the gather is the one exchange step of the path.
"""
from __future__ import annotations

from .renderer import tile_pixel_map, tiles_for_rank  # noqa: F401  (re-exported)


def tiles_per_rank(width: int, height: int, world: int) -> int:
    """Tiles of the largest rank: the padded per-rank slab of the gather."""
    return max(len(tiles_for_rank(width, height, world, r)) for r in range(world))


def gather_tiles(local, tiles_pad: int, group=None, dst: int = 0):
    """Gather the ranks' packed tile framebuffers to rank `dst`. `local` is
    [tiles_pad * 64, 4] float (tiles past the rank's own count are padding). Returns
    [world * tiles_pad * 64, 4], rank-major, on `dst` and None elsewhere.

    A gather, not an all-gather: only `dst` assembles the frame. Over RCCL it is one grouped
    send/recv per peer, so `dst` receives from all peers at once over their own xGMI links
    (1/world of the frame each) instead of a world-1 step ring that moves the whole frame
    through every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    assert local.shape[0] == tiles_pad * 64 and local.is_contiguous()
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal path (several ranks on one GPU): gloo gathers host copies
        out = gather_tiles(local.cpu(), tiles_pad, group, dst)
        return None if out is None else out.to(local.device)
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device) if rank == dst else None
    try:
        dist.gather(local, gather_list=list(out.chunk(world)) if out is not None else None,
                    dst=dst, group=group)
    except NotImplementedError:
        # a backend without gather refuses it up front on every rank: all-gather instead
        full = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]),
                           dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(full, local, group=group)
        out = full if rank == dst else None
    if local.is_cuda:
        # every rank: the collective is ordered on torch's current stream only, and the
        # renderer's next frame (on its own stream) rewrites `local`; wait until it has been sent
        torch.cuda.current_stream(local.device).synchronize()
    return out


def assemble_frame(renderer, gathered, frame, tiles_pad: int) -> None:
    """Re-interleave gathered tiles into `frame` [H, W, 4] on the GPU (vcrt_assemble)."""
    renderer.assemble_tiles(gathered.data_ptr(), frame.data_ptr(), tiles_pad)
