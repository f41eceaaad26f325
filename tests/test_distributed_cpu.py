"""The N>1 path on CPU: world_size-2 (and 3) gloo process groups run the product's gather
(distributed.gather_tiles) on packed rank framebuffers filled from an oracle render for exactly
the tiles each rank owns; re-interleaved with the product's tile map they must equal the
single-rank frame bit for bit. The HIP re-interleave kernel itself is covered by
tests/test_gpu_parity.py::test_sharded_tiles_reassemble_bitwise."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vulkancomputeraytracing_amd import distributed as D
from vulkancomputeraytracing_amd import tile_pixel_map

W, H, SPP, DEPTH = 40, 45, 2, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir, W=W, H=H):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests import oracle_py
        o = oracle_py.load()
        full, _ = o.render(o.config(W, H, SPP, DEPTH), o.scene("three"), threads=1)
        # the rank's packed tile framebuffer (what vcrt renders for rank/world), padded
        pad = D.tiles_per_rank(W, H, world)
        local = np.zeros((pad * 64, 4), dtype=np.float32)
        m = tile_pixel_map(W, H, world)
        mine = m[..., 0] == rank
        local[m[..., 1][mine]] = full[mine]
        gathered = D.gather_tiles(torch.from_numpy(local), pad)
        if rank == 0:
            g = gathered.numpy().reshape(world, pad * 64, 4)
            frame = g[m[..., 0], m[..., 1]]
            np.save(os.path.join(outdir, "frame.npy"), frame)
            np.save(os.path.join(outdir, "full.npy"), full)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h", [(2, W, H), (3, W, H),
                                       (3, 8, 8), (4, 9, 9)])  # ranks that own no tile
def test_gloo_gather_reassembles_bitwise(tmp_path, world, w, h):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), w, h), nprocs=world, join=True)
    frame = np.load(tmp_path / "frame.npy")
    full = np.load(tmp_path / "full.npy")
    assert np.array_equal(frame.view(np.uint32), full.view(np.uint32))


def test_tile_interleave_balances_the_final_scene_load():
    # Per-pixel segment counts of the bench frame (1920x1080, final scene, depth 10) from a
    # 1-spp oracle pass, summed per rank: diagonally interleaved 8x8 tiles give each of 2/4/8
    # ranks the mean load within 1%; contiguous row bands (sky on top, ground below) would not.
    from tests import oracle_py
    o = oracle_py.load()
    w, h = 1920, 1080
    cfg = o.config(w, h, 1, 10)
    scene = o.scene("final")
    # segments per 8-row band of tiles, per tile column: render 8 rows at a time
    per_row = np.array([o.render(cfg, scene, rows=range(y, y + 1))[1] for y in range(h)],
                       dtype=np.float64)
    for world in (2, 4, 8):
        # a tile's cost ~ its rows' cost share over its 8 columns; with (tx + ty) % world every
        # rank gets 1/world of every tile row (and, shifted per row, of every column)
        m = tile_pixel_map(w, h, world)[..., 0]
        loads = [(per_row[:, None] / w * (m == r)).sum() for r in range(world)]
        assert max(loads) / np.mean(loads) < 1.01, loads
    bands = [per_row[r * h // 8:(r + 1) * h // 8].sum() for r in range(8)]
    assert max(bands) / np.mean(bands) > 1.2, bands
