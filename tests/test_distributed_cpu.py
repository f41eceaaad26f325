"""The N>1 path on CPU: world_size-2 (and 3) gloo process groups run the product's gather
(distributed.gather_stripes) on rank framebuffers rendered by the oracle for exactly the rows
each rank owns; the stripes re-interleaved with the product's row map must equal the
single-rank frame bit for bit. The HIP re-interleave kernel itself is covered by
tests/test_gpu_parity.py::test_sharded_stripes_reassemble_bitwise."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from vulkancomputeraytracing_amd import distributed as D
from vulkancomputeraytracing_amd import rows_for_rank

W, H, SPP, DEPTH, STRIPE = 40, 45, 2, 8, 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests import oracle_py
        o = oracle_py.load()
        rows = rows_for_rank(H, STRIPE, world, rank)
        full, _ = o.render(o.config(W, H, SPP, DEPTH), o.scene("three"), threads=1)
        # the rank's packed framebuffer (what vcrt renders for rank/world), padded
        pad = D.rows_per_rank(H, STRIPE, world)
        local = np.zeros((pad, W, 4), dtype=np.float32)
        local[:len(rows)] = full[rows]
        gathered = D.gather_stripes(torch.from_numpy(local), pad)
        if rank == 0:
            g = gathered.numpy().reshape(world, pad, W, 4)
            m = D.stripe_row_map(H, STRIPE, world)
            frame = g[m[:, 0], m[:, 1]]
            np.save(os.path.join(outdir, "frame.npy"), frame)
            np.save(os.path.join(outdir, "full.npy"), full)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_reassembles_bitwise(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    frame = np.load(tmp_path / "frame.npy")
    full = np.load(tmp_path / "full.npy")
    assert np.array_equal(frame.view(np.uint32), full.view(np.uint32))


@pytest.mark.parametrize("h,stripe,world", [(1080, 16, 8), (45, 4, 3), (7, 16, 2), (100, 5, 4)])
def test_row_map_matches_rank_rows(h, stripe, world):
    m = D.stripe_row_map(h, stripe, world)
    for r in range(world):
        rows = rows_for_rank(h, stripe, world, r)
        assert list(np.nonzero(m[:, 0] == r)[0]) == rows
        assert list(m[rows, 1]) == list(range(len(rows)))
    assert D.rows_per_rank(h, stripe, world) == max(
        len(rows_for_rank(h, stripe, world, r)) for r in range(world))


def test_interleaving_balances_the_final_scene_load():
    # Segment counts per row of the bench frame (1920x1080, final scene, depth 10) from a 1-spp
    # oracle pass: row-interleaved shards (stripe height 1, the default) give each of 8 ranks
    # the mean load within 1%; 16-row stripes (67.5 stripes over 8 ranks) and contiguous bands
    # (sky on top, ground below) would not.
    from tests import oracle_py
    o = oracle_py.load()
    w, h = 1920, 1080
    cfg = o.config(w, h, 1, 10)
    scene = o.scene("final")
    per_row = np.array([o.render(cfg, scene, rows=range(y, y + 1))[1] for y in range(h)],
                       dtype=np.float64)
    world = 8

    def imbalance(loads):
        return max(loads) / np.mean(loads)

    rows1 = [per_row[rows_for_rank(h, 1, world, r)].sum() for r in range(world)]
    rows16 = [per_row[rows_for_rank(h, 16, world, r)].sum() for r in range(world)]
    bands = [per_row[r * h // world:(r + 1) * h // world].sum() for r in range(world)]
    assert imbalance(rows1) < 1.01, rows1
    assert imbalance(rows16) > imbalance(rows1)
    assert imbalance(bands) > 1.2, bands
