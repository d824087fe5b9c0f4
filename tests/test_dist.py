"""The N>1 path on CPU: world_size-2 gloo ranks each render their row bands
(with the CPU oracle standing in for the device, as a checker only), gather
the tiles to rank 0 with one collective and assemble the frame with the same
code bench.py uses -- the result must equal the single-rank frame."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import ROOT, data


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import oracle
    from toymeshpathtracer_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, h, spp, band = 96, 70, 2, 16
    tris, bmin, bmax = oracle.load_scene(data("suzanne.obj"))
    cam = oracle.camera_for_scene(bmin, bmax, w, h)
    sc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX)
    rows = shard.all_rows(h, band, world)
    full, rays = sc.render(cam, w, h, spp, seed_mode=oracle.SEED_PIXEL)  # rendered rows only below
    mine = rows[rank]
    frame_part, _ = sc.render(cam, w, h, spp, seed_mode=oracle.SEED_PIXEL, threads=2)
    tile = np.zeros((max(len(r) for r in rows), w, 4), np.uint8)
    tile[: len(mine)] = frame_part[mine]
    t = torch.from_numpy(tile)
    gathered = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, gathered, dst=0)
    if rank == 0:
        frame = np.zeros((h, w, 4), np.uint8)
        shard.assemble([g.numpy() for g in gathered], rows, frame)
        np.save(out_path, np.stack([frame, full]))
    dist.destroy_process_group()


def test_gloo_two_ranks_assemble_frame(tmp_path):
    out = str(tmp_path / "frames.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    frame, full = np.load(out)
    assert np.array_equal(frame, full)
