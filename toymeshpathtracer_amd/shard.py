"""Row-band sharding of a frame over ranks.

Rows are grouped in bands of ``band_rows``; band b goes to rank b % world
(round-robin, so cheap sky rows and expensive interior rows spread evenly).
Each rank renders its bands into a compact tile (``tmpt_render`` with
shard/num_shards); rank 0 gathers the tiles (one collective) and scatters
their rows back into the frame.  Pure index arithmetic: mirrors
``tmpt_tile_rows`` / ``tmpt_tile_row_to_y`` in tmpt_api.cpp and is checked
against them in tests/test_host.py.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def rows_of(height: int, band_rows: int, shard: int, world: int) -> np.ndarray:
    """Global rows (ascending) of ``shard``'s tile, in tile order."""
    band = band_rows if band_rows > 0 else height
    if world <= 1:
        shard, world = 0, 1
    nbands = (height + band - 1) // band
    out: List[int] = []
    for b in range(shard, nbands, world):
        out.extend(range(b * band, min((b + 1) * band, height)))
    return np.asarray(out, np.int64)


def all_rows(height: int, band_rows: int, world: int) -> List[np.ndarray]:
    return [rows_of(height, band_rows, s, world) for s in range(world)]


def assemble(tiles: Sequence, rows: Sequence[np.ndarray], frame):
    """Write tile rows into ``frame`` (numpy or torch, [H, W, 4]); tiles may be
    padded to a common row count (equal-size collectives): extra rows ignored."""
    for t, r in zip(tiles, rows):
        n = len(r)
        if hasattr(frame, "index_copy_"):  # torch, on the device
            import torch

            idx = torch.as_tensor(r, device=frame.device)
            frame.index_copy_(0, idx, t[:n])
        else:
            frame[r] = np.asarray(t)[:n]
    return frame


def placement(devices: Sequence[dict], backend) -> dict:
    """What a multi-rank run ran on, from every rank's device identity
    ({"pci": domain:bus:device, "uuid": ...}, rank order): ``n_gpus`` counts
    DISTINCT devices, so ranks that share a GPU (the gloo rehearsal) are not
    reported as more GPUs; ``ranks`` is the process count; ``rehearsal`` is
    true when some ranks share a device.  ``backend`` is None for a plain
    single-process run (no process group)."""
    distinct = len({(d["pci"], d.get("uuid", "")) for d in devices})
    return {"n_gpus": distinct, "ranks": len(devices), "dist_backend": backend,
            "devices": [d["pci"] for d in devices], "rehearsal": distinct < len(devices)}
