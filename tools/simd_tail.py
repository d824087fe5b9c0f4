"""Per-SIMD / per-wave tail analysis of a saved production-kernel timeline
(tools/tlog.py with TMPT_PROF=0 and TLOG_SAVE=<file.npy>): where the last
pixels ran and how much traversal work each SIMD and wave carried.
  python tools/simd_tail.py <file.npy>"""
import sys

import numpy as np

t = np.load(sys.argv[1]).astype(np.int64)
e = (t[:, 1] - t[:, 0].min()) / 1e5  # ms
st = t[:, 2]
hw = t[:, 3]
xcc, h = hw >> 16, hw & 0xFFFF
sid = (((xcc * 8 + ((h >> 13) & 7)) * 2 + ((h >> 12) & 1)) * 16 + ((h >> 8) & 15)) * 4 + ((h >> 4) & 3)
wid = sid * 16 + (h & 15)
for name, key in (("SIMD", sid), ("wave", wid)):
    u, inv = np.unique(key, return_inverse=True)
    emax, ssum, n = np.zeros(len(u)), np.zeros(len(u)), np.zeros(len(u))
    np.maximum.at(emax, inv, e)
    np.add.at(ssum, inv, st)
    np.add.at(n, inv, 1)
    print(f"{name}s {len(u)}: steps/{name} min {ssum.min() / 1e3:.0f}k p50 {np.median(ssum) / 1e3:.0f}k "
          f"max {ssum.max() / 1e3:.0f}k; last end min {emax.min():.2f} p50 {np.median(emax):.2f} "
          f"p90 {np.percentile(emax, 90):.2f} max {emax.max():.2f} ms; corr(steps, end) "
          f"{np.corrcoef(ssum, emax)[0, 1]:.2f}")
print(f"pixels {len(t)}, span {e.max():.2f} ms, mean end {e.mean():.2f} ms")
