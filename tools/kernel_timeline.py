"""Kernel timeline of a rocprofv3 --kernel-trace database: the dispatches in
time order with their durations and the idle gap before each, and per-kernel
totals of duration and of the gaps that precede it (host launch / sync cost
between the device's kernels).

  python tools/kernel_timeline.py <run_results.db> [last_n]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    c = sqlite3.connect(db)
    views = [r[0] for r in c.execute("select name from sqlite_master where type in ('view','table')")]
    if "kernels" not in views:
        print("no kernels view; objects:", ", ".join(sorted(views)))
        return
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
    start_col = "start" if "start" in cols else None
    end_col = "end" if "end" in cols else None
    if not (name_col and start_col and end_col):
        print("kernels columns:", ", ".join(cols))
        return
    rows = c.execute(f'select {name_col}, "{start_col}", "{end_col}" from kernels order by "{start_col}"').fetchall()
    tot = {}
    prev_end = None
    out = []
    for n, s, e in rows:
        short = n.split("(")[0].replace("void ", "")[:70]
        gap = (s - prev_end) if prev_end is not None else 0
        prev_end = e if prev_end is None else max(prev_end, e)
        t = tot.setdefault(short, [0, 0.0, 0.0])
        t[0] += 1
        t[1] += (e - s) / 1e3
        if 0 <= gap < 5e6:  # gaps over 5 ms: host work between frames, not counted
            t[2] += gap / 1e3
        out.append((short, (e - s) / 1e3, gap / 1e3))
    print(f"{'kernel':<72} {'n':>5} {'dur_us':>12} {'gap_before_us':>14}")
    for k, (n, d, g) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:<72} {n:>5} {d:>12.1f} {g:>14.1f}")
    # device busy time: the union of all dispatch intervals (kernels on several
    # streams overlap), against the span from the first start to the last end
    iv = sorted((s, e) for _, s, e in rows)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        busy += ce - cs
        span = max(e for _, e in iv) - iv[0][0]
        print(f"\nspan {span / 1e6:.3f} ms, device busy (union) {busy / 1e6:.3f} ms ({100.0 * busy / span:.1f} %), "
              f"sum of durations {sum(e - s for s, e in iv) / 1e6:.3f} ms")
    print(f"\nlast {last} dispatches (duration us, idle gap before it us):")
    for k, d, g in out[-last:]:
        print(f"{k:<72} {d:>10.1f} {g:>10.1f}")


if __name__ == "__main__":
    main()
