"""Summarise rocprofv3 rocpd databases: per-kernel dispatch stats (--kernel-trace
--stats run) and per-kernel PMC averages (one --pmc pass per counter).

  python tools/prof_summary.py <trace.db> [<pmc.db> ...]  > profiles/<round>_kernels.txt
  TMPT_PMC_JSON=profiles/pmc_k_path.json python tools/prof_summary.py ...   (also
  writes per-dispatch HBM bytes of the k_path<false,...> dispatches for bench.py)

FETCH_SIZE/WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md (HBM/rocprofv3):
on gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane) reads -- the
corrected column doubles it; other access widths are uncalibrated."""
import json
import os
import sqlite3
import sys


def short(name, n=90):
    return name if len(name) <= n else name[: n - 3] + "..."


def main():
    trace, pmcs = sys.argv[1], sys.argv[2:]
    traffic = {}
    c = sqlite3.connect(trace)
    print(f"# kernel stats: {trace}")
    print(f"{'kernel':<92} {'calls':>6} {'total_ms':>10} {'avg_ms':>10} {'pct':>6}")
    for name, calls, tot, avg, pct in c.execute(
            "select name,total_calls,total_duration,average,percentage from top_kernels "
            "order by total_duration desc limit 25"):
        # top_kernels durations are in microseconds
        print(f"{short(name):<92} {calls:>6} {tot / 1e3:>10.3f} {avg / 1e3:>10.4f} {pct:>6.2f}")
    for p in pmcs:
        c = sqlite3.connect(p)
        print(f"\n# PMC: {p}")
        rows = c.execute("select kernel_name, counter_name, count(*), avg(value), avg(duration) "
                         "from counters_collection group by kernel_name, counter_name "
                         "order by avg(duration)*count(*) desc limit 12").fetchall()
        print(f"{'kernel':<92} {'counter':>11} {'n':>4} {'avg_MB':>10} {'x2_MB':>10} {'avg_ms':>10}")
        for k, cn, n, v, d in rows:
            mb = v * 1024 / 1e6
            if k.startswith("void tmpt::k_path<false"):
                traffic[cn] = {"kernel": k.split("(")[0], "dispatches": n, "raw_bytes": v * 1024,
                               "avg_ms": d / 1e6}
            print(f"{short(k):<92} {cn:>11} {n:>4} {mb:>10.2f} {2 * mb:>10.2f} {d / 1e6:>10.3f}")
    out = os.environ.get("TMPT_PMC_JSON")
    if out and traffic:
        f = traffic.get("FETCH_SIZE", {}).get("raw_bytes", 0.0)
        w = traffic.get("WRITE_SIZE", {}).get("raw_bytes", 0.0)
        rec = {"kernel": next(iter(traffic.values()))["kernel"], "counters": traffic,
               "fetch_bytes_corrected": 2 * f, "write_bytes": w,
               "hbm_bytes_per_launch": 2 * f + w,
               "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM/rocprofv3); WRITE_SIZE as read",
               "source": pmcs}
        with open(out, "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
