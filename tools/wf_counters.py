#!/usr/bin/env python3
"""Lane utilisation, VALU and cache counters of the wavefront engine's traversal
kernels (k_wf_trace closest-hit / any-hit) per variant, from the rocprofv3 --pmc
databases tools/_cmd_r3s3.sh writes (<out>/wf_<variant>[_c]/run_results.db)."""
import glob
import os
import sqlite3
import sys

out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, "wf_*"))):
    db = os.path.join(d, "run_results.db")
    if not os.path.exists(db):
        continue
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, count(*), sum(value), sum(duration) from counters_collection "
                     "where kernel_name like '%k_wf_trace%' group by kernel_name, counter_name").fetchall()
    agg = {}
    for k, cn, n, v, dur in rows:
        kind = "closest-hit" if "k_wf_trace<false" in k else "any-hit"
        agg.setdefault(kind, {})[cn] = (v, dur, n)
    print(os.path.basename(d))
    for kind, cs in sorted(agg.items()):
        v = {k: x[0] for k, x in cs.items()}
        dur = max(x[1] for x in cs.values()) / 1e6
        n = max(x[2] for x in cs.values())
        extra = ""
        if "SQ_THREAD_CYCLES_VALU" in v:
            extra += f" lane_util={v['SQ_THREAD_CYCLES_VALU'] / 64 / v['SQ_ACTIVE_INST_VALU']:.4f}"
            extra += f" valu_insts={v['SQ_INSTS_VALU']:.4g} wait_frac={v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES']:.3f}"
        if "TCC_HIT_sum" in v:
            extra += f" l2_hit={v['TCC_HIT_sum'] / (v['TCC_HIT_sum'] + v['TCC_MISS_sum']):.4f}"
            extra += f" l1_hit={1 - v['TCP_TCC_READ_REQ_sum'] / v['TCP_TOTAL_CACHE_ACCESSES_sum']:.4f}"
            extra += f" l2_req={v['TCP_TCC_READ_REQ_sum']:.4g}"
        print(f"  {kind:12} launches={n} kernel_ms={dur:.1f}{extra}")
