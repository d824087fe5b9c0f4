"""Print per-kernel PMC sums from tools/pmc_pass.sh databases.
  python tools/pmc_read.py gpurun_out/<tag>/p*/run_results.db [--kernel k_path]"""
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
kern = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "k_path"
args = [a for a in args if a != kern]
vals = {}
for f in args:
    c = sqlite3.connect(f)
    for k, cn, v, d in c.execute("select kernel_name, counter_name, sum(value), avg(duration) from "
                                 "counters_collection where kernel_name like ? group by kernel_name, counter_name",
                                 (f"%{kern}%",)):
        vals[(k.split("(")[0], cn)] = (v, d)
for (k, cn), (v, d) in sorted(vals.items()):
    print(f"{k[:60]:<60} {cn:<24} {v:14.5g}  {d / 1e6:8.2f} ms")
