#!/usr/bin/env python3
"""Counter-backed ceilings of k_path from rocprofv3 --pmc passes over bench.py
(tools/pmc_bench.sh + the request-size passes) and the calibration kernel
(tools/pmc_calib.hip), written as one JSON record that bench.py reads.

  python tools/roofline_counters.py <pmc dir> [<ea dir>] > profiles/r03_counters_k_path.json

What the record holds, per k_path launch of the bench frame (all counters are
averaged over the launches of the timed kernel, k_path<false, ...> sample
instantiation):
  valu      SQ_INSTS_VALU, and the VALU issue ceiling: one wave64 VALU
            instruction per SIMD per 2 cycles (MI355X_MICROARCH.md: a wave issues
            each VALU instruction over 2 cycles), 1024 SIMDs, at the measured
            clock (GRBM_GUI_ACTIVE / 8 XCDs / launch time) and at 2.4 GHz
  lanes     SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU): lane utilisation
  l2        TCP_TCC_READ_REQ + TCP_TCC_WRITE_REQ requests x 128 B (the
            calibration: a 16-B gather and a 128-B line are one request each)
            against the ~34.5 TB/s aggregate L2 (MI355X_MICROARCH.md, L2)
  hbm       fabric read requests (TCC_EA0_RDREQ by size: all 128 B here) and
            write requests (TCC_EA0_WRREQ, 32 or 64 B) -> exact bytes; FETCH_SIZE x 2
            agrees with it (the calibration shows every read request is 128 B,
            FETCH_SIZE counts 64 B per request, for streams and 16-B gathers alike)
The ceilings are per-query figures (counter / queries of the profiled launch),
so bench.py scales them by its own queries and launch time."""
import json
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "void tmpt::k_path<false"
SIMDS = 1024
XCDS = 8
SPEC_CLOCK_HZ = 2.4e9
L2_PEAK_BPS = 34.5e12


def counters(db, kernel_prefix=KERNEL, pick="sample"):
    """{counter: (mean value, mean duration ns)} over dispatches of the kernel.
    pick: 'sample' = the instantiation with the most time (the timed launches)."""
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, count(*), avg(value), avg(duration) "
                     "from counters_collection group by kernel_name, counter_name").fetchall()
    by_kernel = {}
    for k, cn, n, v, d in rows:
        if k.startswith(kernel_prefix):
            by_kernel.setdefault(k, {})[cn] = (v, d, n)
    if not by_kernel:
        return None, {}
    k = max(by_kernel, key=lambda kk: max(x[1] * x[2] for x in by_kernel[kk].values()))
    return k, {cn: (v, d) for cn, (v, d, n) in by_kernel[k].items()}


def calib(db):
    c = sqlite3.connect(db)
    out = {}
    for k, cn, v in c.execute("select kernel_name, counter_name, avg(value) from counters_collection "
                              "group by kernel_name, counter_name"):
        name = k.split("(")[0].replace("void ", "")
        if name.startswith(("k_stream", "k_gather", "k_scatter")):
            out.setdefault(name, {})[cn] = v
    return out


def main():
    pmc = sys.argv[1]
    ea = sys.argv[2] if len(sys.argv) > 2 else pmc
    merged = {}
    kernel = None
    for sub in ("sq", "fetch", "write", "l2req"):
        db = os.path.join(pmc, sub, "run_results.db")
        if os.path.exists(db):
            k, c = counters(db)
            kernel = kernel or k
            merged.update(c)
    for sub in ("ea_TCC_EA0_RDREQ_sum", "ea_TCC_EA0_WRREQ_sum"):
        db = os.path.join(ea, sub, "run_results.db")
        if os.path.exists(db):
            merged.update(counters(db)[1])
    v = {k: x[0] for k, x in merged.items()}
    dur = {k: x[1] for k, x in merged.items()}
    t = dur["SQ_INSTS_VALU"] * 1e-9  # launch time of the SQ pass, s
    bench = json.load(open(os.path.join(pmc, "sq.json")))
    queries = bench["config"]["rays_per_step"]
    clock = v["GRBM_GUI_ACTIVE"] / XCDS / (dur["GRBM_GUI_ACTIVE"] * 1e-9)
    valu_slots = SIMDS * clock * t / 2.0
    rd128, rd64, rd32 = (v.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) for s in (128, 64, 32))
    wr, wr64 = v.get("TCC_EA0_WRREQ_sum", 0.0), v.get("TCC_EA0_WRREQ_64B_sum", 0.0)
    hbm_read = 128 * rd128 + 64 * rd64 + 32 * rd32
    hbm_write = 64 * wr64 + 32 * (wr - wr64)
    l2_bytes = 128.0 * (v["TCP_TCC_READ_REQ_sum"] + v["TCP_TCC_WRITE_REQ_sum"])
    lib = os.path.join(ROOT, "toymeshpathtracer_amd", "_lib", "libtmpt.so")
    sha = subprocess.run(["sha256sum", lib], capture_output=True, text=True).stdout.split()[0][:16] \
        if os.path.exists(lib) else None
    rec = {
        "kernel": kernel, "queries_per_launch": queries, "launch_ms": round(t * 1e3, 3),
        "clock_ghz": round(clock / 1e9, 4), "lib_sha256_16": sha, "source": [pmc, ea],
        "per_query": {
            "valu_insts": v["SQ_INSTS_VALU"] / queries,
            "l2_bytes": l2_bytes / queries,
            "hbm_read_bytes": hbm_read / queries,
            "hbm_write_bytes": hbm_write / queries,
        },
        "valu": {"insts": v["SQ_INSTS_VALU"], "issue_slots": valu_slots,
                 "frac": v["SQ_INSTS_VALU"] / valu_slots,
                 "frac_at_2p4ghz": v["SQ_INSTS_VALU"] / (SIMDS * SPEC_CLOCK_HZ * t / 2.0),
                 "lane_utilisation": v["SQ_THREAD_CYCLES_VALU"] / (64.0 * v["SQ_ACTIVE_INST_VALU"]),
                 "salu_insts": v.get("SQ_INSTS_SALU"),
                 "wave_cycles_waiting_frac": v.get("SQ_WAIT_ANY", 0) / v["SQ_WAVE_CYCLES"]},
        "l2": {"read_req": v["TCP_TCC_READ_REQ_sum"], "write_req": v["TCP_TCC_WRITE_REQ_sum"],
               "bytes": l2_bytes, "tbps": l2_bytes / t / 1e12, "frac": l2_bytes / t / L2_PEAK_BPS,
               "hit_rate": v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"])},
        "hbm": {"read_req_128B": rd128, "read_req_64B": rd64, "read_req_32B": rd32,
                "write_req": wr, "write_req_64B": wr64,
                "read_bytes": hbm_read, "write_bytes": hbm_write,
                "fetch_size_x2_bytes": 2 * 1024 * v.get("FETCH_SIZE", 0.0),
                "write_size_bytes": 1024 * v.get("WRITE_SIZE", 0.0),
                "gbps": (hbm_read + hbm_write) / t / 1e9, "frac": (hbm_read + hbm_write) / t / 8e12},
    }
    cal = {}
    for sub in ("cal_FETCH_SIZE", "cal_WRITE_SIZE", "cal_TCP_TCC_READ_REQ_sum", "cal_TCC_HIT_sum"):
        db = os.path.join(pmc, sub, "run_results.db")
        if os.path.exists(db):
            for k, d in calib(db).items():
                cal.setdefault(k, {}).update(d)
    for sub in ("cal_ea_TCC_EA0_RDREQ_sum", "cal_ea_TCC_EA0_WRREQ_sum"):
        db = os.path.join(ea, sub, "run_results.db")
        if os.path.exists(db):
            for k, d in calib(db).items():
                cal.setdefault(k, {}).update(d)
    known = json.load(open(os.path.join(pmc, "cal_FETCH_SIZE.json")))
    names = {"k_stream<0>": "stream", "k_gather<16, 1>": "gather16_big", "k_gather<64, 1>": "gather64_big",
             "k_gather<128, 1>": "gather128_big", "k_gather<16, 0>": "gather16_small", "k_scatter<16>": "scatter16_nt"}
    rec["calibration"] = {names.get(k, k): {"known": known.get(names.get(k, k)), "counters": d} for k, d in cal.items()}
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
