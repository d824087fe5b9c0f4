#!/usr/bin/env python3
"""bench.py -- MRays/s of the hot path (Trace -> Scatter -> Scene::HitScene) on MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it
is launched by torch.distributed.run, one rank per GPU.  One *step* = one full
frame of BASELINE.json configs[3]: sponza.obj 1920x1080, 64 spp (the
deterministic stand-in scene, data/gen_standin_sponza.py; the real sponza.obj
is absent from the reference), sample seeding (below), persistent path engine.  The frame
is sharded over the N GPUs in rows dealt round-robin (1-row bands; total work fixed:
strong scaling); each rank renders its bands straight into a device tensor and
one RCCL gather over xGMI assembles the image on rank 0 -- inside the timed
region.  value = all rays of all ranks / max-over-ranks wall time.

Seeding (--seed-mode): "sample" (default) = every pixel's own xorshift stream
(seed (y*W+x)*9781+1, as pixel mode) with sample s starting 2^16*s steps into
it, so a pixel's samples are independent work units; "pixel" = one stream per
pixel, samples in sequence (the per-pixel chain bounds strong scaling); "row" =
the reference's own seeding, unmodified (main.cpp:204: one stream threaded
through a row's pixels and samples; byte-identical to the reference binary),
run by the speculative row engine.  All three are byte-exact against their
oracle legs (tests/); the line also reports the other modes' throughput
(seed_modes), timed the same way after the main run.

Launch: `python bench.py --gpus N` with N > 1 and no launcher around it (no
WORLD_SIZE in the environment) starts N ranks itself -- this process runs
`torch.distributed.run` as a child before it has touched the GPU, and exits
with its code -- after checking that N GPUs are visible (nccl; the gloo
rehearsal may put several ranks on one GPU).  Under a launcher, WORLD_SIZE must
equal --gpus.

Rank 0 prints ONE JSON line.  Besides the contract keys it carries
  roofline      dominant kernel (k_path: all queries of the frame), its mean
                launch time HIP-event timed on the stream it runs on, against
                three counter-backed ceilings (VALU issue, L2 requests, HBM
                bytes; per-query counts from the committed rocprofv3 record
                profiles/r*_counters_k_path.json); `bound` = the highest.  The
                SURVEY.md §8d algorithmic bytes (B_ray = 32 + 16 + 64*N_node +
                36*N_tri, N_node/N_tri from an instrumented run of the same kernel
                at reduced spp) are reported under roofline.algorithmic
  cpu_baseline  the CPU restatement of the reference algorithm (octree +
                Moller-Trumbore, oracle/, bit-exact to the reference binary on the
                pinned cases) timed on this host on a bounded row sample of the same
                frame, N=1 only
Everything else goes to stderr.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="sponza1080", choices=["sponza1080", "teapot720", "suzanne360", "sponza4k"])
    ap.add_argument("--engine", default="persistent", choices=["wavefront", "persistent", "mega"])
    ap.add_argument("--seed-mode", default="sample", choices=["sample", "pixel", "row"])
    ap.add_argument("--no-compare", action="store_true", help="skip timing the other seeding modes")
    ap.add_argument("--compare", action="store_true",
                    help="time the other seeding modes at N>1 too (default: only at N=1, so the driver's "
                         "multi-GPU runs are not slowed)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the collective path (process group, gather, max-over-ranks) even at one rank "
                         "(tests the RCCL calls on a 1-GPU box)")
    ap.add_argument("--count-spp", type=int, default=4, help="spp of the instrumented run")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline: time budget of the row sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--save", default="", help="rank 0 writes the frame as PNG here")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (default); gloo = CPU rehearsal of the N>1 path "
                         "(ranks may share one GPU)")
    return ap.parse_args(argv)


def visible_gpus_without_hip() -> int:
    """GPUs this process would see, counted without touching HIP: the KFD
    topology's GPU nodes (simd_count > 0), narrowed by the visibility
    variables.  0 without a KFD (no GPU HIP could open); -1 when the topology
    is there but unreadable (each rank then checks its own LOCAL_RANK)."""
    nodes = "/sys/class/kfd/kfd/topology/nodes"
    if not os.path.isdir(nodes):
        return 0
    try:
        n = 0
        for d in os.listdir(nodes):
            with open(os.path.join(nodes, d, "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            n += int(props.get("simd_count", "0")) > 0
    except (OSError, ValueError):
        return -1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def launch_ranks_if_needed() -> None:
    """--gpus N without a launcher: run N ranks under torch.distributed.run (a
    child process; this one makes no HIP call -- it counts GPUs from the KFD
    topology -- and exits with the child's code).  Fails loudly when nccl
    would need more GPUs than are visible."""
    args = parse_args()
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return
    ndev = visible_gpus_without_hip()
    if args.dist_backend == "nccl" and 0 <= ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs for RCCL (one rank per GPU); "
              f"{ndev} visible", file=sys.stderr, flush=True)
        sys.exit(2)
    if ndev == 0:
        print("bench.py: no GPU visible", file=sys.stderr, flush=True)
        sys.exit(2)
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: starting {args.gpus} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    sys.exit(subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode)


if __name__ == "__main__":
    launch_ranks_if_needed()

import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402  (imports torch first: one HIP runtime)
from toymeshpathtracer_amd import shard as sharding  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "MRays/s on sponza.obj 1920x1080 64spp at 1/2/4/8 GPUs; %HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (spec)
L2_PEAK_BPS = 34.5e12  # MI355X_MICROARCH.md, L2 (aggregate over the 8 XCDs)
BAND_ROWS = 1   # rows dealt round-robin: every rank gets H/N rows of statistically equal cost
S_NODE = 64            # bytes per visited node: BVH4Q (4 quantised child boxes + links) or BVH2
S_TRI = 36             # bytes per triangle test (3 x vec3), SURVEY.md §8d
S_RAY = 32 + 16        # ray read + hit write, SURVEY.md §8d

# What each seeding mode is (tmpt.h TMPT_SEED_*).  Only row
# seeding threads the reference's own stream (main.cpp:204) and so reproduces
# the reference binary's image; pixel and sample seeding are the north star's
# "same per-pixel xorshift seed" contract, each byte-exact against its oracle leg.
RNG_CONTRACT = {
    "sample": "per-pixel seed (y*W+x)*9781+1; sample s starts 2^16*s xorshift steps into the pixel's stream "
              "(NOT the reference's row-chained stream: statistically equivalent image, not the reference "
              "binary's bytes; reference-exact row seeding is timed under seed_modes.row)",
    "pixel": "per-pixel seed (y*W+x)*9781+1, the pixel's samples in sequence (NOT the reference's row-chained "
             "stream; reference-exact row seeding is timed under seed_modes.row)",
    "row": "the reference's own seeding, unmodified: y*9781+1 per row, threaded through the row's pixels and "
           "samples (main.cpp:204); byte-identical to the reference binary",
}

CONFIGS = {
    # name: (obj, width, height, spp, is_sponza)
    "sponza1080": ("sponza", 1920, 1080, 64, True),    # BASELINE configs[3]: the metric's config
    "teapot720": ("teapot.obj", 1280, 720, 16, False),  # configs[2]
    "suzanne360": ("suzanne.obj", 640, 360, 4, False),  # configs[1]
    "sponza4k": ("sponza", 3840, 2160, 256, True),      # configs[4] (8-GPU config)
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def scene_path(obj: str) -> str:
    if obj == "sponza":
        import gen_standin_sponza
        return gen_standin_sponza.ensure()
    return os.path.join(ROOT, "data", obj)


def counter_record() -> dict:
    """The newest counter record of k_path (profiles/r*_counters_k_path.json,
    tools/roofline_counters.py over rocprofv3 --pmc passes of this bench, one
    pass per counter set, and the calibration kernel tools/pmc_calib.hip).
    PMC needs rocprofv3 around the process, so the live bench cannot collect
    it itself; it scales the record's per-query figures by its own queries and
    launch time.  stale = the record was taken with another libtmpt.so build."""
    import glob
    import hashlib
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_counters_k_path.json")))
    if not files:
        return {}
    with open(files[-1]) as f:
        rec = json.load(f)
    rec["_source"] = os.path.relpath(files[-1], ROOT)
    try:
        with open(tm.lib_path, "rb") as f:
            rec["_stale"] = hashlib.sha256(f.read()).hexdigest()[:16] != rec.get("lib_sha256_16")
    except OSError:
        rec["_stale"] = None
    return rec


def roofline(queries: float, launch_ms: float, b_ray: float, kernel: str, counters_apply: bool = True) -> dict:
    """Ceilings of the dominant kernel, each as achieved / peak over the live
    launch time (the bound is the resource that binds, from
    counters; the SURVEY §8d algorithmic bytes are reported beside it):
      valu_issue  VALU instructions (per query, counted) / (1024 SIMDs x 2.4 GHz / 2)
      l2          L1->L2 requests x 128 B (per query, counted) / 34.5 TB/s
      hbm         fabric bytes (EA requests by size, counted) / 8 TB/s
    `bound` is the highest; `achieved`, `peak`, `frac` are its.  The algorithmic
    bytes (48 + 64 N_node + 36 N_tri per query, instrumented run) are served by
    L1 / L2 (hit rates in the record), so against HBM they are not a bound."""
    t = launch_ms * 1e-3
    # the record's per-query counts are the sample-seeding k_path's (SAMP=1);
    # another seeding runs other kernels, so its ceilings are not given
    rec = counter_record() if counters_apply else {}
    alg = {"bytes_per_query": round(b_ray, 1), "tbps": round(b_ray * queries / t / 1e12, 3),
           "frac_of_l2_peak": round(b_ray * queries / t / L2_PEAK_BPS, 4),
           "frac_of_hbm_peak": round(b_ray * queries / t / (HBM_PEAK_GBS * 1e9), 4),
           "note": "SURVEY.md 8d algorithmic bytes; served from L1/L2 (see l2.hit_rate), not HBM"}
    out = {"kernel": kernel, "avg_launch_ms": round(launch_ms, 4), "queries_per_launch": int(queries),
           "algorithmic": alg}
    if not rec:
        out.update({"bound": "hbm", "achieved": round(alg["tbps"] * 1e3, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": alg["frac_of_hbm_peak"], "traffic": None,
                    "counter_ceilings": "not applicable: the counter record is the sample-seeding k_path's"
                    if not counters_apply else "no counter record"})
        return out
    pq = rec["per_query"]
    valu_rate = pq["valu_insts"] * queries / t
    valu_peak = 1024 * 2.4e9 / 2.0
    l2_rate = pq["l2_bytes"] * queries / t
    hbm_bytes = (pq["hbm_read_bytes"] + pq["hbm_write_bytes"]) * queries
    ceil = {
        "valu_issue": {"achieved": round(valu_rate / 1e9, 1), "peak": round(valu_peak / 1e9, 1), "unit": "Ginstr/s",
                       "frac": round(valu_rate / valu_peak, 4),
                       "lane_utilisation": round(rec["valu"]["lane_utilisation"], 4)},
        "l2": {"achieved": round(l2_rate / 1e9, 1), "peak": L2_PEAK_BPS / 1e9, "unit": "GB/s",
               "frac": round(l2_rate / L2_PEAK_BPS, 4), "hit_rate": round(rec["l2"]["hit_rate"], 4)},
        "hbm": {"achieved": round(hbm_bytes / t / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(hbm_bytes / t / (HBM_PEAK_GBS * 1e9), 4)},
    }
    bound = max(ceil, key=lambda k: ceil[k]["frac"])
    out.update({"bound": bound, "achieved": ceil[bound]["achieved"], "peak": ceil[bound]["peak"],
                "unit": ceil[bound]["unit"], "frac": ceil[bound]["frac"],
                "traffic": round(hbm_bytes), "traffic_unit": "bytes/launch (HBM: EA read+write requests by size)",
                "ceilings": ceil, "counter_source": rec["_source"], "counter_record_stale": rec["_stale"],
                "counter_kernel": rec["kernel"].split("(")[0]})
    return out


def host_cpus() -> dict:
    """Host cores as the reference's TBB would see them (main.cpp:250-251:
    task_scheduler_init(default_num_threads()) = every core the process may
    run on) and the cgroup CPU quota the box enforces, if any."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return {"nproc": aff, "os_cpu_count": os.cpu_count(), "cgroup_cpu_quota": quota, "cpu_model": model}


def cpu_baseline(args, tris, bmin, bmax, cam, W, H, SPP, frame):
    """The CPU restatement of the reference algorithm (octree + Moller-Trumbore,
    oracle/) on every CPU the process may use -- like TBB's default_num_threads()
    (main.cpp:250-251), but counted as the cgroup quota grants them, not as the
    host's thread count -- timed on a bounded sample
    of the same frame: batches of rows y = o (mod S), S ~ H / (2 threads) (two rows per
    thread), of which the pixels x = c (mod 32) (pixel and sample seeding:
    pixels are independent; row seeding renders whole rows of fewer rows per
    batch, its stream runs along the row), batches in a fixed scattered order
    until ~args.cpu_seconds have passed.  Also compares those pixels with the
    GPU frame (octree tie order)."""
    import oracle
    hc = host_cpus()
    # the CPUs the process may actually use: its affinity, capped by the
    # cgroup's CPU quota (the GPU box grants 16 of 256 host threads; more
    # threads than that only oversubscribe the quota); the oracle's pool holds <= 256
    eff = hc["nproc"] if not hc["cgroup_cpu_quota"] else min(hc["nproc"], max(1, int(hc["cgroup_cpu_quota"])))
    threads = max(1, min(eff, 256))
    osc = oracle.Scene(tris, accel=oracle.ACCEL_OCTREE, tie=oracle.TIE_VISIT, bmin=bmin, bmax=bmax)
    seed = {"sample": oracle.SEED_SAMPLE, "pixel": oracle.SEED_PIXEL, "row": oracle.SEED_ROW}[args.seed_mode]
    row_mode = args.seed_mode == "row"
    xs = 1 if row_mode else 32
    stride = max(1, H // (16 if row_mode else 2 * threads))
    batches = [(o, c) for c in range(xs) for o in range(stride)]
    order = [batches[(k * 7919) % len(batches)] for k in range(len(batches))] \
        if len(batches) % 7919 else batches
    ref = np.zeros((H, W, 4), np.uint8)
    mask = np.zeros((H, W), bool)
    crays, cdt, nb = 0, 0.0, 0
    for o, c in order:
        t1 = time.perf_counter()
        _, r = osc.render(cam.as_array(), W, H, SPP, seed_mode=seed, y0=o, row_step=stride, x0=c, x_step=xs,
                          threads=threads, rgba=ref)
        cdt += time.perf_counter() - t1
        crays += r
        mask[o::stride, c::xs] = True
        nb += 1
        if cdt >= args.cpu_seconds:
            break
    npx = int(mask.sum())
    cpu = {"value": round(crays / cdt / 1e6, 3), "unit": "MRays/s", "cores": threads, "kind": "port",
           "threads": threads, **hc,
           "sample": f"{npx} of {W * H} px ({nb} batches of rows y%{stride}==o, pixels x%{xs}==c) x {SPP} spp, "
                     f"{crays} rays, {cdt:.1f} s on {threads} threads = the effective CPUs (affinity "
                     f"{hc['nproc']}, cgroup quota {hc['cgroup_cpu_quota']}); octree restatement of scene.cpp, "
                     f"{args.seed_mode} seeding"}
    diff = int(((frame != ref).any(-1) & mask).sum())
    parity = {"pixels_checked": npx, "pixels_differ": diff, "oracle": "octree (reference tie order)"}
    return cpu, parity


def device_identity(local: int) -> dict:
    """The physical device this rank opened: PCI domain:bus:device and UUID
    (hipDeviceProp_t via torch), so an N>1 line proves which GPUs it ran on."""
    p = torch.cuda.get_device_properties(local)
    return {"pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", "uuid": str(p.uuid),
            "name": p.name, "local_rank": local}


def world_devices(ident: dict, world: int, dist_on: bool, backend: str) -> dict:
    """Every rank's device identity gathered to all ranks, summarised by
    shard.placement (`n_gpus` = distinct devices; a gloo rehearsal whose ranks
    share one GPU reports 1 with `ranks` N and `rehearsal` true)."""
    devs = [ident]
    if dist_on:
        devs = [None] * world
        dist.all_gather_object(devs, ident)
    return sharding.placement(devs, backend if dist_on else None)


@contextlib.contextmanager
def stdout_to_stderr():
    """Point file descriptor 1 at stderr for the duration (native libraries
    write to the descriptor, not to sys.stdout)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def main() -> None:
    args = parse_args()
    assert set(CONFIGS) == {"sponza1080", "teapot720", "suzanne360", "sponza4k"}

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # measuring another GPU count than asked for would mislabel the line
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world} (the launcher started {world} ranks)")
        sys.exit(2)
    dist_on = world > 1 or args.force_dist  # the collective path (process group, gather, reductions)
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and local >= ndev:
        log(f"bench.py: rank {rank} has LOCAL_RANK {local} but {ndev} visible GPUs (RCCL needs one GPU per rank)")
        sys.exit(2)
    local = local % max(ndev, 1) if args.dist_backend == "gloo" else local
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if dist_on:
        # RCCL prints a version banner on stdout when its communicator comes up;
        # route it to stderr so stdout carries only rank 0's JSON line
        with stdout_to_stderr():
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
            else:
                dist.init_process_group("gloo")
            dist.barrier()
    placement = world_devices(device_identity(local), world, dist_on, args.dist_backend)

    obj, W, H, SPP, sponza = CONFIGS[args.config]
    path = scene_path(obj)
    engine = {"wavefront": tm.ENGINE_WAVEFRONT, "persistent": tm.ENGINE_PERSISTENT,
              "mega": tm.ENGINE_MEGAKERNEL}[args.engine]
    seeds = {"sample": tm.SEED_SAMPLE, "pixel": tm.SEED_PIXEL, "row": tm.SEED_ROW}
    seed = seeds[args.seed_mode]
    tris, bmin, bmax = tm.load_scene(path)
    cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=sponza)
    t0 = time.perf_counter()
    # Scene + BuildOctree (main.cpp:165, 312): the BVH on the device, and the
    # reference's octree for the queries it decides (ties on t, its root box)
    scene = tm.Scene(tris, device=local, bounds=(bmin, bmax))
    init_s = time.perf_counter() - t0
    st0 = scene.stats()

    rows_of = sharding.all_rows(H, BAND_ROWS, world)
    max_rows = max(len(r) for r in rows_of)
    my_rows = len(rows_of[rank])
    tile = torch.zeros((max_rows, W, 4), dtype=torch.uint8, device=dev)
    gloo = dist_on and args.dist_backend == "gloo"
    gdev = torch.device("cpu") if gloo else dev
    gathered = [torch.empty(tile.shape, dtype=tile.dtype, device=gdev) for _ in range(world)] if rank == 0 else None
    image = torch.empty((H, W, 4), dtype=torch.uint8, device=dev) if rank == 0 else None

    def step(seed=seed):
        # out= a device tile: the render waits for torch's current stream
        # (TMPT_FLAG_WAIT_STREAM), on which torch orders the previous step's
        # gather / assembly of the same tile, and returns once the tile is done
        _, rays = scene.trace_image(cam, W, H, SPP, seed_mode=seed, engine=engine,
                                    band_rows=BAND_ROWS, shard=rank, num_shards=world,
                                    out=tile.data_ptr())
        st = scene.stats()
        if dist_on:
            dist.gather(tile.cpu() if gloo else tile, gathered, dst=0)
        if rank == 0:  # de-interleave the bands into the frame, on the device
            parts = [g.to(dev) for g in gathered] if gloo else (gathered if dist_on else [tile])
            sharding.assemble(parts, rows_of, image)
        return rays, st

    for _ in range(args.warmup):
        step()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rays = 0
    ext_ms = sh_ms = 0.0
    ext_rays = sh_rays = 0
    ext_launches = 0
    ties = roots = redo = redo_late = cracks = 0
    redo_launches = redo_rays = 0
    redo_ms = 0.0
    last_tie_path = 0
    for _ in range(args.steps):
        r, st = step()
        ties += st.tie_queries
        roots += st.root_misses
        cracks += st.crack_queries
        redo += st.redo_samples
        redo_late += st.redo_late
        redo_launches += st.redo_launches
        redo_ms += st.redo_ms
        redo_rays += st.redo_rays
        last_tie_path = st.tie_path
        rays += r
        ext_ms += st.extend_ms
        sh_ms += st.shadow_ms
        ext_rays += st.extend_rays
        sh_rays += st.shadow_rays
        ext_launches += st.extend_launches
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=gdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays], dtype=torch.int64, device=gdev)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays = int(r.item())

    value = rays / elapsed / 1e6

    # ---- the other seeding mode, timed the same way (reported, not `value`)
    frame = image.cpu().numpy() if rank == 0 else None
    compare = {}
    if not args.no_compare and (world == 1 or args.compare):
        for name, sd in seeds.items():
            if sd == seed:
                continue
            if name == "row" and W * H * SPP > 1920 * 1080 * 64:  # ~3 s per 1080p64 frame: skip larger ones
                compare[name] = {"skipped": "frame larger than sponza1080 (row seeding ~3 s per 1080p 64 spp frame)"}
                continue
            step(sd)
            if dist_on:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            csteps = min(args.steps, 3)  # informational: a few frames (row seeding takes ~3 s each)
            crays = 0
            engines, fallbacks = set(), 0
            for _ in range(csteps):
                r_, st_ = step(sd)
                crays += r_
                engines.add(st_.row_engine)
                fallbacks += st_.stream_fallbacks
            torch.cuda.synchronize()
            if dist_on:
                dist.barrier()
            cel = time.perf_counter() - t1
            if dist_on:
                t = torch.tensor([cel], dtype=torch.float64, device=gdev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                cel = float(t.item())
                r = torch.tensor([crays], dtype=torch.int64, device=gdev)
                dist.all_reduce(r, op=dist.ReduceOp.SUM)
                crays = int(r.item())
            compare[name] = {"value": round(crays / cel / 1e6, 2), "ms_per_step": round(cel / csteps * 1e3, 2),
                             "rays_per_step": crays // csteps, "steps": csteps}
            if name == "row":  # which row engine ran, and whether the streaming launch fell back
                compare[name].update({"row_engine": sorted({3: "streaming", 2: "iterated", 1: "lane per row"}
                                                           .get(e, str(e)) for e in engines),
                                      "stream_fallbacks": fallbacks})
    # ---- the same frames with ties by the lowest index (option tie_rule=index,
    # the exact-semantics contract of rounds 1-3): what the reference's own tie
    # answer costs (reported, not `value`)
    index_rule = None
    if not args.no_compare and st0.tie_rule == 0:
        scene.set_option("tie_rule", 1)
        step()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        csteps = min(args.steps, 5)
        crays = 0
        for _ in range(csteps):
            crays += step()[0]
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        cel = time.perf_counter() - t1
        if dist_on:
            t = torch.tensor([cel], dtype=torch.float64, device=gdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            cel = float(t.item())
            r = torch.tensor([crays], dtype=torch.int64, device=gdev)
            dist.all_reduce(r, op=dist.ReduceOp.SUM)
            crays = int(r.item())
        scene.set_option("tie_rule", 0)
        index_rule = {"value": round(crays / cel / 1e6, 2), "ms_per_step": round(cel / csteps * 1e3, 2),
                      "steps": csteps, "cost_of_reference_ties": round(1.0 - value / (crays / cel / 1e6), 4)}
    if rank != 0:
        scene.close()
        dist.destroy_process_group()
        return
    if dist_on:
        log(f"gathered frame: {world} ranks ({args.dist_backend}), {rays} rays")

    # ---- roofline of the dominant kernel (extend), from an instrumented run
    _, _ = scene.trace_image(cam, W, H, args.count_spp, seed_mode=seed, engine=engine,
                             band_rows=BAND_ROWS, shard=rank, num_shards=world,
                             count_visits=True, out=tile.data_ptr())
    cs = scene.stats()
    roof = None
    if engine == tm.ENGINE_WAVEFRONT and cs.extend_rays and ext_launches:
        n_node = cs.node_visits / cs.extend_rays
        n_tri = cs.tri_tests / cs.extend_rays
        n_node_s = cs.shadow_node_visits / max(cs.shadow_rays, 1)
        n_tri_s = cs.shadow_tri_tests / max(cs.shadow_rays, 1)
        b_ray = S_RAY + S_NODE * n_node + S_TRI * n_tri
        per_launch_rays = ext_rays / ext_launches
        avg_launch_ms = ext_ms / ext_launches
        achieved = b_ray * per_launch_rays / (avg_launch_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                "kernel": "k_wf_trace<closest-hit> (extend)",
                "bytes_per_ray": round(b_ray, 1), "n_node_per_ray": round(n_node, 2),
                "n_tri_per_ray": round(n_tri, 2), "avg_launch_ms": round(avg_launch_ms, 4),
                "rays_per_launch": round(per_launch_rays, 1),
                "shadow_bytes_per_ray": round(S_RAY + S_NODE * n_node_s + S_TRI * n_tri_s, 1),
                "extend_ms_per_step": round(ext_ms / args.steps, 2),
                "shadow_ms_per_step": round(sh_ms / args.steps, 2)}
    elif engine == tm.ENGINE_PERSISTENT and cs.extend_rays and ext_launches:
        # one launch per frame serves both query kinds: per-query averages over all of them
        q = cs.extend_rays + cs.shadow_rays
        n_node = (cs.node_visits + cs.shadow_node_visits) / q
        n_tri = (cs.tri_tests + cs.shadow_tri_tests) / q
        b_ray = S_RAY + S_NODE * n_node + S_TRI * n_tri
        kernel = {"sample": "k_path<SAMP=1> (persistent: closest-hit + shadow queries + shading, sample units)",
                  "pixel": "k_path<SAMP=0> (persistent, pixel chains; pilot + cost-ordered pass)",
                  "row": "streaming row engine: k_path<SAMP=4> speculative launch + k_path<SAMP=2> chain re-trace; "
                         "reference-chain rays only (the speculative traces are ~11x as many)"}[args.seed_mode]
        # per k_path launch: its own queries and time; a k_redo launch (the
        # deferred-tie samples the main launch's tail left) is reported apart
        roof = roofline((ext_rays + sh_rays - redo_rays) / ext_launches, ext_ms / ext_launches, b_ray, kernel,
                        counters_apply=args.seed_mode == "sample")
        roof.update({"n_node_per_query": round(n_node, 2), "n_tri_per_query": round(n_tri, 2),
                     "k_path_launches": ext_launches, "redo_launches": redo_launches,
                     "redo_ms": round(redo_ms, 3), "redo_queries": redo_rays})

    # ---- CPU baseline: the reference algorithm on this host, bounded row sample
    cpu = None
    parity = None
    if world == 1 and not args.no_cpu:
        cpu, parity = cpu_baseline(args, tris, bmin, bmax, cam, W, H, SPP, frame)

    if args.save:
        tm.write_png(args.save, frame)

    # ---- host paths either side of the hot path: OBJ
    # ingest and PNG encode, sequential vs parallel (off the timed region, as in
    # main.cpp:122-170 / 341-342)
    host = None
    if rank == 0:
        import tempfile

        def timed(fn, env, val):
            old = os.environ.get(env)
            os.environ[env] = str(val)
            try:
                t = time.perf_counter()
                fn()
                return round((time.perf_counter() - t) * 1e3, 2)
            finally:
                if old is None:
                    del os.environ[env]
                else:
                    os.environ[env] = old

        png = os.path.join(tempfile.gettempdir(), f"tmpt_bench_{os.getpid()}.png")
        nt = min(16, os.cpu_count() or 1)
        host = {"obj_parse_ms": {"threads_1": timed(lambda: tm.load_scene(path), "TMPT_OBJ_THREADS", 1),
                                 f"threads_{nt}": timed(lambda: tm.load_scene(path), "TMPT_OBJ_THREADS", nt)},
                "png_encode_ms": {"threads_1": timed(lambda: tm.write_png(png, frame), "TMPT_PNG_THREADS", 1),
                                  f"threads_{nt}": timed(lambda: tm.write_png(png, frame), "TMPT_PNG_THREADS", nt)},
                "obj_bytes": os.path.getsize(path), "png_bytes": os.path.getsize(png)}
        os.remove(png)

    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "MRays/s", "n_gpus": placement["n_gpus"],
        "ranks": placement["ranks"], "dist_backend": placement["dist_backend"], "devices": placement["devices"],
        "rehearsal": placement["rehearsal"],
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: deterministic stand-in for the absent sponza.obj (66,452 tris incl. "
                "floor, data/gen_standin_sponza.py)" if sponza else "data/*.obj from the reference",
        "config": {"workload": f"{args.config}: {os.path.basename(path)} {W}x{H} {SPP}spp",
                   "global_batch": W * H, "spp": SPP, "tris": int(tris.shape[0]),
                   "seed_mode": args.seed_mode, "rng": RNG_CONTRACT[args.seed_mode],
                   "image_is_reference_binary_image": args.seed_mode == "row", "engine": args.engine,
                   "parallelism": f"row-bands{BAND_ROWS}x{world}",
                   "rays_per_step": rays // args.steps},
        "seed_modes": compare,
        "roofline": roof, "cpu_baseline": cpu, "parity_sample": parity, "host_paths": host,
        "scene_init_s": round(init_s, 3), "bvh_build_ms": round(st0.build_ms, 2),
        "bvh": {"lbvh2_depth": st0.bvh_depth, "bvh4_nodes": st0.bvh4_nodes, "bvh4_depth": st0.bvh4_depth,
                "leaf_max": st0.leaf_max, "builder": "ploc" if st0.builder_iters else "lbvh",
                "ploc_iters": st0.builder_iters},
        # the reference's octree (scene.cpp:99-160, host-built) answers the
        # closest hits whose t two or more triangles share, in its visit order
        "reference_octree": {"nodes": st0.octree_nodes, "leaves": st0.octree_leaves, "refs": st0.octree_refs,
                             "build_ms": round(st0.octree_build_ms, 1), "tie_rule": "visit" if st0.tie_rule == 0 else "index",
                             "tie_queries_per_step": ties // max(args.steps, 1),
                             "root_misses_per_step": roots // max(args.steps, 1),
                             # hits that may lie in a crack between the octree's subtree
                             # boxes, answered over it too
                             "crack_queries_per_step": cracks // max(args.steps, 1),
                             # sample seeding at >= 192 samples per lane: tied samples dropped by
                             # the main loop and traced again in the launch's tail
                             "tie_answer": "deferred" if redo else "in the main loop",
                             # tmpt_stats.tie_path of the last timed render: 1 main loop, 2 deferred,
                             # 3 deferral chosen but its list did not fit (main loop)
                             "tie_path": last_tie_path,
                             # triangles flat on an octree plane: with any, shadow answers are
                             # checked too and the deferral / shadow offload are off
                             "octree_flat": st0.octree_flat,
                             "redo_samples_per_step": redo // max(args.steps, 1),
                             "redo_late_total": redo_late,
                             "index_rule": index_rule},
    }
    print(json.dumps(out), flush=True)
    scene.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
