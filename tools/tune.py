"""Interleaved A/B of scene-option variants in ONE process on the bench frame
(sponza stand-in 1920x1080, pixel seeding by default; MI355X_MICROARCH-style
rule: compare variants in one process, interleaved rounds).

  python tools/tune.py "builder=lbvh;ploc_radius=16&leaf_max=4;sample_block=2&ENGINE=wavefront" [spp] [rounds]

Variants are separated by ';', options within a variant by '&' (include/tmpt.h
"Scene options").  Build options select a scene built once per distinct
setting; render options are set on it before each render; ENGINE picks the
engine.  Every variant's image must equal the first one's (bit-exact contract).
Harness settings: TUNE_SCENE, TUNE_SHARDS, TUNE_BAND, TUNE_SEED, TUNE_RES,
TUNE_COUNT, TUNE_OCTREE (0: no reference octree, ties by index); another
library build: TMPT_LIB_PATH (one per process)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

BUILD_KEYS = ("builder", "layout", "leaf_max", "collapse", "ploc_radius", "sah_c_leaf", "sah_c_tri")
ENGINES = {"wavefront": tm.ENGINE_WAVEFRONT, "persistent": tm.ENGINE_PERSISTENT, "mega": tm.ENGINE_MEGAKERNEL}

variants = sys.argv[1].split(";") if len(sys.argv) > 1 else [""]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
scene_name = os.environ.get("TUNE_SCENE", "sponza")
SHARDS = int(os.environ.get("TUNE_SHARDS", "1"))  # >1: render shard 0 of N (per-rank load at N GPUs)
BAND = int(os.environ.get("TUNE_BAND", "16"))  # rows per band dealt round-robin to the shards
SEED = {"pixel": tm.SEED_PIXEL, "sample": tm.SEED_SAMPLE}[os.environ.get("TUNE_SEED", "pixel")]
W, H = map(int, os.environ.get("TUNE_RES", "1920x1080").split("x"))
path = gen_standin_sponza.ensure() if scene_name == "sponza" else os.path.join(ROOT, "data", scene_name)
tris, bmin, bmax = tm.load_scene(path)
cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=scene_name == "sponza")


def parse(v):
    d = {}
    for kv in filter(None, v.split("&")):
        k, _, val = kv.partition("=")
        d[k.strip()] = val.strip()
    return d


scenes = {}
with tm.Scene(tris[:1]) as _probe:  # render-option defaults, restored after each variant
    DEFAULTS = {}
    for _k in ("sample_block", "sbuf_max", "sbuf_pair", "pilot", "help", "pair", "balance", "dprio", "wave_cap", "pixel_chains", "rowspec",
               "rowspec_wmax", "rowspec_windows", "rowspec_spread", "rowspec_groups", "rowspec_noshadow",
               "rowspec_chase", "rowspec_stream", "wf_bins", "tie_rule", "tie_defer", "redo_cap", "redo_inline", "redo_lanes"):
        try:  # an older library build (TMPT_LIB_PATH) may not know every option
            DEFAULTS[_k] = _probe.get_option(_k)
        except tm.TmptError:
            pass


def scene_for(env):
    key = tuple((k, env.get(k)) for k in BUILD_KEYS)
    if key not in scenes:
        sc = tm.Scene(tris, options={k: v for k, v in key if v is not None},
                      bounds=None if os.environ.get("TUNE_OCTREE") == "0" else (bmin, bmax))
        st = sc.stats()
        print(f"scene {dict(key)}: build {st.build_ms:.1f} ms, bvh4 nodes {st.bvh4_nodes}, depth4 "
              f"{st.bvh4_depth}, ploc iters {st.builder_iters}", flush=True)
        if os.environ.get("TUNE_COUNT"):  # node visits / triangle tests per query (4 spp)
            _, q = sc.trace_image(cam, W, H, 4, seed_mode=SEED, band_rows=BAND, count_visits=True)
            cs = sc.stats()
            print(f"  visits per query at 4 spp: nodes {(cs.node_visits + cs.shadow_node_visits) / q:.3f}, "
                  f"tris {(cs.tri_tests + cs.shadow_tri_tests) / q:.3f} ({q} queries)", flush=True)
        scenes[key] = sc
    return scenes[key]


res = {v: [] for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        env = parse(v)
        sc = scene_for(env)
        for k, val in env.items():  # render options: set for this render, defaults otherwise
            if k not in BUILD_KEYS and k != "ENGINE":
                sc.set_option(k, float(val))
        t0 = time.perf_counter()
        img, rays = sc.trace_image(cam, W, H, spp, seed_mode=SEED, band_rows=BAND, shard=0,
                                   num_shards=SHARDS, engine=ENGINES[env.get("ENGINE", "persistent")])
        dt = time.perf_counter() - t0
        st = sc.stats()
        for k in env:
            if k not in BUILD_KEYS and k != "ENGINE":
                sc.set_option(k, DEFAULTS[k])
        if ref is None:
            ref, ref_rays = img, rays
        if "tie_rule" not in env:  # the tie rule alone may change answers (include/tmpt.h)
            assert np.array_equal(img, ref), f"variant {v!r} changed the image"
            assert rays == ref_rays, f"variant {v!r} changed the ray count ({rays} vs {ref_rays})"
        res[v].append((rays / dt / 1e6, st.extend_ms, st.shadow_ms, dt * 1e3))
        if getattr(st, "redo_late", 0):
            print(f"  {v or 'default'} round {r}: {st.redo_late} re-traces left to k_redo, "
                  f"extend {st.extend_ms:.1f} ms", flush=True)
for v, xs in res.items():
    a = np.array(xs)
    print(f"{v or 'default':>48}: {np.median(a[:, 0]):8.1f} MRays/s  extend {np.median(a[:, 1]):7.1f} ms  "
          f"shadow {np.median(a[:, 2]):7.1f} ms  frame {np.median(a[:, 3]):7.1f} ms"
          + (f"  (render ms mean {a[:, 1].mean():.2f} sd {a[:, 1].std():.2f} min {a[:, 1].min():.2f}, n={len(a)}: "
             + " ".join(f"{x:.1f}" for x in a[:, 1]) + ")" if len(a) > 2 else ""), flush=True)
