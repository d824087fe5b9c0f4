"""Row seeding (the reference's unmodified RNG, main.cpp:204) on the bench frame:
the speculative row engine's variants against each other, interleaved in one
process; every variant's image and ray count must equal the first one's.

  python tools/rowspec_time.py "rowspec_groups=1;rowspec_groups=2&rowspec_windows=4" [spp] [rounds]

Variants are scene render options (include/tmpt.h); ENGINE=mega runs the
one-lane-per-row megakernel instead.  With the diagnostic library build
(make DIAG=1, TMPT_LIB_PATH) TMPT_ROWSPEC_LOG=1 prints iterations and the
speculation factor per render."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402



def main():
    variants = sys.argv[1].split(";") if len(sys.argv) > 1 else [""]
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    W, H = map(int, os.environ.get("TUNE_RES", "1920x1080").split("x"))
    shards = int(os.environ.get("TUNE_SHARDS", "1"))
    tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
    cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=True)
    sc = tm.Scene(tris)
    defaults = {}
    for k in ("rowspec", "rowspec_wmax", "rowspec_windows", "rowspec_spread", "rowspec_groups", "rowspec_noshadow",
              "rowspec_chase", "rowspec_stream"):
        try:  # an older library build (TMPT_LIB_PATH) may not know every option
            defaults[k] = sc.get_option(k)
        except tm.TmptError:
            pass
    ref = None
    res = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            env = dict(kv.split("=", 1) for kv in v.split("&") if kv)
            for k, val in defaults.items():
                sc.set_option(k, val)
            for k, val in env.items():
                if k != "ENGINE":
                    sc.set_option(k, float(val))
            eng = tm.ENGINE_MEGAKERNEL if env.get("ENGINE") == "mega" else tm.ENGINE_PERSISTENT
            t0 = time.perf_counter()
            img, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_ROW, engine=eng, band_rows=1,
                                       shard=0, num_shards=shards)
            dt = time.perf_counter() - t0
            if ref is None:
                ref = (img, rays)
            assert rays == ref[1] and np.array_equal(img, ref[0]), f"variant {v!r} changed the image"
            res[v].append((dt * 1e3, rays / dt / 1e6))
            print(f"{v or 'default'}: {dt * 1e3:.1f} ms, {rays / dt / 1e6:.1f} MRays/s", flush=True)
    for v, xs in res.items():
        a = np.array(xs)
        print(f"{v or 'default':>60}: frame {np.median(a[:, 0]):8.1f} ms  {np.median(a[:, 1]):7.1f} MRays/s "
              f"({rays} rays, {spp} spp, 1/{shards} shard)", flush=True)


if __name__ == "__main__":
    main()
