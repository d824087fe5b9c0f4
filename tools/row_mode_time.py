"""Row seeding (the unmodified reference stream, one chain per row) on the bench
frame at reduced spp: frame time and MRays/s (time scales with spp)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
lanes = (sys.argv[2] if len(sys.argv) > 2 else "1").split(",")  # TMPT_ROW_LANES variants
with tm.Scene(tris) as sc:
    ref = None
    for rl in lanes:
        os.environ["TMPT_ROW_LANES"] = rl
        t0 = time.perf_counter()
        img, rays = sc.trace_image(cam, 1920, 1080, spp, seed_mode=tm.SEED_ROW)
        dt = time.perf_counter() - t0
        if ref is None:
            ref = img
        assert (img == ref).all(), f"TMPT_ROW_LANES={rl} changed the image"
        print(f"row, {rl} rows per wave: 1920x1080x{spp}: {dt * 1e3:.1f} ms, {rays / dt / 1e6:.1f} MRays/s",
              flush=True)
    t0 = time.perf_counter()
    img, rays = sc.trace_image(cam, 1920, 1080, spp, seed_mode=tm.SEED_SAMPLE)
    dt = time.perf_counter() - t0
    print(f"sample: 1920x1080x{spp}: {dt * 1e3:.1f} ms, {rays / dt / 1e6:.1f} MRays/s", flush=True)
