import os, sys, time
sys.path.insert(0, '.')
import numpy as np, toymeshpathtracer_amd as tm
for obj, W, H, spp in [("suzanne.obj", 640, 360, 4), ("teapot.obj", 1280, 720, 16)]:
    tris, bmin, bmax = tm.load_scene(os.path.join("data", obj))
    cam = tm.Camera.for_scene(bmin, bmax, W, H)
    with tm.Scene(tris) as sc:
        ref = None
        for look in ["7", "15", "31"]:
            os.environ["TMPT_ROWSPEC_LOOK"] = look
            sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_ROW)
            ts = []
            for _ in range(3):
                t0 = time.perf_counter(); img, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_ROW); ts.append(time.perf_counter() - t0)
            if ref is None: ref = (img, rays)
            assert rays == ref[1] and np.array_equal(img, ref[0])
            print(f"{obj} {W}x{H}x{spp} lookahead {look}: {np.median(ts)*1e3:.1f} ms, {rays/np.median(ts)/1e6:.1f} MRays/s", flush=True)
