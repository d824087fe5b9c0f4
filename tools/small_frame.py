"""Where the time of a small frame goes: per-call wall
time of trace_image split into the k_path launch (HIP events around it), the
render's other device work (memsets, resolve: render_ms - extend_ms) and the
host side (API, stream sync, image readback: wall - render_ms), for the small
BASELINE configs, in sample seeding, host image and device output.

  python tools/small_frame.py [calls]   -> one JSON line per config + a table
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402

CONFIGS = [  # name, obj, W, H, spp
    ("cube640", "cube.obj", 640, 360, 4),        # configs[0]
    ("suzanne640", "suzanne.obj", 640, 360, 4),  # configs[1]
    ("teapot720", "teapot.obj", 1280, 720, 16),  # configs[2]
]


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    import torch
    rows = []
    for name, obj, W, H, spp in CONFIGS:
        tris, bmin, bmax = tm.load_scene(os.path.join(ROOT, "data", obj))
        cam = tm.Camera.for_scene(bmin, bmax, W, H)
        with tm.Scene(tris) as sc:
            out = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda:0")
            rec = {"config": name, "W": W, "H": H, "spp": spp}
            for kind in ("host", "device"):
                wall, rms, kms = [], [], []
                for i in range(calls + 3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    if kind == "host":
                        _, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_SAMPLE)
                    else:
                        _, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_SAMPLE, out=out.data_ptr())
                    t1 = time.perf_counter()
                    st = sc.stats()
                    if i >= 3:
                        wall.append((t1 - t0) * 1e3)
                        rms.append(st.render_ms)
                        kms.append(st.extend_ms)
                w, r, k = (float(np.median(x)) for x in (wall, rms, kms))
                rec[kind] = {"wall_ms": round(w, 4), "render_ms": round(r, 4), "k_path_ms": round(k, 4),
                             "other_device_ms": round(r - k, 4), "host_ms": round(w - r, 4),
                             "rays": int(rays), "mrays_wall": round(rays / w / 1e3, 1),
                             "mrays_k_path": round(rays / k / 1e3, 1)}
            print(json.dumps(rec), flush=True)
            rows.append(rec)
    print("\n| config | rays | wall ms (host img / device out) | k_path ms | other device ms | host ms "
          "| MRays/s wall (device out) | MRays/s k_path |")
    print("|---|---|---|---|---|---|---|---|")
    for r in rows:
        h, d = r["host"], r["device"]
        print(f"| {r['config']} {r['W']}x{r['H']}x{r['spp']} | {d['rays']} | {h['wall_ms']:.3f} / {d['wall_ms']:.3f} "
              f"| {d['k_path_ms']:.3f} | {d['other_device_ms']:.3f} | {d['host_ms']:.3f} | {d['mrays_wall']:.0f} "
              f"| {d['mrays_k_path']:.0f} |")


if __name__ == "__main__":
    main()
