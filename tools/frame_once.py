"""One bench frame (stand-in sponza 1920x1080x64, the reference octree built)
per seeding mode given, for experiment builds that print their own
statistics (TMPT_LIB_PATH=<variant>/libtmpt.so).
  python tools/frame_once.py [sample,pixel,row] [shards] [options, e.g. "sample_tail=8,redo_lanes=16"]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

modes = (sys.argv[1] if len(sys.argv) > 1 else "sample").split(",")
shards = int(sys.argv[2]) if len(sys.argv) > 2 else 1
seeds = {"sample": tm.SEED_SAMPLE, "pixel": tm.SEED_PIXEL, "row": tm.SEED_ROW}
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
opts = sys.argv[3] if len(sys.argv) > 3 else None
with tm.Scene(tris, bounds=(bmin, bmax), options=opts) as sc:
    for m in modes:
        _, rays = sc.trace_image(cam, 1920, 1080, 64, seed_mode=seeds[m], band_rows=1, num_shards=shards)
        st = sc.stats()
        print(f"{m}: rays {rays}, k_path {st.extend_ms:.2f} ms, ties {st.tie_queries}, cracks {st.crack_queries}",
              file=sys.stderr, flush=True)
