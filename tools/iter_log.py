"""Per-iteration queue sizes of one wavefront frame (TMPT_ITER_LOG) and the
longest traversal (steps) of any single query (instrumented build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
os.environ["TMPT_ITER_LOG"] = "1"
import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
sc = tm.Scene(tris)
sc.trace_image(cam, 1920, 1080, spp, seed_mode=tm.SEED_PIXEL, count_visits=True)
st = sc.stats()
print("extend rays", st.extend_rays, "node visits/ray", st.node_visits / st.extend_rays,
      "tris/ray", st.tri_tests / st.extend_rays, file=sys.stderr)
