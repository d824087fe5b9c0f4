"""Wave-round efficiency of the persistent engine (instrumented render, TMPT_ROUND_LOG):
how many lanes step per node/leaf round, how many want shading per shading round.
  python tools/round_log.py [spp] [shards...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
shards = [int(x) for x in sys.argv[2:]] or [1, 8]
W, H = 1920, 1080
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=True)
sc = tm.Scene(tris)
os.environ["TMPT_ROUND_LOG"] = "1"
for n in shards:
    img, rays = sc.trace_image(cam, W, H, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_PERSISTENT,
                               band_rows=1, shard=0, num_shards=n, count_visits=True)
    st = sc.stats()
    print(f"shards {n}: rays {rays} nodes {st.node_visits + st.shadow_node_visits} "
          f"tris {st.tri_tests + st.shadow_tri_tests} render {st.render_ms:.1f} ms", flush=True)
    print(f"  closest-hit: {st.extend_rays} rays, {st.node_visits / st.extend_rays:.2f} nodes + "
          f"{st.tri_tests / st.extend_rays:.2f} tris per ray; shadow: {st.shadow_rays} rays, "
          f"{st.shadow_node_visits / max(st.shadow_rays, 1):.2f} nodes + "
          f"{st.shadow_tri_tests / max(st.shadow_rays, 1):.2f} tris per ray", flush=True)
