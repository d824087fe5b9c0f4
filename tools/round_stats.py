"""Wave-round efficiency of k_path on the bench frame (instrumented build,
TMPT_ROUND_LOG): node / leaf rounds and the lanes stepping in them, shading
rounds, lanes shading vs traversing meanwhile.  usage: python tools/round_stats.py [spp] [shards]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 16
shards = int(sys.argv[2]) if len(sys.argv) > 2 else 1
os.environ["TMPT_ROUND_LOG"] = "1"
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
# optional third argument: render-option variants for sample seeding, "defer=0;defer=1"
variants = sys.argv[3].split(";") if len(sys.argv) > 3 else None
runs = [("pixel", tm.SEED_PIXEL, ""), ("sample", tm.SEED_SAMPLE, "")] if variants is None else \
    [("sample " + v, tm.SEED_SAMPLE, v) for v in variants]
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:  # the product configuration (reference octree)
    defaults = {}
    for name, seed, v in runs:
        for k, val in defaults.items():
            sc.set_option(k, val)
        for kv in filter(None, v.split("&")):
            k, _, val = kv.partition("=")
            defaults.setdefault(k, sc.get_option(k))
            sc.set_option(k, float(val))
        print(f"--- {name} seeding, {spp} spp, shard 0 of {shards}", file=sys.stderr, flush=True)
        _, rays = sc.trace_image(cam, 1920, 1080, spp, seed_mode=seed, band_rows=1, num_shards=shards,
                                 count_visits=True)
        st = sc.stats()
        q = st.extend_rays + st.shadow_rays
        print(f"{name}: rays {rays}, node visits/query {(st.node_visits + st.shadow_node_visits) / q:.2f}, "
              f"tri tests/query {(st.tri_tests + st.shadow_tri_tests) / q:.2f}, k_path {st.extend_ms:.1f} ms",
              file=sys.stderr, flush=True)
