"""Diagnostic: shard ray sums vs the full frame, sample seeding, octree built."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..')); sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'data'))
import numpy as np
import toymeshpathtracer_amd as tm
import gen_standin_sponza
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
w, h, spp = [int(x) for x in sys.argv[1:4]]
cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
    for opts in ({"tie_defer": -1}, {"tie_defer": 0}, {"tie_defer": 1}):
        for k, v in opts.items():
            sc.set_option(k, v)
        full, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        st = sc.stats()
        line = [f"{opts} full rays {rays} redo {st.redo_samples} late {st.redo_late} launches {st.redo_launches} ties {st.tie_queries} crack {st.crack_queries}"]
        full2, rays2 = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        line.append(f"again {rays2} same_img {np.array_equal(full, full2)}")
        tot = 0
        for k in range(8):
            tile, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1, shard=k, num_shards=8)
            st = sc.stats()
            tot += r
            line.append(f"s{k} {r} eq {np.array_equal(tile, full[k::8])} redo {st.redo_samples} late {st.redo_late} ties {st.tie_queries} crack {st.crack_queries}")
        line.append(f"sum {tot} diff {tot - rays}")
        print("\n  ".join(line), flush=True)
