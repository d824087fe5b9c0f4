"""Diagnostic: repeated deferred-tie renders, ray counts and redo stats."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..')); sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'data'))
import numpy as np
import toymeshpathtracer_amd as tm
import gen_standin_sponza
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
w, h, spp, reps = [int(x) for x in sys.argv[1:5]]
cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
for inline in (1, 0):
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        sc.set_option("redo_inline", inline)
        ref = None
        for i in range(reps):
            img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
            st = sc.stats()
            same = ref is None or np.array_equal(img, ref[0])
            if ref is None:
                ref = (img, rays)
            print(f"inline {inline} rep {i} rays {rays} d {rays - ref[1]} same {same} redo {st.redo_samples} late {st.redo_late} "
                  f"launches {st.redo_launches} redo_rays {st.redo_rays} kpath {st.extend_ms:.1f} redo_ms {st.redo_ms:.2f}", flush=True)
