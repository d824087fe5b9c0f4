import sys, os, time
pkg = sys.argv[1]
sys.path.insert(0, pkg); sys.path.insert(0, os.path.join(os.getcwd(), "data"))
import toymeshpathtracer_amd as tm, gen_standin_sponza
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
    for i in range(3):
        img, rays = sc.trace_image(cam, 1920, 1080, 64, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        st = sc.stats(); print(pkg, i, rays, "k_path", round(st.extend_ms, 2), "redo", st.redo_samples, "late", st.redo_late, "redo_launches", st.redo_launches, flush=True)
