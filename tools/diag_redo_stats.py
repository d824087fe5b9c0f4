import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "data"))
import toymeshpathtracer_amd as tm, gen_standin_sponza, torch
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
    for i in range(2):
        img, rays = sc.trace_image(cam, 1920, 1080, 64, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        st = sc.stats(); print("host", i, rays, st.redo_samples, st.redo_late, st.tie_path, st.redo_launches, flush=True)
    t = torch.zeros((1080, 1920, 4), dtype=torch.uint8, device="cuda:0")
    for i in range(2):
        _, rays = sc.trace_image(cam, 1920, 1080, 64, seed_mode=tm.SEED_SAMPLE, band_rows=1, out=t.data_ptr())
        st = sc.stats(); print("dev", i, rays, st.redo_samples, st.redo_late, st.tie_path, st.redo_launches, flush=True)
