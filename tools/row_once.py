"""Three row-seeded bench frames (the reference octree built), for kernel traces of the row engine:
  rocprofv3 --kernel-trace --stats -d <dir> -- python3 tools/row_once.py"""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "data"))
import toymeshpathtracer_amd as tm, gen_standin_sponza
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
    for i in range(3):
        img, rays = sc.trace_image(cam, 1920, 1080, 64, seed_mode=tm.SEED_ROW)
        print(i, rays, sc.stats().render_ms, flush=True)
