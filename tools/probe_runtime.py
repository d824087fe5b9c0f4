"""Which HIP runtime does libtmpt bind to when torch is (or is not) imported first?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1]
if order == "torch_first":
    import torch
    print("torch cuda available:", torch.cuda.is_available(), flush=True)
import toymeshpathtracer_amd as tm
import numpy as np
maps = open("/proc/self/maps").read()
print("hip libs:", sorted({l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l or "libhsa-runtime" in l}))
tris, bmin, bmax = tm.load_scene("data/cube.obj")
cam = tm.Camera.for_scene(bmin, bmax, 64, 32)
with tm.Scene(tris) as sc:
    img, rays = sc.trace_image(cam, 64, 32, 2, seed_mode=tm.SEED_PIXEL)
    print("render ok", rays)
    if order == "torch_first":
        dev = torch.zeros((32, 64, 4), dtype=torch.uint8, device="cuda:0")
        _, r2 = sc.trace_image(cam, 64, 32, 2, seed_mode=tm.SEED_PIXEL, out=dev.data_ptr())
        torch.cuda.synchronize()
        print("device-out equal:", np.array_equal(dev.cpu().numpy(), img), r2 == rays)
if order == "lib_first":
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29511", RANK="0", WORLD_SIZE="1")
    dist.init_process_group("gloo")
    t = torch.ones(4)
    dist.all_reduce(t)
    print("gloo ok", t.tolist())
    dist.destroy_process_group()
