"""Pixel-seeding tail: the instrumented build's wave-time split and cycles per
round kind (TMPT_PROF=3) at a few shard counts of the bench frame, with the
frame's k_path time, to price a lone lane's traversal step against its
shading round.  usage: TMPT_LIB_PATH=toymeshpathtracer_amd/_lib_diag/libtmpt.so
python tools/tail_prof.py [shards,...] [prof]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
shards = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "128,8,1").split(",")]
os.environ.setdefault("TMPT_PROF", sys.argv[2] if len(sys.argv) > 2 else "3")
import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
    for n in shards:
        for rep in range(2):
            print(f"--- pixel seeding, 64 spp, shard 0 of {n}, run {rep}", file=sys.stderr, flush=True)
            _, rays = sc.trace_image(cam, 1920, 1080, 64, seed_mode=tm.SEED_PIXEL, band_rows=1, num_shards=n)
            st = sc.stats()
            print(f"rays {rays}, k_path {st.extend_ms:.2f} ms, launches {st.extend_launches}", file=sys.stderr,
                  flush=True)
