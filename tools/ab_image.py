"""Same-box image check across builds: renders the bench frame (sample seeding)
with each package (a directory holding toymeshpathtracer_amd/, as
tools/ab_kpath.py takes them) at the given shard loads and prints the image's
sha256 and the ray count; every build must print the same lines.

  python tools/ab_image.py <pkgdir_a>,<pkgdir_b>[,...] [loads]   loads: seed:shards, e.g. sample:1,sample:2"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, os, hashlib
pkg = sys.argv[1]
sys.path.insert(0, pkg); sys.path.insert(0, os.path.join(sys.argv[2], "data"))
import toymeshpathtracer_amd as tm
import gen_standin_sponza
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, 1920, 1080, is_sponza=True)
seeds = {"sample": tm.SEED_SAMPLE, "pixel": tm.SEED_PIXEL, "row": tm.SEED_ROW}
with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
    for ld in sys.argv[3].split(","):
        sd, n = ld.split(":"); n = int(n)
        img, rays = sc.trace_image(cam, 1920, 1080, 64, seed_mode=seeds[sd], band_rows=1, shard=n - 1, num_shards=n)
        st = sc.stats()
        print(ld, hashlib.sha256(img.tobytes()).hexdigest()[:16], int(rays), "redo", st.redo_samples, "late",
              st.redo_late, "tie_path", st.tie_path, "ties", st.tie_queries, "cracks", st.crack_queries, flush=True)
'''


def main():
    pkgs = sys.argv[1].split(",")
    loads = sys.argv[2] if len(sys.argv) > 2 else "sample:1,sample:2"
    outs = []
    for p in pkgs:
        r = subprocess.run([sys.executable, "-c", CHILD, p, ROOT, loads], capture_output=True, text=True, timeout=600)
        if r.returncode:
            raise SystemExit(r.stderr[-3000:])
        lines = [ln for ln in r.stdout.splitlines() if ":" in ln]
        print(p, *lines, sep="\n  ", flush=True)
        outs.append([" ".join(ln.split()[:3]) for ln in lines])
    same = all(o == outs[0] for o in outs)
    print("IMAGES AND RAYS IDENTICAL" if same else "DIFFERENT", flush=True)
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
