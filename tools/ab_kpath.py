"""Same-box A/B of k_path time: the package under test (default: this tree)
against another build of it (a directory holding toymeshpathtracer_amd/, e.g.
tools/_bin/base from an earlier commit), alternating, on the bench frame.

  python tools/ab_kpath.py <pkgdir_a>[:opts],<pkgdir_b>[:opts][,...] [frames] [loads]
  opts: scene build options with ';' between them, e.g. .:split=20;leaf_max=4
  loads: comma list of seed:shards, e.g. sample:1,sample:8,pixel:1
Prints per load the median k_path ms (tmpt_stats.extend_ms) of each build.
AB_RES=3840x2160 AB_SPP=256 select another frame of the stand-in sponza (configs[4]);
AB_TIME=render times the whole render (every kernel of the call) instead of k_path."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, os, json, statistics
pkg, _, opts = sys.argv[1].partition(":")  # <package dir>[:<scene options>]
sys.path.insert(0, pkg); sys.path.insert(0, os.path.join(sys.argv[2], "data"))
import toymeshpathtracer_amd as tm
import gen_standin_sponza
frames = int(sys.argv[3]); loads = sys.argv[4].split(",")
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
w, h = map(int, os.environ.get("AB_RES", "1920x1080").split("x")); spp = int(os.environ.get("AB_SPP", "64"))
cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
seeds = {"sample": tm.SEED_SAMPLE, "pixel": tm.SEED_PIXEL, "row": tm.SEED_ROW}
out = {}
with tm.Scene(tris, bounds=(bmin, bmax), options=opts.replace(";", ",") or None) as sc:
    for ld in loads:
        sd, n = ld.split(":"); n = int(n)
        ms = []
        for i in range(frames + 1):
            sc.trace_image(cam, w, h, spp, seed_mode=seeds[sd], band_rows=1, shard=n - 1, num_shards=n)
            # row seeding runs several kernels: the render's whole device time
            if i: ms.append(sc.stats().render_ms if sd == "row" or os.environ.get("AB_TIME") == "render"
                            else sc.stats().extend_ms)
        out[ld] = statistics.median(ms)
print(json.dumps(out))
'''


def run(pkg, frames, loads):
    r = subprocess.run([sys.executable, "-c", CHILD, pkg, ROOT, str(frames), loads], capture_output=True, text=True,
                       timeout=600)
    if r.returncode:
        raise SystemExit(r.stderr)
    return json.loads(r.stdout.strip().splitlines()[-1])


def main():
    pkgs = sys.argv[1].split(",")  # the first is the reference of the comparison
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    loads = sys.argv[3] if len(sys.argv) > 3 else "sample:1,sample:8,pixel:1,pixel:8"
    res = {p: [] for p in pkgs}
    for rep in range(2):  # A B C .. A B C ..
        for p in pkgs:
            res[p].append(run(p, frames, loads))
            print(p, {k: round(v, 3) for k, v in res[p][-1].items()}, flush=True)
    for ld in loads.split(","):
        base = min(r[ld] for r in res[pkgs[0]])
        line = [f"{ld}: {pkgs[0]} {base:.2f} ms"]
        for p in pkgs[1:]:
            m = min(r[ld] for r in res[p])
            line.append(f"{p} {m:.2f} ms ({100 * (m / base - 1):+.2f} %)")
        print(", ".join(line), flush=True)


if __name__ == "__main__":
    main()
