"""The checked build (make CHECK=1 -> toymeshpathtracer_amd/_lib_check): device
index tests in the BVH traversal, both octree walks and the hit-record loads
(tmpt_internal.h kChk*; VERDICT r04 "no device bounds-checked debug build").

Each case runs in a child process that loads the checked library through
TMPT_LIB_PATH (the package loads one library per process):
* on real scenes it answers and renders exactly as the product library does,
  with no check failing -- the checks cost nothing but time;
* with TMPT_CHECK_SELFTEST=1 its scene view claims a single BVH node, so every
  query that descends past the root fails the node test, and the call must
  fail with the report (codes, count, last value), not return answers.
The whole GPU suite against the checked library: tools/check_build.sh."""
import json
import os
import subprocess
import sys

import pytest

import toymeshpathtracer_amd as tm
from conftest import data

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK_LIB = os.path.join(ROOT, "toymeshpathtracer_amd", "_lib_check", "libtmpt.so")

CHILD = r'''
import hashlib, json, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import toymeshpathtracer_amd as tm
name, mode = sys.argv[2], sys.argv[3]
tris, bmin, bmax = tm.load_scene(name)
rng = np.random.default_rng(5)
v = tris.reshape(-1, 3)
lo, hi = v.min(0), v.max(0)
o = lo + rng.random((20000, 3)) * (hi - lo)
d = rng.normal(size=(20000, 3)).astype(np.float32)
d /= np.sqrt((d ** 2).sum(1, keepdims=True))
rays = np.concatenate([o, d], 1).astype(np.float32)
out = {}
try:
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        ids, hits = sc.hit_scene_batch(rays, 0.001, 1.0e7)
        out["ids"] = hashlib.sha256(ids.tobytes()).hexdigest()
        out["hits"] = hashlib.sha256(hits.tobytes()).hexdigest()
        if mode == "render":
            cam = tm.Camera.for_scene(bmin, bmax, 160, 90)
            for sm in (tm.SEED_SAMPLE, tm.SEED_PIXEL, tm.SEED_ROW):
                img, rays_n = sc.trace_image(cam, 160, 90, 8, seed_mode=sm)
                out[f"img{sm}"] = hashlib.sha256(img.tobytes()).hexdigest()
                out[f"rays{sm}"] = int(rays_n)
except tm.TmptError as e:
    out["error"] = str(e)
print(json.dumps(out))
'''

# configs[4] (4K x 256, sample seeding, octree answers deferred): the frame three
# times, then its 8 one-row-band shards; rays per frame and per shard
CHILD_4K = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "data"))
import toymeshpathtracer_amd as tm
import gen_standin_sponza
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
w, h, spp = 3840, 2160, 256
cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
out = {"frames": [], "late": [], "redo": [], "shards": []}
try:
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        for _ in range(3):
            _, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
            st = sc.stats()
            out["frames"].append(int(r)); out["late"].append(int(st.redo_late)); out["redo"].append(int(st.redo_samples))
        for k in range(8):
            _, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1, shard=k, num_shards=8)
            out["shards"].append(int(r))
except tm.TmptError as e:
    out["error"] = str(e)
print(json.dumps(out))
'''


def _child(name, mode, lib=None, selftest=False):
    env = dict(os.environ, TMPT_NO_TORCH="1")
    env.pop("TMPT_CHECK_SELFTEST", None)
    if lib:
        env["TMPT_LIB_PATH"] = lib
    else:
        env.pop("TMPT_LIB_PATH", None)
    if selftest:
        env["TMPT_CHECK_SELFTEST"] = "1"
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, name, mode], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


needs_check_lib = pytest.mark.skipif(not os.path.exists(CHECK_LIB),
                                     reason="checked build not built (make -C toymeshpathtracer_amd/csrc CHECK=1)")


@pytest.mark.gpu
@needs_check_lib
@pytest.mark.parametrize("name", ["suzanne.obj", "teapot.obj"])
def test_checked_build_answers_as_product(gpu, name):
    """HitScene answers and the three seedings' images and ray counts of the
    checked library equal the product library's; no check fails."""
    path = data(name)
    got, err = _child(path, "render", lib=CHECK_LIB)
    assert "error" not in got, got["error"]
    assert "device index check failed" not in err
    want, _ = _child(path, "render")
    assert got == want


@pytest.mark.gpu
@needs_check_lib
def test_checked_build_reports_a_bad_index(gpu):
    """The report path end to end: a view that claims one BVH node makes the
    node test fail on the device; the call fails with the codes, not answers."""
    got, err = _child(data("teapot.obj"), "hit", lib=CHECK_LIB, selftest=True)
    assert "error" in got, got
    assert "device index check failed: codes 0x1 " in got["error"], got["error"]
    assert "device index check failed" in err
    # the product library ignores the self-test variable (no checks compiled in)
    got, _ = _child(data("teapot.obj"), "hit", selftest=True)
    assert "error" not in got


@needs_check_lib
def test_check_lib_loads_with_the_same_abi():
    """CPU: the checked library is its own file, loads without a GPU and has
    the product library's ABI version."""
    import ctypes
    assert os.path.abspath(tm.lib_path) != os.path.abspath(CHECK_LIB)
    assert ctypes.CDLL(CHECK_LIB).tmpt_abi_version() == tm.abi_version()


@pytest.mark.gpu
@needs_check_lib
def test_checked_build_4k_ray_sums(gpu):
    """the in-launch handoffs (DESIGN.md section 4
    inventory) under the checked build on configs[4]: three renders of the 4K x
    256 frame count the same rays, with every deferred sample traced in the
    launch (redo_late 0), the 8 shards' rays add up to the frame's (the check
    that caught round 5's write-back bug), and the product library counts the
    same -- no device index check fails."""
    def run(lib):
        env = dict(os.environ, TMPT_NO_TORCH="1")
        env.pop("TMPT_CHECK_SELFTEST", None)
        if lib:
            env["TMPT_LIB_PATH"] = lib
        else:
            env.pop("TMPT_LIB_PATH", None)
        r = subprocess.run([sys.executable, "-c", CHILD_4K, ROOT], capture_output=True, text=True, timeout=280,
                           env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "device index check failed" not in r.stderr
        return json.loads(r.stdout.strip().splitlines()[-1])
    got = run(CHECK_LIB)
    assert "error" not in got, got["error"]
    assert len(set(got["frames"])) == 1 and got["late"] == [0, 0, 0] and min(got["redo"]) > 0, got
    assert sum(got["shards"]) == got["frames"][0], got
    want = run(None)
    assert want["frames"][0] == got["frames"][0] and want["shards"] == got["shards"]
