#!/usr/bin/env python3
"""Regenerates tests/golden/golden.json from the CPU oracle (oracle/).

The oracle itself is pinned to the reference binary (SURVEY.md §8c hashes,
tests/test_oracle.py) and to the reference's committed result*.png; this file
freezes its outputs (RNG / sampling / camera known answers, image hashes and
ray counts in both seed modes) so later changes to either side are caught.
Values are stored as IEEE-754 bit patterns (hex) where bit-exactness matters.

Usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))

import numpy as np  # noqa: E402

import gen_standin_sponza  # noqa: E402
import oracle  # noqa: E402

SEEDS = [1, 9781 * 5 + 1, 0x12345678, 0xDEADBEEF]
SCENES = ["triangle", "cube", "suzanne", "teapot"]


def bits(a):
    return [f"{x:08x}" for x in np.asarray(a, np.float32).ravel().view(np.uint32)]


def png_sha(img):
    return hashlib.sha256(np.ascontiguousarray(img[::-1]).tobytes()).hexdigest()


def main():
    g = {"kat": {}, "camera": {}, "images": {}}
    for s in SEEDS:
        g["kat"][str(s)] = {
            "xorshift": [int(x) for x in oracle.xorshift_seq(s, 32)],
            "float01": bits(oracle.float01_seq(s, 32)),
            "disk": bits(oracle.disk_seq(s, 16)[0]),
            "unit_vector": bits(oracle.unit_vector_seq(s, 16)[0]),
        }
    g["pixel_seed"] = {f"{x},{y},{w}": oracle.pixel_seed(x, y, w)
                       for (x, y, w) in [(0, 0, 640), (639, 359, 640), (1919, 1079, 1920),
                                         (3839, 2159, 3840), (5, 7, 13)]}
    sponza = gen_standin_sponza.ensure()
    g["sponza_standin_sha256"] = hashlib.sha256(open(sponza, "rb").read()).hexdigest()
    cases = [(n, os.path.join(ROOT, "data", n + ".obj"), 640, 360, 4, False) for n in SCENES]
    cases.append(("sponza_standin", sponza, 320, 180, 2, True))
    for name, path, w, h, spp, is_sponza in cases:
        tris, bmin, bmax = oracle.load_scene(path)
        cam = oracle.camera_for_scene(bmin, bmax, w, h, is_sponza)
        g["camera"][f"{name}_{w}x{h}"] = bits(cam)
        g["images"][name] = {"w": w, "h": h, "spp": spp, "tris": int(tris.shape[0])}
        if not is_sponza:  # row mode: the unmodified reference algorithm (octree, visit order)
            osc = oracle.Scene(tris, accel=oracle.ACCEL_OCTREE, tie=oracle.TIE_VISIT, bmin=bmin, bmax=bmax)
            img, rays = osc.render(cam, w, h, spp, seed_mode=oracle.SEED_ROW)
            g["images"][name]["row"] = {"sha256": png_sha(img), "rays": rays}
        bsc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
        img, rays = bsc.render(cam, w, h, spp, seed_mode=oracle.SEED_PIXEL)
        g["images"][name]["pixel"] = {"sha256": png_sha(img), "rays": rays}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
