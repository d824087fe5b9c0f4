"""CPU oracle for the hot path -- TEST INFRASTRUCTURE ONLY.

ctypes face of ``oracle/build/liboracle.so`` (the C restatement in
``oracle/tmpt_oracle.c``, which cites the reference file:line of every
function).  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module; the product never does.

Pinning: the octree restatement reproduces, bit for bit, the raw-RGBA SHA-256
prefixes and ray counts of the reference binary recorded in SURVEY.md §8c
(tests/test_oracle.py), and the reference's committed result{1..4}*.png to
the statistical level those macOS renders allow.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: another build of it (tools/san_check.sh: the sanitizer build, build_san/)
LIB = os.environ.get("ORACLE_LIB") or os.path.join(HERE, "build", "liboracle.so")

ACCEL_OCTREE, ACCEL_BVH, ACCEL_LINEAR = 0, 1, 2
TIE_VISIT, TIE_INDEX = 0, 1
SEED_ROW, SEED_PIXEL, SEED_SAMPLE = 0, 1, 2
SAMPLE_STRIDE = 65536  # xorshift steps between the starts of a pixel's samples (sample seeding)


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


if not os.path.exists(LIB):
    build()
_lib = ctypes.CDLL(LIB)
_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)


class _Camera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("lower_left", ctypes.c_float * 3),
                ("horizontal", ctypes.c_float * 3), ("vertical", ctypes.c_float * 3),
                ("u", ctypes.c_float * 3), ("v", ctypes.c_float * 3), ("w", ctypes.c_float * 3),
                ("lens_radius", ctypes.c_float)]


def _sig(name, res, args):
    f = getattr(_lib, name)
    f.restype, f.argtypes = res, args
    return f


_xorshift = _sig("orc_xorshift32", ctypes.c_uint32, [_u32p])
_xorshift_jump = _sig("orc_xorshift32_jump", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint64])
_sample_seed = _sig("orc_sample_seed", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32])
_rand01 = _sig("orc_random_float01", ctypes.c_float, [_u32p])
_disk = _sig("orc_random_in_unit_disk", None, [_u32p, _f32p])
_unitv = _sig("orc_random_unit_vector", None, [_u32p, _f32p])
_pixel_seed = _sig("orc_pixel_seed", ctypes.c_uint32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32])
_cam_init = _sig("orc_camera_init", None, [ctypes.POINTER(_Camera), _f32p, _f32p, _f32p, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_float])
_cam_scene = _sig("orc_camera_for_scene", None, [ctypes.POINTER(_Camera), _f32p, _f32p, ctypes.c_int32,
                                                 ctypes.c_int32, ctypes.c_int32])
_get_ray = _sig("orc_camera_get_ray", None, [ctypes.POINTER(_Camera), ctypes.c_float, ctypes.c_float,
                                             _u32p, _f32p, _f32p])
_load = _sig("orc_load_scene", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_f32p), _i32p, _f32p, _f32p])
_free = _sig("orc_free", None, [ctypes.c_void_p])
_create = _sig("orc_scene_create", ctypes.c_void_p, [_f32p, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_int32, _f32p, _f32p])
_destroy = _sig("orc_scene_destroy", None, [ctypes.c_void_p])
_hit_batch = _sig("orc_hit_batch", None, [ctypes.c_void_p, _f32p, ctypes.c_int64, ctypes.c_float,
                                          ctypes.c_float, _f32p, _i32p, ctypes.c_int32])
_stats = _sig("orc_scene_stats", None, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)])
_oct_digest = _sig("orc_octree_digest", ctypes.c_uint64, [ctypes.c_void_p])
_oct_nodes = _sig("orc_octree_nodes", ctypes.c_int64, [ctypes.c_void_p, _f32p, _i32p, ctypes.c_int64])
_oct_leaf = _sig("orc_octree_leaf", ctypes.c_int32, [ctypes.c_void_p, ctypes.c_int64, _i32p, ctypes.c_int32])
_ray_box = _sig("orc_ray_box_batch", None, [_f32p, ctypes.c_int64, _f32p, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_void_p])
_render = _sig("orc_render", ctypes.c_uint64, [ctypes.c_void_p, ctypes.POINTER(_Camera), ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_void_p])
_render_ex = _sig("orc_render_ex", ctypes.c_uint64, [ctypes.c_void_p, ctypes.POINTER(_Camera), ctypes.c_int32,
                                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                     ctypes.c_void_p])
_trace = _sig("orc_trace", None, [ctypes.c_void_p, _f32p, _f32p, _u32p, _f32p,
                                  ctypes.POINTER(ctypes.c_uint64)])
_sincos = _sig("orc_unit_angle_sincos", None, [ctypes.c_uint32, _f32p, _f32p])
_sincos_range = _sig("orc_unit_sincos_range", None, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p])


def _fp(a):
    return a.ctypes.data_as(_f32p)


def xorshift_seq(seed: int, n: int) -> np.ndarray:
    s = ctypes.c_uint32(seed)
    return np.array([_xorshift(ctypes.byref(s)) for _ in range(n)], np.uint32)


def xorshift_jump(seed: int, n: int) -> int:
    """State after n xorshift steps from `seed` (GF(2) matrix power, maths.cpp:5-13)."""
    return int(_xorshift_jump(seed, n))


def sample_seed(seed: int, smp: int) -> int:
    """Start state of sample `smp` in sample seeding: xorshift_jump(seed, smp * 2^16)."""
    return int(_sample_seed(seed, smp))


def float01_seq(seed: int, n: int) -> np.ndarray:
    s = ctypes.c_uint32(seed)
    return np.array([_rand01(ctypes.byref(s)) for _ in range(n)], np.float32)


def disk_seq(seed: int, n: int):
    s = ctypes.c_uint32(seed)
    out = np.zeros((n, 3), np.float32)
    for i in range(n):
        _disk(ctypes.byref(s), _fp(out[i]))
    return out, s.value


def unit_vector_seq(seed: int, n: int):
    s = ctypes.c_uint32(seed)
    out = np.zeros((n, 3), np.float32)
    for i in range(n):
        _unitv(ctypes.byref(s), _fp(out[i]))
    return out, s.value


def pixel_seed(x: int, y: int, w: int) -> int:
    return int(_pixel_seed(x, y, w))


def unit_angle_sincos(key24: int):
    c, s = ctypes.c_float(), ctypes.c_float()
    _sincos(key24, ctypes.byref(c), ctypes.byref(s))
    return c.value, s.value


def unit_sincos_range(key0: int, n: int) -> np.ndarray:
    """(cos a, sin a) of the host libm for keys [key0, key0 + n), n x 2 float32."""
    out = np.empty((n, 2), dtype=np.float32)
    _sincos_range(key0, n, out.ctypes.data)
    return out


def _cam_arr(c: _Camera) -> np.ndarray:
    return np.array(list(c.origin) + list(c.lower_left) + list(c.horizontal) + list(c.vertical)
                    + list(c.u) + list(c.v) + list(c.w) + [c.lens_radius], np.float32)


def camera(look_from, look_at, vup, vfov, aspect, aperture, focus) -> np.ndarray:
    c = _Camera()
    a = [np.asarray(x, np.float32) for x in (look_from, look_at, vup)]
    _cam_init(ctypes.byref(c), _fp(a[0]), _fp(a[1]), _fp(a[2]), vfov, aspect, aperture, focus)
    return _cam_arr(c)


def camera_for_scene(bmin, bmax, w, h, is_sponza=False) -> np.ndarray:
    c = _Camera()
    lo, hi = np.asarray(bmin, np.float32), np.asarray(bmax, np.float32)
    _cam_scene(ctypes.byref(c), _fp(lo), _fp(hi), w, h, int(is_sponza))
    return _cam_arr(c)


def _cam_from_arr(a) -> _Camera:
    a = np.asarray(a, np.float32)
    c = _Camera()
    for i, name in enumerate(("origin", "lower_left", "horizontal", "vertical", "u", "v", "w")):
        getattr(c, name)[:] = [float(x) for x in a[3 * i:3 * i + 3]]
    c.lens_radius = float(a[21])
    return c


def get_ray(cam_arr, s: float, t: float, seed: int):
    c = _cam_from_arr(cam_arr)
    st = ctypes.c_uint32(seed)
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    _get_ray(ctypes.byref(c), s, t, ctypes.byref(st), _fp(o), _fp(d))
    return o, d, st.value


def load_scene(path: str):
    p = _f32p()
    n = ctypes.c_int32()
    bmin = np.zeros(3, np.float32)
    bmax = np.zeros(3, np.float32)
    if _load(path.encode(), ctypes.byref(p), ctypes.byref(n), _fp(bmin), _fp(bmax)):
        raise IOError(path)
    try:
        tris = np.ctypeslib.as_array(p, shape=(n.value * 9,)).copy().reshape(n.value, 3, 3)
    finally:
        _free(p)
    return tris, bmin, bmax


def ray_box(rays, box, t_min, t_max) -> np.ndarray:
    """RayHitAabb (maths.h:116-134) of each ray {o, d} against box {min, max},
    over 1/d as HitScene forms it (scene.cpp:92-93): bool per ray."""
    rays = np.ascontiguousarray(np.asarray(rays, np.float32).reshape(-1, 6))
    b = np.ascontiguousarray(np.asarray(box, np.float32).reshape(6))
    out = np.zeros(rays.shape[0], np.uint8)
    _ray_box(_fp(rays), rays.shape[0], _fp(b), t_min, t_max, out.ctypes.data)
    return out.astype(bool)


class Scene:
    """Oracle scene: accel = ACCEL_OCTREE (the reference's, scene.cpp:75-83, 99-160),
    ACCEL_BVH (exact linear-scan semantics, own BVH) or ACCEL_LINEAR."""

    def __init__(self, tris, accel=ACCEL_OCTREE, tie=TIE_VISIT, bmin=None, bmax=None):
        t = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
        self.n = t.shape[0]
        if bmin is None:  # main.cpp:296-297,312 octree bounds from the OBJ bounds
            v = t.reshape(-1, 3)
            bmin = v.min(0) if len(v) else np.zeros(3, np.float32)
            bmax = v.max(0) if len(v) else np.zeros(3, np.float32)
        bmin = np.asarray(bmin, np.float32)
        bmax = np.asarray(bmax, np.float32)
        extra = (bmax - bmin) * np.float32(0.7)
        omin = (bmin - extra).astype(np.float32)
        omax = (bmax + extra).astype(np.float32)
        self._h = _create(_fp(t), self.n, accel, tie, _fp(omin), _fp(omax))

    def __del__(self):
        if getattr(self, "_h", None):
            _destroy(self._h)
            self._h = None

    def hit_batch(self, rays, t_min, t_max, threads=8):
        rays = np.ascontiguousarray(np.asarray(rays, np.float32).reshape(-1, 6))
        n = rays.shape[0]
        hits = np.zeros((n, 7), np.float32)
        ids = np.full(n, -1, np.int32)
        _hit_batch(self._h, _fp(rays), n, t_min, t_max, _fp(hits), ids.ctypes.data_as(_i32p), threads)
        return ids, hits

    def stats(self):
        a = (ctypes.c_int64 * 4)()
        _stats(self._h, a)
        return list(a)

    def octree_digest(self) -> int:
        """FNV-1a of the octree's preorder walk (0 for other accelerators' scenes
        it is the empty hash)."""
        return int(_oct_digest(self._h))

    def octree_nodes(self):
        """(boxes n x 6 {min, max}, info n x 3 {first child or -1, leaf
        triangle count, depth}) of the octree in storage order."""
        n = int(_oct_nodes(self._h, None, None, 0))
        boxes = np.zeros((n, 6), np.float32)
        info = np.zeros((n, 3), np.int32)
        if n:
            _oct_nodes(self._h, _fp(boxes), info.ctypes.data_as(_i32p), n)
        return boxes, info

    def octree_leaf(self, node: int) -> np.ndarray:
        """Triangle ids of leaf `node`, in the reference's order."""
        n = int(_oct_leaf(self._h, node, None, 0))
        ids = np.zeros(n, np.int32)
        if n:
            _oct_leaf(self._h, node, ids.ctypes.data_as(_i32p), n)
        return ids

    def render(self, cam_arr, w, h, spp, seed_mode=SEED_ROW, y0=0, y1=None, row_step=1,
               threads=None, rgba=None, x0=0, x_step=1):
        """Rows y0, y0+row_step, ... < y1 into a full-frame rgba (H, W, 4), row 0 = bottom;
        of each row the pixels x0, x0+x_step, ... (pixel / sample seeding; row
        seeding always renders whole rows).  threads: default every CPU this
        process may run on."""
        if rgba is None:
            rgba = np.zeros((h, w, 4), np.uint8)
        threads = threads or len(os.sched_getaffinity(0)) or 1
        rays = _render_ex(self._h, ctypes.byref(_cam_from_arr(cam_arr)), w, h, spp, seed_mode, y0,
                          h if y1 is None else y1, row_step, x0, x_step, threads,
                          rgba.ctypes.data_as(ctypes.c_void_p))
        return rgba, int(rays)

    def trace(self, orig, direction, seed):
        st = ctypes.c_uint32(seed)
        col = np.zeros(3, np.float32)
        rays = ctypes.c_uint64(0)
        o = np.asarray(orig, np.float32)
        d = np.asarray(direction, np.float32)
        _trace(self._h, _fp(o), _fp(d), ctypes.byref(st), _fp(col), ctypes.byref(rays))
        return col, st.value, rays.value
