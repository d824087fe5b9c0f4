"""toymeshpathtracer_amd -- MI355X-native (gfx950) hot path of pr0g/ToyMeshPathTracer.

Python face of ``libtmpt.so`` (C ABI: ``include/tmpt.h``), mirroring the
reference's host interface for the path (``/root/reference/source``):

==========================  ==============================================
reference                   here
==========================  ==============================================
``LoadScene`` main.cpp:122  :func:`load_scene`
``Camera`` maths.cpp:40     :class:`Camera` (+ :meth:`Camera.for_scene`, main.cpp:295-307)
``Scene`` scene.h:17        :class:`Scene` (LBVH on the GPU)
``BuildOctree`` scene.h:26  :meth:`Scene.build_octree` (+ :func:`octree_bounds`, main.cpp:312)
``Scene::HitScene`` :36     :meth:`Scene.hit_scene` / :meth:`Scene.hit_scene_batch`
``TraceImageBody`` :180     :meth:`Scene.trace_image` (parallel_for, main.cpp:329)
``stbi_write_png`` :342     :func:`write_png`
==========================  ==============================================

The compute path is the HIP library only: if ``libtmpt.so`` is missing this
module raises on import -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

__all__ = [
    "Camera", "Scene", "Hit", "RenderStats", "load_scene", "write_png", "device_count",
    "SEED_ROW", "SEED_PIXEL", "SEED_SAMPLE", "ENGINE_WAVEFRONT", "ENGINE_MEGAKERNEL", "ENGINE_PERSISTENT", "lib_path", "TmptError",
    "tile_rows", "tile_row_to_y", "render_multi", "octree_bounds", "octree_digest", "octree_flags",
]

SEED_ROW, SEED_PIXEL, SEED_SAMPLE = 0, 1, 2
ENGINE_WAVEFRONT, ENGINE_MEGAKERNEL, ENGINE_PERSISTENT = 0, 1, 2
FLAG_OUT_DEVICE, FLAG_COUNT_VISITS, FLAG_WAIT_STREAM, FLAG_REQUIRE_RCCL = 1, 2, 4, 8

_HERE = os.path.dirname(os.path.abspath(__file__))
# TMPT_LIB_PATH: another in-tree build of the library (compiler-flag A/B in tools/)
lib_path = os.environ.get("TMPT_LIB_PATH") or os.path.join(_HERE, "_lib", "libtmpt.so")


class TmptError(RuntimeError):
    pass


if not os.path.exists(lib_path):
    raise ImportError(
        f"libtmpt.so not built ({lib_path}); run `python -c 'import __graft_entry__ as g; g.build()'` "
        "or `make -C toymeshpathtracer_amd/csrc`. There is no CPU fallback.")

# One HIP runtime per process: torch wheels bundle their own libamdhip64 /
# libhsa-runtime64 (same sonames as /opt/rocm's).  Importing torch first makes
# libtmpt bind to the runtime torch already loaded, so torch CUDA tensors,
# torch.distributed (RCCL) and our kernels share one device context.  Without
# torch, the system ROCm runtime is used.
# (TMPT_NO_TORCH=1: not even that -- the host sanitizer runs, tools/san_check.sh)
try:  # pragma: no cover - depends on the environment
    if os.environ.get("TMPT_NO_TORCH") == "1":
        raise ImportError("TMPT_NO_TORCH")
    import torch  # noqa: F401
except Exception:  # torch is optional for the C ABI itself
    torch = None

_lib = ctypes.CDLL(lib_path)

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)


class _Camera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("lower_left", ctypes.c_float * 3),
                ("horizontal", ctypes.c_float * 3), ("vertical", ctypes.c_float * 3),
                ("u", ctypes.c_float * 3), ("v", ctypes.c_float * 3), ("w", ctypes.c_float * 3),
                ("lens_radius", ctypes.c_float)]


class _Desc(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("seed_mode", ctypes.c_int32), ("band_rows", ctypes.c_int32),
                ("shard", ctypes.c_int32), ("num_shards", ctypes.c_int32),
                ("engine", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("spp_begin", ctypes.c_int32), ("spp_count", ctypes.c_int32),
                ("reserved0", ctypes.c_int32), ("wait_stream", ctypes.c_uint64),
                ("reserved", ctypes.c_int32 * 2)]


class _Stats(ctypes.Structure):
    _fields_ = [("render_ms", ctypes.c_double), ("extend_ms", ctypes.c_double),
                ("shadow_ms", ctypes.c_double), ("extend_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("extend_launches", ctypes.c_int64),
                ("shadow_launches", ctypes.c_int64), ("iterations", ctypes.c_int64),
                ("node_visits", ctypes.c_uint64), ("tri_tests", ctypes.c_uint64),
                ("shadow_node_visits", ctypes.c_uint64), ("shadow_tri_tests", ctypes.c_uint64),
                ("build_ms", ctypes.c_double), ("bvh_nodes", ctypes.c_int32),
                ("bvh_depth", ctypes.c_int32), ("n_tris", ctypes.c_int32),
                ("device", ctypes.c_int32), ("bvh4_nodes", ctypes.c_int32),
                ("bvh4_depth", ctypes.c_int32), ("leaf_max", ctypes.c_int32),
                ("builder_iters", ctypes.c_int32), ("octree_nodes", ctypes.c_int32),
                ("octree_leaves", ctypes.c_int32), ("octree_refs", ctypes.c_int64),
                ("octree_build_ms", ctypes.c_double), ("tie_queries", ctypes.c_uint64),
                ("root_misses", ctypes.c_uint64), ("row_engine", ctypes.c_int32),
                ("stream_fallbacks", ctypes.c_int32), ("octree_depth", ctypes.c_int32),
                ("tie_rule", ctypes.c_int32), ("chain_pixels", ctypes.c_int64),
                ("redo_samples", ctypes.c_int64), ("redo_late", ctypes.c_int64),
                ("crack_queries", ctypes.c_uint64), ("octree_flat", ctypes.c_int32),
                ("redo_launches", ctypes.c_int32), ("redo_ms", ctypes.c_double),
                ("redo_rays", ctypes.c_uint64), ("tie_path", ctypes.c_int32), ("reserved_stats", ctypes.c_int32)]


def _sig(name, res, args):
    fn = getattr(_lib, name)
    fn.restype = res
    fn.argtypes = args
    return fn


_load_obj = _sig("tmpt_load_obj", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(_f32p), _i32p, _f32p, _f32p])
_free = _sig("tmpt_free", None, [ctypes.c_void_p])
_cam_init = _sig("tmpt_camera_init", ctypes.c_int, [ctypes.POINTER(_Camera), _f32p, _f32p, _f32p,
                                                     ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                     ctypes.c_float])
_cam_scene = _sig("tmpt_camera_for_scene", ctypes.c_int, [ctypes.POINTER(_Camera), _f32p, _f32p,
                                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32])
_dev_count = _sig("tmpt_device_count", ctypes.c_int, [])
_scene_create = _sig("tmpt_scene_create", ctypes.c_int, [_f32p, ctypes.c_int32, ctypes.c_int32,
                                                         ctypes.POINTER(ctypes.c_void_p)])
_scene_create_ex = _sig("tmpt_scene_create_ex", ctypes.c_int, [_f32p, ctypes.c_int32, ctypes.c_int32,
                                                               ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)])
_set_option = _sig("tmpt_scene_set_option", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double])
_get_option = _sig("tmpt_scene_get_option", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p,
                                                           ctypes.POINTER(ctypes.c_double)])
_scene_destroy = _sig("tmpt_scene_destroy", ctypes.c_int, [ctypes.c_void_p])
_scene_hit = _sig("tmpt_scene_hit", ctypes.c_int, [ctypes.c_void_p, _f32p, ctypes.c_int64,
                                                   ctypes.c_float, ctypes.c_float, ctypes.c_int32,
                                                   _f32p, _i32p])
_scene_hit_ranged = _sig("tmpt_scene_hit_ranged", ctypes.c_int, [ctypes.c_void_p, _f32p, ctypes.c_int64,
                                                                 ctypes.c_int32, _f32p, _i32p])
_render = _sig("tmpt_render", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(_Camera),
                                             ctypes.POINTER(_Desc), ctypes.c_void_p, _u64p])
_build_octree = _sig("tmpt_scene_build_octree", ctypes.c_int, [ctypes.c_void_p, _f32p, _f32p])
_octree_bounds = _sig("tmpt_octree_bounds", ctypes.c_int, [_f32p, _f32p, _f32p])
_octree_digest = _sig("tmpt_octree_digest", ctypes.c_int, [_f32p, ctypes.c_int32, _f32p, _f32p, _u64p])
_octree_flags = _sig("tmpt_octree_flags", ctypes.c_int, [_f32p, ctypes.c_int32, _f32p, _f32p, _f32p, _f32p, _i32p,
                                                         ctypes.c_int64, ctypes.c_void_p, _f32p])
_render_multi = _sig("tmpt_render_multi", ctypes.c_int,
                     [_f32p, ctypes.c_int32, _f32p, ctypes.POINTER(_Camera), ctypes.POINTER(_Desc),
                      ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, ctypes.c_void_p, _u64p,
                      ctypes.POINTER(ctypes.c_double)])
_tile_rows = _sig("tmpt_tile_rows", ctypes.c_int32, [ctypes.POINTER(_Desc)])
_tile_row_to_y = _sig("tmpt_tile_row_to_y", ctypes.c_int32, [ctypes.POINTER(_Desc), ctypes.c_int32])
_stats = _sig("tmpt_get_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(_Stats)])
_write_png = _sig("tmpt_write_png", ctypes.c_int, [ctypes.c_char_p, _u8p, ctypes.c_int32, ctypes.c_int32])
_last_error = _sig("tmpt_last_error", ctypes.c_char_p, [])
_abi = _sig("tmpt_abi_version", ctypes.c_int, [])
_unit_sincos = _sig("tmpt_unit_sincos", ctypes.c_int, [ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint32,
                                                       ctypes.c_void_p])

#: every symbol include/tmpt.h declares (checked by tests/test_abi.py)
EXPORTS = ("tmpt_load_obj", "tmpt_free", "tmpt_camera_init", "tmpt_camera_for_scene",
           "tmpt_device_count", "tmpt_scene_create", "tmpt_scene_create_ex", "tmpt_scene_set_option",
           "tmpt_scene_get_option", "tmpt_scene_destroy", "tmpt_scene_hit", "tmpt_scene_hit_ranged",
           "tmpt_render", "tmpt_render_multi", "tmpt_tile_rows", "tmpt_tile_row_to_y", "tmpt_get_stats",
           "tmpt_write_png", "tmpt_last_error", "tmpt_abi_version", "tmpt_unit_sincos",
           "tmpt_scene_build_octree", "tmpt_octree_bounds", "tmpt_octree_digest",
           "tmpt_octree_flags")


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise TmptError(f"{what} failed ({rc}): {_last_error().decode(errors='replace')}")


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


def unit_sincos(key0: int, n: int, device: int = 0) -> np.ndarray:
    """RandomUnitVector's (cos a, sin a) for RNG keys [key0, key0 + n) (maths.cpp:33-36),
    n x 2 float32: computed on `device`, or by the host restatement when device < 0."""
    out = np.empty((n, 2), dtype=np.float32)
    _check(_unit_sincos(device, key0, n, out.ctypes.data), "tmpt_unit_sincos")
    return out


def device_count() -> int:
    return int(_dev_count())


def abi_version() -> int:
    return int(_abi())


# ----------------------------------------------------------------------------- scene ingest
def load_scene(path: str) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """LoadScene (main.cpp:122-170): returns (tris[n,3,3] float32 incl. the 2
    floor triangles, bounds_min[3], bounds_max[3]) -- bounds of the OBJ only."""
    p = _f32p()
    n = ctypes.c_int32()
    bmin = np.zeros(3, np.float32)
    bmax = np.zeros(3, np.float32)
    _check(_load_obj(path.encode(), ctypes.byref(p), ctypes.byref(n), _fp(bmin), _fp(bmax)),
           f"load_scene({path!r})")
    try:
        tris = np.ctypeslib.as_array(p, shape=(n.value * 9,)).copy().reshape(n.value, 3, 3)
    finally:
        _free(p)
    return tris, bmin, bmax


def octree_bounds(bmin, bmax) -> Tuple[np.ndarray, np.ndarray]:
    """The root box main.cpp:312 gives BuildOctree for a scene whose OBJ bounds
    are (bmin, bmax): bmin - extra, bmax + extra, extra = 0.7 x the size
    (main.cpp:296-297), in float32."""
    lo, hi = np.asarray(bmin, np.float32), np.asarray(bmax, np.float32)
    box = np.zeros(6, np.float32)
    _check(_octree_bounds(_fp(lo), _fp(hi), _fp(box)), "octree_bounds")
    return box[:3].copy(), box[3:].copy()


def octree_digest(tris: np.ndarray, box_min, box_max) -> dict:
    """The octree Scene.build_octree(box_min, box_max) builds, summarised on
    the host (no GPU): nodes, leaves, triangle references, depth and an FNV-1a
    digest of its preorder walk -- the check hook tests compare with the oracle."""
    t = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
    lo, hi = np.asarray(box_min, np.float32), np.asarray(box_max, np.float32)
    out = (ctypes.c_uint64 * 5)()
    _check(_octree_digest(_fp(t), t.shape[0], _fp(lo), _fp(hi), out), "octree_digest")
    return dict(zip(("nodes", "leaves", "refs", "depth", "digest"), (int(v) for v in out)))


def octree_flags(tris: np.ndarray, box_min, box_max, rays, t, ids):
    """Which answered queries the octree re-answers besides ties (host, no GPU):
    per ray 1 = the hit triangle lies flat on an octree plane, 2 = the hit may
    lie in a crack (the device's test), 0 = the BVH's answer stands; and the
    crack grid {r0, 1/cell, cell, band, reach}."""
    tr = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
    lo, hi = np.asarray(box_min, np.float32), np.asarray(box_max, np.float32)
    r = np.ascontiguousarray(np.asarray(rays, np.float32)[:, :6])
    tt = np.ascontiguousarray(np.asarray(t, np.float32))
    ii = np.ascontiguousarray(np.asarray(ids, np.int32))
    out = np.zeros(r.shape[0], np.uint8)
    grid = np.zeros(13, np.float32)
    _check(_octree_flags(_fp(tr), tr.shape[0], _fp(lo), _fp(hi), _fp(r), _fp(tt), ii.ctypes.data_as(_i32p),
                         r.shape[0], out.ctypes.data, _fp(grid)), "octree_flags")
    return out, grid


# ----------------------------------------------------------------------------- camera
@dataclass
class Camera:
    """Camera of maths.h:83-112 (fields as computed by Camera::Camera)."""
    origin: np.ndarray
    lower_left: np.ndarray
    horizontal: np.ndarray
    vertical: np.ndarray
    u: np.ndarray
    v: np.ndarray
    w: np.ndarray
    lens_radius: float

    @staticmethod
    def _from_c(c: _Camera) -> "Camera":
        a = lambda f: np.array(list(f), np.float32)
        return Camera(a(c.origin), a(c.lower_left), a(c.horizontal), a(c.vertical), a(c.u),
                      a(c.v), a(c.w), float(c.lens_radius))

    def _to_c(self) -> _Camera:
        c = _Camera()
        for name in ("origin", "lower_left", "horizontal", "vertical", "u", "v", "w"):
            getattr(c, name)[:] = [float(x) for x in np.asarray(getattr(self, name), np.float32)]
        c.lens_radius = self.lens_radius
        return c

    @staticmethod
    def create(look_from, look_at, vup, vfov: float, aspect: float, aperture: float,
               focus_dist: float) -> "Camera":
        """Camera::Camera (maths.cpp:40-59)."""
        c = _Camera()
        lf, la, up = (np.asarray(x, np.float32) for x in (look_from, look_at, vup))
        _check(_cam_init(ctypes.byref(c), _fp(lf), _fp(la), _fp(up), vfov, aspect, aperture,
                         focus_dist), "Camera")
        return Camera._from_c(c)

    @staticmethod
    def for_scene(bmin, bmax, width: int, height: int, is_sponza: bool = False) -> "Camera":
        """Camera placement of main.cpp:295-307."""
        c = _Camera()
        lo, hi = np.asarray(bmin, np.float32), np.asarray(bmax, np.float32)
        _check(_cam_scene(ctypes.byref(c), _fp(lo), _fp(hi), width, height, int(is_sponza)),
               "Camera.for_scene")
        return Camera._from_c(c)

    def as_array(self) -> np.ndarray:
        return np.concatenate([self.origin, self.lower_left, self.horizontal, self.vertical,
                               self.u, self.v, self.w, [self.lens_radius]]).astype(np.float32)


# ----------------------------------------------------------------------------- scene
@dataclass
class Hit:
    """Hit of maths.h:46-51."""
    pos: np.ndarray
    normal: np.ndarray
    t: float


@dataclass
class RenderStats:
    render_ms: float
    extend_ms: float
    shadow_ms: float
    extend_rays: int
    shadow_rays: int
    extend_launches: int
    shadow_launches: int
    iterations: int
    node_visits: int
    tri_tests: int
    shadow_node_visits: int
    shadow_tri_tests: int
    build_ms: float
    bvh_nodes: int
    bvh_depth: int
    n_tris: int
    device: int
    bvh4_nodes: int
    bvh4_depth: int
    leaf_max: int
    builder_iters: int
    octree_nodes: int
    octree_leaves: int
    octree_refs: int
    octree_build_ms: float
    tie_queries: int
    root_misses: int
    row_engine: int
    stream_fallbacks: int
    octree_depth: int
    tie_rule: int
    chain_pixels: int
    redo_samples: int
    redo_late: int
    crack_queries: int
    octree_flat: int
    redo_launches: int
    redo_ms: float
    redo_rays: int
    tie_path: int


def _desc(width, height, spp, seed_mode, band_rows=0, shard=0, num_shards=1,
          engine=ENGINE_PERSISTENT, flags=0, spp_begin=0, spp_count=0, wait_stream=None) -> _Desc:
    d = _Desc()
    d.width, d.height, d.spp, d.seed_mode = width, height, spp, seed_mode
    d.band_rows, d.shard, d.num_shards = band_rows, shard, num_shards
    d.engine, d.flags = engine, flags
    d.spp_begin, d.spp_count = spp_begin, spp_count
    if wait_stream is not None:
        d.flags |= FLAG_WAIT_STREAM
        d.wait_stream = int(wait_stream)
    return d


def _current_stream(device: int):
    """hipStream_t of torch's current stream on `device` (0 = its null stream),
    or None when torch has not initialised its GPU context (a caller whose
    device buffer does not come from torch has no torch work to wait for, and
    asking would initialise torch's context)."""
    if torch is None or not torch.cuda.is_initialized():
        return None
    return int(torch.cuda.current_stream(device).cuda_stream)


def tile_rows(width, height, band_rows=0, shard=0, num_shards=1) -> int:
    return int(_tile_rows(ctypes.byref(_desc(width, height, 1, 0, band_rows, shard, num_shards))))


def tile_row_to_y(width, height, band_rows, shard, num_shards) -> np.ndarray:
    d = _desc(width, height, 1, 0, band_rows, shard, num_shards)
    n = int(_tile_rows(ctypes.byref(d)))
    return np.array([_tile_row_to_y(ctypes.byref(d), r) for r in range(n)], np.int64)


def _options_text(options) -> Optional[bytes]:
    if options is None:
        return None
    if isinstance(options, str):
        return options.encode()
    return ",".join(f"{k}={v}" for k, v in dict(options).items()).encode()


class Scene:
    """Scene (scene.h:17-43): triangles copied to the GPU, BVH built there.

    ``options``: build and render options (include/tmpt.h "Scene options"),
    a dict or "key=value,..." string, e.g. ``{"builder": "lbvh", "leaf_max": 4}``;
    render options can also be changed later with :meth:`set_option`.
    ``bounds``: the OBJ bounds (bmin, bmax) :func:`load_scene` returns; given,
    the reference's octree is built over them as main.cpp:312 does
    (:meth:`build_octree`), so tied closest hits get the reference's answer."""

    def __init__(self, triangles: np.ndarray, device: int = 0, options=None, bounds=None):
        tris = np.ascontiguousarray(np.asarray(triangles, np.float32).reshape(-1, 9))
        self._h = ctypes.c_void_p()
        self.n = tris.shape[0]
        self.device = device
        _check(_scene_create_ex(_fp(tris), self.n, device, _options_text(options), ctypes.byref(self._h)),
               "Scene")
        if bounds is not None:
            self.build_octree(*octree_bounds(*bounds))

    def build_octree(self, box_min, box_max) -> None:
        """Scene::BuildOctree(min, max) (scene.cpp:75-83): the reference's octree
        over the scene, kept on the device to answer closest hits tied on t in
        its visit order and to apply its root box test (include/tmpt.h)."""
        lo, hi = np.asarray(box_min, np.float32), np.asarray(box_max, np.float32)
        _check(_build_octree(self._h, _fp(lo), _fp(hi)), "build_octree")

    def set_option(self, key: str, value: float) -> None:
        """A render option (include/tmpt.h); applies to the renders after it."""
        _check(_set_option(self._h, key.encode(), float(value)), f"set_option({key!r})")

    def get_option(self, key: str) -> float:
        v = ctypes.c_double()
        _check(_get_option(self._h, key.encode(), ctypes.byref(v)), f"get_option({key!r})")
        return v.value

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- Scene::HitScene (scene.cpp:86-97)
    def hit_scene_batch(self, rays: np.ndarray, t_min: Optional[float] = None, t_max: Optional[float] = None,
                        any_hit: bool = False) -> Tuple[np.ndarray, np.ndarray]:
        """rays [n,6] (orig, dir) with one [t_min, t_max] for all, or rays [n,8]
        (orig, dir, tmin, tmax: the range per ray, as HitScene takes it,
        scene.h:36-37) with t_min = t_max = None
        -> (ids[n] triangle index or -1, hits[n,7] pos/normal/t)."""
        rays = np.asarray(rays, np.float32)
        if (t_min is None) != (t_max is None):
            raise ValueError("hit_scene_batch: give both t_min and t_max, or neither (ranged rays [n,8])")
        ranged = t_min is None and t_max is None
        rays = np.ascontiguousarray(rays.reshape(-1, 8 if ranged else 6))
        n = rays.shape[0]
        hits = np.zeros((n, 7), np.float32)
        ids = np.full(n, -1, np.int32)
        if ranged:
            _check(_scene_hit_ranged(self._h, _fp(rays), n, int(any_hit), _fp(hits), ids.ctypes.data_as(_i32p)),
                   "hit_scene")
        else:
            _check(_scene_hit(self._h, _fp(rays), n, t_min, t_max, int(any_hit), _fp(hits),
                              ids.ctypes.data_as(_i32p)), "hit_scene")
        return ids, hits

    def hit_scene(self, orig, direction, t_min: float, t_max: float) -> Tuple[int, Optional[Hit]]:
        """Same contract as the reference: returns (-1, None) on a miss and
        (1, Hit) on a hit (scene.cpp:37 sets 1, not the index)."""
        ids, hits = self.hit_scene_batch(np.concatenate([orig, direction])[None], t_min, t_max)
        if ids[0] < 0:
            return -1, None
        h = hits[0]
        return 1, Hit(h[0:3].copy(), h[3:6].copy(), float(h[6]))

    # -- TraceImageBody over parallel_for (main.cpp:180-246, 329-331)
    def trace_image(self, camera: Camera, width: int, height: int, spp: int,
                    seed_mode: int = SEED_ROW, engine: int = ENGINE_PERSISTENT, band_rows: int = 0,
                    shard: int = 0, num_shards: int = 1, count_visits: bool = False,
                    out=None, spp_begin: int = 0, spp_count: int = 0,
                    wait_stream="current") -> Tuple[np.ndarray, int]:
        """Render one shard.  Returns (rgba[tile_rows, width, 4] uint8, rays).
        Row 0 is the lowest rendered row (main.cpp:229; flipped on PNG write).
        ``out`` may be a device pointer (int) with tile_rows*width*4 bytes; the
        render then starts after the work already enqueued on ``wait_stream``
        ("current": torch's current stream on the scene's device when torch's
        GPU context is up, so a fill of ``out`` or a collective still reading
        it is ordered before the render; an int: a raw hipStream_t; None: no
        ordering).  The call returns once
        the frame is complete on the device.
        ``spp_begin``/``spp_count``: one progressive pass (persistent engine,
        pixel or sample seeding) -- see :meth:`trace_progressive`."""
        if out is None:
            ws = None
        elif isinstance(wait_stream, str):
            ws = _current_stream(self.device)
        else:
            ws = wait_stream
        d = _desc(width, height, spp, seed_mode, band_rows, shard, num_shards, engine,
                  (FLAG_COUNT_VISITS if count_visits else 0) | (FLAG_OUT_DEVICE if out is not None else 0),
                  spp_begin, spp_count, ws)
        rows = int(_tile_rows(ctypes.byref(d)))
        rays = ctypes.c_uint64()
        cam = camera._to_c()
        if out is not None:
            _check(_render(self._h, ctypes.byref(cam), ctypes.byref(d), ctypes.c_void_p(int(out)),
                           ctypes.byref(rays)), "trace_image")
            return None, int(rays.value)
        img = np.zeros((rows, width, 4), np.uint8)
        _check(_render(self._h, ctypes.byref(cam), ctypes.byref(d), img.ctypes.data_as(ctypes.c_void_p),
                       ctypes.byref(rays)), "trace_image")
        return img, int(rays.value)

    def trace_progressive(self, camera: Camera, width: int, height: int, spp: int, passes,
                          band_rows: int = 0, shard: int = 0, num_shards: int = 1, seed_mode: int = SEED_PIXEL):
        """Progressive spp: yields (samples_done, preview rgba, rays of the pass) per
        pass; ``passes`` = samples per pass (int) or a list of them summing to spp.
        The last preview is the final image, bit-identical to one full render;
        pixel or sample seeding (the samples of a pass run side by side there)."""
        if isinstance(passes, int):
            passes = [min(passes, spp - b) for b in range(0, spp, passes)]
        if sum(passes) != spp or min(passes) < 1:
            raise ValueError("passes must be positive and sum to spp")
        done = 0
        for n in passes:
            img, rays = self.trace_image(camera, width, height, spp, seed_mode=seed_mode,
                                         engine=ENGINE_PERSISTENT, band_rows=band_rows, shard=shard,
                                         num_shards=num_shards, spp_begin=done, spp_count=n)
            done += n
            yield done, img, rays

    def stats(self) -> RenderStats:
        s = _Stats()
        _check(_stats(self._h, ctypes.byref(s)), "stats")
        return RenderStats(*[getattr(s, f) for f, _ in _Stats._fields_ if not f.startswith("reserved")])


def render_multi(tris: np.ndarray, camera: "Camera", width: int, height: int, spp: int, devices,
                 seed_mode: int = SEED_PIXEL, engine: int = ENGINE_PERSISTENT,
                 require_rccl: bool = False, bounds=None) -> Tuple[np.ndarray, int, float]:
    """One frame over several devices in this process (tmpt_render_multi: the
    tiles gathered to devices[0] by one RCCL gather): returns (rgba[height,
    width, 4], rays, seconds from the renders' start to the assembled frame).
    A device may repeat (then the gather is device-to-device copies; with
    require_rccl that is an error instead).  ``bounds`` (OBJ bounds): every
    device's scene builds the reference's octree (main.cpp:312)."""
    t = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
    devs = (ctypes.c_int32 * len(devices))(*devices)
    img = np.zeros((height, width, 4), np.uint8)
    rays = ctypes.c_uint64()
    secs = ctypes.c_double()
    d = _desc(width, height, spp, seed_mode, 0, 0, 1, engine, FLAG_REQUIRE_RCCL if require_rccl else 0)
    cam = camera._to_c()
    box = None if bounds is None else np.concatenate(octree_bounds(*bounds)).astype(np.float32)
    _check(_render_multi(t.ctypes.data_as(_f32p), t.shape[0], None if box is None else _fp(box),
                         ctypes.byref(cam), ctypes.byref(d), devs,
                         len(devices), img.ctypes.data_as(ctypes.c_void_p), ctypes.byref(rays),
                         ctypes.byref(secs)), "render_multi")
    return img, int(rays.value), float(secs.value)


def write_png(path: str, rgba: np.ndarray) -> None:
    """stbi_write_png with flip-on-write (main.cpp:341-342): rgba rows bottom-up."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    h, w = rgba.shape[:2]
    _check(_write_png(path.encode(), rgba.ctypes.data_as(_u8p), w, h), "write_png")
