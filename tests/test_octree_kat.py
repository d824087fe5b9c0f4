"""The reference's octree against the exact closest hit, on rays aimed at its
cracks (CPU, oracle + the library's host check hook; no GPU).

The library answers closest hits from its BVH and sends to the reference's
octree only the queries where the two can differ.  tests/octree_kat.py aims
rays at the octree's own faces, edges and corners, at triangles crossing them,
along them (axis-parallel and in-plane directions) and at triangle vertices,
and sorts every difference between the reference's answer (oracle octree,
visit order, scene.cpp:21-52) and the exact closest hit into ties, root-box
misses and the rest.  The rest is the crack class (tmpt_internal.h OctGrid):
this test checks that the library's own predicate (tmpt_octree_flags, the
device's octree_crack and the flat-triangle marks) flags every such ray, so
the GPU answers it over the octree (tests/test_gpu_parity.py checks that).
"""
import numpy as np
import pytest

import oracle
import octree_kat as K
import toymeshpathtracer_amd as tm
from conftest import data


def _scene(name):
    if name == "grid":
        return K.grid_scene()
    return oracle.load_scene(data(name + ".obj"))


@pytest.mark.parametrize("name", ["cube", "suzanne", "teapot", "grid"])
def test_excluded_class_is_flagged(name):
    tris, bmin, bmax = _scene(name)
    osc = K.ref_scene(tris, bmin, bmax)
    rays, kind = K.adversarial_rays(tris, bmin, bmax, 6000, seed=5, osc=osc)
    c = K.classify(tris, bmin, bmax, rays, osc=osc)
    lo, hi = tm.octree_bounds(bmin, bmax)
    flags, grid = tm.octree_flags(tris, lo, hi, rays, c["eh"][:, 6], c["eid"])
    other = c["other"]
    per_kind = {K.KINDS[k]: int((kind[other] == k).sum()) for k in range(len(K.KINDS))}
    print(name, "rays", c["n"], "ties", len(c["tie"]), "root", len(c["root"]), "other", len(other), per_kind,
          "flagged", int((flags > 0).sum()))
    assert c["hits"] > c["n"] // 2
    unflagged = other[flags[other] == 0]
    assert unflagged.size == 0, f"{unflagged.size} unflagged deviations, first {rays[unflagged[:3]]}"
    if name == "teapot":  # the class exists: axis-parallel and in-plane rays along a crack
        assert len(other) > 0 and per_kind["axis_edge"] + per_kind["axis_face"] + per_kind["in_plane"] == len(other)


def test_near_parallel_rays_flagged():
    """Rays leaving an octree plane with one direction component 1e-7 .. 1e-2
    (the drift that decides whether a ray can run inside a crack): every
    deviation from the exact closest hit that is not a tie or a root miss is
    flagged."""
    tris, bmin, bmax = _scene("teapot")
    osc = K.ref_scene(tris, bmin, bmax)
    boxes, _ = osc.octree_nodes()
    rng = np.random.default_rng(1)
    v = tris.reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    n, total_other = 4000, 0
    olo, ohi = tm.octree_bounds(bmin, bmax)
    for mag in (0.0, 1e-7, 1e-6, 1e-5, 1e-4, 1e-2):
        o = K._origins(rng, lo, hi, n)
        ax, ar = rng.integers(0, 3, n), np.arange(n)
        b = boxes[rng.integers(0, len(boxes), n)]
        o[ar, ax] = b[ar, ax + 3 * rng.integers(0, 2, n)]
        d = K._unit(K._box_points(rng, boxes, n, "face") - o)
        d[ar, ax] = mag * rng.choice([-1.0, 1.0], n) * (1 + rng.random(n))
        rays = np.concatenate([o, K._unit(d)], 1).astype(np.float32)
        c = K.classify(tris, bmin, bmax, rays, osc=osc)
        flags, _ = tm.octree_flags(tris, olo, ohi, rays, c["eh"][:, 6], c["eid"])
        assert (flags[c["other"]] > 0).all(), mag
        total_other += len(c["other"])
    assert total_other > 0


def test_crack_wall_is_flat_and_lost():
    """A wall lying inside a crack of teapot's octree (in no leaf): the
    reference sees through it -- every ray aimed at it answers differently
    from the exact closest hit -- and the library marks it flat, so every hit
    on it is flagged."""
    tris, bmin, bmax = _scene("teapot")
    got = K.crack_wall_scene(tris, bmin, bmax)
    assert got is not None
    t2, ax, _ = got
    rays = K.crack_wall_rays(t2[-1], ax, 2000, seed=3)
    c = K.classify(t2, bmin, bmax, rays)
    wall = len(t2) - 1
    assert (c["eid"] == wall).sum() > 1500 and (c["rid"] == wall).sum() == 0
    lo, hi = tm.octree_bounds(bmin, bmax)
    flags, _ = tm.octree_flags(t2, lo, hi, rays, c["eh"][:, 6], c["eid"])
    on_wall = c["eid"] == wall
    assert (flags[on_wall] & 1).all() and (flags[c["other"]] > 0).all()
    # the scene's own triangles are not flat (teapot has no triangle on a plane)
    f_all, _ = tm.octree_flags(tris, lo, hi, rays[:1], np.ones(1, np.float32), np.zeros(1, np.int32))
    assert f_all[0] & 1 == 0


def test_child_order_case_pins_the_oracle():
    """The oracle's octree gives the hand-derived answer (Tb, t = 1) and its
    exact-semantics BVH the lowest index (Ta)."""
    tris, ray, _ = K.child_order_case()
    # oracle.Scene takes OBJ bounds and pads them by 0.7 x size (main.cpp:296-297): pass
    # bounds whose padded box is [-1, 1]^3 exactly
    s = np.float32(1.0 / 2.4)
    ob = (np.full(3, -s, np.float32), np.full(3, s, np.float32))
    octree = oracle.Scene(tris, accel=oracle.ACCEL_OCTREE, tie=oracle.TIE_VISIT, bmin=ob[0], bmax=ob[1])
    boxes, info = octree.octree_nodes()
    assert np.allclose(boxes[0], [-1, -1, -1, 1, 1, 1]) and len(boxes) == 17 and info[0, 0] == 1
    ids, hits = octree.hit_batch(ray, 0.001, 1.0e7)
    assert ids[0] == 1 and hits[0, 6] == 1.0
    ex = oracle.Scene(tris, accel=oracle.ACCEL_LINEAR)
    eids, ehits = ex.hit_batch(ray, 0.001, 1.0e7)
    assert eids[0] == 0 and ehits[0, 6] == 1.0


SPANS = (1 / 256, 1 / 64, 1 / 16, 1 / 8, 1 / 4, 1 / 2, 1.0, 2.0, 4.0)  # crossing spans, in finest cells


def _scene_any(name):
    if name == "sponza":
        import gen_standin_sponza
        return oracle.load_scene(gen_standin_sponza.ensure())
    return _scene(name)


@pytest.mark.parametrize("name", ["cube", "suzanne", "teapot", "grid", "sponza"])
def test_crack_span_sweep(name):
    """the crack flag's guarantee, swept.  Rays cross an
    octree face plane exactly where a leaf triangle meets it (tri_plane
    points) with the drift across the plane set by the crossing span
    S = g / |d_k| (g = the crack width W of the grid, at least 1 ulp of the
    root's coordinates: the t-span the ray spends inside the crack), S = 1/256
    .. 4 finest cells, from origins 0.05 .. 3 cells back along the ray.  The
    derived bound says the reference's walk can miss the
    exact closest hit (besides a tie or its root box) only where
    |d_k| min(t, reach) <= 2 (W + delta_k) with the hit within W + delta_k of
    the plane -- inside the flagged region |d_k| min(t, reach) <= 2 band,
    hit within band.  Every deviation that is not a tie or a root-box miss
    must be flagged, at every span; the table shows where deviations occur."""
    import sys
    sys.path.insert(0, data(""))
    tris, bmin, bmax = _scene_any(name)
    osc = K.ref_scene(tris, bmin, bmax)
    boxes, info = osc.octree_nodes()
    refs = K.leaf_lists(tris, osc, info)
    olo, ohi = tm.octree_bounds(bmin, bmax)
    _, grid = tm.octree_flags(tris, olo, ohi, np.zeros((1, 6), np.float32), np.ones(1, np.float32),
                              -np.ones(1, np.int32))
    cell, band = grid[6:9].astype(np.float64), grid[9:12].astype(np.float64)
    top = np.maximum(np.abs(olo), np.abs(ohi)).astype(np.float32)
    ulp = (np.nextafter(top, np.float32(np.inf)) - top).astype(np.float64)
    gap = np.maximum((band - 8.0 * ulp) / 4.0, ulp)  # band = 4 W + 8 ulp (OctGrid)
    rng = np.random.default_rng(11)
    n = 1500 if name == "sponza" else 2500
    report, unflagged_total, other_total = [], 0, 0
    for span in SPANS:
        p = K._tri_plane_points(rng, tris, boxes, info, refs, n, False).astype(np.float64)
        m = len(p)
        # the axis whose plane each point lies on
        rel = (p - grid[0:3]) / cell
        ax = np.argmin(np.abs(rel - np.rint(rel)) * cell / band, axis=1)
        ar = np.arange(m)
        dk = gap[ax] / (span * cell[ax]) * rng.choice([-1.0, 1.0], m) * rng.uniform(0.5, 1.0, m)
        u = rng.normal(size=(m, 3))
        u[ar, ax] = 0.0
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        d = u * np.sqrt(1.0 - dk * dk)[:, None]
        d[ar, ax] = dk
        L = cell[ax] * rng.uniform(0.05, 3.0, m)
        o = p - L[:, None] * d
        rays = np.concatenate([o, d], 1).astype(np.float32)
        c = K.classify(tris, bmin, bmax, rays, osc=osc)
        flags, _ = tm.octree_flags(tris, olo, ohi, rays, c["eh"][:, 6], c["eid"])
        other = c["other"]
        unf = other[flags[other] == 0]
        report.append((span, m, len(c["tie"]), len(c["root"]), len(other), int((flags > 0).sum()), len(unf)))
        unflagged_total += len(unf)
        other_total += len(other)
    print(name, "span/cell, rays, ties, root, other, flagged, unflagged:", report)
    assert unflagged_total == 0, report
