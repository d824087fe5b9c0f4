"""Adversarial HitScene rays for the reference's octree (test helper).

The library answers a closest-hit query from its BVH -- the exact closest hit
over all triangles -- except where the reference's octree walk is known to
answer differently: a tie on t (re-answered in the octree's visit order) and a
ray its root box test drops (a miss).  The argument that nothing else differs
rests on the octree's geometry: a unique closest triangle T at hit point p is
in the leaf whose cell holds p (scene.cpp:144-154, TriangleIntersectAabb), and
the ray passes that cell's slab test (maths.h:116-134) -- both robust unless p,
or the ray, sits on a cell's face, edge or corner, where the rounding of the
separating-axis test or of the slab test decides.

So these rays are aimed exactly there, from the octree's own node boxes
(oracle.Scene.octree_nodes, node for node the library's octree,
tests/test_octree.py):

  corner / edge / face   a random point of a node box's corner, edge or face
  tri_plane              a point of a leaf triangle on one of its leaf's face
                         planes (T cut by x = const: a segment; its endpoints,
                         where T's edges cross the plane, included)
  tri_edge               T crossed by one of its leaf's box edge lines
  axis_face, axis_edge   axis-parallel directions travelling inside a face
                         plane or along an edge line (1/d = inf in the slab test)
  vertex                 a leaf triangle's vertices (on split planes in the
                         axis-aligned and grid scenes)

`classify` compares the reference's answer (oracle octree, visit order) with
the exact closest hit (oracle BVH, lowest index on a tie) and sorts every
difference into the two known kinds and the excluded one.
"""
from __future__ import annotations

import numpy as np

import oracle

KINDS = ("corner", "edge", "face", "tri_plane", "tri_edge", "axis_face", "axis_edge", "vertex", "in_plane")


def _unit(d):
    d = d.astype(np.float32)
    n = np.sqrt((d * d).sum(1, keepdims=True, dtype=np.float32)).astype(np.float32)
    n[n == 0] = 1
    return (d / n).astype(np.float32)


def _origins(rng, lo, hi, n):
    ext = hi - lo
    return (lo - 0.3 * ext + rng.random((n, 3)) * 1.6 * ext).astype(np.float32)


def _box_points(rng, boxes, n, kind):
    """n points on random boxes' corners / edges / faces."""
    b = boxes[rng.integers(0, len(boxes), n)]
    lo, hi = b[:, :3], b[:, 3:]
    sel = rng.integers(0, 2, (n, 3)).astype(bool)
    p = np.where(sel, hi, lo)  # a corner
    if kind in ("edge", "face"):
        free = rng.integers(0, 3, n)  # one coordinate moves along the edge
        f = rng.random(n).astype(np.float32)
        ar = np.arange(n)
        p[ar, free] = lo[ar, free] + f * (hi[ar, free] - lo[ar, free])
        if kind == "face":
            free2 = (free + 1 + rng.integers(0, 2, n)) % 3
            f2 = rng.random(n).astype(np.float32)
            p[ar, free2] = lo[ar, free2] + f2 * (hi[ar, free2] - lo[ar, free2])
    return p.astype(np.float32)


def _tri_plane_points(rng, tris, boxes, info, refs, n, on_edge):
    """Points of leaf triangles on their leaf box's face planes (on_edge: on
    the box's edge lines, i.e. two coordinates fixed)."""
    leaves = np.nonzero((info[:, 0] < 0) & (info[:, 1] > 0))[0]
    out = []
    tries = 0
    while len(out) < n and tries < 40 * n:
        tries += 1
        lf = leaves[rng.integers(0, len(leaves))]
        tid = refs[lf][rng.integers(0, len(refs[lf]))]
        T = tris[tid].astype(np.float64)
        box = boxes[lf].astype(np.float64)
        ax = rng.integers(0, 3)
        c = box[ax + 3 * rng.integers(0, 2)]
        s = T[:, ax] - c
        pts = []
        for i in range(3):  # where the triangle's edges cross the plane
            a, b = s[i], s[(i + 1) % 3]
            if a == 0:
                pts.append(T[i])
            elif a * b < 0:
                pts.append(T[i] + (a / (a - b)) * (T[(i + 1) % 3] - T[i]))
        if not pts:
            continue
        if len(pts) >= 2 and not on_edge:
            f = rng.random()
            p = pts[0] + f * (pts[1] - pts[0])
            if rng.random() < 0.25:
                p = pts[rng.integers(0, len(pts))]
        elif on_edge and len(pts) >= 2:
            # the segment crossed by a second plane: an edge line of the box
            ax2 = (ax + 1 + rng.integers(0, 2)) % 3
            c2 = box[ax2 + 3 * rng.integers(0, 2)]
            a, b = pts[0][ax2] - c2, pts[1][ax2] - c2
            if a * b > 0:
                continue
            p = pts[0] if a == b else pts[0] + (a / (a - b)) * (pts[1] - pts[0])
            p = p.copy()
            p[ax2] = c2
        else:
            p = pts[0]
        p = p.copy()
        p[ax] = c
        out.append(p)
    return np.array(out, np.float32).reshape(-1, 3)


def _axis_rays(rng, boxes, n, along_edge, lo, hi):
    """Axis-parallel rays inside a face plane (along_edge=False: two of the
    origin's coordinates free, one on the plane) or on an edge line."""
    b = boxes[rng.integers(0, len(boxes), n)]
    ax = rng.integers(0, 3, n)  # travel axis
    ar = np.arange(n)
    o = (lo + rng.random((n, 3)) * (hi - lo)).astype(np.float32)
    k1 = (ax + 1) % 3
    k2 = (ax + 2) % 3
    side1 = rng.integers(0, 2, n)
    o[ar, k1] = b[ar, k1 + 3 * side1]
    if along_edge:
        side2 = rng.integers(0, 2, n)
        o[ar, k2] = b[ar, k2 + 3 * side2]
    ext = (hi - lo).max()
    sgn = np.where(rng.random(n) < 0.5, -1.0, 1.0).astype(np.float32)
    o[ar, ax] = np.where(sgn > 0, lo[ax] - 0.2 * ext, hi[ax] + 0.2 * ext)
    d = np.zeros((n, 3), np.float32)
    d[ar, ax] = sgn
    return np.concatenate([o, d], 1)


def adversarial_rays(tris, bmin, bmax, n_per_kind, seed, osc=None):
    """Rays of every kind in KINDS, n_per_kind each (fewer for tri_* when
    triangles rarely cross their leaf's planes).  Returns (rays n x 6, kind
    index per ray)."""
    rng = np.random.default_rng(seed)
    osc = osc or ref_scene(tris, bmin, bmax)
    boxes, info = osc.octree_nodes()
    refs = leaf_lists(tris, osc, info)
    v = tris.reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    rays, kind = [], []

    def aim(targets, k):
        o = _origins(rng, lo, hi, len(targets))
        rays.append(np.concatenate([o, _unit(targets - o)], 1).astype(np.float32))
        kind.append(np.full(len(targets), k, np.int32))

    for k, name in enumerate(KINDS):
        if name in ("corner", "edge", "face"):
            aim(_box_points(rng, boxes, n_per_kind, name), k)
        elif name == "tri_plane":
            aim(_tri_plane_points(rng, tris, boxes, info, refs, n_per_kind, False), k)
        elif name == "tri_edge":
            aim(_tri_plane_points(rng, tris, boxes, info, refs, n_per_kind, True), k)
        elif name in ("axis_face", "axis_edge"):
            r = _axis_rays(rng, boxes, n_per_kind, name == "axis_edge", lo, hi)
            rays.append(r.astype(np.float32))
            kind.append(np.full(len(r), k, np.int32))
        elif name == "in_plane":
            # one direction component exactly 0 (a scatter ray off an axis-aligned
            # face can round to that: normalize(target - pos), main.cpp:71-72),
            # the origin's coordinate on a node box's face plane
            o = _origins(rng, lo, hi, n_per_kind)
            ax = rng.integers(0, 3, n_per_kind)
            ar = np.arange(n_per_kind)
            b = boxes[rng.integers(0, len(boxes), n_per_kind)]
            o[ar, ax] = b[ar, ax + 3 * rng.integers(0, 2, n_per_kind)]
            tgt = _box_points(rng, boxes, n_per_kind, "face")
            d = tgt - o
            d[ar, ax] = 0
            rays.append(np.concatenate([o, _unit(d)], 1).astype(np.float32))
            kind.append(np.full(n_per_kind, k, np.int32))
        else:  # vertex
            leaves = np.nonzero((info[:, 0] < 0) & (info[:, 1] > 0))[0]
            lf = leaves[rng.integers(0, len(leaves), n_per_kind)]
            tid = np.array([refs[x][rng.integers(0, len(refs[x]))] for x in lf])
            aim(tris[tid, rng.integers(0, 3, n_per_kind)].astype(np.float32), k)
    return np.concatenate(rays), np.concatenate(kind)


def leaf_lists(tris, osc, info):
    """Triangle ids per non-empty octree leaf, in the reference's order."""
    return {int(lf): osc.octree_leaf(int(lf)) for lf in np.nonzero((info[:, 0] < 0) & (info[:, 1] > 0))[0]}


def _leaf_lists_bruteforce(tris, osc, info):
    """(unused) triangles whose bounding box touches the leaf box."""
    boxes, _ = osc.octree_nodes()
    tlo = tris.min(1)
    thi = tris.max(1)
    out = {}
    for lf in np.nonzero((info[:, 0] < 0) & (info[:, 1] > 0))[0]:
        b = boxes[lf]
        m = np.nonzero(((tlo <= b[3:]) & (thi >= b[:3])).all(1))[0]
        out[lf] = m if len(m) else np.array([0])
    return out


def ref_scene(tris, bmin, bmax):
    return oracle.Scene(tris, accel=oracle.ACCEL_OCTREE, tie=oracle.TIE_VISIT, bmin=bmin, bmax=bmax)


def classify(tris, bmin, bmax, rays, t_min=0.001, t_max=1.0e7, osc=None):
    """Reference answer vs the exact closest hit, per ray.  Returns a dict of
    index arrays: same (no difference), tie (both hit at the same t, another
    triangle: visit order), root (the reference misses and its root box test
    failed), other (anything else -- the class the library does not flag)."""
    osc = osc or ref_scene(tris, bmin, bmax)
    ex = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    rid, rh = osc.hit_batch(rays, t_min, t_max)
    eid, eh = ex.hit_batch(rays, t_min, t_max)
    boxes, _ = osc.octree_nodes()
    root_ok = oracle.ray_box(rays, boxes[0], t_min, t_max) if len(boxes) else np.ones(len(rays), bool)
    diff = rid != eid
    tie = diff & (rid >= 0) & (eid >= 0) & (rh[:, 6].view(np.uint32) == eh[:, 6].view(np.uint32))
    root = diff & (rid < 0) & ~root_ok
    other = diff & ~tie & ~root
    return {"n": len(rays), "hits": int((eid >= 0).sum()), "tie": np.nonzero(tie)[0], "root": np.nonzero(root)[0],
            "other": np.nonzero(other)[0], "rid": rid, "eid": eid, "rh": rh, "eh": eh}


def grid_scene(k=3, n=6, seed=0):
    """A synthetic scene on the octree's split planes: OBJ bounds +-s with
    s = 1/2.4 give the root box +-1 (main.cpp:296-297,312: bounds +- 0.7 x
    size), whose planes are the multiples of 1/2^j; axis-aligned quads on the
    planes c = i / 2^k and triangles with vertices snapped to them.
    Returns (tris, bmin, bmax)."""
    rng = np.random.default_rng(seed)
    planes = np.arange(-(2 ** k) + 1, 2 ** k) / float(2 ** k)
    s = np.float32(1.0 / 2.4)
    planes = planes[np.abs(planes) <= s]
    tris = []
    for _ in range(n * 40):
        ax = rng.integers(0, 3)
        c = rng.choice(planes)
        a, b = np.sort(rng.choice(planes, 2, replace=False)), np.sort(rng.choice(planes, 2, replace=False))
        q = np.zeros((4, 3))
        u, w = (ax + 1) % 3, (ax + 2) % 3
        for i, (x, y) in enumerate(((a[0], b[0]), (a[1], b[0]), (a[1], b[1]), (a[0], b[1]))):
            q[i, ax], q[i, u], q[i, w] = c, x, y
        tris.append(q[[0, 1, 2]])
        tris.append(q[[0, 2, 3]])
    for _ in range(n * 20):
        tris.append(rng.choice(planes, (3, 3)))
    tris = np.array(tris, np.float32)
    # bounds exactly +-s so that the root box lands on +-1 (main.cpp:296-297,312)
    tris[0, 0] = [-s, -s, -s]
    tris[1, 0] = [s, s, s]
    bmin = tris.reshape(-1, 3).min(0)
    bmax = tris.reshape(-1, 3).max(0)
    return tris, bmin, bmax


def crack_wall_scene(tris, bmin, bmax, osc=None):
    """The scene plus one small wall lying flat inside a crack of its octree:
    a plane coordinate strictly between one subtree's box max and the next
    subtree's min, at a spot no leaf box covers (found from the octree's leaf
    boxes).  The reference's walk never meets the wall (it is in no leaf), so
    rays aimed at it see through it; the exact closest hit finds it.  Returns
    (tris with the wall last, the wall's axis, a point on it) or None when the
    octree has no such gap."""
    osc = osc or ref_scene(tris, bmin, bmax)
    boxes, info = osc.octree_nodes()
    lb = boxes[np.nonzero(info[:, 0] < 0)[0]]
    for ax in range(3):
        u, w = (ax + 1) % 3, (ax + 2) % 3
        mn = np.unique(lb[:, ax])
        for a in np.unique(lb[:, ax + 3]):
            jj = np.searchsorted(mn, a, side="right")
            if jj >= len(mn):
                continue
            c = mn[jj]
            if not (c > a and c - a <= 16 * np.spacing(np.float32(abs(c)))):
                continue
            cp = np.nextafter(np.float32(a), np.float32(c))
            if not (a < cp < c):
                continue
            for l in np.nonzero(lb[:, ax + 3] == a)[0]:
                lo, hi = lb[l, [u, w]], lb[l, [u + 3, w + 3]]
                p = np.zeros(3, np.float32)
                p[ax], p[u], p[w] = cp, lo[0] + 0.5 * (hi[0] - lo[0]), lo[1] + 0.5 * (hi[1] - lo[1])
                if ((lb[:, :3] <= p) & (lb[:, 3:] >= p)).all(1).any():
                    continue
                e = 0.2 * (hi - lo)
                v = np.zeros((3, 3), np.float32)
                for i, (du, dw) in enumerate(((-1, -1), (1, -1), (0, 1))):
                    v[i, ax], v[i, u], v[i, w] = cp, p[u] + du * e[0], p[w] + dw * e[1]
                return np.concatenate([tris, v[None]]).astype(np.float32), ax, p
    return None


def crack_wall_rays(wall, ax, n, seed):
    """Rays aimed head-on (tilted) at points of the wall (tris[-1])."""
    rng = np.random.default_rng(seed)
    v = wall.astype(np.float32)
    bary = rng.random((n, 3))
    bary /= bary.sum(1, keepdims=True)
    pts = (bary @ v).astype(np.float32)
    pts[:, ax] = v[0, ax]
    u, w = (ax + 1) % 3, (ax + 2) % 3
    off = np.zeros((n, 3), np.float32)
    off[:, ax] = np.where(rng.random(n) < 0.5, -5.0, 5.0)
    off[:, u] = rng.normal(size=n) * 0.5
    off[:, w] = rng.normal(size=n) * 0.5
    o = pts + off
    return np.concatenate([o, _unit(pts - o)], 1).astype(np.float32)


def child_order_case():
    """A tie whose reference answer follows from scene.cpp's structure alone,
    derived by hand (the visit order pinned independently of the
    oracle).  Root box [-1, 1]^3, 12 triangles, so the root splits
    (scene.cpp:101; 17 nodes: child 6 holds Tb and the fillers and splits
    again); children are built min-corner first (:119-141) and
    visited in that order (:44-49), child 0 = [-1, 0]^3, child 7 = [0, 1]^3.
      Ta (index 0): small, around p = (0.5, 0.5, 0.5), inside child 7 only;
      Tb (index 1): large, coplanar with Ta (plane z = x), through p, with a
                    vertex at (-0.75, -0.75, -0.75) inside child 0;
      10 fillers near (-0.9, 0.9, 0.9), off the ray.
    The ray o = (-0.75, -0.75, -0.25), d = (1.25, 1.25, 0.75) starts in child 0
    and hits both at exactly t = 1 (dyadic coordinates: every Moller-Trumbore
    step is exact).  The walk meets Tb in child 0 first; Ta, met in child 7 at
    the same t, is not nearer (strict '<', scene.cpp:34).  So the reference
    answers Tb, index 1; the lowest-index rule answers Ta."""
    ta = [[0.25, 0.25, 0.25], [0.75, 0.25, 0.75], [0.5, 0.75, 0.5]]
    tb = [[-0.75, -0.75, -0.75], [0.75, -0.75, 0.75], [0.75, 0.875, 0.75]]
    fill = [[[-0.9 + 0.01 * i, 0.9, 0.9], [-0.9 + 0.01 * i, 0.92, 0.9], [-0.9 + 0.01 * i, 0.9, 0.92]]
            for i in range(10)]
    tris = np.array([ta, tb] + fill, np.float32)
    ray = np.array([[-0.75, -0.75, -0.25, 1.25, 1.25, 0.75]], np.float32)
    box = (np.full(3, -1.0, np.float32), np.full(3, 1.0, np.float32))
    return tris, ray, box

