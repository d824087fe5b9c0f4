#!/usr/bin/env python3
"""Deterministic STAND-IN for data/sponza.obj (absent from the reference:
/root/reference/.MISSING_LARGE_BLOBS).

An arcaded, open-roof atrium of exactly 66,450 triangles (66,452 with the two
floor triangles LoadScene adds, readme.md:74) built so that the reference's
hard-coded sponza camera (-5.96, 4.08, -1.22) (main.cpp:300-301) stands inside
it, looking down the long axis.  The file name contains "sponza.obj" so that
camera is selected.  It is a stand-in for the workload's shape (an interior
with columns, arches, galleries, drapes and an open roof: deep multi-bounce
paths), not the Dabrovic model; every number measured on it says so.

Usage: python data/gen_standin_sponza.py [out.obj]   (default data/generated/standin_sponza.obj)
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

TARGET_TRIS = 66450

# atrium extents (x along the nave, y up, z across)
X0, X1 = -15.0, 15.0
Z0, Z1 = -6.6, 6.6
Y_BASE = -0.12          # foundation slab; keeps LoadScene's floor below everything
L1, L2, L3 = 0.0, 5.2, 10.4   # floor, gallery 1, gallery 2 levels
TOP = 14.2


class Mesh:
    def __init__(self):
        self.v: list[np.ndarray] = []
        self.f: list[np.ndarray] = []
        self.nv = 0

    def add(self, verts: np.ndarray, faces: np.ndarray) -> None:
        verts = np.asarray(verts, np.float64).reshape(-1, 3)
        faces = np.asarray(faces, np.int64).reshape(-1, 3)
        self.v.append(verts)
        self.f.append(faces + self.nv)
        self.nv += verts.shape[0]

    @property
    def ntris(self) -> int:
        return int(sum(f.shape[0] for f in self.f))

    def grid(self, P: np.ndarray) -> None:
        """P[nu+1, nv+1, 3] -> 2*nu*nv triangles."""
        nu, nv = P.shape[0] - 1, P.shape[1] - 1
        idx = np.arange((nu + 1) * (nv + 1)).reshape(nu + 1, nv + 1)
        a, b = idx[:-1, :-1].ravel(), idx[1:, :-1].ravel()
        c, d = idx[1:, 1:].ravel(), idx[:-1, 1:].ravel()
        faces = np.stack([np.stack([a, b, c], 1), np.stack([a, c, d], 1)], 1).reshape(-1, 3)
        self.add(P.reshape(-1, 3), faces)

    def box(self, lo, hi) -> None:
        lo, hi = np.asarray(lo, float), np.asarray(hi, float)
        c = np.array([[lo[0] if i & 1 == 0 else hi[0], lo[1] if i & 2 == 0 else hi[1],
                       lo[2] if i & 4 == 0 else hi[2]] for i in range(8)])
        quads = [(0, 2, 3, 1), (4, 5, 7, 6), (0, 1, 5, 4), (2, 6, 7, 3), (0, 4, 6, 2), (1, 3, 7, 5)]
        faces = []
        for q in quads:
            faces += [(q[0], q[1], q[2]), (q[0], q[2], q[3])]
        self.add(c, np.array(faces))


def column(m: Mesh, cx: float, cz: float, y0: float, y1: float, r: float, seg=20, rings=6):
    th = np.linspace(0, 2 * math.pi, seg + 1)
    ys = np.linspace(y0 + 0.35, y1 - 0.45, rings + 1)
    # slight entasis
    rr = r * (1.0 - 0.08 * ((ys - ys[0]) / (ys[-1] - ys[0])) ** 1.5)
    P = np.stack([cx + rr[None, :] * np.cos(th)[:, None],
                  np.broadcast_to(ys[None, :], (seg + 1, rings + 1)),
                  cz + rr[None, :] * np.sin(th)[:, None]], -1)
    m.grid(P)
    m.box((cx - 1.35 * r, y0, cz - 1.35 * r), (cx + 1.35 * r, y0 + 0.35, cz + 1.35 * r))        # base
    m.box((cx - 1.5 * r, y1 - 0.45, cz - 1.5 * r), (cx + 1.5 * r, y1 - 0.2, cz + 1.5 * r))      # capital
    m.box((cx - 1.2 * r, y1 - 0.2, cz - 1.2 * r), (cx + 1.2 * r, y1, cz + 1.2 * r))             # abacus


def arch(m: Mesh, xa: float, xb: float, zc: float, y_spring: float, depth: float, seg=16,
         along_x=True, thick=0.35, crown=None):
    """Semicircular arch between two column centres, extruded across `depth`."""
    rc = 0.5 * (xb - xa)
    xc = 0.5 * (xa + xb)
    crown = crown if crown is not None else y_spring + rc + thick + 0.3
    th = np.linspace(math.pi, 0.0, seg + 1)
    ri, ro = rc - 0.05, rc + thick

    def P(u, y, zoff):
        return (np.stack([u, y, np.full_like(u, zc + zoff)], -1) if along_x
                else np.stack([np.full_like(u, zc + zoff), y, u], -1))

    inner_u, inner_y = xc + ri * np.cos(th), y_spring + ri * np.sin(th)
    for zoff in (-0.5 * depth, 0.5 * depth):  # spandrel faces: arch ring up to the crown line
        top_y = np.full_like(inner_y, crown)
        G = np.stack([P(inner_u, inner_y, zoff), P(inner_u, top_y, zoff)], 1)
        m.grid(G)
    # intrados (soffit)
    G = np.stack([P(inner_u, inner_y, -0.5 * depth), P(inner_u, inner_y, 0.5 * depth)], 1)
    m.grid(G)
    _ = ro


def drape(m: Mesh, xa: float, xb: float, z: float, ytop: float, ybot: float, nu: int, nv: int,
          amp: float, phase: float, along_x=True):
    u = np.linspace(0.0, 1.0, nu + 1)
    v = np.linspace(0.0, 1.0, nv + 1)
    U, V = np.meshgrid(u, v, indexing="ij")
    X = xa + (xb - xa) * U
    Y = ytop + (ybot - ytop) * V
    sway = amp * np.sin(2 * math.pi * (3.0 * U + phase)) * (0.3 + 0.7 * V) \
        + 0.15 * amp * np.sin(2 * math.pi * 7.0 * V + phase)
    if along_x:
        P = np.stack([X, Y, z + sway], -1)
    else:
        P = np.stack([z + sway, Y, X], -1)
    m.grid(P)


def build(target=TARGET_TRIS) -> Mesh:
    m = Mesh()
    # foundation slab and tiled floor of the nave and the aisles
    m.box((X0 - 3.0, Y_BASE, Z0 - 3.2), (X1 + 3.0, L1, Z1 + 3.2))
    xs = np.linspace(X0 - 3.0, X1 + 3.0, 73)
    zs = np.linspace(Z0 - 3.2, Z1 + 3.2, 35)
    Xg, Zg = np.meshgrid(xs, zs, indexing="ij")
    m.grid(np.stack([Xg, np.full_like(Xg, L1 + 0.002), Zg], -1))

    ncol = 11
    cxs = np.linspace(X0 + 1.2, X1 - 1.2, ncol)
    for side, zc in ((-1, Z0), (1, Z1)):
        for lvl, (ya, yb, r) in enumerate(((L1, L2, 0.42), (L2, L3, 0.33), (L3, TOP - 0.6, 0.26))):
            for cx in cxs:
                column(m, cx, zc, ya + (0.25 if lvl else 0.0), yb, r)
            for a, b in zip(cxs[:-1], cxs[1:]):
                arch(m, a, b, zc, yb - (b - a) * 0.5 - 0.55, depth=0.9, along_x=True,
                     crown=yb + 0.25)
            # gallery slab (floor of the next level) and its balustrade
            zi, zo = (zc - 0.8, zc + 3.2) if side > 0 else (zc - 3.2, zc + 0.8)
            m.box((X0 - 3.0, yb, zi), (X1 + 3.0, yb + 0.25, zo))
            zr = zc - 0.55 * side
            m.box((X0 + 0.6, yb + 0.25, zr - 0.08), (X1 - 0.6, yb + 1.2, zr + 0.08))
        # outer aisle wall with two rows of windows (tessellated panels)
        zw = zc + 3.2 * side
        for ya, yb in ((L1, L2), (L2, L3), (L3, TOP)):
            ys = np.linspace(ya, yb, 9)
            xw = np.linspace(X0 - 3.0, X1 + 3.0, 61)
            Xw, Yw = np.meshgrid(xw, ys, indexing="ij")
            win = ((np.sin((Xw - X0) / (X1 - X0) * math.pi * 10) > 0.55)
                   & (Yw > ya + 0.3 * (yb - ya)) & (Yw < ya + 0.8 * (yb - ya)))
            Zw = np.where(win, zw + 0.25 * side, zw)
            m.grid(np.stack([Xw, Yw, Zw], -1))
    # end walls with arched openings
    for xe, s in ((X0 - 3.0, 1), (X1 + 3.0, -1)):
        zs2 = np.linspace(Z0 - 3.2, Z1 + 3.2, 41)
        ys2 = np.linspace(L1, TOP, 31)
        Zg2, Yg2 = np.meshgrid(zs2, ys2, indexing="ij")
        hole = (np.abs(Zg2) < 2.4) & (Yg2 < 4.2 + np.sqrt(np.clip(2.4 ** 2 - Zg2 ** 2, 0, None)))
        Xg2 = np.where(hole, xe - 0.6 * s, xe)
        m.grid(np.stack([Xg2, Yg2, Zg2], -1))
        for zc2 in (-4.0, 0.0, 4.0):
            column(m, xe + 1.0 * s, zc2, L1, L2, 0.36)
    # cornice ring at the open roof
    m.box((X0 - 3.0, TOP, Z0 - 3.2), (X1 + 3.0, TOP + 0.4, Z0 + 0.6))
    m.box((X0 - 3.0, TOP, Z1 - 0.6), (X1 + 3.0, TOP + 0.4, Z1 + 3.2))
    # drapes hanging in the first gallery arches (fill the budget exactly)
    rest = target - m.ntris
    pairs = list(zip(cxs[:-1], cxs[1:]))
    slots = [(a, b, zc - 0.1 * np.sign(zc)) for zc in (Z0, Z1) for (a, b) in pairs[1::2]]
    nd = len(slots)
    per = rest // nd
    nu = 24
    nv = max(1, per // (2 * nu))
    for k, (a, b, z) in enumerate(slots):
        drape(m, a + 0.5, b - 0.5, float(z), L3 - 0.7, L2 + 1.4, nu, nv, 0.18, 0.37 * k)
    rest = target - m.ntris
    # remainder: a tessellated banner on the far wall (2*nu*nv) + one triangle if odd
    if rest >= 2:
        q = rest // 2
        nu2 = 1
        for cand in range(min(q, 60), 0, -1):
            if q % cand == 0:
                nu2 = cand
                break
        nv2 = q // nu2
        drape(m, -3.0, 3.0, X1 + 2.2, TOP - 1.0, L2, nu2, nv2, 0.05, 0.0, along_x=False)
        rest = target - m.ntris
    if rest == 1:
        m.add(np.array([[X1 + 2.0, L2, -0.5], [X1 + 2.0, L2, 0.5], [X1 + 2.0, L2 + 1.0, 0.0]]),
              np.array([[0, 1, 2]]))
    assert m.ntris == target, (m.ntris, target)
    return m


def write_obj(m: Mesh, path: str) -> None:
    V = np.concatenate(m.v)
    F = np.concatenate(m.f) + 1
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as fh:
        fh.write("# STAND-IN for sponza.obj (not the Dabrovic model): generated by "
                 "data/gen_standin_sponza.py\n")
        fh.write(f"# {m.ntris} triangles\n")
        fh.write("".join(f"v {x:.5f} {y:.5f} {z:.5f}\n" for x, y, z in V))
        fh.write("".join(f"f {a} {b} {c}\n" for a, b, c in F))


DEFAULT_OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "generated",
                           "standin_sponza.obj")


def ensure(path: str = DEFAULT_OUT) -> str:
    if not os.path.exists(path):
        write_obj(build(), path)
    return path


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_OUT
    write_obj(build(), out)
    print(out)
