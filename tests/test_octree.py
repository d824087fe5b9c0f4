"""The reference's octree as the library builds it (tmpt_octree.cpp, host
code; no GPU): node for node the oracle's restatement of scene.cpp:99-160 --
the same boxes, the same triangle lists in the same order -- compared through
the preorder digest both sides compute (tmpt_octree_digest / orc_octree_digest)."""
import numpy as np
import pytest

import oracle
import toymeshpathtracer_amd as tm
from conftest import data


def _check(tris, bmin, bmax):
    lo, hi = tm.octree_bounds(bmin, bmax)
    got = tm.octree_digest(tris, lo, hi)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_OCTREE, tie=oracle.TIE_VISIT, bmin=bmin, bmax=bmax)
    nodes, leaves, refs, n = osc.stats()
    assert (got["nodes"], got["leaves"], got["refs"]) == (nodes, leaves, refs)
    assert got["digest"] == osc.octree_digest()
    return got


def test_octree_bounds_main_cpp_312():
    """BuildOctree(sceneMin - extra, sceneMax + extra), extra = size * 0.7f, in float32."""
    bmin = np.array([-1.25, 0.1, 3.0], np.float32)
    bmax = np.array([2.5, 7.75, 3.5], np.float32)
    lo, hi = tm.octree_bounds(bmin, bmax)
    extra = (bmax - bmin) * np.float32(0.7)
    assert np.array_equal(lo, (bmin - extra).astype(np.float32))
    assert np.array_equal(hi, (bmax + extra).astype(np.float32))


@pytest.mark.parametrize("name", ["triangle.obj", "cube.obj", "suzanne.obj", "teapot.obj"])
def test_octree_equals_oracle(name):
    tris, bmin, bmax = tm.load_scene(data(name))
    got = _check(tris, bmin, bmax)
    if name == "teapot.obj":  # SURVEY.md §3 [probe]: 47,681 nodes / 41,721 leaves / 144,583 references
        assert (got["nodes"], got["leaves"], got["refs"], got["depth"]) == (47681, 41721, 144583, 10)


def test_octree_equals_oracle_standin_sponza(sponza_path):
    tris, bmin, bmax = tm.load_scene(sponza_path)
    got = _check(tris, bmin, bmax)
    assert got["depth"] == 10 and got["refs"] > len(tris)


def test_octree_edges():
    """Empty scene and <= 10 triangles: a single leaf (scene.cpp:101); a grid of
    axis-aligned triangles lying exactly on cell planes (the separating-axis
    test's touching cases) and a degenerate (zero-area) triangle."""
    got = tm.octree_digest(np.zeros((0, 9), np.float32), np.zeros(3, np.float32), np.ones(3, np.float32))
    assert (got["nodes"], got["leaves"], got["refs"]) == (1, 1, 0)
    rng = np.random.default_rng(3)
    few = rng.random((10, 3, 3)).astype(np.float32)
    _check(few, few.reshape(-1, 3).min(0), few.reshape(-1, 3).max(0))
    g = []
    for i in range(8):
        for j in range(8):
            x0, z0 = np.float32(i - 4), np.float32(j - 4)
            g.append([[x0, 0, z0], [x0 + 1, 0, z0], [x0, 0, z0 + 1]])
            g.append([[x0, i * 0.25, z0], [x0, i * 0.25, z0 + 1], [x0, i * 0.25 + 1, z0]])
    g.append([[0.5, 0.5, 0.5], [0.5, 0.5, 0.5], [0.5, 0.5, 0.5]])
    grid = np.array(g, np.float32)
    v = grid.reshape(-1, 3)
    got = _check(grid, v.min(0), v.max(0))
    assert got["leaves"] > 8
