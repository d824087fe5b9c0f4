"""GPU parity: the HIP path through the C ABI against the CPU oracle.

Tolerance: none.  BASELINE.json asks for the PNG within 1e-4 per channel of the
reference; on 8-bit channels that is byte equality, so every image comparison
here is exact, and Scene::HitScene results are compared bit for bit.
"""
import hashlib

import os

import numpy as np
import pytest

import oracle
import toymeshpathtracer_amd as tm
from conftest import data

pytestmark = pytest.mark.gpu

# raw-RGBA SHA-256 prefixes (decoded-PNG row order) and ray counts of the
# unmodified reference binary at 640x360x4, row mode: SURVEY.md §8c.
REFERENCE_BINARY = {
    "triangle": ("7aa3820992abf7eb", 1932.5),
    "cube": ("da6b5abfaccbc394", 2419.3),
    "suzanne": ("c9a035a993b4ee32", 2559.7),
    "teapot": ("aa59780a14a04ba5", 2388.5),
}


def _scene(name, device=0, octree=False):
    """octree: build the reference's octree too (main.cpp:312), so the scene
    answers as the reference does (tied closest hits in its visit order, its
    root box test); without it ties go to the lowest index."""
    tris, bmin, bmax = tm.load_scene(data(name))
    return tris, bmin, bmax, tm.Scene(tris, device=device, bounds=(bmin, bmax) if octree else None)


def _ref_oracle(tris, bmin, bmax):
    """The reference's own algorithm: octree, first strict '<' in visit order."""
    return oracle.Scene(tris, accel=oracle.ACCEL_OCTREE, tie=oracle.TIE_VISIT, bmin=bmin, bmax=bmax)


def _png_order_sha(img):
    return hashlib.sha256(np.ascontiguousarray(img[::-1]).tobytes()).hexdigest()[:16]


def _random_rays(tris, n, seed):
    rng = np.random.default_rng(seed)
    v = tris.reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    ext = hi - lo
    o = lo - 0.2 * ext + rng.random((n, 3)) * 1.4 * ext
    # half the rays aim at points on triangles (edges/vertices included), half random
    k = n // 2
    t = rng.integers(0, tris.shape[0], k)
    bary = rng.random((k, 3))
    # snap a third of them onto edges / vertices: grazing and tie cases
    snap = rng.random(k) < 0.33
    bary[snap, rng.integers(0, 3, snap.sum())] = 0.0
    vert = rng.random(k) < 0.1
    bary[vert] = np.eye(3)[rng.integers(0, 3, vert.sum())]
    bary /= bary.sum(1, keepdims=True)
    target = np.einsum("kj,kjc->kc", bary, tris[t])
    d = np.empty((n, 3))
    d[:k] = target - o[:k]
    d[k:] = rng.normal(size=(n - k, 3))
    d = d.astype(np.float32)
    d /= np.sqrt((d.astype(np.float32) ** 2).sum(1, keepdims=True))
    return np.concatenate([o, d], 1).astype(np.float32)


def _same_answers(ids, hits, oids, ohits):
    mism = np.nonzero(ids != oids)[0]
    assert mism.size == 0, f"{mism.size} id mismatches, first {mism[:5]} gpu {ids[mism[:5]]} oracle {oids[mism[:5]]}"
    h = ids >= 0
    assert np.array_equal(hits[h].view(np.uint32), ohits[h].view(np.uint32))


# rays of test_hitscene_kat (seed 7) on which the reference's octree answers
# differently from the exact closest hit (oracle, counted in this container):
# (t ties it breaks in visit order, rays its root box test drops)
KAT_REFERENCE_DEVIATIONS = {"triangle.obj": (0, 296), "cube.obj": (1022, 52), "suzanne.obj": (167, 0),
                            "teapot.obj": (87, 0)}


@pytest.mark.parametrize("name", ["triangle.obj", "cube.obj", "suzanne.obj", "teapot.obj"])
def test_hitscene_kat(gpu, name):
    """Scene::HitScene on 200k rays, a third of the aimed ones snapped onto
    edges and vertices (t ties between triangles sharing them).
    With the reference's octree built (main.cpp:312): the same triangle and
    the same t/pos/normal bits as the reference's own algorithm -- octree,
    first strict '<' in visit order, its root box test (oracle octree) --
    including every tie and root-box miss where that differs from the exact
    closest hit.  With option tie_rule=index: the exact-semantics contract
    (oracle BVH = linear scan with strict '<', lowest index on a tie)."""
    tris, bmin, bmax, sc = _scene(name, octree=True)
    rays = _random_rays(tris, 200_000, seed=7)
    ids, hits = sc.hit_scene_batch(rays, 0.001, 1.0e7)
    st = sc.stats()
    assert (ids >= 0).sum() > 1000
    _same_answers(ids, hits, *_ref_oracle(tris, bmin, bmax).hit_batch(rays, 0.001, 1.0e7))
    ties, roots = KAT_REFERENCE_DEVIATIONS[name]
    # every query the octree decided is counted: ties (>= the ones whose answer
    # changes) and root-box rejections (>= the ones the BVH would have hit)
    assert st.tie_rule == 0 and st.tie_queries >= ties and st.root_misses >= roots
    # any-hit: same hit/miss bit
    aids, _ = sc.hit_scene_batch(rays, 0.001, 1.0e7, any_hit=True)
    assert np.array_equal(aids >= 0, ids >= 0)
    sc.set_option("tie_rule", 1)
    ids, hits = sc.hit_scene_batch(rays, 0.001, 1.0e7)
    assert sc.stats().tie_rule == 1 and sc.stats().tie_queries == 0
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    _same_answers(ids, hits, *osc.hit_batch(rays, 0.001, 1.0e7))
    sc.close()


def test_hitscene_child_order_tie(gpu):
    """The hand-derived visit-order tie (tests/octree_kat.py child_order_case):
    two coplanar triangles at exactly t = 1, met in octree children 0 and 7.
    The reference's walk answers index 1 (child 0 first, scene.cpp:44-49); the
    lowest-index rule answers 0.  Pins the tie order without the oracle."""
    import octree_kat as K
    tris, ray, (lo, hi) = K.child_order_case()
    sc = tm.Scene(tris)
    sc.build_octree(lo, hi)
    assert sc.stats().octree_nodes == 17
    ids, hits = sc.hit_scene_batch(ray, 0.001, 1.0e7)
    assert ids[0] == 1 and hits[0, 6] == 1.0 and sc.stats().tie_queries >= 1
    sc.set_option("tie_rule", 1)
    ids, hits = sc.hit_scene_batch(ray, 0.001, 1.0e7)
    assert ids[0] == 0 and hits[0, 6] == 1.0
    sc.close()


def test_hitscene_per_ray_ranges(gpu):
    """tmpt_scene_hit_ranged: HitScene(ray, tMin, tMax, hit) with the range per
    ray, as scene.h:36-37 takes it (SURVEY §8b rays8 = {o, d, tmin, tmax}).
    Mixed ranges in one batch -- the reference's 0.001..1e7, ranges starting
    at or behind the origin, short, degenerate and empty (tmin > tmax) ones --
    equal the oracle per range: the exact linear scan on suzanne (its BVH
    clamps boxes at t = 0, so it is exact only for tmin >= 0) and the oracle
    BVH on teapot; any-hit agrees on the hit bit."""
    ranges = np.array([(0.001, 1e7), (0.0, 1e7), (-2.0, 1e7), (0.001, 1.5), (0.5, 4.0), (2.0, 2.0001),
                       (3.0, 1.0), (0.001, 0.001), (-1e7, 0.0), (-0.5, 0.25)], np.float32)
    for name, accel, n in (("suzanne.obj", oracle.ACCEL_LINEAR, 60_000), ("teapot.obj", oracle.ACCEL_BVH, 200_000)):
        tris, bmin, bmax, sc = _scene(name)
        rng = np.random.default_rng(21)
        rays = _random_rays(tris, n, seed=23)
        use = np.arange(len(ranges)) if accel == oracle.ACCEL_LINEAR else np.nonzero(ranges[:, 0] >= 0)[0]
        k = use[rng.integers(0, len(use), n)]
        r8 = np.concatenate([rays, ranges[k]], 1).astype(np.float32)
        ids, hits = sc.hit_scene_batch(r8)
        aids, _ = sc.hit_scene_batch(r8, any_hit=True)
        osc = oracle.Scene(tris, accel=accel, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
        for j in use:
            sel = np.nonzero(k == j)[0]
            oids, ohits = osc.hit_batch(rays[sel], float(ranges[j, 0]), float(ranges[j, 1]))
            assert np.array_equal(ids[sel], oids), (name, ranges[j])
            h = oids >= 0
            assert np.array_equal(hits[sel][h].view(np.uint32), ohits[h].view(np.uint32)), (name, ranges[j])
        assert np.array_equal(aids >= 0, ids >= 0)
        assert (ids >= 0).sum() > 1000 and (ids < 0).sum() > 1000
        # the reference's constant range through both entry points: the same answers
        ref = k == 0
        cids, chits = sc.hit_scene_batch(rays[ref], 0.001, 1.0e7)
        assert np.array_equal(cids, ids[ref]) and np.array_equal(chits.view(np.uint32), hits[ref].view(np.uint32))
        sc.close()


@pytest.mark.parametrize("opts", [{"builder": "lbvh"}, {"collapse": "sah"}, {"leaf_max": 4},
                                  {"builder": "lbvh", "leaf_max": 1}, {"ploc_radius": 4, "leaf_max": 16},
                                  {"collapse": "sah", "sah_c_leaf": 0.2, "sah_c_tri": 2.0}, {"layout": "soa"},
                                  {"layout": "soa", "leaf_max": 4}])
def test_build_variants_match_oracle(gpu, opts):
    """Every build option (LBVH builder, SAH collapse and its costs, leaf size,
    PLOC radius, the SoA plane layout) changes the tree or its layout, never the answers: HitScene on 200k
    rays and a sample-seeded frame equal the oracle."""
    tris, bmin, bmax = tm.load_scene(data("teapot.obj"))
    sc = tm.Scene(tris, options=opts)
    rays = _random_rays(tris, 200_000, seed=13)
    ids, hits = sc.hit_scene_batch(rays, 0.001, 1.0e7)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    oids, ohits = osc.hit_batch(rays, 0.001, 1.0e7)
    assert (ids >= 0).sum() > 1000 and np.array_equal(ids, oids)
    h = ids >= 0
    assert np.array_equal(hits[h].view(np.uint32), ohits[h].view(np.uint32))
    aids, _ = sc.hit_scene_batch(rays, 0.001, 1.0e7, any_hit=True)
    assert np.array_equal(aids >= 0, ids >= 0)
    w, hh, spp = 160, 90, 4
    cam = tm.Camera.for_scene(bmin, bmax, w, hh)
    img, nrays = sc.trace_image(cam, w, hh, spp, seed_mode=tm.SEED_SAMPLE)
    ref, ref_rays = osc.render(cam.as_array(), w, hh, spp, seed_mode=oracle.SEED_SAMPLE)
    assert nrays == ref_rays and np.array_equal(img, ref)
    sc.close()


@pytest.mark.parametrize("name", ["cube.obj", "suzanne.obj"])
def test_hitscene_vs_linear_scan(gpu, name):
    """Against the brute-force linear scan (the upstream algorithm)."""
    tris, bmin, bmax, sc = _scene(name)
    rays = _random_rays(tris, 20_000, seed=11)
    ids, hits = sc.hit_scene_batch(rays, 0.001, 1.0e7)
    lin = oracle.Scene(tris, accel=oracle.ACCEL_LINEAR)
    lids, lhits = lin.hit_batch(rays, 0.001, 1.0e7)
    assert np.array_equal(ids, lids)
    h = ids >= 0
    assert np.array_equal(hits[h].view(np.uint32), lhits[h].view(np.uint32))
    sc.close()


def test_hitscene_nan_and_degenerate_rays(gpu):
    """NaN rays (normalize of a zero vector, main.cpp:72) never hit in the
    reference (every Moller-Trumbore comparison is false); rays along a face
    plane, from a vertex, and zero-length directions behave as the oracle."""
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    nan = np.float32("nan")
    c = ((bmin + bmax) / 2).astype(np.float32)
    v = tris[5]
    rays = np.array([
        [*c, nan, nan, nan],
        [*c, nan, 0.0, 1.0],
        [nan, 0.0, 0.0, 0.0, 1.0, 0.0],
        [*v[0], *((v[1] - v[0]) / np.linalg.norm(v[1] - v[0]))],   # along an edge
        [*v[0], 0.0, 1.0, 0.0],                                     # from a vertex
        [*c, 0.0, 0.0, 0.0],                                        # zero direction
        [*(c + 100.0), -0.57735026, -0.57735026, -0.57735026],
    ], np.float32)
    ids, hits = sc.hit_scene_batch(rays, 0.001, 1.0e7)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_LINEAR)
    oids, ohits = osc.hit_batch(rays, 0.001, 1.0e7)
    assert list(ids[:3]) == [-1, -1, -1]
    assert np.array_equal(ids, oids)
    h = ids >= 0
    assert np.array_equal(hits[h].view(np.uint32), ohits[h].view(np.uint32))
    sc.close()


def test_hitscene_reference_contract(gpu):
    """Single-ray form returns 1 / -1 like scene.cpp:86-97."""
    tris, bmin, bmax, sc = _scene("cube.obj")
    c = (bmin + bmax) / 2
    o = np.array([c[0], c[1], c[2] + 10.0], np.float32)
    rid, hit = sc.hit_scene(o, np.array([0, 0, -1], np.float32), 0.001, 1e7)
    assert rid == 1 and hit is not None and abs(hit.t - (10.0 - (bmax[2] - c[2]))) < 1e-4
    rid, hit = sc.hit_scene(o, np.array([0, 0, 1], np.float32), 0.001, 1e7)
    assert rid == -1 and hit is None
    sc.close()


@pytest.mark.parametrize("engine", [tm.ENGINE_MEGAKERNEL, tm.ENGINE_PERSISTENT])
@pytest.mark.parametrize("name", ["triangle", "cube", "suzanne", "teapot"])
def test_row_mode_reproduces_reference_binary(gpu, name, engine):
    """Row mode (main.cpp:204 unmodified) at 640x360x4: the GPU image is the
    reference binary's, byte for byte (SHA-256 recorded in SURVEY.md §8c), and
    the ray count matches.  Megakernel = one lane per row chain; persistent =
    the speculative row engine (render_rowspec)."""
    tris, bmin, bmax, sc = _scene(name + ".obj", octree=True)
    cam = tm.Camera.for_scene(bmin, bmax, 640, 360)
    img, rays = sc.trace_image(cam, 640, 360, 4, seed_mode=tm.SEED_ROW, engine=engine)
    sha, krays = REFERENCE_BINARY[name]
    assert round(rays / 1000.0, 1) == krays
    assert _png_order_sha(img) == sha
    sc.close()


# ---------------------------------------------------------------- speculative row chains
_ITER = {"rowspec_stream": 0}    # the host-driven iterations
_STREAM = {"rowspec_stream": 1}  # the streaming engine


@pytest.mark.parametrize("opts", [{}, {**_STREAM}, {**_STREAM, "rowspec_windows": 1}, {**_STREAM, "rowspec_spread": 0.0},
                                  {**_STREAM, "rowspec_spread": 0.0, "rowspec_windows": 1},
                                  {**_STREAM, "rowspec_windows": 7}, {**_STREAM, "rowstream_dynamic": 0},
                                  {**_ITER}, {**_ITER, "rowspec_wmax": 8}, {**_ITER, "rowspec_wmax": 33},
                                  {**_ITER, "rowspec_windows": 1}, {**_ITER, "rowspec_windows": 1, "rowspec_wmax": 33},
                                  {**_ITER, "rowspec_spread": 0.0}, {**_ITER, "rowspec_spread": 0.0, "rowspec_wmax": 8},
                                  {**_ITER, "rowspec_spread": 0.02, "rowspec_windows": 8},
                                  {**_ITER, "rowspec_windows": 32, "rowspec_groups": 3},
                                  {"rowspec_noshadow": 0}, {"rowspec_noshadow": 0, "rowspec_wmax": 8},
                                  {**_ITER, "rowspec_chase": 0}, {**_ITER, "rowspec_chase": 0, "rowspec_wmax": 33}])
@pytest.mark.parametrize("name,w,h,spp", [("suzanne.obj", 320, 180, 16), ("teapot.obj", 203, 77, 7),
                                          ("cube.obj", 64, 1, 1), ("triangle.obj", 1, 3, 5)])
def test_rowspec_equals_row_chains(gpu, name, w, h, spp, opts):
    """The speculative row engines (every even RNG offset of a window traced,
    then the chain walked through it, into the next pixel's lookahead window
    when its first sample falls there) give the one-lane-per-row megakernel's
    image and ray count exactly.  Iterated engine: windows capped at 8 and 33
    units, or placed with no spread, force many iterations per pixel, chains
    that leave a window mid-pixel and next pixels that start before or after
    the lookahead.  Streaming engine: one window ahead or seven, no spread
    (most pixels then need the chaser's demand or extension windows), windows
    fixed at the launch's load or following the rows still chasing."""
    tris, bmin, bmax, sc = _scene(name)
    for k, v in opts.items():
        sc.set_option(k, v)
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    a, ra = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_MEGAKERNEL)
    b, rb = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
    if opts.get("rowspec_stream") == 1:
        # the streaming engine ran (one launch), not its fallback to iterations
        assert sc.stats().iterations == 1
    assert ra == rb
    diff = np.nonzero((a != b).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"
    sc.close()


def test_rowstream_fallback_wide_rows(gpu):
    """Rows wider than the streaming engine's limit (W > 4094: its 12-bit
    window fields) take the iterated engine instead: the same image and rays
    as the one-lane-per-row chains, and the iterated engine ran (more than one
    iteration)."""
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    w, h, spp = 4100, 3, 2
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    a, ra = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_MEGAKERNEL)
    b, rb = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
    assert sc.stats().iterations > 1 and sc.stats().row_engine == 2 and sc.stats().stream_fallbacks == 0
    assert ra == rb and np.array_equal(a, b)
    sc.close()


def test_rowstream_abort_falls_back_exactly(gpu):
    """The streaming engine's abort path: with its chasers made to
    leave at once (test hook rowstream_test_abort) no chain moves, the
    workers' watchdog aborts the launch, and the frame is rendered again by
    the iterated engine -- whose image and ray count must be the row chains'
    exactly, so nothing the aborted launch left in the shared buffers (chain
    list, colour buffer, counters) leaks into it.  The stats say so; the next
    render, hook off, streams again."""
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    w, h, spp = 320, 180, 8
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    a, ra = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_MEGAKERNEL)
    assert sc.stats().row_engine == 1
    sc.set_option("rowstream_test_abort", 1)
    b, rb = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
    st = sc.stats()
    assert st.stream_fallbacks == 1 and st.row_engine == 2 and st.iterations > 1
    assert rb == ra and np.array_equal(b, a)
    sc.set_option("rowstream_test_abort", 0)
    c, rc = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
    st = sc.stats()
    assert st.stream_fallbacks == 0 and st.row_engine == 3 and st.iterations == 1
    assert rc == ra and np.array_equal(c, a)
    sc.close()


def test_rowspec_shards_and_oracle(gpu):
    """Row seeding over 3 interleaved shards (each row's chain is independent):
    the tiles reassemble to the 1-shard frame, which equals the oracle's row
    loop (main.cpp:202-233) on every 7th row."""
    tris, bmin, bmax, sc = _scene("teapot.obj")
    w, h, spp = 320, 180, 8
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    full, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
    out = np.zeros_like(full)
    total = 0
    for s in range(3):
        tile, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, band_rows=5, shard=s, num_shards=3,
                                 engine=tm.ENGINE_PERSISTENT)
        out[tm.tile_row_to_y(w, h, 5, s, 3)] = tile
        total += r
    assert np.array_equal(out, full) and total == rays
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, _ = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_ROW, row_step=7)
    rows = np.arange(0, h, 7)
    assert np.array_equal(full[rows], ref[rows])
    sc.close()


def test_rowspec_bench_frame_full_spp_vs_oracle(gpu, sponza_path):
    """The bench frame at its full 64 spp in row seeding -- the reference's
    own RNG, each row one chain through 1920 x 64 samples -- with the
    reference's octree built: every 64th row equals the reference algorithm
    (oracle octree, visit-order ties) byte for byte.  A tie answered in
    another order would change one path's draws and with them the rest of its
    row's chain.  The streaming row engine rendered it (no fallback)."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 64
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
        st = sc.stats()
    assert st.row_engine == 3 and st.stream_fallbacks == 0 and st.iterations == 1
    assert st.tie_queries > 0  # ties occurred and took the octree's visit order
    osc = _ref_oracle(tris, bmin, bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_ROW, row_step=64, threads=16)
    rows = np.arange(0, h, 64)
    diff = np.nonzero((img[rows] != ref[rows]).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"


def test_rowspec_bench_frame_rows(gpu, sponza_path):
    """Bench workload (stand-in sponza 1920x1080) in row seeding at 2 spp: the
    speculative engine, with and without shadow-free speculation, equals the
    megakernel's row chains on the whole frame."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 2
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris) as sc:
        a, ra = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_MEGAKERNEL)
        b, rb = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
        sc.set_option("rowspec_noshadow", 0)
        c, rc = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
    assert ra == rb == rc and np.array_equal(a, b) and np.array_equal(a, c)


@pytest.mark.parametrize("engine", [tm.ENGINE_WAVEFRONT, tm.ENGINE_MEGAKERNEL, tm.ENGINE_PERSISTENT])
@pytest.mark.parametrize("name,w,h,spp", [("cube.obj", 640, 360, 4), ("suzanne.obj", 640, 360, 4),
                                          ("teapot.obj", 320, 180, 4)])
def test_pixel_mode_matches_oracle(gpu, engine, name, w, h, spp):
    tris, bmin, bmax, sc = _scene(name)
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=engine)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL)
    assert rays == ref_rays
    diff = np.nonzero((img != ref).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"
    sc.close()


@pytest.mark.parametrize("bins", [2, 8])
def test_wavefront_octant_binned_queues(gpu, bins):
    """Wavefront engine with each segment's extend queue split by direction
    octant (option wf_bins, sort-by-bounce binning): the same pixels and ray
    count as the oracle, on a frame and on a ragged shard."""
    tris, bmin, bmax, sc = _scene("teapot.obj")
    sc.set_option("wf_bins", bins)
    w, h, spp = 320, 180, 4
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_WAVEFRONT)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL)
    assert rays == ref_rays and np.array_equal(img, ref)
    tile, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_WAVEFRONT, band_rows=7,
                             shard=2, num_shards=3)
    assert np.array_equal(tile, ref[tm.tile_row_to_y(w, h, 7, 2, 3)])
    sc.close()


@pytest.mark.parametrize("engine", [tm.ENGINE_WAVEFRONT, tm.ENGINE_PERSISTENT])
def test_shards_assemble_to_full_frame(gpu, engine):
    """Interleaved 16-row bands over 3 shards reassemble to the 1-shard frame."""
    tris, bmin, bmax, sc = _scene("teapot.obj")
    w, h, spp = 320, 180, 2
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    full, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL)
    out = np.zeros_like(full)
    total = 0
    for s in range(3):
        tile, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=16, shard=s,
                                 num_shards=3, engine=engine)
        ys = tm.tile_row_to_y(w, h, 16, s, 3)
        out[ys] = tile
        total += r
    assert np.array_equal(out, full) and total == rays
    sc.close()


def test_sponza_standin_rows_match_oracle(gpu, sponza_path):
    """Bench workload (stand-in sponza, 1920x1080) at 4 spp: every 64th row
    against the oracle, plus determinism of a second run."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 4
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris) as sc:
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL)
        img2, rays2 = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL)
        img3, rays3 = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_PERSISTENT)
    assert rays == rays2 == rays3 and np.array_equal(img, img2) and np.array_equal(img, img3)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, _ = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL, row_step=64)
    rows = np.arange(0, h, 64)
    assert np.array_equal(img[rows], ref[rows])


def test_full_size_teapot_engine_independence(gpu):
    """configs[2] at full size (teapot 1280x720x16) with the reference's
    octree built, as the product's CLI and bench build it (main.cpp:312):
    wavefront == megakernel == persistent byte for byte with the same ray
    count (a size-independent property), every 48th row equal to the
    reference algorithm (oracle octree, visit-order ties) in pixel seeding,
    and the sample-seeded frame's rows too."""
    tris, bmin, bmax, sc = _scene("teapot.obj", octree=True)
    w, h, spp = 1280, 720, 16
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    a, ra = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_WAVEFRONT)
    b, rb = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_MEGAKERNEL)
    c, rc = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_PERSISTENT)
    assert sc.stats().tie_rule == 0
    assert ra == rb == rc and np.array_equal(a, b) and np.array_equal(a, c)
    smp, _ = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
    osc = _ref_oracle(tris, bmin, bmax)
    rows = np.arange(0, h, 48)
    ref, _ = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL, row_step=48)
    diff = np.nonzero((a[rows] != ref[rows]).any(-1))
    assert diff[0].size == 0, f"pixel: {diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"
    ref_s, _ = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE, row_step=48)
    diff = np.nonzero((smp[rows] != ref_s[rows]).any(-1))
    assert diff[0].size == 0, f"sample: {diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"
    sc.close()


def test_pixel_bench_frame_full_spp_octree_vs_oracle(gpu, sponza_path):
    """The bench frame (stand-in sponza 1920x1080) at its full 64 spp in PIXEL
    seeding (bench.py's seed_modes.pixel line: the pilot-ordered persistent
    engine) with the reference's octree built: every 64th row equals the
    reference algorithm (oracle octree, visit-order ties) byte for byte, and
    the octree answered queries (ties met)."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 64
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=1)
        st = sc.stats()
    assert st.tie_rule == 0 and st.tie_queries > 0
    rows = np.arange(0, h, 64)
    ref, _ = _ref_oracle(tris, bmin, bmax).render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL,
                                                  row_step=64)
    diff = np.nonzero((img[rows] != ref[rows]).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"


def test_device_output_pointer(gpu):
    """TMPT_FLAG_OUT_DEVICE: render straight into a torch CUDA tensor."""
    import torch

    tris, bmin, bmax, sc = _scene("cube.obj")
    w, h, spp = 200, 100, 2
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    host, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL)
    dev = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda:0")
    _, rays2 = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, out=dev.data_ptr())
    assert rays2 == rays and np.array_equal(dev.cpu().numpy(), host)
    sc.close()


def test_device_output_ordered_after_caller_stream(gpu):
    """TMPT_FLAG_WAIT_STREAM (bench.py's N>1 step): two cameras rendered back to
    back into ONE device tile while torch's stream still has a delayed reader
    of the first frame queued (a stand-in for the RCCL gather): the reader must
    see the first frame, and the second render must not start before it."""
    import torch

    tris, bmin, bmax, sc = _scene("suzanne.obj")
    w, h, spp = 160, 90, 2
    cam_a = tm.Camera.for_scene(bmin, bmax, w, h)
    cam_b = tm.Camera.create(bmin - (bmax - bmin), (bmin + bmax) / 2, [0, 1, 0], 40.0, w / h, 0.0, 3.0)
    host_a, _ = sc.trace_image(cam_a, w, h, spp, seed_mode=tm.SEED_PIXEL)
    host_b, _ = sc.trace_image(cam_b, w, h, spp, seed_mode=tm.SEED_PIXEL)
    assert not np.array_equal(host_a, host_b)
    tile = torch.full((h, w, 4), 7, dtype=torch.uint8, device="cuda:0")  # the caller's fill, ordered too
    seen = []
    for cam in (cam_a, cam_b):
        sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, out=tile.data_ptr())
        torch.cuda._sleep(50_000_000)  # the reader waits behind 20-500 ms of GPU time
        seen.append(tile.clone())
    torch.cuda.synchronize()
    assert np.array_equal(seen[0].cpu().numpy(), host_a)
    assert np.array_equal(seen[1].cpu().numpy(), host_b)
    sc.close()


def test_count_visits_instrumentation(gpu):
    """TMPT_FLAG_COUNT_VISITS (the roofline's node / triangle counts): both
    query kinds counted, the same image as the plain render; closest-hit
    traversal is the same ordered walk in the wavefront and the persistent
    engine, so their closest-hit work is identical."""
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    cam = tm.Camera.for_scene(bmin, bmax, 160, 90)
    seen = {}
    for engine in (tm.ENGINE_WAVEFRONT, tm.ENGINE_PERSISTENT):
        img, rays = sc.trace_image(cam, 160, 90, 2, seed_mode=tm.SEED_PIXEL, engine=engine, count_visits=True)
        st = sc.stats()
        img2, _ = sc.trace_image(cam, 160, 90, 2, seed_mode=tm.SEED_PIXEL, engine=engine)
        assert st.extend_rays + st.shadow_rays == rays
        assert st.node_visits > st.extend_rays and st.tri_tests > 0 and st.shadow_node_visits > 0
        assert np.array_equal(img, img2)
        seen[engine] = (img, st.extend_rays, st.node_visits, st.tri_tests)
    a, b = seen[tm.ENGINE_WAVEFRONT], seen[tm.ENGINE_PERSISTENT]
    assert np.array_equal(a[0], b[0]) and a[1:] == b[1:]
    sc.close()


# ---------------------------------------------------------------- progressive spp
@pytest.mark.parametrize("seed", [tm.SEED_PIXEL, tm.SEED_SAMPLE])
@pytest.mark.parametrize("name,w,h,spp,passes", [("suzanne.obj", 160, 90, 16, [1, 3, 4, 8]),
                                                 ("teapot.obj", 320, 180, 8, [5, 3]),
                                                 ("teapot.obj", 96, 54, 64, [6, 2, 24, 32])])
def test_progressive_passes_equal_full_render(gpu, name, w, h, spp, passes, seed):
    """Passes of spp_count samples continue each pixel's RNG stream (pixel
    seeding) or start its samples where sample seeding puts them, and carry
    its colour sum: the last pass is the full render bit for bit, every
    preview equals a full render at that sample count, and the passes' rays
    sum to the full count.  Sample seeding: passes starting at odd and even
    samples (block sizes 1, 2, 8), small frames where a pass is one block per
    pixel; the octree built (the reference's answers, deferred ties)."""
    tris, bmin, bmax, sc = _scene(name, octree=seed == tm.SEED_SAMPLE)
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    full, rays = sc.trace_image(cam, w, h, spp, seed_mode=seed)
    total = 0
    for done, img, r in sc.trace_progressive(cam, w, h, spp, passes, seed_mode=seed):
        total += r
        ref, _ = sc.trace_image(cam, w, h, done, seed_mode=seed)
        assert np.array_equal(img, ref), done
    assert np.array_equal(img, full) and total == rays
    if seed == tm.SEED_SAMPLE:
        ref, ref_rays = _ref_oracle(tris, bmin, bmax).render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE)
        assert ref_rays == rays and np.array_equal(full, ref)
    sc.close()


def test_progressive_sample_seeding_shards_and_blocks(gpu, sponza_path):
    """Sample seeding progressive on the bench frame's 1/8 shard (1-row bands,
    the per-rank load at 8 GPUs) at 64 spp in passes of 8, 24, 32 and with
    every block size of the persistent engine forced (option sample_block):
    the last pass equals the one-call shard, which equals those rows of the
    full frame."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 64
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    kw = dict(band_rows=1, shard=3, num_shards=8)
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        one, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, **kw)
        for blk in (0, 1, 4):
            sc.set_option("sample_block", blk)
            total = 0
            for done, img, r in sc.trace_progressive(cam, w, h, spp, [8, 24, 32], seed_mode=tm.SEED_SAMPLE, **kw):
                total += r
            assert total == rays and np.array_equal(img, one), blk
        sc.set_option("sample_block", 0)
        full, _ = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
    assert np.array_equal(one, full[3::8])


def test_progressive_shards_and_errors(gpu):
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    w, h, spp = 160, 90, 6
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    full, _ = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=16, shard=1, num_shards=3)
    full0, _ = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL)
    *_, (done, img, _) = sc.trace_progressive(cam, w, h, spp, 2, band_rows=16, shard=1, num_shards=3)
    assert done == spp and np.array_equal(img, full)
    # a continuation needs the previous pass of the same shard
    with pytest.raises(tm.TmptError, match="continue"):
        sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, spp_begin=2, spp_count=2)
    # ... and of the same camera: another camera's samples must not blend in
    sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, spp_begin=0, spp_count=2)
    other = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with pytest.raises(tm.TmptError, match="same camera"):
        sc.trace_image(other, w, h, spp, seed_mode=tm.SEED_PIXEL, spp_begin=2, spp_count=2)
    img, _ = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, spp_begin=2, spp_count=4)
    assert np.array_equal(img, full0)
    with pytest.raises(tm.TmptError, match="persistent"):
        sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_WAVEFRONT,
                       spp_begin=0, spp_count=2)
    with pytest.raises(tm.TmptError, match="spp_begin"):
        sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, spp_begin=6, spp_count=1)
    sc.close()


def test_progressive_sample_pass_unit_bound(gpu):
    """a sample-seeding pass whose first sample forces small
    blocks can need more than 2^31 sample units (unit ids are 32-bit); it is
    refused with an error, not wrapped.  4096 x 4096 x 258 spp from sample 2:
    blocks of 2, 16.8 M pixels x 128 blocks = 2.15 G units (the colour buffer,
    69 GB, fits the device, so the call reaches the bound)."""
    tris, bmin, bmax, sc = _scene("cube.obj")
    w = h = 4096
    spp = 258
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, spp_begin=0, spp_count=2)
    with pytest.raises(tm.TmptError, match="2\\^31"):
        sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, spp_begin=2, spp_count=spp - 2)
    # a fresh first pass of the same frame still renders
    sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, spp_begin=0, spp_count=2)
    sc.close()


# ---------------------------------------------------------------- edge cases
def _oracle_pixel(tris, cam, w, h, spp):
    osc = oracle.Scene(tris, accel=oracle.ACCEL_LINEAR if len(tris) < 64 else oracle.ACCEL_BVH,
                       tie=oracle.TIE_INDEX)
    return osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL)


@pytest.mark.parametrize("w,h,spp", [(1, 1, 1), (3, 2, 5), (65, 1, 2), (1, 130, 2), (97, 33, 1)])
@pytest.mark.parametrize("engine", [tm.ENGINE_PERSISTENT, tm.ENGINE_WAVEFRONT, tm.ENGINE_MEGAKERNEL])
def test_ragged_image_sizes(gpu, w, h, spp, engine):
    """Images smaller than a wave, a band or a segment, odd sizes, one row or
    one column: same pixels and ray count as the oracle."""
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=engine)
    ref, rrays = _oracle_pixel(tris, cam, w, h, spp)
    assert rays == rrays and np.array_equal(img, ref)
    sc.close()


@pytest.mark.parametrize("ntris", [0, 1, 2])
@pytest.mark.parametrize("engine", [tm.ENGINE_PERSISTENT, tm.ENGINE_WAVEFRONT, tm.ENGINE_MEGAKERNEL])
def test_tiny_scenes(gpu, ntris, engine):
    """Scenes of 0, 1 and 2 triangles (no floor): the BVH degenerates to a
    single leaf or nothing; every query still matches the linear scan."""
    tris, bmin, bmax = tm.load_scene(data("cube.obj"))
    sub = np.ascontiguousarray(tris[:ntris])
    cam = tm.Camera.for_scene(bmin, bmax, 48, 27)
    with tm.Scene(sub) as sc:
        img, rays = sc.trace_image(cam, 48, 27, 3, seed_mode=tm.SEED_PIXEL, engine=engine)
        o = np.tile(cam.as_array()[:3], (64, 1)).astype(np.float32)
        d = np.random.default_rng(ntris).normal(size=(64, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        ids, _ = sc.hit_scene_batch(np.concatenate([o, d], 1), 0.001, 1e7)
    ref, rrays = _oracle_pixel(sub, cam, 48, 27, 3)
    assert rays == rrays and np.array_equal(img, ref)
    if ntris == 0:
        assert (ids == -1).all()


def test_max_spp_and_sample_count_edges(gpu):
    """spp at the reference's maximum (1024, main.cpp:258-280) on a tiny image."""
    tris, bmin, bmax, sc = _scene("cube.obj")
    cam = tm.Camera.for_scene(bmin, bmax, 8, 4)
    img, rays = sc.trace_image(cam, 8, 4, 1024, seed_mode=tm.SEED_PIXEL)
    ref, rrays = _oracle_pixel(tris, cam, 8, 4, 1024)
    assert rays == rrays and np.array_equal(img, ref)
    with pytest.raises(tm.TmptError, match="samplesPerPixel"):
        sc.trace_image(cam, 8, 4, 1025, seed_mode=tm.SEED_PIXEL)
    sc.close()


def test_bench_frame_full_size_shards(gpu, sponza_path):
    """BASELINE configs[3] at full size (1920x1080x64): the 8 row-band shards
    reassemble to the single-GPU frame, ray counts add up, run to run identical
    (size-independent properties of the full workload)."""
    from toymeshpathtracer_amd import shard

    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 64
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris) as sc:
        full, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=16)
        again, rays2 = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=16)
        tiles, total = [], 0
        for k in range(8):
            t, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=16, shard=k, num_shards=8)
            tiles.append(t)
            total += r
    frame = np.zeros_like(full)
    shard.assemble(tiles, shard.all_rows(h, 16, 8), frame)
    assert rays == rays2 == total and np.array_equal(full, again) and np.array_equal(full, frame)


@pytest.mark.parametrize("opts", [{}, {"help": 0}, {"help": 1, "pair": 0},
                                  {"help": 1, "pair": 40, "wave_cap": 48},
                                  {"help": 1, "pilot": 0}, {"pilot": 3, "wave_cap": 17},
                                  {"balance": 0}, {"dprio": 0}])
def test_shadow_offload_matches_oracle(gpu, opts):
    """Low-load shadow offload (k_path HELP: idle lanes trace other lanes' shadow
    queries; pending light slots; paired expensive/cheap chunks).  A small frame
    is far below one pixel per resident lane, so the default already offloads;
    every variant must give the oracle's image and ray count."""
    tris, bmin, bmax, sc = _scene("teapot.obj")
    for k, v in opts.items():
        sc.set_option(k, v)
    w, h, spp = 320, 180, 16
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, engine=tm.ENGINE_PERSISTENT)
    sc.close()
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL)
    assert rays == ref_rays
    diff = np.nonzero((img != ref).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"


def test_shadow_offload_bench_frame_shard(gpu, sponza_path):
    """The bench frame's 1/8 and 1/4 shards (where the offload, the SIMD-balanced
    first chunks and the dynamic priority are on by default) equal the same
    shards rendered with all three forced off, bit for bit."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 64
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris) as sc:
        for n in (8, 4):
            for k, v in (("help", -1), ("balance", 1), ("dprio", 1)):
                sc.set_option(k, v)
            a, ra = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=1, shard=n - 1,
                                   num_shards=n)
            for k in ("help", "balance", "dprio"):
                sc.set_option(k, 0)
            b, rb = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=1, shard=n - 1,
                                   num_shards=n)
            assert ra == rb and np.array_equal(a, b)


# ---------------------------------------------------------------- single-process multi-device
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_render_multi_equals_single_device(gpu, devices):
    """tmpt_render_multi (SURVEY §8e single-process form): rows dealt to one
    scene per listed device, one host thread each, the tiles gathered to the
    first device -- over RCCL (ncclCommInitAll / ncclGather / ncclReduce) when
    the devices are distinct, which [0] is on this box, so the test demands it
    -- and de-interleaved there: the frame == the single-call frame, rays add
    up.  A repeated device (the 1-GPU stand-in for several) takes the
    device-to-device gather, and refuses RCCL when it is demanded."""
    tris, bmin, bmax, sc = _scene("teapot.obj")
    w, h, spp = 320, 200, 4
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    ref, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL)
    unique = len(set(devices)) == len(devices)
    img, mrays, secs = tm.render_multi(tris, cam, w, h, spp, devices, require_rccl=unique)
    assert mrays == rays and np.array_equal(img, ref) and secs > 0
    if not unique:
        with pytest.raises(tm.TmptError, match="distinct devices"):
            tm.render_multi(tris, cam, w, h, spp, devices, require_rccl=True)
    with pytest.raises(tm.TmptError, match="device"):
        tm.render_multi(tris, cam, w, h, spp, [0, 99])
    sc.close()


# ---------------------------------------------------------------- the drop-in CLI
@pytest.mark.parametrize("name", ["cube", "teapot"])
def test_cli_reproduces_reference_binary(gpu, tmp_path, name):
    """`tmpt 640 360 4 <obj>` (the reference's command line, row seeding by
    default) writes the PNG whose pixels hash to the reference binary's
    (SURVEY §8c pins, the same as test_oracle's) and logs its ray count."""
    import subprocess
    from PIL import Image

    cli = os.path.join(os.path.dirname(tm.lib_path), "tmpt")
    out = tmp_path / "o.png"
    r = subprocess.run([cli, "640", "360", "4", data(name + ".obj"), "--out", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    img = np.asarray(Image.open(out).convert("RGBA"))  # top-down as written
    sha = hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()[:16]
    want_sha, want_krays = REFERENCE_BINARY[name]
    assert sha == want_sha
    assert f"- {want_krays:.1f} K Rays" in r.stdout


def test_unit_sincos_device_matches_host_libm_every_key(gpu):
    """The device's cosf/sinf restatement (no libm table) equals the host libm
    on all 2^24 RNG keys of RandomUnitVector (maths.cpp:33-36)."""
    n = 1 << 24
    dev = tm.unit_sincos(0, n, device=0)
    ref = oracle.unit_sincos_range(0, n)
    bad = np.nonzero((dev.view(np.uint32) != ref.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} keys differ, first {bad[:8]}"


# ---------------------------------------------------------------- sample seeding
@pytest.mark.parametrize("engine", [tm.ENGINE_PERSISTENT, tm.ENGINE_WAVEFRONT, tm.ENGINE_MEGAKERNEL])
@pytest.mark.parametrize("name,w,h,spp", [("cube.obj", 320, 180, 4), ("suzanne.obj", 320, 180, 6),
                                          ("teapot.obj", 160, 90, 5)])
def test_sample_mode_matches_oracle(gpu, engine, name, w, h, spp):
    """TMPT_SEED_SAMPLE (sample s of a pixel starts 2^16*s steps into its
    stream): byte-identical to the oracle's sample-seeded loop with every
    block size of the persistent engine -- 1 sample per unit (per-sample
    colours + in-order resolve), 2 and 4, and the whole pixel per unit."""
    tris, bmin, bmax, sc = _scene(name)
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE)
    for blk in ([1, 2, 4, 1024] if engine == tm.ENGINE_PERSISTENT else [None]):
        if blk is not None:
            sc.set_option("sample_block", blk)
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, engine=engine)
        assert rays == ref_rays, blk
        diff = np.nonzero((img != ref).any(-1))
        assert diff[0].size == 0, f"block {blk}: {diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"
    sc.close()


@pytest.mark.parametrize("octree", [False, True])
def test_sample_mode_tail_units(gpu, octree):
    """Sample seeding's tail (option sample_tail): the last blocks are handed
    out as single-sample units.  With blocks of 2 and one tail block per
    resident lane the frame mixes both kinds of unit; it equals the oracle
    and the render without a tail (every block a unit), with the octree's
    deferred ties too; the whole frame as single units as well."""
    tris, bmin, bmax, sc = _scene("teapot.obj", octree=octree)
    w, h, spp = 320, 180, 16
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    osc = _ref_oracle(tris, bmin, bmax) if octree else \
        oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE)
    sc.set_option("sample_block", 2)
    if octree:
        sc.set_option("tie_defer", 1)
    for tail in (0, 1, 64):  # none; 262 k of 460,800 blocks (mixed); every block
        sc.set_option("sample_tail", tail)
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE)
        assert rays == ref_rays, tail
        diff = np.nonzero((img != ref).any(-1))
        assert diff[0].size == 0, f"tail {tail}: {diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"
    sc.close()


def test_sample_mode_shards_and_sizes(gpu, monkeypatch):
    """Sample seeding: 1-row bands over 3 and 8 shards reassemble to the
    1-shard frame with the same ray count (auto block size differs per
    shard load: a property, not an oracle run), ragged sizes match the
    oracle, and spp = 1 equals pixel mode."""
    tris, bmin, bmax, sc = _scene("teapot.obj")
    w, h, spp = 320, 180, 8
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    full, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE)
    for n in (3, 8):
        out = np.zeros_like(full)
        total = 0
        for k in range(n):
            tile, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1, shard=k, num_shards=n)
            out[tm.tile_row_to_y(w, h, 1, k, n)] = tile
            total += r
        assert np.array_equal(out, full) and total == rays, n
    a, ra = sc.trace_image(cam, w, h, 1, seed_mode=tm.SEED_SAMPLE)
    b, rb = sc.trace_image(cam, w, h, 1, seed_mode=tm.SEED_PIXEL)
    assert ra == rb and np.array_equal(a, b)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    for (ww, hh, ss) in ((1, 1, 3), (65, 3, 7), (97, 33, 2)):
        c2 = tm.Camera.for_scene(bmin, bmax, ww, hh)
        img, r = sc.trace_image(c2, ww, hh, ss, seed_mode=tm.SEED_SAMPLE)
        ref, rr = osc.render(c2.as_array(), ww, hh, ss, seed_mode=oracle.SEED_SAMPLE)
        assert r == rr and np.array_equal(img, ref), (ww, hh, ss)
    with pytest.raises(tm.TmptError, match="progressive"):
        sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_ROW, spp_begin=0, spp_count=2)
    sc.close()


def test_sample_mode_bench_frame(gpu, sponza_path):
    """The bench frame (stand-in sponza 1920x1080x64) in sample seeding: the
    1/8 shard (the per-rank load at 8 GPUs) equals the same rows of the
    single-GPU frame, ray counts add up, a row sample at 4 spp matches the
    oracle, and a second render is identical (determinism)."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h = 1920, 1080
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris) as sc:
        full, rays = sc.trace_image(cam, w, h, 64, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        tile, r0 = sc.trace_image(cam, w, h, 64, seed_mode=tm.SEED_SAMPLE, band_rows=1, shard=0, num_shards=8)
        assert np.array_equal(tile, full[0::8])
        rest = sum(sc.trace_image(cam, w, h, 64, seed_mode=tm.SEED_SAMPLE, band_rows=1, shard=k,
                                  num_shards=8)[1] for k in range(1, 8))
        assert r0 + rest == rays
        small, _ = sc.trace_image(cam, w, h, 4, seed_mode=tm.SEED_SAMPLE)
        small2, _ = sc.trace_image(cam, w, h, 4, seed_mode=tm.SEED_SAMPLE)
    assert np.array_equal(small, small2)
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, _ = osc.render(cam.as_array(), w, h, 4, seed_mode=oracle.SEED_SAMPLE, row_step=64)
    rows = np.arange(0, h, 64)
    assert np.array_equal(small[rows], ref[rows])


def test_sample_mode_bench_frame_full_spp_vs_oracle(gpu, sponza_path):
    """The headline workload itself -- the bench frame (stand-in sponza
    1920x1080) at its full 64 spp in sample seeding, rendered exactly as
    bench.py renders it (1-row bands, the auto block size) -- against the
    oracle's sample-seeded image loop (main.cpp:202-233) on every 64th row,
    byte for byte, with the reference's octree built: the reference's own
    HitScene answers (ties in its visit order), as the oracle octree gives
    them.  With tie_rule=index the same rows equal the exact-semantics oracle
    (lowest index on a tie)."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 1920, 1080, 64
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        st = sc.stats()
        assert st.tie_queries > 0 and st.redo_samples > 0  # ties left to the redo pass (tie_defer auto)
        sc.set_option("tie_rule", 1)
        img_ix, rays_ix = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
    rows = np.arange(0, h, 64)
    osc_ix = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref_ix, _ = osc_ix.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE, row_step=64)
    assert np.array_equal(img_ix[rows], ref_ix[rows])
    osc = _ref_oracle(tris, bmin, bmax)
    ref, _ = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE, row_step=64)
    rows = np.arange(0, h, 64)
    diff = np.nonzero((img[rows] != ref[rows]).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"


@pytest.mark.parametrize("seed", ["sample", "pixel"])
def test_path_waves_same_frame_and_rays(gpu, sponza_path, seed):
    """The 5-wave path kernels (option path_waves 5: a 12-entry LDS stack,
    the pending ray's direction only, 80 LDS top nodes) render the same
    frame and ray count as the 4-wave ones (path_waves 4), in sample seeding
    (deferred ties, whole frame and a 1/8 shard) and pixel seeding (cost-
    ordered passes, with and without the shadow offload), and the tie_path
    stat says which answer path ran."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 480, 270, 16
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    sd = tm.SEED_SAMPLE if seed == "sample" else tm.SEED_PIXEL
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        for shards in (1, 8):
            kw = dict(seed_mode=sd, band_rows=1, shard=0, num_shards=shards)
            out = {}
            for waves in (4, 5):
                sc.set_option("path_waves", waves)
                if seed == "sample":
                    sc.set_option("tie_defer", 1)
                    img, rays = sc.trace_image(cam, w, h, spp, **kw)
                    st = sc.stats()
                    assert st.tie_path == 2 and st.redo_samples > 0 and st.redo_late == 0
                    out[waves] = (img, rays)
                else:
                    for help_ in (0, 1):
                        sc.set_option("help", help_)
                        img, rays = sc.trace_image(cam, w, h, spp, **kw)
                        assert sc.stats().tie_path == 1
                        out[(waves, help_)] = (img, rays)
                    sc.set_option("help", -1)
            first = next(iter(out.values()))
            for k, (img, rays) in out.items():
                assert rays == first[1] and np.array_equal(img, first[0]), (shards, k)
        sc.set_option("path_waves", 0)
        sc.set_option("tie_defer", -1)


@pytest.mark.parametrize("shards", [1, 8])
def test_tie_defer_same_frame_and_rays(gpu, sponza_path, shards):
    """Deferred ties (option tie_defer): the sample kernel's main loop, built
    without the octree walk, drops each sample whose closest hit is a tie; the
    launch's waves trace those samples again, ties settled, once their main
    loop is done.  The frame and its ray count equal the render that settles
    ties in the main loop (tie_defer=0), for the whole frame and a 1/8 shard;
    a redo list too small for the frame (test hook redo_cap=1) overflows, and
    the frame is rendered again with the list grown; with the tail's redo
    phase off (test hook redo_inline=0) the k_redo launch traces them all --
    same frame, same rays each time.  Rows every 16th
    against the oracle octree close the loop to the reference's answers."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 480, 270, 16
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    kw = dict(seed_mode=tm.SEED_SAMPLE, band_rows=1, shard=0, num_shards=shards)
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        sc.set_option("tie_defer", 0)
        exact, rays_exact = sc.trace_image(cam, w, h, spp, **kw)
        st0 = sc.stats()
        assert st0.redo_samples == 0 and st0.tie_queries > 0
        sc.set_option("tie_defer", 1)
        img, rays = sc.trace_image(cam, w, h, spp, **kw)
        st1 = sc.stats()
        assert st1.redo_samples > 0
        assert st1.tie_queries == st0.tie_queries  # the redo pass meets the same ties
        # the list entries are written through to memory (sc1): every listed
        # sample is visible to the waiting lanes at once, so none is left late
        assert st1.redo_late == 0 and st1.redo_launches == 0
        assert rays == rays_exact and np.array_equal(img, exact)
        sc.set_option("redo_cap", 1)
        img2, rays2 = sc.trace_image(cam, w, h, spp, **kw)
        assert sc.stats().redo_samples == st1.redo_samples
        assert rays2 == rays_exact and np.array_equal(img2, exact)
        sc.set_option("redo_cap", 0)
        sc.set_option("redo_inline", 0)  # every dropped sample to the k_redo launch
        img3, rays3 = sc.trace_image(cam, w, h, spp, **kw)
        st3 = sc.stats()
        assert st3.redo_samples == st1.redo_samples
        assert st3.redo_launches == 1 and st3.redo_late == st1.redo_samples and st3.redo_rays > 0
        assert rays3 == rays_exact and np.array_equal(img3, exact)
    if shards == 1:
        ref, _ = _ref_oracle(tris, bmin, bmax).render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE,
                                                      row_step=16)
        rows = np.arange(0, h, 16)
        assert np.array_equal(img[rows], ref[rows])


def test_sponza4k_config4_shard_oracle_and_fallback(gpu, sponza_path):
    """BASELINE configs[4] -- stand-in sponza 3840x2160 at 256 spp, the 8-GPU
    configuration -- in sample seeding (bench.py --config sponza4k):
    (a) shard k of 8 (1-row bands: rank k's load at 8 GPUs, main.cpp:329-331
        dealt round-robin) equals those rows of the single-GPU frame, and the
        8 shards' rays add up to the frame's;
    (b) 3 rows of the full frame equal the oracle's row loop at 256 spp
        (main.cpp:202-233) over the reference's octree (visit-order ties),
        byte for byte -- the octree is built, as bench.py --config sponza4k
        builds it;
    (c) the same frame with the per-sample colour buffer capped (option
        sbuf_max: the path a frame too large for HBM takes -- here the buffer
        is 34 GB) renders whole pixels as units: the same bytes, same rays."""
    tris, bmin, bmax = tm.load_scene(sponza_path)
    w, h, spp = 3840, 2160, 256
    cam = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=True)
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:  # the reference's octree, as bench.py builds it
        full, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        assert sc.stats().tie_rule == 0 and sc.stats().tie_queries > 0
        total = 0
        for k in range(8):
            tile, r = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1, shard=k, num_shards=8)
            assert np.array_equal(tile, full[k::8]), k
            total += r
        assert total == rays
        sc.set_option("sbuf_max", 1 << 20)
        capped, rays_c = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE, band_rows=1)
        assert rays_c == rays and np.array_equal(capped, full)
    osc = _ref_oracle(tris, bmin, bmax)
    rows = np.array([5, 1080, 2150])
    ref = np.zeros((h, w, 4), np.uint8)
    for y in rows:
        osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE, y0=int(y), y1=int(y) + 1, rgba=ref)
    diff = np.nonzero((full[rows] != ref[rows]).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"


def test_cli_and_render_multi_sample_seeding(gpu, tmp_path):
    """`tmpt ... --seed sample` writes the sample-seeded oracle's image, and
    tmpt_render_multi (device repeated: two scenes, rows dealt round-robin,
    one host thread each) assembles the same frame."""
    import subprocess
    from PIL import Image

    cli = os.path.join(os.path.dirname(tm.lib_path), "tmpt")
    out = tmp_path / "s.png"
    w, h, spp = 200, 120, 3
    r = subprocess.run([cli, str(w), str(h), str(spp), data("suzanne.obj"), "--seed", "sample", "--out", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    img = np.asarray(Image.open(out).convert("RGBA"))[::-1]  # back to row 0 = bottom
    tris, bmin, bmax = tm.load_scene(data("suzanne.obj"))
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    osc = _ref_oracle(tris, bmin, bmax)  # the CLI builds the reference's octree (main.cpp:312)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE)
    assert np.array_equal(img, ref)
    multi, rays, _ = tm.render_multi(tris, cam, w, h, spp, [0, 0], seed_mode=tm.SEED_SAMPLE, bounds=(bmin, bmax))
    assert rays == ref_rays and np.array_equal(multi, ref)


def test_sample_mode_without_colour_buffer(gpu):
    """When the per-sample colour buffer would not fit (option sbuf_max stands
    in for a frame too large for HBM), sample seeding runs whole pixels as
    units: the same image and ray count."""
    tris, bmin, bmax, sc = _scene("teapot.obj")
    w, h, spp = 160, 90, 6
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    sc.set_option("sample_block", 1)
    a, ra = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE)
    sc2 = tm.Scene(tris, options={"sample_block": 1, "sbuf_max": 1024})  # no buffer held yet
    b, rb = sc2.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE)
    assert ra == rb and np.array_equal(a, b)
    sc.close()
    sc2.close()


# ---------------------------------------------------------------- the reference's tie order
@pytest.mark.parametrize("engine", [tm.ENGINE_PERSISTENT, tm.ENGINE_WAVEFRONT, tm.ENGINE_MEGAKERNEL])
@pytest.mark.parametrize("seed,oseed", [(tm.SEED_PIXEL, oracle.SEED_PIXEL), (tm.SEED_SAMPLE, oracle.SEED_SAMPLE)])
def test_octree_rule_every_engine(gpu, engine, seed, oseed):
    """With the reference's octree built every engine answers closest hits as
    the reference does (ties re-answered over the octree where they are met:
    k_path's shading round, k_wf_trace, the megakernel's query; camera rays
    from a lens that reaches outside the root box take its root test -- the
    cube's camera sits on the root's face, main.cpp:297 vs :312): the frame
    equals the oracle octree's (visit-order ties) byte for byte."""
    tris, bmin, bmax, sc = _scene("cube.obj", octree=True)
    w, h, spp = 320, 180, 4
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    img, rays = sc.trace_image(cam, w, h, spp, seed_mode=seed, engine=engine)
    ref, ref_rays = _ref_oracle(tris, bmin, bmax).render(cam.as_array(), w, h, spp, seed_mode=oseed)
    assert rays == ref_rays and np.array_equal(img, ref)
    sc.close()


@pytest.mark.parametrize("seed,oseed", [(tm.SEED_PIXEL, oracle.SEED_PIXEL), (tm.SEED_SAMPLE, oracle.SEED_SAMPLE)])
def test_octree_many_way_ties(gpu, seed, oseed):
    """Every hit a many-way tie: suzanne's triangles 12 times over (the floor
    once), so each closest hit on the mesh is tied between >= 12 identical
    triangles, the octree (10 M references) bottoms out at depth 10 with
    leaves of dozens of references, and every tied query walks it (k_path's
    wave walk, 64 nodes / triangles per round trip; the batched HitScene's
    serial walk).  The frame and the batched answers equal the oracle's
    octree in its visit order (scene.cpp:21-52: the first copy met wins)."""
    tris, bmin, bmax = tm.load_scene(data("suzanne.obj"))
    reps = (12,) + (1,) * (tris.ndim - 1)
    many = np.ascontiguousarray(np.concatenate([np.tile(tris[:-2], reps), tris[-2:]]))
    w, h, spp = 96, 64, 2
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    osc = _ref_oracle(many, bmin, bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oseed)
    with tm.Scene(many, bounds=(bmin, bmax)) as sc:
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=seed)
        assert sc.stats().tie_queries > 0
        rays_in = _random_rays(many, 4000, seed=11)
        ids, hits = sc.hit_scene_batch(rays_in, 0.001, 1.0e7)
    assert rays == ref_rays and np.array_equal(img, ref)
    _same_answers(ids, hits, *osc.hit_batch(rays_in, 0.001, 1.0e7))


def test_octree_render_multi_and_rebuild(gpu):
    """tmpt_render_multi with the octree box builds it on every device's scene
    (the frame equals the oracle octree's); building the octree again on a
    scene (another box) replaces the first one."""
    tris, bmin, bmax = tm.load_scene(data("teapot.obj"))
    w, h, spp = 200, 120, 2
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    ref, ref_rays = _ref_oracle(tris, bmin, bmax).render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_SAMPLE)
    img, rays, _ = tm.render_multi(tris, cam, w, h, spp, [0], seed_mode=tm.SEED_SAMPLE, bounds=(bmin, bmax),
                                   require_rccl=True)
    assert rays == ref_rays and np.array_equal(img, ref)
    with tm.Scene(tris) as sc:
        assert sc.stats().octree_nodes == 0 and sc.stats().tie_rule == 1
        sc.build_octree(np.array([-50, -50, -50], np.float32), np.array([50, 50, 50], np.float32))
        sc.build_octree(*tm.octree_bounds(bmin, bmax))
        st = sc.stats()
        want = tm.octree_digest(tris, *tm.octree_bounds(bmin, bmax))
        assert st.octree_nodes == want["nodes"] and st.octree_refs == want["refs"] and st.tie_rule == 0
        img2, rays2 = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_SAMPLE)
    assert rays2 == ref_rays and np.array_equal(img2, ref)


@pytest.mark.parametrize("per1024", [0, 16, 200, 1024])
def test_pixel_chains_match_oracle(gpu, per1024):
    """Pixel seeding with the heaviest pixels run as speculative chains
    (option pixel_chains: that many per 1024 of the cost order, up to all of
    them): every even RNG offset past a pixel's pilot state traced
    shadow-free, the chain walked through them, its samples traced again in
    full and summed after the pilot's sum -- the frame and the ray count equal
    the pixel-seeded oracle's, whole and as shard 1 of 3."""
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    w, h, spp = 320, 180, 8
    cam = tm.Camera.for_scene(bmin, bmax, w, h)
    sc.set_option("pixel_chains", per1024)
    img, rays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL)
    n = sc.stats().chain_pixels
    assert n == (0 if per1024 == 0 else min(w * h, (w * h * per1024 + 1023) // 1024))
    osc = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax)
    ref, ref_rays = osc.render(cam.as_array(), w, h, spp, seed_mode=oracle.SEED_PIXEL)
    assert rays == ref_rays and np.array_equal(img, ref)
    tile, trays = sc.trace_image(cam, w, h, spp, seed_mode=tm.SEED_PIXEL, band_rows=1, shard=1, num_shards=3)
    assert np.array_equal(tile, ref[1::3])
    sc.close()


# ---------------------------------------------------------------- the octree's cracks
@pytest.mark.parametrize("name", ["cube", "suzanne", "teapot", "grid", "crack_wall"])
def test_hitscene_adversarial_octree(gpu, name):
    """HitScene on rays aimed at the reference octree's faces, edges and
    corners, at triangles crossing them, along them (axis-parallel and
    in-plane rays: the crack class) and at vertices (tests/octree_kat.py);
    'grid' puts its geometry on the octree's planes, 'crack_wall' adds a wall
    lying inside one of teapot's cracks (in no leaf: the reference sees
    through it).  The GPU's answers equal the reference algorithm's (oracle
    octree) on every ray -- ties, root-box misses and crack queries included --
    and the any-hit query's hit bit equals it.  Reports the deviation counts."""
    import octree_kat as K
    if name == "grid":
        tris, bmin, bmax = K.grid_scene()
    else:
        tris, bmin, bmax = oracle.load_scene(data(("teapot" if name == "crack_wall" else name) + ".obj"))
    extra = None
    if name == "crack_wall":
        tris, ax, _ = K.crack_wall_scene(tris, bmin, bmax)
        extra = K.crack_wall_rays(tris[-1], ax, 4000, seed=3)
    osc = K.ref_scene(tris, bmin, bmax)
    rays, kind = K.adversarial_rays(tris, bmin, bmax, 8000, seed=9, osc=osc)
    if extra is not None:
        rays = np.concatenate([rays, extra])
    c = K.classify(tris, bmin, bmax, rays, osc=osc)
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        ids, hits = sc.hit_scene_batch(rays, 0.001, 1.0e7)
        st = sc.stats()
        aids, _ = sc.hit_scene_batch(rays, 0.001, 1.0e7, any_hit=True)
    print(name, "rays", len(rays), "ties", len(c["tie"]), "root", len(c["root"]), "crack class", len(c["other"]),
          "gpu tie_queries", st.tie_queries, "crack_queries", st.crack_queries, "flat", st.octree_flat)
    _same_answers(ids, hits, c["rid"], c["rh"])
    assert np.array_equal(aids >= 0, c["rid"] >= 0)
    if name in ("teapot", "crack_wall"):
        assert len(c["other"]) > 0 and st.crack_queries + st.tie_queries >= len(c["other"])
    if name == "crack_wall":
        assert st.octree_flat == 1


@pytest.mark.parametrize("engine", [tm.ENGINE_PERSISTENT, tm.ENGINE_WAVEFRONT, tm.ENGINE_MEGAKERNEL])
@pytest.mark.parametrize("seed,oseed", [(tm.SEED_PIXEL, oracle.SEED_PIXEL), (tm.SEED_SAMPLE, oracle.SEED_SAMPLE),
                                        (tm.SEED_ROW, oracle.SEED_ROW)])
def test_crack_wall_render(gpu, engine, seed, oseed):
    """A frame looking at a wall that lies inside a crack of teapot's octree
    (in no leaf, so the reference's camera and shadow rays pass through it):
    every engine and seeding gives the reference algorithm's frame (oracle
    octree) byte for byte -- the wall's hits are flagged (a flat triangle) and
    answered over the octree, shadow queries included (PathCtl::oct_shadow)."""
    import octree_kat as K
    tris, bmin, bmax = oracle.load_scene(data("teapot.obj"))
    tris, ax, p = K.crack_wall_scene(tris, bmin, bmax)
    frm = p.astype(np.float64).copy()
    frm[ax] -= 3.0
    frm[(ax + 1) % 3] += 0.7
    w, h, spp = 96, 64, 3
    cam = tm.Camera.create(frm.astype(np.float32), p, [0, 1, 0] if ax != 1 else [1, 0, 0], 20.0, w / h, 0.0, 3.0)
    ref, ref_rays = _ref_oracle(tris, bmin, bmax).render(cam.as_array(), w, h, spp, seed_mode=oseed)
    exact, _ = oracle.Scene(tris, accel=oracle.ACCEL_BVH, tie=oracle.TIE_INDEX, bmin=bmin, bmax=bmax).render(
        cam.as_array(), w, h, spp, seed_mode=oseed)
    assert not np.array_equal(ref, exact)  # the wall is in view: the reference sees through it
    with tm.Scene(tris, bounds=(bmin, bmax)) as sc:
        img, rays = sc.trace_image(cam, w, h, spp, seed_mode=seed, engine=engine)
        st = sc.stats()
    assert st.octree_flat == 1
    assert rays == ref_rays
    diff = np.nonzero((img != ref).any(-1))
    assert diff[0].size == 0, f"{diff[0].size} pixels differ, first at {list(zip(*diff))[:5]}"


def test_hitscene_negative_single_range(gpu):
    """one range for the batch that starts behind the origin
    (t_min = -1e7): the traversal's far-distance slack by magnitude (NEG), so
    no box behind the origin is culled -- the same answers as the oracle's
    linear scan."""
    tris, bmin, bmax, sc = _scene("suzanne.obj")
    rays = _random_rays(tris, 40_000, seed=31)
    for lo, hi in ((-1.0e7, 1.0e7), (-3.0, 0.5)):
        ids, hits = sc.hit_scene_batch(rays, lo, hi)
        oids, ohits = oracle.Scene(tris, accel=oracle.ACCEL_LINEAR).hit_batch(rays, lo, hi)
        assert (ids >= 0).sum() > 1000 and np.array_equal(ids, oids), (lo, hi)
        h = ids >= 0
        assert np.array_equal(hits[h].view(np.uint32), ohits[h].view(np.uint32))
    sc.close()
