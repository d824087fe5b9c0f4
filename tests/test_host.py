"""Host side of the drop-in (no GPU): OBJ ingest, camera placement, PNG writer
and the row-band sharding arithmetic, each against the oracle or an
independent decoder."""
import os

import numpy as np
import pytest
from PIL import Image

import oracle
import toymeshpathtracer_amd as tm
from conftest import data
from toymeshpathtracer_amd import shard


@pytest.mark.parametrize("name", ["triangle.obj", "cube.obj", "suzanne.obj", "teapot.obj"])
def test_load_scene_matches_oracle(name):
    a, amin, amax = tm.load_scene(data(name))
    b, bmin, bmax = oracle.load_scene(data(name))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(amin, bmin) and np.array_equal(amax, bmax)


def test_load_sponza_standin(sponza_path):
    a, amin, amax = tm.load_scene(sponza_path)
    b, _, _ = oracle.load_scene(sponza_path)
    assert a.shape == (66452, 3, 3) and np.array_equal(a.view(np.uint32), b.view(np.uint32))


OBJ_CASES = {
    "quad_fan": "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0.5 1.5 0\nf 1 2 3 4 5\n",
    "negative_idx": "v 0 0 0\nv 1 0 0\nv 0 1 0\nf -3 -2 -1\nv 0 0 1\nf -1 -3 -2\n",
    "slashes": "v 0 0 0\nvt 0 0\nvn 0 0 1\nv 1 0 0\nv 0 1 0\nf 1/1/1 2//1 3/1\nf 1//1 3//1 2//1\n",
    "exponents": "v 1e2 -2.5E-1 +3.0e+0\nv .5 -0. 1e-30\nv 123456789012345678 0 7\nf 1 2 3\n",
    "crlf_no_trailing_newline": "v 0 0 0\r\nv 2 0 0\r\nv 0 2 0\r\nf 1 2 3",
    "comments_groups": "# c\ng grp\nusemtl m\ns 1\nv 0 0 0\nv 1 0 0\nv 0 0 1\no x\nf 1 2 3\n",
    "empty": "",
}


@pytest.mark.parametrize("case", sorted(OBJ_CASES))
def test_obj_edge_cases_match_oracle(tmp_path, case):
    p = tmp_path / f"{case}.obj"
    p.write_bytes(OBJ_CASES[case].encode())
    a, amin, amax = tm.load_scene(str(p))
    b, bmin, bmax = oracle.load_scene(str(p))
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(amin.view(np.uint32), bmin.view(np.uint32))


def test_obj_fan_triangulation_order(tmp_path):
    p = tmp_path / "fan.obj"
    p.write_text(OBJ_CASES["quad_fan"])
    t, _, _ = tm.load_scene(str(p))
    # (v1,v2,v3), (v1,v3,v4), (v1,v4,v5) + 2 floor triangles (objparser.cpp:263-276)
    assert t.shape[0] == 5
    assert np.array_equal(t[1], np.array([[0, 0, 0], [1, 1, 0], [0, 1, 0]], np.float32))


def test_load_missing_file_errors():
    with pytest.raises(tm.TmptError, match="cannot open"):
        tm.load_scene("/nonexistent/file.obj")


@pytest.mark.parametrize("name,w,h,sponza", [("cube.obj", 640, 360, False), ("teapot.obj", 1280, 720, False),
                                             ("suzanne.obj", 37, 1000, False), ("sponza", 1920, 1080, True)])
def test_camera_matches_oracle(sponza_path, name, w, h, sponza):
    path = sponza_path if name == "sponza" else data(name)
    _, bmin, bmax = oracle.load_scene(path)
    a = tm.Camera.for_scene(bmin, bmax, w, h, is_sponza=sponza).as_array()
    b = oracle.camera_for_scene(bmin, bmax, w, h, sponza)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_camera_ctor_matches_oracle():
    args = ([1.5, 2.0, -3.0], [0.1, -0.2, 0.3], [0, 1, 0], 47.0, 1.25, 0.07, 3.3)
    a = tm.Camera.create(*args).as_array()
    b = oracle.camera(*args)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_png_writer_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    p = tmp_path / "x.png"
    tm.write_png(str(p), img)
    back = np.asarray(Image.open(p).convert("RGBA"))
    assert np.array_equal(back, img[::-1])  # flipped on write, main.cpp:341


@pytest.mark.parametrize("h,band,world", [(1080, 16, 1), (1080, 16, 2), (1080, 16, 8), (360, 16, 3),
                                          (7, 16, 4), (2160, 16, 8), (100, 1, 7), (90, 0, 1)])
def test_row_bands_partition_the_frame(h, band, world):
    rows = shard.all_rows(h, band, world)
    allr = np.sort(np.concatenate(rows))
    assert np.array_equal(allr, np.arange(h))
    for s in range(world):
        n = tm.tile_rows(16, h, band, s, world)
        assert n == len(rows[s])
        if n:
            assert np.array_equal(tm.tile_row_to_y(16, h, band, s, world), rows[s])


def test_assemble_numpy():
    h, w = 50, 3
    rows = shard.all_rows(h, 4, 3)
    frame = np.full((h, w, 4), 255, np.uint8)
    tiles = [np.repeat(r[:, None, None], w, 1).repeat(4, 2).astype(np.uint8) for r in rows]
    tiles = [np.concatenate([t, np.zeros((2, w, 4), np.uint8)]) for t in tiles]  # padded
    shard.assemble(tiles, rows, frame)
    assert np.array_equal(frame[:, 0, 0], np.arange(h))


# ---------------------------------------------------------------- parallel host paths
@pytest.fixture
def small_chunks(monkeypatch):
    """Force the parallel OBJ parser and PNG encoder to cut tiny pieces."""
    monkeypatch.setenv("TMPT_OBJ_CHUNK", "7")
    monkeypatch.setenv("TMPT_OBJ_THREADS", "4")
    monkeypatch.setenv("TMPT_PNG_STRIP", "3")
    monkeypatch.setenv("TMPT_PNG_THREADS", "4")


@pytest.mark.parametrize("case", sorted(OBJ_CASES))
def test_parallel_obj_chunks_match_oracle(tmp_path, small_chunks, case):
    """Chunks cut at every few bytes (negative indices resolved across chunk
    boundaries) give exactly the sequential parse."""
    p = tmp_path / f"{case}.obj"
    p.write_bytes((OBJ_CASES[case] * 3).encode())
    a, amin, amax = tm.load_scene(str(p))
    b, bmin, bmax = oracle.load_scene(str(p))
    assert a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(amin.view(np.uint32), bmin.view(np.uint32))


@pytest.mark.parametrize("name", ["suzanne.obj", "teapot.obj"])
def test_parallel_obj_files_match_oracle(small_chunks, monkeypatch, name):
    monkeypatch.setenv("TMPT_OBJ_CHUNK", "4096")
    a, _, _ = tm.load_scene(data(name))
    b, _, _ = oracle.load_scene(data(name))
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("h,w", [(1, 1), (2, 5), (37, 53), (200, 91)])
def test_parallel_png_decodes_exactly(tmp_path, small_chunks, h, w):
    rng = np.random.default_rng(h * 1000 + w)
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    img[h // 2:] = img[h // 2:] // 17 * 17  # compressible half: long matches across strips
    p = tmp_path / "x.png"
    tm.write_png(str(p), img)
    back = np.asarray(Image.open(p).convert("RGBA"))
    assert np.array_equal(back, img[::-1])


def test_parallel_png_same_pixels_as_sequential(tmp_path, monkeypatch):
    img = (np.arange(120 * 77 * 4) % 251).astype(np.uint8).reshape(120, 77, 4)
    monkeypatch.setenv("TMPT_PNG_THREADS", "1")
    tm.write_png(str(tmp_path / "a.png"), img)
    monkeypatch.setenv("TMPT_PNG_THREADS", "8")
    monkeypatch.setenv("TMPT_PNG_STRIP", "5")
    tm.write_png(str(tmp_path / "b.png"), img)
    a = np.asarray(Image.open(tmp_path / "a.png").convert("RGBA"))
    b = np.asarray(Image.open(tmp_path / "b.png").convert("RGBA"))
    assert np.array_equal(a, b) and np.array_equal(a, img[::-1])


def test_unit_sincos_restatement_matches_host_libm_every_key():
    """RandomUnitVector's cosf/sinf (maths.cpp:35-36): the restatement of glibc's
    algorithm the device runs (tmpt_math.h glibc_sincosf_unit), evaluated on the
    host, equals the host libm bit for bit on all 2^24 reachable angles."""
    n = 1 << 24
    mine = tm.unit_sincos(0, n, device=-1)
    ref = oracle.unit_sincos_range(0, n)
    bad = np.nonzero((mine.view(np.uint32) != ref.view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} keys differ, first {bad[:8]}"
