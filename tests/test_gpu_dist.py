"""bench.py's N>1 path end to end on the one GPU of the box: two ranks under
torch.distributed.run share cuda:0 with the gloo backend (the driver's 8-GPU
run uses nccl = RCCL; the band partition, device tiles, gather, assembly and
max-over-ranks timing are the same code).  Rank 0's frame must equal the
single-process frame byte for byte."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(args, env_extra=None, timeout=600):
    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    # the contract: stdout is exactly one JSON line (RCCL's init banner is
    # routed to stderr by bench.py)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_ranks_gloo_matches_single(gpu, tmp_path, ranks):
    one = tmp_path / "one.png"
    two = tmp_path / "two.png"
    common = ["--config", "teapot720", "--steps", "1", "--warmup", "0", "--no-cpu"]
    r1 = _bench(["bench.py", "--gpus", "1", "--save", str(one)] + common)
    port = _free_port()
    r2 = _bench(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ranks),
                 "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(ranks),
                 "--dist-backend", "gloo", "--save", str(two)] + common)
    # ranks sharing the box's one GPU: a rehearsal, one distinct device
    assert r2["n_gpus"] == 1 and r2["ranks"] == ranks and r2["rehearsal"] is True and r2["scaling"] == "strong"
    assert r2["dist_backend"] == "gloo" and len(r2["devices"]) == ranks and len(set(r2["devices"])) == 1
    assert r1["n_gpus"] == 1 and r1["ranks"] == 1 and r1["rehearsal"] is False and r1["dist_backend"] is None
    assert r2["config"]["rays_per_step"] == r1["config"]["rays_per_step"]
    a = np.asarray(Image.open(one).convert("RGBA"))
    b = np.asarray(Image.open(two).convert("RGBA"))
    assert np.array_equal(a, b)


def test_bench_rccl_path_one_rank(gpu, tmp_path):
    """The nccl (= RCCL) calls of bench.py's N>1 step -- process group on the
    device, gather of the device tile, device-side max/sum reductions,
    barriers -- run on the box's one GPU with --force-dist at world size 1
    (RCCL refuses two ranks on one device); the frame must equal the plain
    single-process frame."""
    one = tmp_path / "one.png"
    rccl = tmp_path / "rccl.png"
    common = ["--config", "teapot720", "--steps", "2", "--warmup", "1", "--no-cpu", "--no-compare"]
    r1 = _bench(["bench.py", "--gpus", "1", "--save", str(one)] + common)
    port = _free_port()
    r2 = _bench(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
                 "--master-port", str(port), "bench.py", "--gpus", "1", "--force-dist", "--save", str(rccl)] + common)
    assert r2["n_gpus"] == 1 and r2["config"]["rays_per_step"] == r1["config"]["rays_per_step"]
    # the RCCL line names its backend and the one device's PCI address
    assert r2["dist_backend"] == "nccl" and r2["ranks"] == 1 and r2["rehearsal"] is False
    assert len(r2["devices"]) == 1 and r2["devices"] == r1["devices"] and ":" in r2["devices"][0]
    a = np.asarray(Image.open(one).convert("RGBA"))
    b = np.asarray(Image.open(rccl).convert("RGBA"))
    assert np.array_equal(a, b)


def test_bench_gpus_n_launches_its_own_ranks(gpu, tmp_path):
    """`python bench.py --gpus 2` with no launcher around it starts its two
    ranks itself (torch.distributed.run as a child, before any GPU call): with
    the gloo rehearsal both share the box's GPU and the line says ranks 2 on
    n_gpus 1 (one distinct device, rehearsal true);
    with nccl (one rank per GPU) on a box with fewer GPUs it exits non-zero
    and says why, instead of measuring one GPU."""
    import toymeshpathtracer_amd as tm
    two = tmp_path / "two.png"
    one = tmp_path / "one.png"
    common = ["--config", "teapot720", "--steps", "1", "--warmup", "0", "--no-cpu", "--no-compare"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r1 = _bench(["bench.py", "--gpus", "1", "--save", str(one)] + common)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--dist-backend", "gloo", "--save", str(two)] + common,
                       cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["ranks"] == 2 and line["rehearsal"] is True
    assert line["config"]["rays_per_step"] == r1["config"]["rays_per_step"]
    assert np.array_equal(np.asarray(Image.open(one)), np.asarray(Image.open(two)))
    if tm.device_count() < 2:
        r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"] + common, cwd=ROOT, capture_output=True,
                           text=True, timeout=300, env=env)
        assert r.returncode != 0 and "visible GPUs" in r.stderr and not r.stdout.strip()
