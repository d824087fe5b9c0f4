"""Per-pixel timeline of the persistent engine's final launch (PROF build,
TMPT_TLOG): when each pixel started and ended (s_memrealtime, 100 MHz), its
traversal steps and the shading rounds its wave ran while it held the pixel.
Shows where a shard's frame time goes at low pixel-per-lane loads.
  python tools/tlog.py <shards> [env assignments ...]   e.g. tools/tlog.py 8 TMPT_HELP=1"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))
import numpy as np  # noqa: E402

import toymeshpathtracer_amd as tm  # noqa: E402
import gen_standin_sponza  # noqa: E402

shards = int(sys.argv[1]) if len(sys.argv) > 1 else 8
for kv in sys.argv[2:]:
    k, _, v = kv.partition("=")
    os.environ[k] = v
PROD = os.environ.pop("TMPT_PROF", "1") == "0"  # TMPT_PROF=0: the production kernel
W, H, SPP = 1920, 1080, 64
tris, bmin, bmax = tm.load_scene(gen_standin_sponza.ensure())
cam = tm.Camera.for_scene(bmin, bmax, W, H, is_sponza=True)
sc = tm.Scene(tris)
path = os.path.join(tempfile.gettempdir(), f"tlog_{os.getpid()}.bin")
if not PROD:
    os.environ["TMPT_PROF"] = "1"
os.environ["TMPT_TLOG"] = path
img, rays = sc.trace_image(cam, W, H, SPP, seed_mode=tm.SEED_PIXEL, band_rows=1, shard=0, num_shards=shards)
st = sc.stats()
t = np.fromfile(path, dtype=np.uint32).reshape(-1, 4).astype(np.int64)
os.unlink(path)
if os.environ.get("TLOG_SAVE"):
    np.save(os.environ["TLOG_SAVE"], t.astype(np.uint32))
t0 = t[:, 0].min()
s, e, steps, nsh = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, t[:, 2], t[:, 3]  # us
dur = e - s
print(f"shards {shards} {' '.join(sys.argv[2:])}: pixels {len(t)}, render {st.render_ms:.1f} ms, "
      f"final launch span {e.max() / 1e3:.2f} ms", flush=True)
print(f"  steps/pixel: mean {steps.mean():.0f} p50 {np.percentile(steps, 50):.0f} p99 {np.percentile(steps, 99):.0f} "
      f"max {steps.max()}")
print(f"  chain us/step: mean {np.mean(dur / np.maximum(steps, 1)):.3f}; pixels ended by 25/50/75/90/99/100 % "
      f"of the span: " + " ".join(f"{np.mean(e <= q * e.max()) * 100:.1f}" for q in (0.25, 0.5, 0.75, 0.9, 0.99, 1.0)))
span = e.max()
print("  time window   active px   steps/us of px ending   mean us/step (px active in window)")
for i in range(10):
    a, b = span * i / 10, span * (i + 1) / 10
    act = np.sum((s < b) & (e > a))
    sel = (e > a) & (e <= b)
    print(f"  {a / 1e3:6.2f}-{b / 1e3:6.2f} ms {act:9d}   {sel.sum():8d} px end   "
          f"{np.mean(dur[sel] / np.maximum(steps[sel], 1)) if sel.any() else 0:.3f}")
order = np.argsort(-e)[:12]
print("  last pixels to finish: start_ms end_ms steps us/step shade_rounds")
for i in order:
    print(f"    {s[i] / 1e3:7.2f} {e[i] / 1e3:7.2f} {steps[i]:7d} {dur[i] / max(steps[i], 1):.3f} {nsh[i]:6d}")
top = np.argsort(-steps)[:12]
print("  most steps: start_ms end_ms steps us/step shade_rounds")
for i in top:
    print(f"    {s[i] / 1e3:7.2f} {e[i] / 1e3:7.2f} {steps[i]:7d} {dur[i] / max(steps[i], 1):.3f} {nsh[i]:6d}")
