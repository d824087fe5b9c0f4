#!/bin/bash
# r03 session 10: streaming row engine -- first run, parity, A/B at N=1 and 1/8
out=gpurun_out/r03s10; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 120 python -u - > $out/first.log 2>&1 <<'PY'
import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import toymeshpathtracer_amd as tm
tris, bmin, bmax = tm.load_scene("data/suzanne.obj")
cam = tm.Camera.for_scene(bmin, bmax, 64, 16)
with tm.Scene(tris) as sc:
    a, ra = sc.trace_image(cam, 64, 16, 4, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_MEGAKERNEL)
    b, rb = sc.trace_image(cam, 64, 16, 4, seed_mode=tm.SEED_ROW, engine=tm.ENGINE_PERSISTENT)
    print("stream iterations", sc.stats().iterations, "rays", ra, rb, "pixels differ", int((a != b).any(-1).sum()))
PY
rc=$?; cat $out/first.log | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "rowspec or row_mode" > $out/pytest_row.log 2>&1
rc=$?; tail -2 $out/pytest_row.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_row.log | head -20; exit $rc; fi
for n in 1 8; do
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "rowspec_stream=0;rowspec_stream=1" 64 3 > $out/stream_$n.log 2>&1 || exit $?
  tail -n2 $out/stream_$n.log | cut -c1-150
done
TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so TMPT_ROWSPEC_LOG=1 timeout -k 10 120 python -u tools/rowspec_time.py "rowspec_stream=1" 64 1 > $out/stream_diag.log 2>&1
grep -E "rowstream|rowspec:" $out/stream_diag.log | head -5
echo session-done
