#!/bin/bash
set -e
o=gpurun_out/${1:-r2c}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -2 $o/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
tail -2 $o/smoke.log
TUNE_RES=3840x2160 TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py "" 256 2 > $o/4k_n1.log 2>&1
TUNE_RES=3840x2160 TUNE_BAND=1 TUNE_SHARDS=8 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py "" 256 3 > $o/4k_n8.log 2>&1
TUNE_RES=3840x2160 TUNE_BAND=1 TUNE_SHARDS=8 TUNE_SEED=pixel timeout -k 10 300 python tools/tune.py "" 256 2 > $o/4k_n8_pixel.log 2>&1
grep -h MRays $o/4k_*.log
