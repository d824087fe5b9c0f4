#!/bin/bash
# sample-seeding session: new parity tests, then N=1 and 1/8-shard timings
set -e
o=gpurun_out/${1:-samp}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "sample or ordered or progressive or device_output" > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -3 $o/pytest.log
TUNE_BAND=1 timeout -k 10 200 python tools/tune.py "" 64 3 > $o/n1_pixel.log 2>&1
TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py ";TMPT_SAMPLE_BLOCK=1;TMPT_SAMPLE_BLOCK=4;TMPT_SAMPLE_BLOCK=16;TMPT_SAMPLE_BLOCK=64" 64 3 > $o/n1_sample.log 2>&1
TUNE_BAND=1 TUNE_SHARDS=8 timeout -k 10 200 python tools/tune.py "" 64 5 > $o/n8_pixel.log 2>&1
TUNE_BAND=1 TUNE_SHARDS=8 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py ";TMPT_SAMPLE_BLOCK=1;TMPT_SAMPLE_BLOCK=2;TMPT_SAMPLE_BLOCK=4;TMPT_SAMPLE_BLOCK=8" 64 5 > $o/n8_sample.log 2>&1
grep -h "MRays" $o/*.log
