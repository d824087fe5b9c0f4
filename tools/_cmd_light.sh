#!/bin/bash
set -e
o=gpurun_out/${1:-light}; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -30 $o/pytest.log; exit 1; }
tail -2 $o/pytest.log
timeout -k 10 200 python tools/round_stats.py 16 1 > $o/rs.log 2>&1; TMPT_LIGHT_BVH=0 timeout -k 10 200 python tools/round_stats.py 16 1 > $o/rs0.log 2>&1
grep -h "node visits" $o/rs.log $o/rs0.log
bash tools/_cmd_ab.sh $1 "TMPT_LIGHT_BVH=0;TMPT_LIGHT_BVH=1" 3 5
