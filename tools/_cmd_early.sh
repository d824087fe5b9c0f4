#!/bin/bash
set -e
o=gpurun_out/${1:-early}; mkdir -p $o; export TMPDIR=/tmp
V="TMPT_TUNE=902,16,16,0;TMPT_TUNE=902,32,16,16;TMPT_TUNE=902,32,16,24;TMPT_TUNE=902,32,24,24;TMPT_TUNE=902,32,32,32;TMPT_TUNE=902,24,16,20;TMPT_TUNE=902,16,16,24;TMPT_TUNE=902,64,16,16;TMPT_TUNE=902,32,12,12;TMPT_TUNE=902,16,8,16"
TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 400 python tools/tune.py "$V" 64 3 > $o/n1.log 2>&1
TUNE_BAND=1 TUNE_SHARDS=8 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py "$V" 64 5 > $o/n8.log 2>&1
grep -h "MRays" $o/n1.log $o/n8.log
