#!/bin/bash
set -e
o=gpurun_out/${1:-sbuf}; mkdir -p $o; export TMPDIR=/tmp
TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py "TMPT_SBUF=0;TMPT_SBUF=1;TMPT_SBUF=2" 64 4 > $o/n1.log 2>&1
TUNE_BAND=1 TUNE_SHARDS=8 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py "TMPT_SBUF=0;TMPT_SBUF=1;TMPT_SBUF=2" 64 5 > $o/n8.log 2>&1
for v in 0 1 2; do
  TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $o/f$v -o run -- python3 tools/tune.py "TMPT_SBUF=$v" 64 1 > $o/f$v.log 2>&1
  TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $o/w$v -o run -- python3 tools/tune.py "TMPT_SBUF=$v" 64 1 > $o/w$v.log 2>&1
done
grep -h "MRays" $o/n1.log $o/n8.log
