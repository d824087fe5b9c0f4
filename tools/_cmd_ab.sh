#!/bin/bash
# generic sample-mode A/B: bash tools/_cmd_ab.sh <tag> "<variants>" [n1 rounds] [n8 rounds]
set -e
o=gpurun_out/$1; mkdir -p $o; export TMPDIR=/tmp
TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 400 python tools/tune.py "$2" 64 ${3:-3} > $o/n1.log 2>&1
TUNE_BAND=1 TUNE_SHARDS=8 TUNE_SEED=sample timeout -k 10 300 python tools/tune.py "$2" 64 ${4:-5} > $o/n8.log 2>&1
grep -h "MRays" $o/n1.log $o/n8.log
