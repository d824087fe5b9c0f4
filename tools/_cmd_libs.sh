#!/bin/bash
# compiler-flag A/B: the bench frame (sample seeding) at N=1 and the 1/8 shard
# with each in-tree library build, two interleaved passes
# usage: bash tools/_cmd_libs.sh <tag> <lib dir> [<lib dir> ...]
set -e
o=gpurun_out/$1; shift; mkdir -p $o; export TMPDIR=/tmp
for pass in 1 2; do
  for d in "$@"; do
    n=$(basename $d)
    TMPT_LIB_PATH=$d/libtmpt.so TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 200 python tools/tune.py "" 64 3 2>&1 | grep MRays | sed "s/^ *default/$n n1 p$pass/" >> $o/libs.log
    TMPT_LIB_PATH=$d/libtmpt.so TUNE_BAND=1 TUNE_SHARDS=8 TUNE_SEED=sample timeout -k 10 200 python tools/tune.py "" 64 3 2>&1 | grep MRays | sed "s/^ *default/$n n8 p$pass/" >> $o/libs.log
  done
done
cat $o/libs.log
