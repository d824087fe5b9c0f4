#!/bin/bash
# per-rank load at N = 1, 2, 4, 8, 16 (shard 0 of N, 1-row bands); seeding modes as $2 (default "sample pixel")
set -e
o=gpurun_out/${1:-scale}; mkdir -p $o; export TMPDIR=/tmp
for n in 1 2 4 8 16; do
  for m in ${2:-sample pixel}; do
    TUNE_BAND=1 TUNE_SHARDS=$n TUNE_SEED=$m timeout -k 10 200 python tools/tune.py "" 64 5 > $o/${m}_$n.log 2>&1
  done
done
for f in $o/*_*.log; do echo "$f $(grep MRays $f)"; done
