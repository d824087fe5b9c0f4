#!/bin/bash
# per-rank load at N = 1, 2, 4, 8 (shard 0 of N, 1-row bands) for both seeding modes
set -e
o=gpurun_out/${1:-scale}; mkdir -p $o; export TMPDIR=/tmp
for n in 1 2 4 8 16; do
  TUNE_BAND=1 TUNE_SHARDS=$n TUNE_SEED=sample timeout -k 10 200 python tools/tune.py "" 64 5 > $o/sample_$n.log 2>&1
  TUNE_BAND=1 TUNE_SHARDS=$n TUNE_SEED=pixel timeout -k 10 200 python tools/tune.py "" 64 5 > $o/pixel_$n.log 2>&1
done
for f in $o/*_*.log; do echo "$f $(grep MRays $f)"; done
