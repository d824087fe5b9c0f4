#!/bin/bash
# PMC passes on one rank's load at N GPUs (tools/tune.py TUNE_SHARDS=N).
# usage: bash tools/pmc_shard.sh <tag> <N> "<counters pass 1>" ["<pass 2>" ...]
set -e
tag=$1; n=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  TUNE_SHARDS=$n timeout -k 10 300 rocprofv3 --pmc $set -d $out/p$i -o run -- python3 tools/tune.py ENGINE=persistent 64 1 > $out/p$i.log 2>&1
done
echo done
