#!/bin/bash
# PMC passes over one render of the bench frame (tools/tune.py), one rocprofv3
# process per counter set (never combined with traces).
# usage: bash tools/pmc_pass.sh <tag> "<tune variant>" "<counters pass 1>" ["<counters pass 2>" ...]
set -e
tag=$1; var=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $out/p$i -o run -- python3 tools/tune.py "$var" 64 1 > $out/p$i.log 2>&1
done
echo done
