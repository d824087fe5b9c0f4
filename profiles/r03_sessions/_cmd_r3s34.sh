#!/bin/bash
# r03 session 34: sample block size re-checked at the closing library
out=gpurun_out/r03s34; mkdir -p $out; export TMPDIR=/tmp
for cfg in "1 sample_block=0;sample_block=4;sample_block=16" "2 sample_block=0;sample_block=2;sample_block=8" "4 sample_block=0;sample_block=1;sample_block=4" "8 sample_block=0;sample_block=2"; do
  n=${cfg%% *}; V=${cfg#* }
  TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 300 python -u tools/tune.py "$V" 64 3 > $out/blk_$n.log 2>&1
  rc=$?; grep "MRays" $out/blk_$n.log | tail -n3 | cut -c1-140; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
