#!/bin/bash
# r03 session 13: row engine variants re-measured at HEAD (the previous session's
# logs were lost): chase over LDS-staged units vs one thread per row, streaming
# engine vs host-driven iterations, whole frame and 1/8 shard
out=gpurun_out/r03s13; mkdir -p $out; export TMPDIR=/tmp
V="rowspec_chase=1;rowspec_chase=0;rowspec_stream=1;rowspec_stream=1&rowspec_chase=0"
for n in 1 8; do
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "$V" 64 3 > $out/row_$n.log 2>&1
  rc=$?; tail -n4 $out/row_$n.log | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
