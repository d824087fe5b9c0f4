#!/bin/bash
# r03 session 16: streaming row engine -- windows per row by load
out=gpurun_out/r03s16; mkdir -p $out; export TMPDIR=/tmp
for cfg in "1 2;3" "2 2;3;4" "4 2;3;4;6" "8 2;3;4;7"; do
  n=${cfg%% *}; ws=${cfg#* }
  V=""; for w in ${ws//;/ }; do V="$V;rowspec_stream=1&rowspec_windows=$w"; done; V=${V#;}
  [ $n -eq 1 ] && V="$V;rowspec_chase=0"
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "$V" 64 3 > $out/sw_$n.log 2>&1
  rc=$?; grep "frame" $out/sw_$n.log | tail -n5 | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
