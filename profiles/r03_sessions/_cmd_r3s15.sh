#!/bin/bash
# r03 session 15: row engine choice by load -- iterated (chase per thread / per
# wave) vs streaming at 1/2 and 1/4 of the bench frame; streaming window count at N=1
out=gpurun_out/r03s15; mkdir -p $out; export TMPDIR=/tmp
V="rowspec_chase=1;rowspec_chase=0;rowspec_stream=1"
for n in 2 4; do
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "$V" 64 3 > $out/row_$n.log 2>&1
  rc=$?; tail -n3 $out/row_$n.log | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
W="rowspec_chase=0;rowspec_stream=1&rowspec_windows=2;rowspec_stream=1&rowspec_windows=4;rowspec_stream=1&rowspec_windows=8;rowspec_stream=1&rowspec_spread=0.1"
TUNE_SHARDS=1 timeout -k 10 300 python -u tools/rowspec_time.py "$W" 64 2 > $out/stream_w_1.log 2>&1
rc=$?; tail -n5 $out/stream_w_1.log | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so TMPT_ROWSPEC_LOG=1 TUNE_SHARDS=1 timeout -k 10 120 python -u tools/rowspec_time.py "rowspec_stream=1" 64 1 > $out/stream_diag_1.log 2>&1
grep -E "rowstream" $out/stream_diag_1.log | cut -c1-250
TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so TMPT_ROWSPEC_LOG=1 TUNE_SHARDS=8 timeout -k 10 120 python -u tools/rowspec_time.py "rowspec_stream=1" 64 1 > $out/stream_diag_8.log 2>&1
grep -E "rowstream" $out/stream_diag_8.log | cut -c1-250
echo session-done
