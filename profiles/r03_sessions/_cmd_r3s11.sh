#!/bin/bash
# r03 session 11: streaming row engine statistics (diagnostic build), small loads first
out=gpurun_out/r03s12; mkdir -p $out; export TMPDIR=/tmp
export TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so TMPT_ROWSPEC_LOG=1
for cfg in "8 16" "8 64" "1 16" "1 64"; do
  set -- $cfg
  TUNE_SHARDS=$1 timeout -k 10 150 python -u tools/rowspec_time.py "rowspec_stream=0;rowspec_stream=1" $2 1 > $out/s_$1_$2.log 2>&1
  rc=$?; grep -E "rowstream|rowspec:|frame" $out/s_$1_$2.log | cut -c1-220; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
