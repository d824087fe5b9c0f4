#!/bin/bash
# r03 session 18: wave-time split of the sample kernel (diagnostic build,
# TMPT_PROF 1/2/3) at N=1 and 1/8; streaming row engine spread sweep
out=gpurun_out/r03s18; mkdir -p $out; export TMPDIR=/tmp
for p in 1 2 3; do for n in 1 8; do
  TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so TMPT_PROF=$p TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n \
    timeout -k 10 120 python -u tools/tune.py "" 16 1 > $out/prof${p}_$n.log 2>&1
  rc=$?; echo "PROF=$p 1/$n"; grep -E "wave time|cycles per round|shading split" $out/prof${p}_$n.log | head -4 | cut -c1-220; if [ $rc -ne 0 ]; then exit $rc; fi
done; done
for n in 1 8; do
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "rowspec_spread=0.06;rowspec_spread=0.08;rowspec_spread=-1;rowspec_spread=0.14" 64 3 > $out/spread_$n.log 2>&1
  rc=$?; grep frame $out/spread_$n.log | tail -n4 | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
