#!/bin/bash
# r03 session 9: the shadow-free pass's unit throughput against its launch
# size (one row group, so kernels do not overlap): default windows vs 8 and 32
out=gpurun_out/r03s9; mkdir -p $out; export TMPDIR=/tmp
export TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so TMPT_ROWSPEC_LOG=1
for v in "rowspec_groups=1" "rowspec_groups=1&rowspec_windows=8" "rowspec_groups=1&rowspec_windows=32"; do
  tag=$(echo $v | tr '=&' '__')
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/$tag -o run -- python3 tools/rowspec_time.py "$v" 64 1 > $out/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $out/$tag.log; exit $rc; fi
  python3 tools/kernel_timeline.py $(find $out/$tag -name "*.db" | head -1) 5 > $out/${tag}_timeline.txt 2>&1
  grep -E "rowspec:|frame" $out/$tag.log | cut -c1-200; head -6 $out/${tag}_timeline.txt
done
find $out -name "*.db" -delete
echo session-done
