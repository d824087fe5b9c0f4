#!/bin/bash
# r03 session 31: streaming row engine's worker kernel at 4 waves per SIMD (no
# spills) vs 5 (the closing library), alternating processes, N=1 and 1/8
out=gpurun_out/r03s31; mkdir -p $out; export TMPDIR=/tmp
for r in 1 2; do for lib in base occ4; do
  L=$PWD/toymeshpathtracer_amd/_lib/libtmpt.so; [ $lib != base ] && L=$PWD/toymeshpathtracer_amd/_lib_var_$lib/libtmpt.so
  for n in 1 8; do
    TMPT_LIB_PATH=$L TUNE_SHARDS=$n timeout -k 10 200 python -u tools/rowspec_time.py "" 64 2 > $out/${lib}_${n}_$r.log 2>&1 || exit $?
    echo "$lib 1/$n r$r: $(tail -n1 $out/${lib}_${n}_$r.log | cut -c50-140)"
  done
done; done
echo session-done
