#!/bin/bash
# r03 session 30: issue priority by phase in the sample kernel (A: shading
# rounds at priority 1, traversal 0; B: the reverse) vs the closing library
out=gpurun_out/r03s30; mkdir -p $out; export TMPDIR=/tmp
for r in 1 2; do for lib in base prioA prioB; do
  L=$PWD/toymeshpathtracer_amd/_lib/libtmpt.so; [ $lib != base ] && L=$PWD/toymeshpathtracer_amd/_lib_var_$lib/libtmpt.so
  for n in 1 8; do
    TMPT_LIB_PATH=$L TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 200 python -u tools/tune.py "" 64 3 > $out/${lib}_${n}_$r.log 2>&1 || exit $?
    echo "$lib 1/$n r$r: $(tail -n1 $out/${lib}_${n}_$r.log | cut -c40-140)"
  done
done; done
echo session-done
