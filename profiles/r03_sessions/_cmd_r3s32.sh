#!/bin/bash
# r03 session 32: vote threshold of the sample kernel's traversal rounds
# (leaf round when n_leaf > t * n_node; t = 1 closing library, 1.25, 0.8, 1.5)
out=gpurun_out/r03s32; mkdir -p $out; export TMPDIR=/tmp
for r in 1 2; do for lib in base v125 v080 v150; do
  L=$PWD/toymeshpathtracer_amd/_lib/libtmpt.so; [ $lib != base ] && L=$PWD/toymeshpathtracer_amd/_lib_var_$lib/libtmpt.so
  for n in 1 8; do
    TMPT_LIB_PATH=$L TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 200 python -u tools/tune.py "" 64 3 > $out/${lib}_${n}_$r.log 2>&1 || exit $?
    echo "$lib 1/$n r$r: $(tail -n1 $out/${lib}_${n}_$r.log | cut -c40-140)"
  done
done; done
echo session-done
