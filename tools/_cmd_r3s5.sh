#!/bin/bash
# r03 session 5: the wavefront engine after the pruning -- kind-specialised
# voted steps with (lib) and without (lib_var) the LDS top-node copy -- against
# the round-2 library, N=1 and the 1/8 shard, pixel seeding
out=gpurun_out/r03s5; mkdir -p $out; export TMPDIR=/tmp
for n in 1 8; do
  TUNE_SHARDS=$n TUNE_BAND=1 timeout -k 10 300 python -u tools/tune.py "ENGINE=wavefront" 64 3 > $out/wf_new_topc_$n.log 2>&1 || exit $?
  TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_var/libtmpt.so TUNE_SHARDS=$n TUNE_BAND=1 timeout -k 10 300 python -u tools/tune.py "ENGINE=wavefront" 64 3 > $out/wf_new_notopc_$n.log 2>&1 || exit $?
  (cd _old_r02 && TUNE_SHARDS=$n TUNE_BAND=1 timeout -k 10 300 python -u tools/tune.py "ENGINE=wavefront" 64 3 > ../$out/wf_old_r02_$n.log 2>&1) || exit $?
  tail -qn1 $out/wf_new_topc_$n.log $out/wf_new_notopc_$n.log $out/wf_old_r02_$n.log
done
echo session-done
