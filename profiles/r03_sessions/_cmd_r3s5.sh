#!/bin/bash
# r03 session 5: wavefront trace variants (TMPT_WF_VARIANT builds in _lib_var<v>)
# and octant bins, N=1 and the 1/8 shard, pixel seeding
out=gpurun_out/r03s5e; mkdir -p $out; export TMPDIR=/tmp
for n in 1 8; do
  TUNE_SHARDS=$n TUNE_BAND=1 timeout -k 10 300 python -u tools/tune.py "ENGINE=wavefront;ENGINE=wavefront&wf_bins=8" 64 3 > $out/wf_v0_$n.log 2>&1 || exit $?
  TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_var4/libtmpt.so TUNE_SHARDS=$n TUNE_BAND=1 timeout -k 10 300 python -u tools/tune.py "ENGINE=wavefront;ENGINE=wavefront&wf_bins=8" 64 3 > $out/wf_v4_$n.log 2>&1 || exit $?
  tail -qn2 $out/wf_v0_$n.log $out/wf_v4_$n.log | cut -c1-130
done
echo session-done
