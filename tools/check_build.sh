#!/bin/bash
# The GPU suite against the checked build (make CHECK=1: device index tests in
# the traversal, the octree walks and the hit-record loads; tmpt_internal.h
# kChk*).  Build it here first (make -C toymeshpathtracer_amd/csrc CHECK=1 or
# __graft_entry__.build()); on the GPU box:
#   bash tools/check_build.sh <outdir>
# Any failed index test fails its API call (TmptError "device index check
# failed"), so a green run means no index test failed anywhere in the suite.
out=${1:-gpurun_out/check}; mkdir -p $out
export TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_check/libtmpt.so
test -f $TMPT_LIB_PATH || { echo "no checked build at $TMPT_LIB_PATH"; exit 2; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu_check.log 2>&1
rc=$?; tail -2 $out/pytest_gpu_check.log
grep -c "device index check failed" $out/pytest_gpu_check.log
exit $rc
