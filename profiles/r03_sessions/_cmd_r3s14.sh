#!/bin/bash
# r03 session 14: postponed leaves (option defer) -- parity, then A/B in sample
# seeding on the bench frame at N=1 and the 1/8 shard, and the round counters
out=gpurun_out/r03s14; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "postponed or sample_mode_matches" > $out/pytest_sel.log 2>&1
rc=$?; tail -2 $out/pytest_sel.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_sel.log | head -20; exit $rc; fi
for n in 1 8; do
  TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 300 python -u tools/tune.py "defer=0;defer=1" 64 5 > $out/defer_$n.log 2>&1
  rc=$?; tail -n2 $out/defer_$n.log | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so timeout -k 10 300 python -u tools/round_stats.py 16 1 "defer=0;defer=1" > $out/defer_rounds.log 2>&1
grep -v amdgpu $out/defer_rounds.log | cut -c1-250

bash tools/_cmd_r3s13.sh || exit $?
echo session-done
