#!/bin/bash
# r03 session 27: cost-ordered sample seeding (option sample_pilot) -- parity,
# then base library vs this one (off / on) in alternating processes
out=gpurun_out/r03s27; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sample_mode" > $out/pytest_sel.log 2>&1
rc=$?; tail -1 $out/pytest_sel.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_sel.log | head -20; exit $rc; fi
for r in 1 2; do for n in 1 8; do
  TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_base/libtmpt.so TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 200 python -u tools/tune.py "" 64 3 > $out/base_${n}_$r.log 2>&1 || exit $?
  echo "base 1/$n r$r: $(tail -n1 $out/base_${n}_$r.log | cut -c40-140)"
  TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 300 python -u tools/tune.py "sample_pilot=0;sample_pilot=1" 64 3 > $out/new_${n}_$r.log 2>&1 || exit $?
  tail -n2 $out/new_${n}_$r.log | cut -c1-140
done; done
echo session-done
