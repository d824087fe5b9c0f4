#!/bin/bash
# r03 session 25: seed-table loads issued together (sample_seed) -- A/B of two
# library builds in alternating processes, sample seeding at N=1 and 1/8, row seeding
out=gpurun_out/r03s25; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "sample_mode or rowspec or row_mode" > $out/pytest_sel.log 2>&1
rc=$?; tail -1 $out/pytest_sel.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_sel.log | head -20; exit $rc; fi
for r in 1 2 3; do for lib in base new; do
  L=$PWD/toymeshpathtracer_amd/_lib/libtmpt.so; [ $lib = base ] && L=$PWD/toymeshpathtracer_amd/_lib_base/libtmpt.so
  for n in 1 8; do
    TMPT_LIB_PATH=$L TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 200 python -u tools/tune.py "" 64 3 > $out/${lib}_${n}_$r.log 2>&1 || exit $?
    echo "$lib 1/$n r$r: $(tail -n1 $out/${lib}_${n}_$r.log | cut -c40-140)"
  done
  TMPT_LIB_PATH=$L TUNE_SHARDS=8 timeout -k 10 200 python -u tools/rowspec_time.py "" 64 2 > $out/${lib}_row8_$r.log 2>&1 || exit $?
  echo "$lib row 1/8 r$r: $(tail -n1 $out/${lib}_row8_$r.log | cut -c50-140)"
done; done
for n in 1 8; do
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "rowspec_abandon=0;rowspec_abandon=1" 64 3 > $out/abandon_$n.log 2>&1
  rc=$?; grep frame $out/abandon_$n.log | tail -n2 | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
