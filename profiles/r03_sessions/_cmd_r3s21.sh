#!/bin/bash
# r03 session 21: streaming row engine with the spread rule -- windows re-checked, row tests
out=gpurun_out/r03s21; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "row or smoke or cli" > $out/pytest_row.log 2>&1
rc=$?; tail -2 $out/pytest_row.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_row.log | head -20; exit $rc; fi
for cfg in "1 rowspec_windows=1;rowspec_windows=3" "2 rowspec_windows=3" "4 rowspec_windows=2;rowspec_windows=4" "8 rowspec_windows=4;rowspec_windows=7"; do
  n=${cfg%% *}; V="rowspec_stream=1;${cfg#* }"
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "$V" 64 3 > $out/win_$n.log 2>&1
  rc=$?; grep "frame" $out/win_$n.log | tail -n3 | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
