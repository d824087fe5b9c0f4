#!/bin/bash
# r03 session 26: pixel seeding, pilot order by 64-pixel runs (option pilot_strips)
out=gpurun_out/r03s26; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pilot_strips or pixel_mode or progressive" > $out/pytest_sel.log 2>&1
rc=$?; tail -1 $out/pytest_sel.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_sel.log | head -20; exit $rc; fi
for n in 1 2 4 8; do
  TUNE_SEED=pixel TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 300 python -u tools/tune.py "pilot_strips=0;pilot_strips=1" 64 5 > $out/strips_$n.log 2>&1
  rc=$?; tail -n2 $out/strips_$n.log | cut -c1-150; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
