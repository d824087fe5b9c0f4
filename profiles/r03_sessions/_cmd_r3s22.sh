#!/bin/bash
# r03 session 22: lean pixel kernel (option pixel_lean) -- parity, A/B at 1, 1/2, 1/4, 1/8
out=gpurun_out/r03s22; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "lean or pixel_mode" > $out/pytest_sel.log 2>&1
rc=$?; tail -2 $out/pytest_sel.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_sel.log | head -20; exit $rc; fi
for n in 1 2 4 8; do
  TUNE_SEED=pixel TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 300 python -u tools/tune.py "pixel_lean=0;pixel_lean=1" 64 5 > $out/lean_$n.log 2>&1
  rc=$?; tail -n2 $out/lean_$n.log | cut -c1-150; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
