#!/bin/bash
# r03 session 8: LDS chase for the row engine -- parity, A/B at N=1 and 1/8, timeline
out=gpurun_out/r03s8; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "rowspec or row_mode" > $out/pytest_row.log 2>&1
rc=$?; tail -2 $out/pytest_row.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $out/pytest_row.log | head; exit $rc; fi
for n in 1 8; do
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "rowspec_chase=0;rowspec_chase=1" 64 3 > $out/chase_$n.log 2>&1 || exit $?
  tail -n2 $out/chase_$n.log | cut -c1-150
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 tools/rowspec_time.py "" 64 1 > $out/row_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 tools/kernel_timeline.py $(find $out/prof -name "*.db" | head -1) 30 > $out/timeline.txt 2>&1
head -16 $out/timeline.txt
find $out -name "*.db" -delete
echo session-done
