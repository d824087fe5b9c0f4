#!/bin/bash
# r03 session 17: streaming row engine as the row-seeding default -- the row
# tests, the full GPU suite, the bench (seed_modes.row), the per-scene table
out=gpurun_out/r03s17; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['seed_modes'])"
TUNE_SHARDS=8 timeout -k 10 300 python -u tools/rowspec_time.py "rowspec_stream=1;rowspec_stream=0" 64 3 > $out/row_8.log 2>&1
rc=$?; tail -n2 $out/row_8.log | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u tools/scene_table.py 3 > $out/scene_table.log 2>&1 || exit $?
tail -9 $out/scene_table.log
echo session-done
