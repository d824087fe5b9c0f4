#!/bin/bash
# r03 session 12 (re-entry): HEAD check -- GPU suite, smoke, bench, rocprof stats
out=gpurun_out/r03s12h; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $out/pytest_gpu.log | head; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $out/smoke.log; exit 1; }
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-compare > $out/prof_bench.json 2> $out/prof.err
echo "prof rc=$?"
python3 tools/prof_summary.py $out/prof/run_results.db > $out/rocprof_stats.txt 2>&1
find $out -name "*.db" -delete
echo session-done
