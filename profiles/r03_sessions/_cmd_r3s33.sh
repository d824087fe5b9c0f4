#!/bin/bash
# r03 session 33: the GPU suite with the wide-row fallback test
out=gpurun_out/r03s33; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_gpu.log | head -20; exit $rc; fi
echo session-done
