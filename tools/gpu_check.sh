#!/bin/bash
# GPU-box session: parity suite (+ optional bench line).  usage: bash tools/gpu_check.sh <tag> [bench_steps]
set -o pipefail
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
if [ -n "$2" ]; then
    timeout -k 10 300 python bench.py --steps $2 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
    head -c 700 $out/bench.json; echo
fi
