#!/bin/bash
# One GPU-box session: parity suite, default bench line, rocprofv3 kernel stats and
# the two HBM PMC passes (FETCH_SIZE / WRITE_SIZE cannot share a pass on gfx950).
# usage: bash tools/gpu_round.sh <tag>
set -e
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err
cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format rocpd csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-compare > $out/prof_bench.json 2> $out/prof.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare > $out/pmc_fetch.json 2> $out/pmc_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $out/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare > $out/pmc_write.json 2> $out/pmc_write.err
echo done
