#!/bin/bash
# One GPU-box session: the GPU parity suite (all of it, failures listed, not
# stopped at the first), then -- unless a test crashed the process -- a short
# bench line.  usage: bash tools/gpu_session.sh <tag> [bench args...]
tag=${1:-run}; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -40
tail -2 $out/pytest_gpu.log
# 0 = all passed, 1 = some failed: the GPU is fine; anything else (crash, timeout) ends the session
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python bench.py "$@" > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], {k: v.get('value') for k, v in d['seed_modes'].items()}, d['roofline']['frac'], d.get('parity_sample'), d.get('reference_octree'))"
echo session-done
