#!/bin/bash
# r03 session 35: the bench as the driver runs it (20 steps) at the closing library
out=gpurun_out/r03s35; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python3 bench.py --steps 20 --warmup 2 > $out/bench20.json 2> $out/bench20.err || { echo "bench rc=$?"; tail -20 $out/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench20.json')); print(d['value'], d['ms_per_step'], d['seed_modes'], d['roofline']['bound'], d['roofline']['frac'], d['roofline']['counter_record_stale'], d['cpu_baseline']['value'])"
echo session-done
