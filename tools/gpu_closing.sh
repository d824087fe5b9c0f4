#!/bin/bash
# Closing artifacts of a round on one GPU box: the GPU suite, smoke, the bench
# line as the driver runs it, rocprofv3 kernel stats of the bench, the k_path
# counter passes (roofline record: tools/pmc_bench.sh + the EA request-size
# passes, each its own rocprofv3 process), the configs[4] line and the 2-rank
# gloo rehearsal of the N>1 path through bench.py's own rank launch.
# usage: bash tools/gpu_closing.sh <tag> [steps]
tag=${1:-closing}; steps=${2:-20}
out=gpurun_out/$tag; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; grep -E "FAILED|ERROR" $out/pytest_gpu.log | head -20; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $out/smoke.log; exit 1; }
grep "smoke ok" $out/smoke.log
timeout -k 10 600 python3 bench.py --steps $steps --warmup 2 > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], {k: v.get('value') for k, v in d['seed_modes'].items()}, d['roofline']['bound'], d['roofline']['frac'], d['cpu_baseline']['value'], d['parity_sample'], d['reference_octree'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-compare > $out/prof_bench.json 2> $out/prof.err
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 tools/prof_summary.py $out/prof/run_results.db > $out/rocprof_stats.txt 2>&1
head -4 $out/rocprof_stats.txt | cut -c1-150
bash tools/pmc_bench.sh $out/pmc || exit $?
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare"
for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  ptag=ea_$(echo $set | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $set -d $out/pmc/$ptag -o run -- $BENCH > $out/pmc/$ptag.json 2> $out/pmc/$ptag.err
  rc=$?; echo "$ptag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
python3 tools/roofline_counters.py $out/pmc $out/pmc > $out/counters_k_path.json 2> $out/counters.err
echo "counters rc=$?"; tail -3 $out/counters.err
find $out -name "*.db" -delete
timeout -k 10 400 python3 bench.py --config sponza4k --steps 2 --warmup 1 --no-cpu > $out/bench_sponza4k.json 2> $out/bench_sponza4k.err || { echo "4k rc=$?"; tail -5 $out/bench_sponza4k.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench_sponza4k.json')); print('4k', d['value'], d['ms_per_step'])"
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 2 --warmup 1 > $out/gloo2.json 2> $out/gloo2.err || { echo "gloo2 rc=$?"; tail -20 $out/gloo2.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/gloo2.json')); print('gloo2', d['value'], d['n_gpus'], d['ranks'], d['rehearsal'], d['devices'])"
timeout -k 10 400 python3 bench.py --gpus 4 --dist-backend gloo --steps 2 --warmup 1 > $out/gloo4.json 2> $out/gloo4.err || { echo "gloo4 rc=$?"; tail -20 $out/gloo4.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/gloo4.json')); print('gloo4', d['value'], d['n_gpus'], d['ranks'], d['rehearsal'], d['devices'])"
echo session-done
