#!/bin/bash
# r03 session 24: closing artifacts at HEAD -- GPU suite, smoke, bench, rocprof
# stats, the k_path counter passes (roofline record), configs[4] bench line,
# 2-rank gloo rehearsal of the N>1 bench path
out=gpurun_out/r03s24; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail $out/smoke.log; exit 1; }
grep "smoke ok" $out/smoke.log
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['seed_modes'], d['roofline']['bound'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-compare > $out/prof_bench.json 2> $out/prof.err
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 tools/prof_summary.py $out/prof/run_results.db > $out/rocprof_stats.txt 2>&1
head -4 $out/rocprof_stats.txt | cut -c1-150
bash tools/pmc_bench.sh $out/pmc || exit $?
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare"
for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=ea_$(echo $set | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $set -d $out/pmc/$tag -o run -- $BENCH > $out/pmc/$tag.json 2> $out/pmc/$tag.err
  rc=$?; echo "$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
  timeout -s KILL 60 rocprofv3 --pmc $set -d $out/pmc/cal_$tag -o run -- ./tools/_bin/pmc_calib > $out/pmc/cal_$tag.json 2> $out/pmc/cal_$tag.err
  rc=$?; echo "cal_$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
python3 tools/roofline_counters.py $out/pmc $out/pmc > $out/counters_k_path.json 2> $out/counters.err
echo "counters rc=$?"; tail -3 $out/counters.err
find $out -name "*.db" -delete
timeout -k 10 400 python3 bench.py --config sponza4k --steps 2 --warmup 1 --no-cpu > $out/bench_sponza4k.json 2> $out/bench_sponza4k.err || { echo "4k rc=$?"; tail -5 $out/bench_sponza4k.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench_sponza4k.json')); print('4k', d['value'], d['ms_per_step'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 2 --warmup 1 > $out/gloo2.json 2> $out/gloo2.err || { echo "gloo2 rc=$?"; tail -20 $out/gloo2.err; exit 1; }
python3 -c "import json; d=json.load(open('$out/gloo2.json')); print('gloo2', d['value'], d['n_gpus'])"
echo session-done
