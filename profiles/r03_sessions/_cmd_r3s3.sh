#!/bin/bash
# r03 session 3: wavefront octant-binned queues (A/B + counters), the k_path
# counter passes on the pruned library (roofline record), bench
out=gpurun_out/r03s3; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "octant or pixel_mode or render_multi or ranges" > $out/pytest_sel.log 2>&1
rc=$?; tail -2 $out/pytest_sel.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $out/pytest_sel.log | head; exit $rc; fi
for v in "ENGINE=wavefront" "ENGINE=wavefront&wf_bins=8"; do
  tag=wf_$(echo $v | tr '=&' '__')
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $out/$tag -o run -- python3 tools/tune.py "$v" 64 1 > $out/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $out/${tag}_c -o run -- python3 tools/tune.py "$v" 64 1 > $out/${tag}_c.log 2>&1
  rc=$?; echo "${tag}_c rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
bash tools/pmc_bench.sh $out/pmc || exit $?
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare"
for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=ea_$(echo $set | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $set -d $out/pmc/$tag -o run -- $BENCH > $out/pmc/$tag.json 2> $out/pmc/$tag.err
  rc=$?; echo "$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
  timeout -s KILL 60 rocprofv3 --pmc $set -d $out/pmc/cal_$tag -o run -- ./tools/_bin/pmc_calib > $out/pmc/cal_$tag.json 2> $out/pmc/cal_$tag.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-compare > $out/prof_bench.json 2> $out/prof.err
echo "prof rc=$?"
# summaries on the box (the rocpd databases exceed the 64 MiB pull limit)
python3 tools/roofline_counters.py $out/pmc $out/pmc > $out/counters_k_path.json 2> $out/counters.err
python3 tools/prof_summary.py $out/prof/run_results.db > $out/rocprof_stats.txt 2>&1
python3 tools/wf_counters.py $out > $out/wf_counters.txt 2>&1
find $out -name "*.db" -delete
echo session-done
