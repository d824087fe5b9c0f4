#!/bin/bash
# r03 session 2: GPU suite on the pruned library (options API, RCCL multi-device,
# per-ray ranges, configs[4] and full-spp sample tests), smoke, bench, and the
# request-size passes (EA read requests by size: exact HBM bytes)
out=gpurun_out/r03s2; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -3 $out/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|error" $out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare"
for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=ea_$(echo $set | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $set -d $out/$tag -o run -- $BENCH > $out/$tag.json 2> $out/$tag.err
  rc=$?; echo "$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
  timeout -s KILL 60 rocprofv3 --pmc $set -d $out/cal_$tag -o run -- ./tools/_bin/pmc_calib > $out/cal_$tag.json 2> $out/cal_$tag.err
  rc=$?; echo "cal_$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
echo session-done
