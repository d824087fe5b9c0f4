#!/bin/bash
# r03 session 1: host facts, counter list, default bench (all-core CPU baseline),
# counter passes + calibration, write attribution (no colour buffer / plain stores)
out=gpurun_out/r03s1; mkdir -p $out; export TMPDIR=/tmp
{ nproc; python3 -c "import os;print(os.cpu_count(), len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max; lscpu; } > $out/host.txt 2>&1
timeout -k 10 60 rocprofv3 --list-avail > $out/counters.txt 2>&1
echo "list rc=$?"
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
bash tools/pmc_bench.sh $out/pmc || exit $?
for v in "TMPT_SAMPLE_BLOCK=1024" "TMPT_SBUF=1"; do
  tag=w_$(echo $v | tr '=' '_')
  env $v timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $out/$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare > $out/$tag.json 2> $out/$tag.err
  rc=$?; echo "$tag rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
echo session-done
