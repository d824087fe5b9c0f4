#!/bin/bash
# r03 session 23: kernel split of a row-seeded bench frame (streaming engine) at N=1 and 1/8
out=gpurun_out/r03s23; mkdir -p $out; export TMPDIR=/tmp
for n in 1 8; do
  TUNE_SHARDS=$n timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$n -o run -- python3 tools/rowspec_time.py "rowspec_stream=1" 64 2 > $out/row_$n.log 2>&1
  rc=$?; echo "prof $n rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $out/row_$n.log; exit $rc; fi
  python3 tools/prof_summary.py $(find $out/prof_$n -name "*.db" | head -1) > $out/stats_$n.txt 2>&1
  head -8 $out/stats_$n.txt | cut -c1-150
done
find $out -name "*.db" -delete
echo session-done
