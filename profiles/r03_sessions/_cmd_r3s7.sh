#!/bin/bash
# r03 session 7: kernel timeline of one row-seeded bench frame (speculative row engine)
out=gpurun_out/r03s7b; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 tools/rowspec_time.py "rowspec_groups=1" 64 1 > $out/row_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $out/row_prof.log; exit $rc; fi
python3 tools/kernel_timeline.py $(find $out/prof -name "*.db" | head -1) 30 > $out/timeline.txt 2>&1
cat $out/timeline.txt | head -20
find $out -name "*.db" -delete
echo session-done
