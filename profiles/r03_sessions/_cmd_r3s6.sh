#!/bin/bash
# r03 session 6: small-frame time split (host / other device work / k_path),
# kernel timeline of the small configs, per-scene table at HEAD
out=gpurun_out/r03s6; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/small_frame.py 50 > $out/small_frame.log 2>&1 || exit $?
tail -6 $out/small_frame.log
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 tools/small_frame.py 10 > $out/small_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
python3 tools/kernel_timeline.py $(find $out/prof -name "*.db" | head -1) 60 > $out/timeline.txt 2>&1
head -30 $out/timeline.txt
find $out -name "*.db" -delete
timeout -k 10 600 python -u tools/scene_table.py 3 > $out/scene_table.log 2>&1 || exit $?
tail -9 $out/scene_table.log
echo session-done
