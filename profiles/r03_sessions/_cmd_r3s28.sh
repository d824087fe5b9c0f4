#!/bin/bash
# r03 session 28: per-scene, per-load table at the closing library
out=gpurun_out/r03s28; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/scene_table.py 3 > $out/scene_table.log 2>&1 || exit $?
tail -9 $out/scene_table.log
echo session-done
