#!/bin/bash
# r03 session 19: streaming row engine -- window spread by load
out=gpurun_out/r03s19; mkdir -p $out; export TMPDIR=/tmp
for cfg in "1 0.02 0.035 0.05 0.06" "2 0.04 0.06 0.08 0.102" "4 0.06 0.09 0.118 0.15" "8 0.1 0.12 0.15 0.18"; do
  set -- $cfg; n=$1; shift
  V=""; for s in "$@"; do V="$V;rowspec_spread=$s"; done; V=${V#;}
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "$V" 64 3 > $out/spread_$n.log 2>&1
  rc=$?; grep "frame" $out/spread_$n.log | tail -n4 | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
