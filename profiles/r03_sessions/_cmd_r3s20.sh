#!/bin/bash
# r03 session 20: streaming row engine spread -- the edges (N=1 low, 1/8 high)
out=gpurun_out/r03s20; mkdir -p $out; export TMPDIR=/tmp
for cfg in "1 0 0.01 0.02" "8 0.18 0.22 0.27"; do
  set -- $cfg; n=$1; shift
  V=""; for s in "$@"; do V="$V;rowspec_spread=$s"; done; V=${V#;}
  TUNE_SHARDS=$n timeout -k 10 300 python -u tools/rowspec_time.py "$V" 64 3 > $out/spread_$n.log 2>&1
  rc=$?; grep "frame" $out/spread_$n.log | tail -n3 | cut -c1-160; if [ $rc -ne 0 ]; then exit $rc; fi
done
echo session-done
