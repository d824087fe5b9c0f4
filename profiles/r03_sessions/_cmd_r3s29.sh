#!/bin/bash
# r03 session 29: diagnostics -- (1) the sample kernel with its colour stores
# removed (wrong image; an upper bound on what the stores' write acks cost at
# the traversal loop's entry wait), alternating processes; (2) the streaming
# row engine's speculation statistics at the closing defaults
out=gpurun_out/r03s29; mkdir -p $out; export TMPDIR=/tmp
for r in 1 2; do for lib in base nostore; do
  L=$PWD/toymeshpathtracer_amd/_lib/libtmpt.so; [ $lib = nostore ] && L=$PWD/toymeshpathtracer_amd/_lib_var_nostore/libtmpt.so
  for n in 1 8; do
    TMPT_LIB_PATH=$L TUNE_SEED=sample TUNE_BAND=1 TUNE_SHARDS=$n timeout -k 10 200 python -u tools/tune.py "" 64 3 > $out/${lib}_${n}_$r.log 2>&1 || exit $?
    echo "$lib 1/$n r$r: $(tail -n1 $out/${lib}_${n}_$r.log | cut -c40-140)"
  done
done; done
for n in 1 8; do
  TMPT_LIB_PATH=$PWD/toymeshpathtracer_amd/_lib_diag/libtmpt.so TMPT_ROWSPEC_LOG=1 TUNE_SHARDS=$n timeout -k 10 120 python -u tools/rowspec_time.py "" 64 1 > $out/stream_diag_$n.log 2>&1 || exit $?
  grep -E "rowstream" $out/stream_diag_$n.log | cut -c1-250
done
echo session-done
