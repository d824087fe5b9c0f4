#!/bin/bash
# r03 session 4: GPU suite, bench, wavefront bins at the 1/8 shard, round-2
# library A/B of the wavefront engine, per-call overhead at the 1/8 shard, and a
# 2-rank gloo rehearsal of bench.py's N>1 path
out=gpurun_out/r03s4; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; tail -2 $out/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $out/pytest_gpu.log | head; exit $rc; fi
timeout -k 10 400 python3 bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc=$?"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
TUNE_SHARDS=8 TUNE_BAND=1 timeout -k 10 300 python -u tools/tune.py "ENGINE=wavefront;ENGINE=wavefront&wf_bins=8;ENGINE=persistent" 64 3 > $out/tune_bins_shard8.log 2>&1 || exit $?
tail -4 $out/tune_bins_shard8.log
TUNE_SHARDS=8 TUNE_BAND=1 TUNE_SEED=sample timeout -k 10 300 python -u tools/tune.py "ENGINE=persistent" 64 5 > $out/tune_sample_shard8.log 2>&1 || exit $?
tail -1 $out/tune_sample_shard8.log
(cd _old_r02 && timeout -k 10 300 python -u tools/tune.py "ENGINE=wavefront;ENGINE=persistent" 64 3 > ../$out/old_r02_wavefront.log 2>&1) || exit $?
tail -3 $out/old_r02_wavefront.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 2 --warmup 1 > $out/gloo2.json 2> $out/gloo2.err || { echo "gloo2 rc=$?"; tail -20 $out/gloo2.err; exit 1; }
cat $out/gloo2.json
echo session-done
