set -e
mkdir -p gpurun_out/prof8
export TMPDIR=/tmp TUNE_BAND=1 TUNE_SHARDS=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8/p -o run --output-format csv -- python3 tools/tune.py "" 64 2 > gpurun_out/prof8/tune.log 2>&1
