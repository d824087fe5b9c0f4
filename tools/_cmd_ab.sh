set -e
tag=$1; shift
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp TUNE_BAND=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$tag/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
python -c "import json;d=json.load(open('gpurun_out/$tag/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
for n in 8 32 128; do TUNE_SHARDS=$n timeout -k 10 200 python tools/tune.py "" 64 3 2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/shards $n /"; done
