set -e
tag=$1
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$tag/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/$tag/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/$tag/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
python -c "import json;d=json.load(open('gpurun_out/$tag/bench.json'));print('bench',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])"
ROUNDS=6 bash tools/_cmd_multi.sh $tag ";TMPT_BALANCE=0&TMPT_DPRIO=0,0,0" 8 4 2 1
