set -e
tag=$1; shards=$2; variants=$3; rounds=${4:-2}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp TUNE_BAND=1
TUNE_SHARDS=$shards timeout -k 10 500 python tools/tune.py "$variants" 64 $rounds > gpurun_out/$tag/s$shards.log 2>&1
grep -v amdgpu.ids gpurun_out/$tag/s$shards.log
