# usage: bash tools/_cmd_multi.sh <tag> "<variants>" <shards...>
set -e
tag=$1; variants=$2; shift 2
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp TUNE_BAND=1
for n in "$@"; do
  TUNE_SHARDS=$n timeout -k 10 300 python tools/tune.py "$variants" 64 ${ROUNDS:-2} > gpurun_out/$tag/s$n.log 2>&1
  grep -v "amdgpu.ids\|^scene" gpurun_out/$tag/s$n.log | sed "s/^/[$n] /"
done
