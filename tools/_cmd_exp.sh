set -e
mkdir -p gpurun_out/exp1
export TMPDIR=/tmp TUNE_BAND=1
TUNE_SHARDS=128 timeout -k 10 200 python tools/tune.py "TMPT_HELP=0;TMPT_WAVE_CAP=8&TMPT_HELP=0;TMPT_WAVE_CAP=16&TMPT_HELP=0;TMPT_LEAF_MAX=4&TMPT_HELP=0;TMPT_COLLAPSE=sah&TMPT_HELP=0" 64 2 > gpurun_out/exp1/s128.log 2>&1
TUNE_SHARDS=128 timeout -k 10 200 python tools/tune.py "TMPT_PROF=3;TMPT_PROF=3&TMPT_WAVE_CAP=8" 64 1 > gpurun_out/exp1/s128_prof.log 2>&1
TUNE_SHARDS=8 timeout -k 10 200 python tools/tune.py ";TMPT_LEAF_MAX=4;TMPT_COLLAPSE=sah;TMPT_LEAF_MAX=3" 64 2 > gpurun_out/exp1/s8.log 2>&1
echo ok
