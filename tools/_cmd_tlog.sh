set -e
mkdir -p gpurun_out/tlog
export TMPDIR=/tmp
for n in 8 32 128; do timeout -k 10 200 python tools/tlog.py $n > gpurun_out/tlog/tlog_$n.log 2>&1; done
echo ok
