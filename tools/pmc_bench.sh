#!/bin/bash
# Counter passes over bench.py's k_path (one rocprofv3 process per counter set,
# never combined with traces; each pass bounded by its own timeout) and over the
# calibration microbenchmark tools/_bin/pmc_calib (known byte counts).
# usage: bash tools/pmc_bench.sh <out dir> [extra bench.py args]
# Summaries: python tools/roofline_counters.py <out dir> > profiles/<round>_counters.json
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-compare $*"
run_pass() {  # name, counters..., (env in PASS_ENV)
    local name=$1; shift
    env $PASS_ENV timeout -s KILL 150 rocprofv3 --pmc "$@" -d "$out/$name" -o run -- $BENCH > "$out/$name.json" 2> "$out/$name.err"
    local rc=$?
    echo "pass $name rc=$rc"
    if [ $rc -ge 124 ]; then echo "stopping: pass $name rc=$rc"; exit $rc; fi
    return 0
}
PASS_ENV= run_pass sq SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
PASS_ENV= run_pass fetch FETCH_SIZE
PASS_ENV= run_pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
PASS_ENV= run_pass l2req TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
if [ -x tools/_bin/pmc_calib ]; then
  for set in "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=cal_$(echo $set | cut -d' ' -f1)
    timeout -s KILL 60 rocprofv3 --pmc $set -d "$out/$tag" -o run -- ./tools/_bin/pmc_calib > "$out/$tag.json" 2> "$out/$tag.err"
    rc=$?; echo "calib $tag rc=$rc"
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
fi
echo done
