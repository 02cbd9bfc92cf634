#!/bin/bash
# TA / TD occupancy of the C3 kernels (GPU box): is the L1 address (TA) or data-return (TD) path a
# co-limiter of k_raster's gathers? Lists the counters first; one rocprofv3 run per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/tatd
rm -rf $OUT; mkdir -p $OUT
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --no-secondary --inflight 1"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -oE "\b(TA|TD|TCP)_[A-Z0-9_]+" $OUT/counters.txt | sort -u > $OUT/tatd_names.txt
pass() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
    echo "$name rc=$?"
}
pass a TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
pass b TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TD_SPI_STALL_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
python3 tools/prof_summary.py $OUT tatd $OUT/summary.json | grep -E "^k_raster|^k_setup|^k_vertex"
