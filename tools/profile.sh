#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes over a short bench run (GPU box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
# one frame in flight: overlapping kernels of two contexts would stretch every traced duration (and
# mix the PMC attribution), while the bench times its kernels in a separate single-context event pass
ARGS="${BENCH_ARGS:---steps 50 --warmup 5 --no-cpu-baseline --no-secondary --inflight 1}"
run() {  # name, rocprofv3 options...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc
}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run trace --kernel-trace --stats || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
# sized L2->fabric read requests: the byte count the FETCH_SIZE calibration validates (tools/fetch_calib.sh)
run pmc_sized --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum || exit $?
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit $?
run pmc_sq2 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit $?
run pmc_tcc --pmc TCC_HIT_sum TCC_MISS_sum || exit $?
# L1 address (TA) and data-return (TD) occupancy: every wave-level gather costs the CU ~16 cycles there
# (tools/td_probe), so k_raster's fragment gathers load these units about as much as its VALU work
run pmc_tatd --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE || exit $?
find $OUT -name "*.csv" | head -50
