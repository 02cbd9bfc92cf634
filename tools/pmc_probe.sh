#!/bin/bash
# Extra PMC passes (memory pipeline occupancy) over the C3 bench, one rocprofv3 run per pass (GPU box):
#   bash tools/pmc_probe.sh [bench args]   -> gpurun_out/probe/*, summary on stdout
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/probe
rm -rf $OUT; mkdir -p $OUT
ARGS="${*:---steps 30 --warmup 5 --no-cpu-baseline --no-secondary}"
pass() {
    local name=$1; shift
    timeout -k 10 120 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
    local rc=$?; [ $rc = 0 ] || { echo "$name rc=$rc"; tail -3 $OUT/$name.log; exit $rc; }
}
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
pass sqa SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES
pass sqb SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_INSTS_VALU_TRANS_F32 SQ_WAVES
python3 tools/prof_summary.py $OUT probe $OUT/summary.json | grep -E "^k_"
