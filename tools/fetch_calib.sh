#!/bin/bash
# GPU box: FETCH_SIZE calibration (tools/fetch_calib/fetch_calib.hip, built on the CPU side with
#   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib/fetch_calib tools/fetch_calib/fetch_calib.hip).
# One kernel-trace pass and one PMC pass per counter group, each its own short run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${CAL_OUT:-gpurun_out/fetch_calib}
BIN=./tools/fetch_calib/fetch_calib
mkdir -p $OUT
timeout -k 10 60 $BIN 3 > $OUT/plain.json || exit 1
run() {  # name, rocprofv3 options...
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- $BIN 2 > $OUT/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc
}
run trace --kernel-trace --stats || exit $?
run pmc_fetch --pmc FETCH_SIZE || exit $?
run pmc_sized --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum || exit $?
run pmc_misc --pmc TCC_BUBBLE_sum TCC_READ_SECTORS_sum TCC_EA0_RDREQ_DRAM_sum || exit $?
run pmc_req --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum || exit $?
run pmc_write --pmc WRITE_SIZE || exit $?
python3 tools/fetch_calib_summary.py $OUT
