#!/bin/bash
# Instruction-cache PMC passes over the C3 bench (GPU box), one rocprofv3 run per pass:
#   bash tools/pmc_icache.sh [bench args]   -> gpurun_out/icache/*, summary on stdout
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/icache
rm -rf $OUT; mkdir -p $OUT
ARGS="${*:---steps 30 --warmup 5 --no-cpu-baseline --no-secondary}"
pass() {
    local name=$1; shift
    timeout -k 10 120 rocprofv3 --pmc "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
    local rc=$?; [ $rc = 0 ] || { echo "$name rc=$rc"; tail -3 $OUT/$name.log; exit $rc; }
}
pass ic SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
pass if SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_WAVE_CYCLES
python3 tools/prof_summary.py $OUT icache $OUT/summary.json | grep -E "^k_"
