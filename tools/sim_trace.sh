#!/bin/bash
# rocprofv3 kernel trace of one rank of the N-way row-band split on one GPU (SURVEY 8(e) per-rank cost):
# the kernels' own durations, next to the bench's event-pass stage times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W=${SIM_WORLD:-8}; R=${SIM_RANK:-4}
OUT=${PROF_OUT:-gpurun_out/prof_sim${W}_${R}}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- \
  python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary --sim-world $W --sim-rank $R --inflight ${INFLIGHT:-2} \
  > $OUT/trace.log 2>&1 || { echo "sim trace failed"; tail -5 $OUT/trace.log; exit 1; }
tail -1 $OUT/trace.log
python3 tools/prof_summary.py $OUT sim${W}_${R} $OUT/summary.json
