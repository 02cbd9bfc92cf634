#!/bin/bash
# Per-rank render cost of the N-way row-band split, measured on one GPU without the collective.
# SPECS="8 4,1 0" (comma-separated "world rank" pairs) limits the runs; TRI_RASTER_LIB picks a library;
# SIM_DISPLAY_ROWS sizes the display band (rank 0) of an uneven split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=, read -ra SPECLIST <<< "${SPECS:-1 0,2 0,4 0,4 2,8 0,8 4,8 7}"
for spec in "${SPECLIST[@]}"; do
  set -- $spec
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary --sim-world $1 --sim-rank $2 --inflight ${INFLIGHT:-2} ${SIM_DISPLAY_ROWS:+--sim-display-rows $SIM_DISPLAY_ROWS} \
    > gpurun_out/sim_$1_$2.log 2>&1 || { echo "sim $spec failed"; tail -3 gpurun_out/sim_$1_$2.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/sim_$1_$2.log').read().strip().splitlines()[-1])
print('world=$1 rank=$2 fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
