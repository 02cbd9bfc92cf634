#!/bin/bash
# Bin size A/B for the N-way band split (one GPU, no collective): TRI_BIN_LOG2=4/5 per band size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "1 5" "1 4" "4 5" "4 4" "8 5" "8 4"; do
  set -- $spec
  TRI_BIN_LOG2=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary --sim-world $1 \
    > gpurun_out/simbin_$1_$2.log 2>&1 || { echo "sim $spec failed"; tail -3 gpurun_out/simbin_$1_$2.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/simbin_$1_$2.log').read().strip().splitlines()[-1])
print('world=$1 bin_log2=$2 fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
for bl in 5 4; do
  TRI_BIN_LOG2=$bl timeout -k 10 200 python bench.py --config c2 --steps 300 --warmup 30 --no-cpu-baseline --no-secondary > gpurun_out/c2_$bl.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c2_$bl.log').read().strip().splitlines()[-1])
print('c2 bin_log2=$bl fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
