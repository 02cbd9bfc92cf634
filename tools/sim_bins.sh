#!/bin/bash
# Bin size A/B for the N-way band split (one GPU, no collective). Build the variants first, on the CPU:
#   tools/build_variant.sh bl4 -DTRI_FORCE_BIN_LOG2=4 && tools/build_variant.sh bl5 -DTRI_FORCE_BIN_LOG2=5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBDIR=3d-renderer_amd/lib/variants
for spec in "1 5" "1 4" "4 5" "4 4" "8 5" "8 4"; do
  set -- $spec
  TRI_RASTER_LIB=$LIBDIR/bl$2.so timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-secondary --sim-world $1 \
    > gpurun_out/simbin_$1_$2.log 2>&1 || { echo "sim $spec failed"; tail -3 gpurun_out/simbin_$1_$2.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/simbin_$1_$2.log').read().strip().splitlines()[-1])
print('world=$1 bin_log2=$2 fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
for bl in 5 4; do
  TRI_RASTER_LIB=$LIBDIR/bl$bl.so timeout -k 10 200 python bench.py --config c2 --steps 300 --warmup 30 --no-cpu-baseline --no-secondary > gpurun_out/c2_$bl.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c2_$bl.log').read().strip().splitlines()[-1])
print('c2 bin_log2=$bl fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
