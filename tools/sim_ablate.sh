#!/bin/bash
# k_setup / k_raster cost split on the 8-way band (rank 4, one GPU, no collective) with the compile-time
# ablation variants (build them first: bash tools/build_variant.sh ablate_N -DTRI_ABLATE=N).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base ${VARIANTS:-ablate_4 ablate_16 ablate_32}; do
  lib=""
  [ "$v" != base ] && lib="TRI_RASTER_LIB=3d-renderer_amd/lib/variants/$v.so"
  env $lib TRI_NOOP=1 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-secondary \
    --sim-world ${WORLD:-8} --sim-rank ${RANK_:-4} > gpurun_out/sa_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/sa_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/sa_$v.log').read().strip().splitlines()[-1])
print('$v fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
