#!/bin/bash
# k_raster cost split: full / coverage only (TRI_ABLATE=1) / shading only (TRI_ABLATE=2).
# The ablations are compile-time (the shipped library carries none of them): build the variants on the
# CPU first,
#   for a in 1 2; do bash tools/build_variant.sh ablate_$a -DTRI_ABLATE=$a; done
# then run this on the GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for a in 0 1 2; do
  lib=""
  [ "$a" != 0 ] && lib="TRI_RASTER_LIB=3d-renderer_amd/lib/variants/ablate_$a.so"
  env $lib TRI_NOOP=1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${EXTRA} > gpurun_out/ablate_$a.log 2>&1 || exit $?
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ablate_$a.log').read().strip().splitlines()[-1])
print('ablate=$a fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()})"
done
