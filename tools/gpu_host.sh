#!/bin/bash
# tri_render's host cost by phase (tools/host_breakdown.py) under HIP runtime settings. Build the diagnostics
# library first: tools/build_variant.sh hostt -DTRI_HOST_TIMING
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
L=3d-renderer_amd/lib/variants/hostt.so
for setting in "" ROC_USE_FGS_KERNARG=0 ROC_USE_FGS_KERNARG=1 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1 \
               DEBUG_HIP_KERNARG_COPY_OPT=0 DEBUG_HIP_KERNARG_COPY_OPT=1 HIP_FORCE_DEV_KERNARG=0 ""; do
  for c in c2 c3; do
    env ${setting:-TRI_NOOP=1} TRI_RASTER_LIB=$L timeout -k 10 120 python tools/host_breakdown.py $c 100 > gpurun_out/hb.txt 2>&1 || { cat gpurun_out/hb.txt; exit 1; }
    echo "[${setting:-base}] $(cat gpurun_out/hb.txt)"
  done
done
