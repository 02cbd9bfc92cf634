#!/bin/bash
# Round 4 (d): device-resident arguments — where the C3 frame rate went. C3 A/B of r3trims (round-3 kernels with
# by-value arguments), the current build (graphs), nograph (same launches one by one), preload (the argument
# pointer preloaded into SGPRs); host cost per tri_render for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
V=3d-renderer_amd/lib/variants
for lib in $V/r3trims.so 3d-renderer_amd/lib/libtri_raster.so $V/nograph.so $V/preload.so; do
  TRI_RASTER_LIB=$lib timeout -k 10 120 python tools/host_overhead.py c2 2000 > gpurun_out/host.txt 2>&1 || { cat gpurun_out/host.txt; exit 1; }
  echo "$(basename $lib): $(head -1 gpurun_out/host.txt)"
done
EXTRA="--no-secondary" bash tools/ab.sh "TRI_RASTER_LIB=$V/r3trims.so" "" "TRI_RASTER_LIB=$V/nograph.so" "TRI_RASTER_LIB=$V/preload.so" "TRI_RASTER_LIB=$V/r3trims.so" "" "TRI_RASTER_LIB=$V/nograph.so" "TRI_RASTER_LIB=$V/preload.so"
