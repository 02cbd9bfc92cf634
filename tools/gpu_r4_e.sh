#!/bin/bash
# Round 4 (e): the first kernel carries the frame's arguments by value (no ring, no fetch kernel, no graphs):
# GPU suite, host cost, and C3 A/B against r3trims (round-3 kernels) and nograph (argument ring + fetch kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
V=3d-renderer_amd/lib/variants
for lib in $V/r3trims.so 3d-renderer_amd/lib/libtri_raster.so; do
  for cfg in c2 c3; do
    TRI_RASTER_LIB=$lib timeout -k 10 120 python tools/host_overhead.py $cfg 2000 > gpurun_out/host.txt 2>&1 || { cat gpurun_out/host.txt; exit 1; }
    echo "$(basename $lib): $(head -1 gpurun_out/host.txt)"
  done
done
bash tools/ab.sh "TRI_RASTER_LIB=$V/r3trims.so" "" "TRI_RASTER_LIB=$V/nograph.so" "TRI_RASTER_LIB=$V/r3trims.so" "" "TRI_RASTER_LIB=$V/nograph.so"
