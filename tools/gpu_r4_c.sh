#!/bin/bash
# Round 4 (c): the GPU suite on the fetch-kernel argument ring, host cost per tri_render, then A/Bs:
# C3 r3trims (round-3 kernels) / notrims / current; C5 novis (inline shadow lookup) / vis6 / current.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
for cfg in c2 c3; do timeout -k 10 120 python tools/host_overhead.py $cfg 2000 > gpurun_out/host_$cfg.txt 2>&1 || exit 1; cat gpurun_out/host_$cfg.txt; done
V=3d-renderer_amd/lib/variants
EXTRA="--no-secondary" bash tools/ab.sh "TRI_RASTER_LIB=$V/r3trims.so" "TRI_RASTER_LIB=$V/notrims.so" "" "TRI_RASTER_LIB=$V/r3trims.so" "TRI_RASTER_LIB=$V/notrims.so" "" || exit 1
EXTRA="--config c5 --no-secondary" bash tools/ab.sh "TRI_RASTER_LIB=$V/novis.so" "TRI_RASTER_LIB=$V/vis6.so" "" "TRI_RASTER_LIB=$V/novis.so" "TRI_RASTER_LIB=$V/vis6.so" ""
