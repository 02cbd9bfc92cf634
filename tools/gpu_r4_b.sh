#!/bin/bash
# Round 4: launch-cost probe (graphs), host cost of tri_render, the GPU suite, then an A/B on the bench:
# r3trims = round-3 kernels (by-value arguments, no trims), notrims = device-resident arguments + graphs
# without the k_raster trims, "" = the current build; interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 60 ./tools/launch_probe/launch_probe > gpurun_out/launch_probe.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/launch_probe.txt
timeout -k 10 120 python tools/host_overhead.py c2 2000 > gpurun_out/host_c2.txt 2>&1; echo "host rc=$?"; cat gpurun_out/host_c2.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
V=3d-renderer_amd/lib/variants
bash tools/ab.sh "TRI_RASTER_LIB=$V/r3trims.so" "TRI_RASTER_LIB=$V/notrims.so" "" "TRI_RASTER_LIB=$V/r3trims.so" "TRI_RASTER_LIB=$V/notrims.so" ""
