#!/bin/bash
# Round-4 first GPU check: launch-cost probe, host cost of tri_render, the GPU suite, a quick C3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 60 ./tools/launch_probe/launch_probe > gpurun_out/launch_probe.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/launch_probe.txt
timeout -k 10 120 python tools/host_overhead.py c2 2000 > gpurun_out/host_c2.txt 2>&1; echo "host rc=$?"; cat gpurun_out/host_c2.txt
bash tools/gpu_quick.sh
