cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 60 ./tools/launch_probe/launch_probe > gpurun_out/launch_probe.txt 2>&1; echo "probe rc=$?"; cat gpurun_out/launch_probe.txt
timeout -k 10 120 python tools/host_overhead.py c2 2000 > gpurun_out/host_c2.txt 2>&1 && cat gpurun_out/host_c2.txt
PYTEST_K=reference_frame bash tools/gpu_quick.sh
