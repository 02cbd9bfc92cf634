#!/bin/bash
# GPU-box validation: smoke -> parity tests -> short bench. Stops at the first fault/abort/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
(ls /usr/share/vulkan/icd.d /etc/vulkan/icd.d; ldconfig -p | grep -i -E "vulkan|lvp") > gpurun_out/vulkan_probe.txt 2>&1
nproc > gpurun_out/host.txt; lscpu | head -20 >> gpurun_out/host.txt 2>&1
fatal() { case "$1" in 124|134|137|139) return 0;; *) [ "$1" -gt 128 ] && return 0; return 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; fatal $rc && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -q --tb=short ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; fatal $rc && exit $rc
timeout -k 10 400 python bench.py ${BENCH_ARGS:---steps 100 --warmup 10} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
exit $rc
