#!/bin/bash
# One GPU call: the GPU parity suite on the in-tree library, then tools/ab.sh over the settings given
# as arguments (kernel-variant libraries via TRI_RASTER_LIB, diagnostics via TRI_ABLATE, ...).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/ab.sh "$@"
