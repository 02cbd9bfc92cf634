#!/bin/bash
# One GPU-box session: GPU tests, the default bench line, then rocprofv3 trace + PMC passes for C3
# and C5 (tools/profile.sh). Every GPU step has its own time limit and the chain stops at the first
# failure. Usage on the box: bash tools/gpu_session.sh [tests|bench|prof|all]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
what=${1:-all}
set -o pipefail
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
  echo bench ok
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  PROF_OUT=gpurun_out/prof_c3 bash tools/profile.sh > gpurun_out/prof_c3.log 2>&1 || { tail -5 gpurun_out/prof_c3.log; exit 1; }
  PROF_OUT=gpurun_out/prof_c5 BENCH_ARGS="--config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --inflight 1" \
    bash tools/profile.sh > gpurun_out/prof_c5.log 2>&1 || { tail -5 gpurun_out/prof_c5.log; exit 1; }
  echo prof ok
fi
