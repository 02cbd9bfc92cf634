#!/bin/bash
# Round-6 closing session on one GPU box: the GPU suite, the driver-shaped bench line (20 steps, and 200 for the
# steady state), then rocprofv3 kernel traces + PMC passes for C3 and C5 (tools/profile.sh). Every GPU step has its own
# time limit and the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  || { tail -5 gpurun_out/gpu_tests.log; grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --steps 20 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --no-secondary > gpurun_out/bench200.json 2> gpurun_out/bench200.err || { tail -5 gpurun_out/bench200.err; exit 1; }
echo bench ok
PROF_OUT=gpurun_out/prof_c3 bash tools/profile.sh > gpurun_out/prof_c3.log 2>&1 || { tail -5 gpurun_out/prof_c3.log; exit 1; }
PROF_OUT=gpurun_out/prof_c5 BENCH_ARGS="--config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --inflight 1" \
  bash tools/profile.sh > gpurun_out/prof_c5.log 2>&1 || { tail -5 gpurun_out/prof_c5.log; exit 1; }
echo prof ok
# N = 8 per-rank rates on this GPU (assemble-only display: rank 0 decodes the seven bands; senders 1, 4, 7)
DROWS=0 RANKS="0 1 4 7" timeout -k 10 900 bash tools/sim_split.sh > gpurun_out/sim_split6.txt 2>&1 || { tail -5 gpurun_out/sim_split6.txt; exit 1; }
cat gpurun_out/sim_split6.txt
