#!/bin/bash
# GPU box: parity tests (stop at the first failure), then a C3-only bench line (20 and 200 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit $rc
for s in 20 200; do
  timeout -k 10 200 python -u bench.py --steps $s --warmup 5 --no-cpu-baseline --no-secondary ${BENCH_EXTRA} > gpurun_out/bq$s.json 2> gpurun_out/bq$s.err || { tail -5 gpurun_out/bq$s.err; exit 1; }
done
python3 - <<'PY'
import json
for f in ["bq20", "bq200"]:
    d = json.loads([l for l in open(f"gpurun_out/{f}.json") if l.startswith("{")][-1])
    print(f, round(d["value"]), round(d["ms_per_step"], 5), "k_raster", round(d["roofline"]["kernel_ms"], 5), d["stage_ms"])
PY
