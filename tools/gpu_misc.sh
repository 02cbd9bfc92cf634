#!/bin/bash
# Round 4: frames in flight at C3 (2 vs 3, twice) and the C2 rate at 20 vs 200 steps (is C2 GPU-bound?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary "$@" > gpurun_out/misc_$n.json 2> gpurun_out/misc_$n.err || { echo "$n failed"; tail -3 gpurun_out/misc_$n.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/misc_$n.json').read().strip().splitlines()[-1])
print('%-12s %8.0f fps  %7.1f us/frame  raster %.1f us' % ('$n', d['value'], d['ms_per_step']*1e3, d['stage_ms']['ms_raster']*1e3))"
}
run c3_if2a --inflight 2 && run c3_if3a --inflight 3 && run c3_if2b --inflight 2 && run c3_if3b --inflight 3 &&
run c2_s20 --config c2 --steps 20 && run c2_s200 --config c2 --steps 200 && run c2_s20b --config c2 --steps 20 && run c2_s200b --config c2 --steps 200
