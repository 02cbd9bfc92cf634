#!/bin/bash
# Round 4: the full bench line (C3 + C2 + C5 secondaries) at 2 and 3 frames in flight, twice, and at 20 steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/misc_$n.json 2> gpurun_out/misc_$n.err || { echo "$n failed"; tail -3 gpurun_out/misc_$n.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/misc_$n.json').read().strip().splitlines()[-1])
print('%-10s c3 %6.0f fps %6.1f us' % ('$n', d['value'], d['ms_per_step']*1e3), ' '.join('%s %.0f' % (k[:2], v['frames_per_s']) for k, v in d['secondary'].items()))"
}
run if2a --inflight 2 && run if3a --inflight 3 && run if2b --inflight 2 && run if3b --inflight 3 && run s20_if2 --steps 20 --inflight 2 && run s20_if3 --steps 20 --inflight 3
