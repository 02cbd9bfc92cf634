#!/bin/bash
# A/B a list of environment settings on the bench (GPU box). Usage:
#   bash tools/ab.sh "TRI_SETUP_STRIDE=1" "" "TRI_ABLATE=1" ...
# Prints fps and per-stage microseconds per setting; stops at the first failing run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for setting in "$@"; do
  i=$((i + 1))
  log=gpurun_out/ab_$i.log
  env ${setting:-TRI_NOOP=1} timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline ${EXTRA} > $log 2>&1 || { echo "[$setting] failed rc=$?"; tail -5 $log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
print('[$setting] fps=%.0f'%d['value'], {k:round(v*1e3,1) for k,v in d['stage_ms'].items()}, 'c2', {k:round(v,4) for k,v in d['secondary'].get('c2_sphere50k_1920x1080',{}).items()})"
done
