#!/bin/bash
# A/B bench.py argument sets on the GPU box: bash tools/ab_args.sh "" "--front-priority 1" ...
# Prints fps and per-stage microseconds (C3 headline, C2 and C5 secondaries) per argument set; stops at
# the first failing run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i + 1))
  log=gpurun_out/abargs_$i.log
  timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline $a > $log 2>&1 || { echo "[$a] failed rc=$?"; tail -5 $log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
st=lambda x: {k[3:]:round(v*1e3,1) for k,v in x.items() if v}
print('[${a:-base}] c3 %.0f'%d['value'], st(d['stage_ms']))
for k,v in d.get('secondary', {}).items(): print('    %s %.0f'%(k[:12], v['frames_per_s']), st(v['stage_ms']))"
done
