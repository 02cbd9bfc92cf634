#!/bin/bash
# A/B a list of environment settings on the bench (GPU box). Usage:
#   bash tools/ab.sh "" "TRI_RASTER_LIB=3d-renderer_amd/lib/variants/w5.so" ...
# Prints fps and per-stage microseconds (C3 headline, C2 and C5 secondaries) per setting; stops at the
# first failing run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for setting in "$@"; do
  i=$((i + 1))
  log=gpurun_out/ab_$i.log
  env ${setting:-TRI_NOOP=1} timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline ${EXTRA} > $log 2>&1 || { echo "[$setting] failed rc=$?"; tail -5 $log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$log').read().strip().splitlines()[-1])
st=lambda x: {k[3:]:round(v*1e3,1) for k,v in x.items() if v}
print('[${setting:-base}] c3 %.0f'%d['value'], st(d['stage_ms']))
for k,v in d['secondary'].items(): print('    %s %.0f'%(k[:24], v['frames_per_s']), st(v.get('stage_ms', {})))"
done
