#!/bin/bash
# One measurement cycle on the GPU box: the GPU suite, per-kernel durations (rocprofv3 kernel trace, one frame
# in flight, C3) of the current build and each named variant (3d-renderer_amd/lib/variants/NAME.so), then the
# C3/C2/C5 rate A/B of [variants..., current], twice.   usage: bash tools/gpu_cycle.sh [NAME...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
V=3d-renderer_amd/lib/variants
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head; exit 1; }
libs=""; ab=""
for n in "$@"; do libs="$libs $V/$n.so"; ab="$ab TRI_RASTER_LIB=$V/$n.so"; done
for cfg in ${TRACE_CFGS:-c3}; do
for lib in $libs 3d-renderer_amd/lib/libtri_raster.so; do
  n=$(basename $lib .so)_$cfg
  TRI_RASTER_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$n -o kt --output-format csv -- python3 bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --inflight 1 > gpurun_out/kt_$n.log 2>&1 || { echo "$n trace failed"; tail -5 gpurun_out/kt_$n.log; exit 1; }
  f=$(find gpurun_out/kt_$n -name "*kernel_stats.csv" | head -1)
  echo "== $n"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('k_vertex','k_setup','k_raster','k_reset','k_shadow')): print('  %-60s %8s calls avg %8.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
done
done
bash tools/ab.sh $ab "" $ab ""
timeout -k 10 120 python tools/host_overhead.py c2 > gpurun_out/host_c2.txt 2>&1 && timeout -k 10 120 python tools/host_overhead.py c3 > gpurun_out/host_c3.txt 2>&1; cat gpurun_out/host_c2.txt gpurun_out/host_c3.txt
