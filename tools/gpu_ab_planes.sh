#!/bin/bash
# GPU box: phase split of k_raster (old per-pixel gather path vs attribute-plane path) and a C3 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=3d-renderer_amd/lib/variants
TRI_RASTER_LIB=$V/phase_old.so timeout -k 10 120 python -u tools/phase_times.py c3 > gpurun_out/phase_old.txt 2>&1 || { tail -5 gpurun_out/phase_old.txt; exit 1; }
TRI_PHASES_PLANES=1 TRI_RASTER_LIB=$V/phase_planes.so timeout -k 10 120 python -u tools/phase_times.py c3 > gpurun_out/phase_planes.txt 2>&1 || { tail -5 gpurun_out/phase_planes.txt; exit 1; }
cat gpurun_out/phase_old.txt gpurun_out/phase_planes.txt | grep -v "^k_setup\|fetch+setup\|binning\|rest\|start offsets"
for lib in $V/old.so 3d-renderer_amd/lib/libtri_raster.so; do
  TRI_RASTER_LIB=$lib timeout -k 10 200 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-secondary ${BENCH_EXTRA} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ab.json') if l.startswith('{')][-1]); print('$lib', round(d['value']), 'k_raster', round(d['roofline']['kernel_ms']*1e3,1), 'us')"
done
