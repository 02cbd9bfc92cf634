#!/bin/bash
# A/B of the current build against variants (bench lines twice each, alternating), then the C5 kernel trace and a
# WRITE_SIZE / FETCH_SIZE pass of the current build (C5's per-kernel bytes).  usage: bash tools/gpu_ab_c5.sh [NAME...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
V=3d-renderer_amd/lib/variants
ab=""
for n in "$@"; do ab="$ab TRI_RASTER_LIB=$V/$n.so"; done
bash tools/ab.sh $ab "" $ab "" || exit 1
A="--config c5 --steps 50 --warmup 5 --no-cpu-baseline --no-secondary --inflight 1"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_c5 -o kt --output-format csv -- python3 bench.py $A > gpurun_out/kt_c5.log 2>&1 || { echo trace failed; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c5_write -o pmc_write --output-format csv -- python3 bench.py $A > gpurun_out/pmc_c5_write.log 2>&1 || { echo write pass failed; exit 1; }
timeout -k 10 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/pmc_c5_sized -o pmc_sized --output-format csv -- python3 bench.py $A > gpurun_out/pmc_c5_sized.log 2>&1 || { echo sized pass failed; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/kt_c5/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('k_vertex', 'k_setup', 'k_raster', 'k_shadow')):
        print('%-50s %6s calls avg %8.2f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
for name in ('pmc_c5_write', 'pmc_c5_sized'):
    g = glob.glob(f'gpurun_out/{name}/**/*counter_collection.csv', recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(g)):
        k = r['Kernel_Name']
        for t in ('k_vertex', 'k_setup', 'k_raster', 'k_shadow'):
            if t in k:
                acc[t][(r['Counter_Name'], r.get('Dispatch_Id', ''))].append(float(r['Counter_Value']))
    for t, d in acc.items():
        per = collections.defaultdict(list)
        for (c, disp), v in d.items():
            per[c].append(sum(v))
        print(name, t, {c: round(sum(v) / len(v)) for c, v in per.items()})
PY
