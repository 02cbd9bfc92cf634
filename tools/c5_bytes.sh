#!/bin/bash
# C5 k_raster's HBM read bytes by ablation (sized L2->fabric read requests, one PMC pass per library):
# the full kernel, without the texture sample (TRI_ABLATE=128) and without the shadow lookup (TRI_ABLATE=2048).
# Build first: for a in 128 2048; do bash tools/build_variant.sh A$a -DTRI_ABLATE=$a; done
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5b
for v in base A128 A2048; do
  if [ $v = base ]; then unset TRI_RASTER_LIB; else export TRI_RASTER_LIB=3d-renderer_amd/lib/variants/$v.so; fi
  timeout -k 10 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/c5b/$v -o $v --output-format csv \
    -- python3 bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --inflight 1 > gpurun_out/c5b/$v.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
f = glob.glob(f"gpurun_out/c5b/{v}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "k_raster" not in r["Kernel_Name"]: continue
    acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
w = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}
by = [sum(c[k] * w[k] for k in w) for c in acc.values()]
print(f"{v}: k_raster reads {sum(by) / len(by) / 1e6:.1f} MB per launch over {len(by)} launches")
PY
done
