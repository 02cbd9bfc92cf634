#!/bin/bash
# Per-kernel instruction counters for a list of environment settings (GPU box). Usage:
#   bash tools/pmc_ab.sh "" "TRI_ABLATE=1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
i=0
for setting in "$@"; do
  i=$((i + 1))
  for v in ${setting}; do export "$v"; done
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES \
    -d $OUT/run$i -o run$i --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary \
    > $OUT/run$i.log 2>&1 || { echo "[$setting] rc=$?"; tail -5 $OUT/run$i.log; exit 1; }
  for v in ${setting}; do unset "${v%%=*}"; done
  python3 - "$OUT/run$i" "$setting" <<'EOF'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/*/*counter_collection.csv") + glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        n = n[n.find("k_"):].split("(")[0] if "k_" in n else n[:30]
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("[%s]" % sys.argv[2])
for k, d in sorted(acc.items()):
    print("  %-28s" % k, " ".join("%s=%.3g" % (c, sum(v) / len(v)) for c, v in sorted(d.items())))
EOF
done
