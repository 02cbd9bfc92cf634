#!/bin/bash
# rocprofv3 counters of the dbp codec kernels (tools/dbp_scaling.py), one PMC pass per group; summary printed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_codec
mkdir -p $OUT
run() {
    local name=$1; shift
    DBP_SIZES=8 timeout -k 10 120 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 tools/dbp_scaling.py > $OUT/$name.log 2>&1
    local rc=$?; echo "$name rc=$rc"; return $rc
}
run trace --kernel-trace --stats || exit $?
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY || exit $?
run sq2 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE || exit $?
python3 - <<'P'
import csv, glob, collections
for name in ("sq1", "sq2"):
    f = glob.glob(f"gpurun_out/prof_codec/{name}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(name, "no csv"); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    disp = collections.defaultdict(set)
    for row in csv.DictReader(open(f[0])):
        k = row["Kernel_Name"]
        if "dbp" not in k:
            continue
        kk = "unpack" if "unpack" in k else "pack"
        acc[kk][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[kk].add(row["Dispatch_Id"])
    for kk, d in acc.items():
        n = len(disp[kk])
        print(name, kk, "dispatches", n, {c: round(v / n) for c, v in sorted(d.items())})
        if "SQ_WAVES" in d:
            wv = d["SQ_WAVES"]
            print("   per wave: VALU %.0f SALU %.0f LDS %.0f; wait_inst/wave_cycles %.2f" % (d["SQ_INSTS_VALU"] / wv,
                  d["SQ_INSTS_SALU"] / wv, d["SQ_INSTS_LDS"] / wv, d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]))
P
for f in $(find $OUT/trace -name "*kernel_stats.csv"); do grep -i dbp $f | cut -c1-200; done
