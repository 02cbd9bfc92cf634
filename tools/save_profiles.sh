#!/bin/bash
# Copy the summaries of a tools/gpu_session.sh prof run (gpurun_out/prof_c3, prof_c5) into profiles/<round>/
# and refresh profiles/pmc_summary.json. Usage: bash tools/save_profiles.sh round2
set -e
cd "$(dirname "$0")/.."
dst=profiles/${1:?round name}
mkdir -p $dst
for w in c3 c5; do
  src=gpurun_out/prof_$w
  cp $src/trace/trace_kernel_stats.csv $dst/${w}_kernel_stats.csv
  for p in fetch write sized sq sq2 tcc tatd; do
    [ -f $src/pmc_$p/pmc_${p}_counter_collection.csv ] || continue
    gzip -c $src/pmc_$p/pmc_${p}_counter_collection.csv > $dst/${w}_pmc_$p.csv.gz
  done
done
python3 tools/prof_summary.py gpurun_out/prof_c3 c3_grid1m_3840x2160 profiles/pmc_summary.json
python3 tools/prof_summary.py gpurun_out/prof_c5 c5_textured4x2048_shadow2048_3840x2160 profiles/pmc_summary.json
[ -f gpurun_out/bench.json ] && tail -1 gpurun_out/bench.json > $dst/bench_line.json
echo saved to $dst
