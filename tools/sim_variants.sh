#!/bin/bash
# N = 8 per-rank rates on one GPU (bench.py --sim-world 8 --sim-codec dbp, assemble-only split) for library
# variants: LIBS = space-separated TRI_RASTER_LIB paths ("" = the default build), RANKS = sim ranks.
set -o pipefail
mkdir -p gpurun_out
i=0
for lib in "" $LIBS; do
  i=$((i + 1))
  for r in ${RANKS:-4}; do
    TRI_RASTER_LIB=$lib timeout -k 10 200 python -u bench.py --steps 400 --warmup 50 --no-secondary --sim-world 8 --sim-rank $r \
      --sim-display-rows ${DROWS:-0} --sim-codec dbp --no-cpu-baseline > gpurun_out/simv_${i}_$r.json 2> gpurun_out/simv_${i}_$r.err || { tail -20 gpurun_out/simv_${i}_$r.err; exit 1; }
    python - "$i" "$r" "${lib:-default}" <<'P'
import json, sys
d = json.loads(open(f"gpurun_out/simv_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[3]} rank {sys.argv[2]}: {d['value']:.0f} frames/s")
P
  done
done
