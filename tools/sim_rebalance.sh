#!/bin/bash
# N = 8 sender rates on one GPU (bench.py --sim-world 8 --sim-codec dbp) with an assemble-only display, for the
# equal sender bands and for the re-cut that rebalance_sizes computes from those rates (SPLIT: comma-separated
# band sizes, rank 0 first).
set -o pipefail
mkdir -p gpurun_out
for split in "0" "${SPLIT:-0,309,311,313,312,309,306,300}"; do
  for r in ${RANKS:-1 4 7}; do
    tag=$(echo $split | tr , _)
    timeout -k 10 200 python -u bench.py --steps 400 --warmup 50 --no-secondary --sim-world 8 --sim-rank $r \
      --sim-display-rows $split --sim-codec dbp > gpurun_out/simr_${tag}_$r.json 2> gpurun_out/simr_${tag}_$r.err || { tail -20 gpurun_out/simr_${tag}_$r.err; exit 1; }
    python - "$tag" "$r" <<'P'
import json, sys
d = json.loads(open(f"gpurun_out/simr_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"split {sys.argv[1]} rank {sys.argv[2]}: rows {d['config']['bands']}, {d['value']:.0f} frames/s ({d['ms_per_step'] * 1e3:.1f} us per frame)")
P
  done
done
