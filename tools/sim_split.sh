#!/bin/bash
# N = 8 per-rank rates on one GPU with the dbp codec folded in, at display bands of 0.5x and 1x the equal share
# (bench.py --sim-world 8 --sim-display-rows D --sim-codec dbp): the display rank (0) and a sender (4), or RANKS.
# D = 0: the display rank renders nothing and only decodes the other bands (an assemble-only display).
set -o pipefail
mkdir -p gpurun_out
for d in ${DROWS:-135 270}; do
  for r in ${RANKS:-0 4}; do
    timeout -k 10 200 python -u bench.py --steps 400 --warmup 50 --no-secondary --sim-world 8 --sim-rank $r \
      --sim-display-rows $d --sim-codec dbp > gpurun_out/simd_${d}_$r.json 2> gpurun_out/simd_${d}_$r.err || { tail -20 gpurun_out/simd_${d}_$r.err; exit 1; }
    python - "$d" "$r" <<'P'
import json, sys
d = json.loads(open(f"gpurun_out/simd_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"display rows {sys.argv[1]} rank {sys.argv[2]}: {d['value']:.0f} frames/s ({d['ms_per_step'] * 1e3:.1f} us per frame)")
P
  done
done
