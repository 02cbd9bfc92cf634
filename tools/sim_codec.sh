#!/bin/bash
# Per-rank frame rates at N = 8 on one GPU with the band codec's per-frame work folded in (bench.py --sim-world 8
# --sim-codec): the display rank (0) decoding the 7 other bands, a sender (4) packing its band; each format and none.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sim_codec.txt
: > $out
for codec in ${CODECS:-none bgr24 dbp}; do
  for r in 0 4; do
    timeout -k 10 200 python -u bench.py --steps 400 --warmup 50 --no-secondary --sim-world 8 --sim-rank $r \
      --sim-codec $codec > gpurun_out/simc_${codec}_$r.json 2> gpurun_out/simc_${codec}_$r.err || { tail -20 gpurun_out/simc_${codec}_$r.err; exit 1; }
    python - "$codec" "$r" >> $out <<'P'
import json, sys
d = json.loads(open(f"gpurun_out/simc_{sys.argv[1]}_{sys.argv[2]}.json").read().strip().splitlines()[-1])
print(f"codec {sys.argv[1]:5s} rank {sys.argv[2]}: {d['value']:.0f} frames/s ({d['ms_per_step'] * 1e3:.1f} us per frame)")
P
    tail -1 $out
  done
done
