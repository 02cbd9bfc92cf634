#!/bin/bash
# GPU box: the driver's bench command (20 steps, 5 warm-up) and a 200-step run of the same build, to check
# that ms_per_step does not depend on the step count, plus a short C3-only run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/b20.json 2> gpurun_out/b20.err || { tail -5 gpurun_out/b20.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu-baseline > gpurun_out/b200.json 2> gpurun_out/b200.err || { tail -5 gpurun_out/b200.err; exit 1; }
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/b20b.json 2> gpurun_out/b20b.err || exit 1
python3 - <<'EOF'
import json
for f in ["b20", "b200", "b20b"]:
    d = json.loads([l for l in open(f"gpurun_out/{f}.json") if l.startswith("{")][-1])
    cpu = d["cpu_baseline"]
    print(f, round(d["value"]), round(d["ms_per_step"], 5), "warm", d["warmup_frames_run"], "k_raster", round(d["roofline"]["kernel_ms"], 5),
          {k: round(v["frames_per_s"]) for k, v in d["secondary"].items()}, cpu and (round(cpu["value"], 3), cpu["cores"], cpu["host_cpus"]))
EOF
