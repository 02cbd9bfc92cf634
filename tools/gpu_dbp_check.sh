set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_band_dbp.py tests/test_multidevice_gpu.py -x -q -s -m gpu --timeout 120 --timeout-method thread > gpurun_out/dbp_gpu.log 2>&1 || { tail -40 gpurun_out/dbp_gpu.log; exit 1; }
tail -3 gpurun_out/dbp_gpu.log
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for r in 1 7; do timeout -k 10 200 python -u bench.py --steps 300 --warmup 50 --no-secondary --sim-world 8 --sim-rank $r > gpurun_out/sim8_r$r.json 2> gpurun_out/sim8_r$r.err || { tail -20 gpurun_out/sim8_r$r.err; exit 1; }; done
python - <<'P'
import json
for r in (1,7):
    d=json.loads(open(f"gpurun_out/sim8_r{r}.json").read().strip().splitlines()[-1])
    print(r, d["value"], json.dumps(d.get("assembly")))
P
