set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?; tail -3 gpurun_out/t2.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 1000 --warmup 20 --no-cpu-baseline > gpurun_out/b2.json 2>gpurun_out/b2.err || exit 1
python - <<'PY'
import json
for f in ["b2"]:
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"], d["roofline"].get("step_breakdown_us"))
PY
