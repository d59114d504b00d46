set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?; tail -3 gpurun_out/t3.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c4s --no-cpu-baseline > gpurun_out/b4s.json 2>gpurun_out/b4s.err || { tail -5 gpurun_out/b4s.err; exit 1; }
timeout -k 10 200 python -u bench.py --config c4 --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/b4.json 2>gpurun_out/b4.err || exit 1
python - <<'PY'
import json
for f in ["b4s", "b4"]:
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["bound"], r["achieved"], r["frac"], r.get("step_breakdown_us"))
PY
cat gpurun_out/b4s.err | tail -3
