set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t4.log 2>&1; rc=$?; tail -3 gpurun_out/t4.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t4.log | head -20; exit $rc; }
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/b3.json 2>gpurun_out/b3.err || { tail -5 gpurun_out/b3.err; exit 1; }
DLR_RELABEL=0 timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/b3n.json 2>gpurun_out/b3n.err || { tail -5 gpurun_out/b3n.err; exit 1; }
python - <<'PY'
import json
for f in ["b3", "b3n"]:
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["frac"], r.get("kernel_avg_us"))
PY
grep "rank 0" gpurun_out/b3.err gpurun_out/b3n.err
