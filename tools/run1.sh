set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_layouts.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?; tail -3 gpurun_out/t1.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config c4 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/b4.json 2>gpurun_out/b4.err || exit 1
timeout -k 10 200 python -u bench.py --config c5 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/b5.json 2>gpurun_out/b5.err || exit 1
timeout -k 10 200 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/btr.json 2>gpurun_out/btr.err || exit 1
python - <<'PY'
import json
for f in ["b4", "b5", "btr"]:
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"])
PY
