set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_relabel.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?; tail -3 gpurun_out/t5.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/t5.log | head -20; exit $rc; }
for arm in "DLR_LONG_SCHED=1" "DLR_LONG_SCHED=0"; do
  env $arm timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b5.json 2>gpurun_out/b5.err || { tail -5 gpurun_out/b5.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/b5.json').read().strip().splitlines()[-1]);print('$arm', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])"
done
