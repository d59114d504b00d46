# A/B of environment settings on the default bench (value only, no rocprof):
#   ARMS="DLR_PREFETCH=0 DLR_PREFETCH=1" bash tools/ab_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abenv
i=0
for rep in 1 2; do
for arm in ${ARMS:-base}; do
  i=$((i+1))
  ( [ "$arm" = base ] || export $arm
    timeout -k 10 200 python -u bench.py ${BENCH_ARGS:---steps 1000 --warmup 50} --no-cpu-baseline > gpurun_out/abenv/arm$i.json 2> gpurun_out/abenv/arm$i.err ) || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/abenv/arm$i.json').read().strip().splitlines()[-1]);print('$arm', d['value'], d['ms_per_step'], d['roofline'].get('kernel_avg_us'))"
done
done
