#!/bin/bash
# One GPU session on the box: a list of steps, each under its own time limit,
# chained so that the first failure ends the call (gpurun's rules: no retry,
# nothing after a fault).  Output under gpurun_out/<session>/.
#
#   bash tools/gpu_session.sh <session> <step> [<step> ...]
#
# steps:
#   suite[:<pytest -k expr>]     the -m gpu suite (or the tests matching expr)
#   tests:<path>[:<-k expr>]     one test file
#   smoke                        __graft_entry__.smoke()
#   bench:<name>:<bench args>    one bench.py line -> <name>.json (+ .err); prints value / frac
#   env:<name>:<VAR=V,...>:<bench args>   the same with extra environment
#   prof:<name>:<bench args>     rocprofv3 --kernel-trace --stats (csv) of a bench line
#   stamps:<c2|c4>[:<args>]      tools/c2_stamps.py / tools/c4_stamps.py (the DLR_STAMPS library)
#   pmc:<name>:<counters>:<bench args>   one rocprofv3 --pmc pass (its own run, 60 s limit)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
S="$1"
shift
OUT="gpurun_out/$S"
mkdir -p "$OUT"
export TMPDIR=/tmp

summary() {
    python3 - "$1" <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = j["roofline"]
print("   value %.4g samples/s  ms/step %.5f  frac %s  kernels %s  layout %s  order %s" % (
    j["value"], j["ms_per_step"], r["frac"], r["kernel_avg_us"], j["config"]["gradient_layout"],
    j["config"]["summation_order"][:9]))
PY
}

for step in "$@"; do
    kind="${step%%:*}"
    rest="${step#*:}"
    [ "$rest" = "$step" ] && rest=""
    echo "== $step"
    case "$kind" in
    suite)
        if [ -n "$rest" ]; then sel=(-k "$rest"); else sel=(); fi
        timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --durations=12 --timeout 600 \
            --timeout-method thread -p no:cacheprovider "${sel[@]}" > "$OUT/pytest.log" 2>&1
        rc=$?
        tail -15 "$OUT/pytest.log"
        [ $rc -eq 0 ] || exit $rc
        ;;
    tests)
        path="${rest%%:*}"
        expr="${rest#*:}"
        [ "$expr" = "$rest" ] && expr=""
        if [ -n "$expr" ]; then sel=(-k "$expr"); else sel=(); fi
        log="$OUT/$(basename "$path" .py).log"
        timeout -k 10 900 python -u -m pytest "$path" -x -v --timeout 600 --timeout-method thread \
            -p no:cacheprovider "${sel[@]}" > "$log" 2>&1
        rc=$?
        grep -E "PASSED|FAILED|ERROR|passed|failed" "$log" | tail -40
        [ $rc -eq 0 ] || exit $rc
        ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
        ;;
    bench)
        name="${rest%%:*}"
        args="${rest#*:}"
        timeout -k 10 600 python -u bench.py $args > "$OUT/$name.json" 2> "$OUT/$name.err" || {
            tail -5 "$OUT/$name.err"
            exit 1
        }
        summary "$OUT/$name.json"
        ;;
    env)
        name="${rest%%:*}"
        rest2="${rest#*:}"
        envs="${rest2%%:*}"
        args="${rest2#*:}"
        env ${envs//,/ } timeout -k 10 600 python -u bench.py $args > "$OUT/$name.json" 2> "$OUT/$name.err" || {
            tail -5 "$OUT/$name.err"
            exit 1
        }
        summary "$OUT/$name.json"
        ;;
    prof)
        name="${rest%%:*}"
        args="${rest#*:}"
        (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof_$name" \
            -o run -- python3 "$R/bench.py" $args > "$R/$OUT/prof_$name.log" 2>&1) || exit 1
        find "$R/$OUT/prof_$name" -name "*kernel_stats.csv" -exec head -8 {} \;
        ;;
    stamps)
        which="${rest%%:*}"
        args="${rest#*:}"
        [ "$args" = "$rest" ] && args=""
        timeout -k 10 400 python -u "tools/${which}_stamps.py" $args > "$OUT/stamps_$which.txt" 2>&1 || {
            tail -5 "$OUT/stamps_$which.txt"
            exit 1
        }
        cat "$OUT/stamps_$which.txt"
        ;;
    pmc)
        name="${rest%%:*}"
        rest2="${rest#*:}"
        ctrs="${rest2%%:*}"
        args="${rest2#*:}"
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc ${ctrs//,/ } --output-format csv -d "$R/$OUT/pmc_$name" \
            -o run -- python3 "$R/bench.py" $args > "$R/$OUT/pmc_$name.log" 2>&1) || exit 1
        ;;
    *)
        echo "unknown step $step"
        exit 2
        ;;
    esac
done
echo "session $S done"
