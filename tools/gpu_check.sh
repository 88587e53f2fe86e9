#!/usr/bin/env bash
# One GPU session: tests -> smoke -> bench (-> optional profile).  Every GPU step has its own
# time limit; a fault / abort / timeout (exit >= 124 or signal) ends the script at once.
# Ordinary test failures (pytest exit 1) do not stop the later steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
step() {  # step <name> <timeout> <cmd...>
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -5 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 5 ]; then
        echo "stopping after $name (rc=$rc)"; exit $rc
    fi
}
PYTEST_ARGS=${PYTEST_ARGS:-"tests -m gpu -q"}
[ "${SKIP_TESTS:-0}" = 1 ] || step tests 900 python -m pytest $PYTEST_ARGS
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-0}" = 1 ]; then
    export TMPDIR=/tmp
    step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 2
fi
echo "=== done"
