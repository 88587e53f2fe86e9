#!/usr/bin/env bash
# GPU session for the bf16x3 persistent engine: -m gpu suite, smoke, bench, phase traces (x3
# and f32 A/B at cfg4 / cfg2).  Every GPU step has its own limit; a crash ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-x3}
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ge 124 ] || [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${TESTS:-1}" = 1 ] && step tests 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step trace_cfg4 120 python3 tools/trace_persist.py --config cfg4
step trace_cfg2 120 python3 tools/trace_persist.py --config cfg2
AMP_VAMP_GEMM=f32 step trace_cfg4_f32 120 python3 tools/trace_persist.py --config cfg4
echo "=== done"
