#!/usr/bin/env bash
# Round-3 measurement session (run from the repo root on the box): bench.py's rocprofv3 kernel
# trace + PMC passes (tools/profile.sh), the persistent engine's phase traces at cfg4 / cfg2 and
# every config's throughput (tools/configs_bench.py).  Every GPU step has its own time limit; any
# non-zero exit ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03p}
mkdir -p "$OUT"
run() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${TRACE:-1}" = 1 ] && run trace_cfg4 120 python3 tools/trace_persist.py --config cfg4
[ "${TRACE:-1}" = 1 ] && run trace_cfg2 120 python3 tools/trace_persist.py --config cfg2
[ "${CONFIGS:-1}" = 1 ] && run configs 300 python3 tools/configs_bench.py ${CONFIG_NAMES:-}
[ "${PROF:-1}" = 1 ] && run profile 900 bash tools/profile.sh
echo "=== done"
