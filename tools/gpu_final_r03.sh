#!/usr/bin/env bash
# Round-end session (run from the repo root on the box): the whole GPU test suite, smoke(),
# bench.py at its defaults, then tools/profile.sh (kernel trace + the PMC passes of the headline).
# Each GPU step has its own time limit; any non-zero exit ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p "$OUT"
run() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${TESTS:-1}" = 1 ] && run tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
[ "${SMOKE:-1}" = 1 ] && run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
[ "${BENCH:-1}" = 1 ] && run bench 300 python3 bench.py
[ "${PROF:-1}" = 1 ] && run profile 900 bash tools/profile.sh
echo "=== done"
