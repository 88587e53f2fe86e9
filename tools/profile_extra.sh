#!/usr/bin/env bash
# Kernel-trace sessions for the round's secondary workloads (run from the repo root on the box):
#   steady-state cfg4 bench (default warmup, so the average is past the clock ramp),
#   the cfg5-shape BAMP tool and the Shrink kernel tool.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof2
mkdir -p "$OUT"
run() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run kt 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 30
run cfg5 600 rocprofv3 --kernel-trace --stats -d "$OUT/cfg5" -o cfg5 --output-format csv -- python3 tools/cfg5_bench.py
run shrink 600 rocprofv3 --kernel-trace --stats -d "$OUT/shrink" -o shrink --output-format csv -- python3 tools/shrink_bench.py
echo "=== done"
