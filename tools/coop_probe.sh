#!/usr/bin/env bash
# Cooperative-launch check for the persistent engines: GPU tests of the persistent paths with
# AMP_PERSIST_LAUNCH=coop, then one forward under rocprofv3 with and without the explicit unload.
# Every step has its own limit; any failure ends the script (nothing more runs on the GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/coop; mkdir -p $O
step() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "$O/$name.log"
    [ $rc -ne 0 ] && exit $rc
    return 0
}
export AMP_PERSIST_LAUNCH=coop
step tests 600 python -u -m pytest tests/test_gpu_vamp.py tests/test_gpu_bamp_scamp.py -m gpu -q -x --timeout 120 --timeout-method thread
step bench 300 python bench.py --no-cpu-baseline
step prof_unload 150 rocprofv3 --kernel-trace --stats -d $O/pu -o p --output-format csv -- python3 tools/exit_probe.py persistent profile unload
step prof_plain 150 rocprofv3 --kernel-trace --stats -d $O/pp -o p --output-format csv -- python3 tools/exit_probe.py persistent profile keep
echo "=== done"
