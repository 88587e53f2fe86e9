#!/usr/bin/env bash
# Round-2 measurement session (run from the repo root on the box): per-config throughput,
# persistent-engine phase traces at cfg2 / cfg4, kernel-trace summaries of the secondary
# configs (cfg2 VAMP, cfg3 SCAMP) and one SQ PMC pass on each of them.
# Every GPU step has its own time limit; any non-zero exit ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02p}
mkdir -p "$OUT"
run() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${CONFIGS:-1}" = 1 ] && run configs 300 python3 tools/configs_bench.py
[ "${TRACE:-1}" = 1 ] && run trace_cfg2 120 python3 tools/trace_persist.py --config cfg2
[ "${TRACE:-1}" = 1 ] && run trace_cfg4 120 python3 tools/trace_persist.py --config cfg4
if [ "${KT:-1}" = 1 ]; then
    run kt_cfg2 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_cfg2" -o kt --output-format csv -- python3 tools/configs_bench.py cfg2
    run kt_cfg3 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_cfg3" -o kt --output-format csv -- python3 tools/configs_bench.py cfg3 cfg3-qpsk
fi
if [ "${SQ:-1}" = 1 ]; then
    C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
    run sq_cfg2 120 rocprofv3 --pmc $C -d "$OUT/sq_cfg2" -o sq --output-format csv -- python3 tools/configs_bench.py cfg2
    run sq_cfg3 120 rocprofv3 --pmc $C -d "$OUT/sq_cfg3" -o sq --output-format csv -- python3 tools/configs_bench.py cfg3
fi
echo "=== done"
