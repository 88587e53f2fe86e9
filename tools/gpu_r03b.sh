#!/usr/bin/env bash
# Round-3 verification session (run from the repo root on the box): GPU tests of the engines the
# last changes touched, cfg5 throughput, the per-phase LDS attribution (tools/ubench), the headline
# kernel's LDS counters, bench.py, and the ISI-shape kernel trace.  Each GPU step has its own time
# limit; any non-zero exit ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03b}
mkdir -p "$OUT"
run() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -4 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
[ "${TESTS:-1}" = 1 ] && run tests 700 python3 -u -m pytest ${TEST_FILES:-tests/test_gpu_vamp.py tests/test_gpu_bamp_scamp.py tests/test_gpu_cfg5.py tests/test_gpu_shard_trials.py tests/test_gpu_isi_model.py tests/test_gpu_random.py tests/test_gpu_segmented.py} -m gpu -q -x --timeout 300 --timeout-method thread
[ "${CFG5:-1}" = 1 ] && run cfg5 300 python3 tools/cfg5_bench.py
[ "${LDS:-1}" = 1 ] && run lds 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d "$OUT/lds" -o lds --output-format csv -- tools/ubench/bin/lds_phase
[ "${LDS:-1}" = 1 ] && run lds_sum 30 python3 tools/lds_phase_summary.py "$OUT/lds"
[ "${SQ:-1}" = 1 ] && run sq 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d "$OUT/sq" -o sq --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --prewarm-ms 0
[ "${BENCH:-1}" = 1 ] && run bench 300 python3 bench.py
[ "${ISI:-1}" = 1 ] && run isi 300 rocprofv3 --kernel-trace --stats -d "$OUT/isi" -o isi --output-format csv -- python3 tools/isi_bench.py 512 50
echo "=== done"
