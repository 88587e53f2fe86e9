#!/usr/bin/env bash
# rocprofv3 session for bench.py: kernel trace + stats, then separate PMC passes for HBM
# traffic (FETCH_SIZE, WRITE_SIZE; one counter group per pass as MI355X_MICROARCH.md says).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${PROF_TAG:-prof}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --steps 5 --warmup 1"}
run() {
    local name=$1 lim=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"; tail -3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run kt 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- python3 bench.py $ARGS
[ "${PMC:-1}" = 1 ] || exit 0
run fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --prewarm-ms 0
run write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --prewarm-ms 0
[ "${SQ:-1}" = 1 ] || { echo "=== done"; exit 0; }
run sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d "$OUT/sq" -o sq --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --prewarm-ms 0
run grbm 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES -d "$OUT/grbm" -o grbm --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --prewarm-ms 0
echo "=== done"
