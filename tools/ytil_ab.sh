#!/usr/bin/env bash
# Same-box A/B of the y~ launch: rocprofv3 kernel trace of bench.py with the shipped library and with
# lib_diag/libampsparc_prev.so, twice each, plus the y~ bit-identity test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ytil}; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_vamp.py -m gpu -k "ytil or engines_agree or n256 or reproducible" > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -20 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for v in def prev def2 prev2; do
  L=""; case $v in prev*) L="AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_prev.so";; esac
  if [ -n "$L" ]; then export AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_prev.so; else unset AMP_LIB_PATH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o kt --output-format csv -- python3 bench.py --no-cpu-baseline > "$OUT/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/$v.log"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$v.log") $(grep -h 'ytil\|build_cweights\|vamp_persist' "$OUT"/$v/*kernel_stats.csv | awk -F, '{print $1, $4}' | tr '\n' ' ')"
done
