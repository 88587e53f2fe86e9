# Same-box A/B of the batched partial reduction (part_reduce_all) against lib_diag prev: launch-
# engine parity, then tools/cfg5_bench.py and tools/isi_bench.py, two rounds.
set -o pipefail
OUT=${OUT:-gpurun_out/r5red}
mkdir -p $OUT
D=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bamp_scamp.py tests/test_gpu_shard_trials.py tests/test_gpu_cfg5.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vamp.py -k "launches or engines" > $OUT/tests_vl.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 tools/cfg5_bench.py > $OUT/cfg5_def_$r.log 2>&1 || exit 1
  AMP_LIB_PATH=$D timeout -k 10 200 python3 tools/cfg5_bench.py > $OUT/cfg5_prev_$r.log 2>&1 || exit 1
done
