# Same-box A/B of the launch tiles: default, lib_diag old (the tree before the staging change),
# and the bf16x3 launch tiles (AMP_BAMP_GEMM=x3 AMP_SCAMP_LAUNCH_GEMM=x3); tools/cfg5_bench.py and
# tools/isi_bench.py, two rounds, after the launch-engine parity tests.  OUT=gpurun_out/<tag>
set -o pipefail
OUT=${OUT:-gpurun_out/r5ab}
mkdir -p $OUT
D=amp-sparc-spatialmodulation_amd/lib_diag
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bamp_scamp.py tests/test_gpu_cfg5.py tests/test_gpu_isi_model.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vamp.py -k "launches" > $OUT/tests_vl.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 tools/cfg5_bench.py > $OUT/cfg5_def_$r.log 2>&1 || exit 1
  AMP_LIB_PATH=$D/libampsparc_old.so timeout -k 10 200 python3 tools/cfg5_bench.py > $OUT/cfg5_old_$r.log 2>&1 || exit 1
  AMP_BAMP_GEMM=x3 timeout -k 10 200 python3 tools/cfg5_bench.py > $OUT/cfg5_x3_$r.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/isi_bench.py > $OUT/isi_def_$r.log 2>&1 || exit 1
  AMP_LIB_PATH=$D/libampsparc_old.so timeout -k 10 200 python3 tools/isi_bench.py > $OUT/isi_old_$r.log 2>&1 || exit 1
  AMP_BAMP_GEMM=x3 AMP_SCAMP_LAUNCH_GEMM=x3 timeout -k 10 200 python3 tools/isi_bench.py > $OUT/isi_x3_$r.log 2>&1 || exit 1
done
