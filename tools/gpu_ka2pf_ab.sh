# Same-box A/B: bamp_ka2 epilogue loads issued before the GEMM (default) against after it
# (lib_diag nopf, -DAMP_KA2_PF=0); cfg5 and the ISI shape, two rounds, parity subset first.
set -o pipefail
OUT=${OUT:-gpurun_out/r5pf}
mkdir -p $OUT
D=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_nopf.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bamp_scamp.py tests/test_gpu_cfg5.py tests/test_gpu_isi_model.py -k "bamp or cfg5" > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 tools/cfg5_bench.py > $OUT/cfg5_def_$r.log 2>&1 || exit 1
  AMP_LIB_PATH=$D timeout -k 10 200 python3 tools/cfg5_bench.py > $OUT/cfg5_nopf_$r.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/isi_bench.py > $OUT/isi_def_$r.log 2>&1 || exit 1
  AMP_LIB_PATH=$D timeout -k 10 200 python3 tools/isi_bench.py > $OUT/isi_nopf_$r.log 2>&1 || exit 1
done
