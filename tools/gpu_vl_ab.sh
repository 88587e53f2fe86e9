# Same-box A/B of the VAMP launch engine (bench.py --engine launches, cfg4) against lib_diag prev,
# after the launch-engine parity tests.
set -o pipefail
OUT=${OUT:-gpurun_out/r5vl}
mkdir -p $OUT
D=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vamp.py -k "launches or engines" > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --engine launches > $OUT/def_$r.log 2>&1 || exit 1
  AMP_LIB_PATH=$D timeout -k 10 200 python3 bench.py --no-cpu-baseline --engine launches > $OUT/prev_$r.log 2>&1 || exit 1
done
