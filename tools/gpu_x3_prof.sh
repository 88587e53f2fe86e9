# Launch-tile staging A/B: parity of the launch engines (BAMP / SCAMP / VAMP launches, cfg5, ISI),
# then kernel traces of tools/cfg5_bench.py (bf16x3 and f32 tiles) and tools/isi_bench.py.
# OUT=gpurun_out/<tag>
set -o pipefail
OUT=${OUT:-gpurun_out/r5x3d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bamp_scamp.py tests/test_gpu_cfg5.py tests/test_gpu_isi_model.py > $OUT/tests.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vamp.py -k "launches" > $OUT/tests_vl.log 2>&1 && \
AMP_BAMP_GEMM=x3 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_x3 -o run -- python3 tools/cfg5_bench.py > $OUT/x3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_f32 -o run -- python3 tools/cfg5_bench.py > $OUT/f32.log 2>&1 && \
timeout -k 10 300 python3 tools/isi_bench.py > $OUT/isi_f32.log 2>&1 && \
AMP_BAMP_GEMM=x3 AMP_SCAMP_LAUNCH_GEMM=x3 timeout -k 10 300 python3 tools/isi_bench.py > $OUT/isi_x3.log 2>&1
