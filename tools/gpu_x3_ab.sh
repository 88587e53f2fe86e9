set -o pipefail
mkdir -p gpurun_out/r5x3a
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bamp_scamp.py -k "bamp_split" > gpurun_out/r5x3a/t_split.log 2>&1 || { echo split-fail; exit 1; }
timeout -k 10 300 python -u tools/cfg5_bench.py > gpurun_out/r5x3a/cfg5_f32.log 2>&1 && \
AMP_BAMP_GEMM=x3 timeout -k 10 300 python -u tools/cfg5_bench.py > gpurun_out/r5x3a/cfg5_x3.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cfg5.py tests/test_gpu_isi_model.py -k "x3" > gpurun_out/r5x3a/t_cfg5.log 2>&1
