set -o pipefail
OUT=gpurun_out/r5c27
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bamp_scamp.py tests/test_gpu_shard_trials.py > $OUT/tests.log 2>&1 && \
timeout -k 10 300 python3 tools/configs_bench.py cfg3 cfg3-qpsk > $OUT/cfg3.log 2>&1 && \
AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_old.so timeout -k 10 300 python3 tools/configs_bench.py cfg3 cfg3-qpsk > $OUT/cfg3_old.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof5 -o run -- python3 tools/cfg5_bench.py > $OUT/cfg5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r5c27/profisi -o run -- python3 tools/isi_bench.py > gpurun_out/r5c27/isi.log 2>&1
