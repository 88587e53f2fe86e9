# Diagnostic: where the bf16x3 launch tile's time goes (cfg5, AMP_BAMP_GEMM=x3): kernel traces of
# the default library and of lib_diag builds without the MFMAs (AMP_X3T_NOMMA) or without the
# operator stream (AMP_X3T_NOWLOAD); their results are wrong by construction.  OUT=gpurun_out/<tag>
set -o pipefail
OUT=${OUT:-gpurun_out/r5x3diag}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=amp-sparc-spatialmodulation_amd/lib_diag
AMP_BAMP_GEMM=x3 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/def -o run -- python3 tools/cfg5_bench.py > $OUT/def.log 2>&1 && \
AMP_BAMP_GEMM=x3 AMP_LIB_PATH=$D/libampsparc_nomma.so timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/nomma -o run -- python3 tools/cfg5_bench.py > $OUT/nomma.log 2>&1 && \
AMP_BAMP_GEMM=x3 AMP_LIB_PATH=$D/libampsparc_nowload.so timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/nowload -o run -- python3 tools/cfg5_bench.py > $OUT/nowload.log 2>&1
