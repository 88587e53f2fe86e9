#!/usr/bin/env bash
# Cross-compiles the micro-benchmarks for gfx950 into tools/ubench/bin (run on the box by run.sh).
set -eu
cd "$(dirname "$0")"
mkdir -p bin
H="/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -w"
$H -o bin/valu_rate valu_rate.hip
$H -shared -fPIC -o bin/libdenoise_ubench.so denoise_ubench.hip
$H -o bin/pk_occ2 pk_occ2.hip
$H -o bin/gemm_x3 gemm_x3_ubench.hip
$H -o bin/gemm_h2 gemm_h2_ubench.hip
$H -o bin/gemm_i8 gemm_i8_ubench.hip
$H -o bin/pk_dpp pk_dpp.hip
$H -o bin/trans_pk trans_pk.hip
$H -o bin/pair pair_ubench.hip
$H -o bin/mfma_rd mfma_rd.hip
$H -o bin/store_war store_war.hip
