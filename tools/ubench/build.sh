#!/usr/bin/env bash
# Cross-compiles the micro-benchmarks for gfx950 into tools/ubench/bin (run on the box by run.sh).
set -eu
cd "$(dirname "$0")"
mkdir -p bin
H="/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -w"
$H -o bin/valu_rate valu_rate.hip
$H -shared -fPIC -o bin/libdenoise_ubench.so denoise_ubench.hip
