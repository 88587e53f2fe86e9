#!/usr/bin/env bash
# Runs the prebuilt micro-benchmarks (built in the container by tools/ubench/build.sh).
set -eu
cd "$(dirname "$0")"
./bin/valu_rate
python3 -c "import ctypes; ctypes.CDLL('./bin/libdenoise_ubench.so').ubench_main()"
