#!/bin/bash
# One GPU session: the -m gpu suite, then (only if it did not crash / time out) the bench.
# Exit statuses >= 124 (timeout, abort, segfault) end the session: nothing more runs on the GPU.
# Usage: tools/gpu_run.sh TAG [pytest-args...]
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests.log
if [ $rc -ge 124 ]; then echo "GPU step ended abnormally ($rc): stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -1 gpurun_out/${TAG}_bench.log
exit $(( rc > rc2 ? rc : rc2 ))
