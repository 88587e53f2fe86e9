set -u
T=${TAG:-exp2}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?
tail -3 gpurun_out/$T/tests.log
[ $rc -ge 124 ] && exit $rc
for c in cfg2 cfg4; do timeout -k 10 120 python3 tools/trace_persist.py --config $c > gpurun_out/$T/trace_$c.log 2>&1 || exit $?; done
timeout -k 10 300 python3 tools/configs_bench.py > gpurun_out/$T/configs.log 2>&1 || exit $?
cat gpurun_out/$T/trace_*.log | grep -v amdgpu.ids
grep config gpurun_out/$T/configs.log | cut -c1-60,200-420
timeout -k 10 300 python3 tools/cfg5_bench.py > gpurun_out/$T/cfg5.log 2>&1; tail -3 gpurun_out/$T/cfg5.log; AMP_GRID_DENOISER=0 timeout -k 10 300 python3 tools/cfg5_bench.py > gpurun_out/$T/cfg5_nogrid.log 2>&1; tail -3 gpurun_out/$T/cfg5_nogrid.log; AMP_GRID_DENOISER=0 timeout -k 10 300 python3 tools/configs_bench.py cfg2 cfg3 cfg4 > gpurun_out/$T/configs_nogrid.log 2>&1
grep config gpurun_out/$T/configs_nogrid.log | cut -c1-60,200-420
exit $rc
