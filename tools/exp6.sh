set -u
mkdir -p gpurun_out/exp6
for u in 2 4 8; do for c in cfg2 cfg4; do AMP_DEN_U=$u timeout -k 10 120 python3 tools/trace_persist.py --config $c > gpurun_out/exp6/u${u}_$c.log 2>&1 || exit $?; done; done
for u in 2 4 8; do for c in cfg2 cfg4; do echo "U=$u $c"; grep "per iteration\|denoiser" gpurun_out/exp6/u${u}_$c.log; done; done
