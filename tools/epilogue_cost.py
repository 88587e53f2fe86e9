#!/usr/bin/env python3
"""Diagnostic (GPU): what the end of a cfg4 forward costs beyond the iteration loop.

Times, with HIP events on the detector's stream, back-to-back forwards of the bench workload as
(a) VAMP.detect (amp_vamp_run: prepare + the persistent loop + the r / xmmse / var outputs, no
decision) and (b) the fused VAMP.forward (amp_vamp_detect_count: the same plus the MAP decision
and counters in the kernel's epilogue and the in-kernel counter fold), so (b) - (a) is the fused
decision's cost per forward.

  python tools/epilogue_cost.py [--reps 50]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..'), os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=50)
    a = ap.parse_args()
    from config import Config
    from vamp import VAMP
    dev = torch.device('cuda', 0)
    Nt, Na, Nr, B, alph, iters = bench.CONFIGS['cfg4']
    cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=iters, alphabet=alph,
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    inp = bench.make_inputs(cfg, 0, 8.0, dev)
    det = VAMP(cfg)
    args = (inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])

    def timed(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    t_detect = timed(lambda: det.detect(*args))
    t_fused = timed(lambda: det(*args, inp['x'], inp['sym'], inp['idx']))
    det.L.resolve()
    print(f'cfg4 B={B}: detect (loop + outputs) {t_detect * 1e3:.1f} us, fused forward (+ decision, counters) '
          f'{t_fused * 1e3:.1f} us, difference {(t_fused - t_detect) * 1e3:.1f} us per forward', flush=True)


if __name__ == '__main__':
    main()
