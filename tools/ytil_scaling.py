#!/usr/bin/env python3
"""Diagnostic (GPU, run under rocprofv3 --kernel-trace): the y~ launch of the bf16x3 engine at
several batch sizes of the cfg4 shape (ten forwards each), so its duration per B shows whether it
scales with the work (a throughput bound) or not (a latency / startup bound).

  rocprofv3 --kernel-trace --stats -d out -o yt -- python3 tools/ytil_scaling.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..'), os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from config import Config
    from vamp import VAMP
    dev = torch.device('cuda', 0)
    Nt, Na, Nr, _, alph, _ = bench.CONFIGS['cfg4']
    for B in (512, 1024, 2048, 4096):
        cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=1, alphabet=alph,
                     channel_profile='uniform', channel_truncation='tail', device='cuda')
        inp = bench.make_inputs(cfg, 0, 8.0, dev)
        det = VAMP(cfg)
        for _ in range(10):
            det.detect(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])
        torch.cuda.synchronize()
        print('B', B, 'done', flush=True)


if __name__ == '__main__':
    main()
