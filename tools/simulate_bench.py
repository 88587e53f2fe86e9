#!/usr/bin/env python3
"""End-to-end Model.simulate throughput (epochs/s and symbol-vectors/s including input
generation), parity mode (rng='host': the reference's numpy / torch-CPU streams, LAPACK SVD)
against throughput mode (rng='device': channel, messages, noise and SVD on the GPU).

  python tools/simulate_bench.py [--config cfg4] [--epochs 8] [--res 1] [--ebn0 8]
"""
import argparse
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd'))
sys.path.insert(0, REPO)

import json  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    from config import Config
    from model import Model
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='cfg4')
    ap.add_argument('--epochs', type=int, default=8)
    ap.add_argument('--res', type=int, default=1)
    ap.add_argument('--ebn0', type=float, default=8.0)
    args = ap.parse_args()
    Nt, Na, Nr, B, alph, iters = bench.CONFIGS[args.config]
    out = {}
    for rng in ('host', 'device'):
        cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=iters, alphabet=alph,
                     channel_profile='uniform', channel_truncation='tail', device='cuda')
        with tempfile.TemporaryDirectory() as d:
            m = Model(cfg, 'vamp', path=d, seed=0, rng=rng)
            m.simulate(1, start=args.ebn0, final=args.ebn0, res=args.res)          # warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = m.simulate(args.epochs, start=args.ebn0, final=args.ebn0, res=args.res)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        out[rng] = dict(epochs_per_s=args.epochs / dt, symbol_vectors_per_s=args.epochs * B / dt,
                        ver=res[-1]['ver'], ser=res[-1]['ser'], T=res[-1]['T'])
    print(json.dumps(dict(config=args.config, epochs=args.epochs, res=args.res, ebn0=args.ebn0, **out)))


if __name__ == '__main__':
    main()
