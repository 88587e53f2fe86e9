#!/usr/bin/env python3
"""Long-sequence (ISI / spatially coupled) detectors at the reference's published shape
(Simulations/SCAMP/QPSK,sparc/uniform,tail/Nt=128,Na=8,Nr=32,Lh=3,Lin=32: N = 4096, n = 1088),
launch engines: time per forward and the block-banded GEMMs' effect.  Run once as is and once
with AMP_BAND_GEMM=0 (the dense GEMMs) to compare; inputs from the reference's generators
(host replica, seed 0), resident in HBM.  Prints one JSON line per detector.
Roofline: the operator has Lin Lh nonzero Nr x Nt blocks (channel.py:89-91); per trial-iteration
SCAMP does two complex mat-vecs on them (A x, A^H s: 8 flop per complex MAC) and BAMP two complex
plus two real (|A|^2 var, |A|^2^T (1/u): 2 flop per MAC), priced against the fp32 MFMA peak
(157.3 TFLOP/s, MI355X_MICROARCH.md).
  python tools/isi_bench.py [B] [iterations]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import amp_native as nat  # noqa: E402
from bamp import BAMP  # noqa: E402
from channel import Channel  # noqa: E402
from config import Config  # noqa: E402
from data import Data  # noqa: E402
from scamp import SCAMP  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device('cuda:0')
    band = os.environ.get('AMP_BAND_GEMM', '1') != '0'
    for algo in ('scamp', 'bamp'):
        np.random.seed(0)
        torch.manual_seed(0)
        cfg = Config(128, 8, 32, 32, 3, batch=B, generator_mode='sparc', iterations=iters, alphabet='QPSK',
                     channel_profile='uniform', channel_truncation='tail', device='cpu')
        ch, da = Channel(cfg), Data(cfg)
        W, A = ch.generate_as_sparc()
        x, s, i = da.generate_message()
        SNR = cfg.snr(6.0)
        y = A @ x + ch.awgn(SNR)
        cfg.device = 'cuda'
        mv = lambda t: t.to(dev).contiguous()  # noqa: E731
        lab = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int64)).to(dev)  # noqa: E731
        if algo == 'scamp':
            det, args = SCAMP(cfg), (mv(W), mv(A), mv(y), SNR, mv(x), lab(s), lab(i))
        else:
            det, args = BAMP(cfg), (mv(A), mv(y), SNR, mv(x), lab(s), lab(i))
        L = det(*args)
        L.resolve()
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            L = det(*args)
        L.resolve()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        T = int(L.loss['T'])
        nz = 32 * 3 * 32 * 128                      # Lin Lh Nr Nt nonzero complex entries
        flop = nz * (2 * 8 if algo == 'scamp' else 2 * 8 + 2 * 2)
        tf = flop * B / (ms / T * 1e-3) / 1e12
        print(json.dumps({'algo': algo, 'shape': 'Nt=128 Na=8 Nr=32 Lin=32 Lh=3 QPSK (N=4096, n=1088)', 'B': B,
                          'EbN0': 6.0, 'band_gemm': band, 'T': T, 'fer': float(L.loss['fer']),
                          'ver': float(L.loss['ver']), 'ser': float(L.loss['ser']), 'ms_per_forward': round(ms, 3),
                          'ms_per_iteration': round(ms / T, 4),
                          'nz_mflop_per_trial_iteration': round(flop / 1e6, 3), 'tflops_nonzero': round(tf, 2),
                          'frac_fp32_peak': round(tf / 157.3, 4)}), flush=True)
    nat.unload()


if __name__ == '__main__':
    main()
