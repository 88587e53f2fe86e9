#!/usr/bin/env python3
"""BASELINE cfg5 shape on one MI355X: BAMP Nt=512 Nr=1024 Na=16, B=8192 trials, on the
correlated channel (rho = 0.5): 64-QAM as named (injected into Config, which rejects it like the
reference, exactly as tests/cfg5_inputs.py does) and its QPSK / 16-QAM twins.

Times `amp_bamp_run` (detector iterations only: 5 GEMM-class launches per iteration) and the
whole forward (+ GPU decision / counters + the 256-byte readback) with HIP events on the stream
the work runs on; inputs resident in HBM.  Algorithmic work per trial-iteration (SURVEY.md
§8(d), BAMP): 20 n N flop = 10,485,760 and 24N + 32n + 12nN/B bytes = 45,824 B at cfg5.
Prints one JSON line per alphabet."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import amp_native as nat  # noqa: E402
from bamp import BAMP  # noqa: E402
from channel import Channel  # noqa: E402
from config import Config  # noqa: E402
from data import Data  # noqa: E402

Nt, Na, Nr, B = 512, 16, 1024, 8192
FLOP_TI = 20.0 * Nr * Nt
BYTES_TI = 24 * Nt + 32 * Nr + 12 * Nr * Nt / B
PEAK_TF = 157.3


def main():
    dev = torch.device('cuda:0')
    for alph, ebn0 in (('64QAM', 16.0), ('QPSK', 2.0), ('16QAM', 10.0)):
        cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=20,
                     alphabet='16QAM' if alph == '64QAM' else alph,
                     channel_profile='uniform', channel_truncation='tail', device='cpu')
        if alph == '64QAM':
            cfg.inject_square_qam(64)
        np.random.seed(0)
        torch.manual_seed(0)
        ch, da = Channel(cfg), Data(cfg)
        A = ch.generate_correlated(0.5)
        x, sym, idx = da.generate_message()
        SNR = cfg.snr(ebn0)
        y = A @ x + ch.awgn(SNR)
        cfg.device = 'cuda'
        A, x, y = A.to(dev), x.to(dev), y.to(dev)
        det = BAMP(cfg)
        st = torch.cuda.current_stream()
        for _ in range(3):
            L = det(A, y, SNR, x, sym, idx)
        T = int(L.loss['T'])
        reps = 10
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(st)
        for _ in range(reps):
            det.detect(A, y, SNR)
        e[1].record(st)
        torch.cuda.synchronize()
        e[2].record(st)
        for _ in range(reps):
            L = det(A, y, SNR, x, sym, idx)
        e[3].record(st)
        torch.cuda.synchronize()
        det_ms = e[0].elapsed_time(e[1]) / reps
        fwd_ms = e[2].elapsed_time(e[3]) / reps
        tflops = B * T * FLOP_TI / (det_ms * 1e-3) / 1e12
        print(json.dumps({'workload': f'cfg5 shape: BAMP Nt={Nt} Nr={Nr} Na={Na} {alph} B={B}, correlated rho=0.5, '
                                      f'EbN0={ebn0} dB', 'T': T, 'ver': float(L.loss['ver']),
                          'ser': float(L.loss['ser']), 'detector_ms': round(det_ms, 4),
                          'forward_ms': round(fwd_ms, 4), 'symbol_vectors_per_s': B / (fwd_ms * 1e-3),
                          'trial_iterations_per_s': B * T / (det_ms * 1e-3),
                          'achieved_TFLOPs': round(tflops, 2), 'peak_TFLOPs': PEAK_TF,
                          'mfma_frac': round(tflops / PEAK_TF, 3),
                          'algorithmic_GBs': round(B * T * BYTES_TI / (det_ms * 1e-3) / 1e9, 1)}), flush=True)
    nat.unload()


if __name__ == '__main__':
    main()
