#!/usr/bin/env python3
"""Throughput of every BASELINE config on one MI355X (bench.py measures only the headline cfg4).

cfg1 BAMP Nt=4 Nr=8 Na=1 QPSK B=100 T<=10 (the reference's CPU-plumbing case: launch-bound)
cfg2 VAMP Nt=64 Nr=128 Na=4 16-QAM B=1024 T<=20
cfg3 SCAMP Nt=128 Nr=256 Na=8 16-QAM B=4096 T<=20
cfg4 VAMP Nt=256 Nr=512 Na=8 16-QAM B=4096 T<=20 (bench.py's workload; repeated for reference)
(cfg5: tools/cfg5_bench.py.)  Inputs: the reference's generators on the host replica, resident
in HBM.  Each forward (detector + GPU decision + 256-byte readback) is timed over 50 epochs
after 30 warm-up epochs; algorithmic flops per trial-iteration from SURVEY.md §8(d):
VAMP 16 N k, SCAMP 16 n N, BAMP 20 n N.  Prints one JSON line per config."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import amp_native as nat  # noqa: E402
from bamp import BAMP  # noqa: E402
from channel import Channel  # noqa: E402
from config import Config  # noqa: E402
from data import Data  # noqa: E402
from scamp import SCAMP  # noqa: E402
from vamp import VAMP  # noqa: E402

PEAK_TF = 157.3
CFGS = {
    'cfg1': ('bamp', 4, 1, 8, 100, 'QPSK', 10, 8.0),
    'cfg2': ('vamp', 64, 4, 128, 1024, '16QAM', 20, 8.0),
    'cfg3': ('scamp', 128, 8, 256, 4096, '16QAM', 20, 8.0),
    'cfg3-launches': ('scamp', 128, 8, 256, 4096, '16QAM', 20, 8.0),   # the launch engine, for comparison
    'cfg3-qpsk': ('scamp', 128, 8, 256, 4096, 'QPSK', 20, 2.0),
    'cfg4': ('vamp', 256, 8, 512, 4096, '16QAM', 20, 8.0),
    # cfg2 with the 4 epochs of one res = 4 block side by side (VAMP.forward_epochs: 256 workgroups)
    'cfg2-epochs4': ('vamp', 64, 4, 128, 1024, '16QAM', 20, 8.0),
    # 8 epochs: two workgroups per CU, diagnostic build only since round 6 (AMP_EPOCHS_TWO_PER_CU=1)
    'cfg2-epochs8': ('vamp', 64, 4, 128, 1024, '16QAM', 20, 8.0),
    # cfg2 at the reference's default res = 1: max_epochs (4; 8 at two per CU) epochs with a channel
    # each side by side
    # (amp_vamp_detect_count_epochs_ch); the inputs include each epoch's own SVD factors
    'cfg2-res1': ('vamp', 64, 4, 128, 1024, '16QAM', 20, 8.0),
}
EPOCHS = {'cfg2-epochs4': 4, 'cfg2-epochs8': 8, 'cfg2-res1': 8}


def main(steps=50, warmup=30, only=None):
    dev = torch.device('cuda:0')
    for name, (algo, Nt, Na, Nr, B, alph, iters, ebn0) in CFGS.items():
        if only and name not in only:
            continue
        cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=iters, alphabet=alph,
                     channel_profile='uniform', channel_truncation='tail', device='cpu')
        np.random.seed(0)
        torch.manual_seed(0)
        ch, da = Channel(cfg), Data(cfg)
        W, A = ch.generate_as_sparc()
        x, sym, idx = da.generate_message()
        SNR = cfg.snr(ebn0)
        y = A @ x + ch.awgn(SNR)
        cfg.device = 'cuda'
        mv = lambda t: t.to(dev).contiguous()  # noqa: E731
        lab = lambda a: torch.as_tensor(np.asarray(a, dtype=np.int64)).to(dev)  # noqa: E731  (resident in HBM)
        sym, idx = lab(sym), lab(idx)
        E = EPOCHS.get(name, 1)
        if E > 1:
            cap = VAMP(cfg).max_epochs(Nt)
            if E > cap:   # two workgroups per CU: diagnostic build only (AMP_EPOCHS_TWO_PER_CU=1)
                if name == 'cfg2-epochs8':
                    print(json.dumps({'config': name, 'skipped': f'{E} epochs need two workgroups per CU '
                                      f'(max_epochs {cap})'}), flush=True)
                    continue
                E = cap
            res1 = name.endswith('res1')
            eps = [(x, sym, idx, y)]
            chans = [torch.linalg.svd(A, full_matrices=False)]
            for _ in range(E - 1):
                if res1:
                    _, A = ch.generate_as_sparc()
                    chans.append(torch.linalg.svd(A, full_matrices=False))
                xe, se, ie = da.generate_message()
                eps.append((xe, lab(se), lab(ie), A @ xe + ch.awgn(SNR)))
            if res1:   # stacked [E, ...] channel factors: one channel per epoch
                U, s, Vh = (torch.stack([c[i] for c in chans]) for i in range(3))
            else:
                U, s, Vh = chans[0]
            det = VAMP(cfg)
            # the epochs' inputs stacked [E, B, ...] in HBM (forward_epochs uses them without a copy)
            ea = (mv(U), mv(s), mv(Vh), torch.stack([mv(e[3]) for e in eps]), SNR,
                  torch.stack([mv(e[0]) for e in eps]), torch.stack([e[1] for e in eps]),
                  torch.stack([e[2] for e in eps]))
            flop = 16.0 * Nt * min(Nt, Nr)
            for _ in range(warmup):
                Ls = det.forward_epochs(*ea)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                Ls = det.forward_epochs(*ea)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            Ts = [int(L.loss['T']) for L in Ls]
            tf = B * sum(Ts) * flop / (ms * 1e-3) / 1e12
            print(json.dumps({'config': name, 'algo': algo, 'engine': 'persistent (side-by-side epochs)',
                              'channels': E if res1 else 1,
                              'epochs_per_launch': E, 'Nt': Nt, 'Nr': Nr, 'Na': Na, 'alphabet': alph, 'B': B,
                              'EbN0': ebn0, 'T': Ts, 'ser': [float(L.loss['ser']) for L in Ls],
                              'ms_per_launch': round(ms, 4), 'ms_per_epoch': round(ms / E, 4),
                              'symbol_vectors_per_s': E * B / (ms * 1e-3),
                              'trial_iterations_per_s': B * sum(Ts) / (ms * 1e-3), 'achieved_TFLOPs': round(tf, 2),
                              'mfma_frac_incl_decision': round(tf / PEAK_TF, 4)}), flush=True)
            continue
        if algo == 'vamp':
            U, s, Vh = torch.linalg.svd(A, full_matrices=False)
            det, args = VAMP(cfg), (mv(U), mv(s), mv(Vh), mv(y), SNR, mv(x), sym, idx)
            flop = 16.0 * Nt * min(Nt, Nr)
        elif algo == 'scamp':
            eng = nat.ENGINE_LAUNCHES if name.endswith('launches') else nat.ENGINE_AUTO
            det, args = SCAMP(cfg, engine=eng), (mv(W), mv(A), mv(y), SNR, mv(x), sym, idx)
            flop = 16.0 * Nr * Nt
        else:
            det, args = BAMP(cfg), (mv(A), mv(y), SNR, mv(x), sym, idx)
            flop = 20.0 * Nr * Nt
        for _ in range(warmup):
            L = det(*args)
        L.resolve()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            L = det(*args)
        L.resolve()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        T = int(L.loss['T'])
        tf = B * T * flop / (ms * 1e-3) / 1e12
        print(json.dumps({'config': name, 'algo': algo, 'engine': getattr(det, 'engine', None), 'Nt': Nt, 'Nr': Nr, 'Na': Na, 'alphabet': alph, 'B': B,
                          'EbN0': ebn0, 'T': T, 'ver': float(L.loss['ver']), 'ser': float(L.loss['ser']),
                          'ms_per_epoch': round(ms, 4), 'symbol_vectors_per_s': B / (ms * 1e-3),
                          'trial_iterations_per_s': B * T / (ms * 1e-3), 'achieved_TFLOPs': round(tf, 2),
                          'mfma_frac_incl_decision': round(tf / PEAK_TF, 4)}), flush=True)
    nat.unload()


if __name__ == '__main__':
    main(only=sys.argv[1:] or None)
