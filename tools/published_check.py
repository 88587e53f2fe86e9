"""The published ISI SCAMP shape (Nt=128 Na=8 Nr=32 Lin=32 Lh=3, QPSK, 6 dB) on the GPU with the
reference's own random streams (host replica), for comparison with the reference run on the CPU
at the same seed:  python tools/published_check.py B SEED"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..'), os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from channel import Channel  # noqa: E402
from config import Config  # noqa: E402
from data import Data  # noqa: E402
from scamp import SCAMP  # noqa: E402

for spec in sys.argv[1:]:
    B, seed = (int(v) for v in spec.split(':'))
    np.random.seed(seed)
    torch.manual_seed(seed)
    cfg = Config(128, 8, 32, 32, 3, batch=B, generator_mode='sparc', iterations=200, alphabet='QPSK',
                 channel_profile='uniform', channel_truncation='tail', device='cpu')
    ch, da = Channel(cfg), Data(cfg)
    W, A = ch.generate_as_sparc()
    x, s, i = da.generate_message()
    SNR = cfg.snr(6.0)
    y = A @ x + ch.awgn(SNR)
    cfg.device = 'cuda'
    dev = torch.device('cuda:0')
    det = SCAMP(cfg)
    L = det(W.to(dev), A.to(dev), y.to(dev), SNR, x.to(dev), s, i)
    print('B', B, 'seed', seed, 'T', L.loss['T'], 'fer', float(L.loss['fer']), 'ver', float(L.loss['ver']), flush=True)
