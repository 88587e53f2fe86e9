"""Generator of the reference-run values pinned in tests/test_gpu_published.py: the reference's
own SCAMP (imported from /root/reference, CPU, 8 threads) at the published ISI shape
(Nt=128 Na=8 Nr=32 Lin=32 Lh=3, QPSK, EbN0 6 dB), one epoch drawn by the reference's generators
at the given seed.  Run here only (the reference is not on the GPU box), from a scratch CWD:
    PYTHONDONTWRITEBYTECODE=1 python3 tests/golden/ref_scamp_published_shape.py B SEED"""
import sys, time
sys.dont_write_bytecode = True
sys.path.insert(0, '/root/reference')
import numpy as np, torch
torch.set_num_threads(8)
from config import Config
from channel import Channel
from data import Data
from scamp import SCAMP
B = int(sys.argv[1]); seed = int(sys.argv[2])
np.random.seed(seed); torch.manual_seed(seed)
cfg = Config(N_transmit_antenna=128, N_active_antenna=8, N_receive_antenna=32, block_length=32, channel_length=3,
             channel_truncation='tail', alphabet='QPSK', channel_profile='uniform', generator_mode='sparc', batch=B,
             iterations=200, device='cpu')
ch, da = Channel(cfg), Data(cfg)
det = SCAMP(cfg)
EbN0 = 6.0
SNRdB = EbN0 + 10 * np.log10(cfg.code_rate)
SNR = 10 ** (SNRdB / 10)
t0 = time.time()
W, A = ch.generate_as_sparc()
x, s, i = da.generate_message()
y = A @ x + ch.awgn(SNR)
L = det(W, A, y, SNR, x, s, i)
print('B', B, 'seed', seed, 'T', L.loss['T'], 'fer', L.loss['fer'], 'ver', L.loss['ver'], 'time', round(time.time() - t0, 1), flush=True)
