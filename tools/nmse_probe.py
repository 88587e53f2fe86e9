"""Diagnostic: Loss values of 8 side-by-side cfg2 epochs (two workgroups per CU) against the
sequential forwards, and nMSE recomputed on the host from each run's xmmse (loss.py:105-120)."""
import sys

sys.path[:0] = ['tests', '.', 'amp-sparc-spatialmodulation_amd']
import numpy as np  # noqa: E402
import torch  # noqa: E402
from test_gpu_epochs import _cfg, _epochs, _run_both  # noqa: E402

for alph, eb in (('QPSK', 6.0),):
    cfg = _cfg(64, 4, 128, 1024, alph)
    chan, SNR, eps = _epochs(cfg, 8, eb, seed=3)
    det, seq, grp = _run_both(cfg, chan, SNR, eps, torch.device('cuda:0'))
    r, xm, var = det.last_epochs
    for e in range(8):
        x = eps[e][0].numpy().reshape(1024, 64).astype(np.complex128)
        ns = 1024 * cfg.Na * cfg.Lin
        h_seq = float((np.abs(seq[e][3].cpu().numpy().reshape(1024, 64) - x) ** 2).sum() / ns)
        h_grp = float((np.abs(xm[e].cpu().numpy().reshape(1024, 64) - x) ** 2).sum() / ns)
        print(e, 'seq', float(seq[e][0]['nMSE']), 'grp', float(grp[e].loss['nMSE']), 'host(seq xm)', h_seq,
              'host(grp xm)', h_grp, flush=True)
