"""generator_mode='random' on the GPU (amp_random_decide_count), B = 1 as in the reference.

g8 decision cases: decisions and all 14 metrics equal the reference's (continuous noisy inputs:
no exact magnitude ties).  g8 curves: BAMP end to end at B = 1 on the reference's inputs
(6 seeds x 5 EbN0 per curve); at most one single-trial point per curve may differ."""
import pytest
import torch
import numpy as np

import golden_io as gio
from test_gpu_vamp import _regen_inputs
from test_random_cpu import CURVES, G8

pytestmark = pytest.mark.gpu


def _cfg(Nt, Na, Nr, Lin, Lh, B, alphabet, iterations=5):
    from config import Config
    return Config(Nt, Na, Nr, Lin, Lh, batch=B, generator_mode='random', iterations=iterations,
                  alphabet=alphabet, channel_profile='uniform', channel_truncation='tail', device='cuda')


@pytest.mark.parametrize('name', sorted(G8, key=lambda k: int(k[4:])))
def test_random_decision_matches_reference(device, name):
    from loss import Loss
    c = G8[name]
    Nt, Na, Nr, B, Lin, Lh = (int(v) for v in c.dims)
    L = Loss(_cfg(Nt, Na, Nr, Lin, Lh, B, str(c.alphabet)))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device).view(B, -1, 1)  # noqa: E731
    xhat, shat, ihat = L.random_decision(t(c.xmap))
    np.testing.assert_array_equal(xhat, c.xhat)
    np.testing.assert_array_equal(shat, c.shat)
    np.testing.assert_array_equal(ihat, c.ihat)
    L.dump()
    L(t(c.xmap), t(c.xmmse), t(c.x), c.sym, c.idx, 3)
    bad = gio.loss_close(L.loss, c.loss_ref, count_tol=0.0, mse_rtol=1e-5)
    assert not bad, bad


@pytest.mark.parametrize('name', ['rand_bamp_QPSK', 'rand_bamp_16QAM'])
def test_random_mode_bamp_b1(device, name):
    from bamp import BAMP
    ent = CURVES[name]
    cfg = _cfg(ent['Nt'], ent['Na'], ent['Nr'], 1, 1, 1, ent['alphabet'], iterations=ent['iterations'])
    det = BAMP(cfg)
    diff = []
    for key, ref in sorted(ent['points'].items()):
        seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
        inp = _regen_inputs(cfg, seed, EbN0, svd=False)
        L = det(inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        if float(L.loss['ver']) != ref['ver'] or float(L.loss['ser']) != ref['ser']:
            diff.append((key, float(L.loss['ver']), ref['ver'], float(L.loss['ser']), ref['ser']))
    assert len(diff) <= 1, diff
