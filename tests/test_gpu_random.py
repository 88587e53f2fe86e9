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


@pytest.mark.parametrize('name', sorted(__import__('test_random_cpu').G9, key=lambda k: int(k[4:])))
def test_bamp_random_denoiser_layer(device, name):
    """BAMPLayer.random_denoiser on the GPU (amp_bamp_random_denoise) against the reference's
    layer (g9): float64 arithmetic, float32/complex64 outputs within 1e-5 relative."""
    from bamp import BAMPLayer
    from test_random_cpu import G9
    c = G9[name]
    layer = BAMPLayer(_cfg(32, 4, 64, 1, 1, 4, str(c.alphabet)))
    r = torch.from_numpy(c.r).to(device).view(4, 32, 1)
    cov = torch.from_numpy(c.cov).to(device).view(4, 32, 1)
    xm, var = layer.denoiser(r, cov)
    assert xm.dtype == torch.complex64 and var.shape == (4, 32, 1)
    np.testing.assert_allclose(xm.cpu().numpy()[..., 0], c.xmmse, rtol=1e-5, atol=1e-6, equal_nan=True)
    np.testing.assert_allclose(var.cpu().numpy()[..., 0], c.var, rtol=1e-5, atol=1e-6, equal_nan=True)
