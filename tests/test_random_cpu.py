"""generator_mode='random' (B = 1): the oracle's random_decision and metrics match the reference's
own Loss (g8: tests/golden/make_goldens.py g8); the reference's random-mode VAMP raises, and so
does the host VAMP."""
import json
import os

import numpy as np
import pytest

import golden_io as gio
from oracle import OracleConfig, loss_dict, random_decision

G8 = gio._group(np.load(os.path.join(gio.GOLDEN, 'g8_random.npz')))
for _c in G8.values():
    _c['loss_ref'] = json.loads(str(_c['loss']))
with open(os.path.join(gio.GOLDEN, 'g8_random_curves.json')) as _f:
    CURVES = json.load(_f)


@pytest.mark.parametrize('name', sorted(G8))
def test_g8_random_decision_metrics(name):
    c = G8[name]
    Nt, Na, Nr, B, Lin, Lh = (int(v) for v in c.dims)
    cfg = OracleConfig(Nt, Na, Nr, Lin=Lin, Lh=Lh, B=B, alphabet=str(c.alphabet), mode='random')
    xhat, shat, ihat = random_decision(c.xmap, cfg)
    np.testing.assert_array_equal(xhat, c.xhat)
    np.testing.assert_array_equal(shat, c.shat)
    np.testing.assert_array_equal(ihat, c.ihat)
    got = loss_dict(c.xmap, c.xmmse, c.x, c.sym, c.idx, 3, cfg)
    bad = gio.loss_close(got, c.loss_ref, count_tol=0.0, mse_rtol=1e-6)
    assert not bad, bad


def test_random_mode_vamp_raises_like_reference():
    import torch
    from config import Config
    from vamp import VAMP
    err = CURVES['vamp_random_error']
    assert err[0] == 'ValueError'
    cfg = Config(32, 4, 64, 1, 1, batch=1, generator_mode='random', alphabet='QPSK', device='cpu',
                 channel_profile='uniform', channel_truncation='tail')
    z = torch.zeros(1)
    with pytest.raises(ValueError, match=err[1].split('(')[0].strip()):
        VAMP(cfg)(z, z, z, z, 1.0, z, None, None)


@pytest.mark.parametrize('name', ['rand_bamp_QPSK', 'rand_bamp_16QAM'])
def test_random_mode_inputs_replica(name):
    """The build's Data.random / channel replica reproduces the reference's inputs bit for bit."""
    import hashlib
    import torch
    from channel import Channel
    from config import Config
    from data import Data
    ent = CURVES[name]
    cfg = Config(ent['Nt'], ent['Na'], ent['Nr'], 1, 1, batch=1, generator_mode='random', iterations=20,
                 alphabet=ent['alphabet'], channel_profile='uniform', channel_truncation='tail', device='cpu')
    sha = lambda t: hashlib.sha256(np.ascontiguousarray(t.numpy()).tobytes()).hexdigest()  # noqa: E731
    for key in ['0/0', '3/8', '5/16']:
        seed = int(key.split('/')[0])
        np.random.seed(seed)
        torch.manual_seed(seed)
        _, A = Channel(cfg).generate_as_sparc()
        x, _, _ = Data(cfg).generate_message()
        assert sha(A) == ent['points'][key]['sha_A'] and sha(x) == ent['points'][key]['sha_x']


@pytest.mark.parametrize('name', ['rand_bamp_QPSK', 'rand_bamp_16QAM'])
def test_oracle_random_mode_bamp_curves(name):
    """The oracle's BAMP with random_denoiser (bamp.py:79-88) against the reference's B = 1 curve
    points (single trials; at most one point may flip on float summation order)."""
    from oracle import bamp_detect, loss_dict
    from config import Config
    from test_gpu_vamp import _regen_inputs
    ent = CURVES[name]
    cfg = Config(ent['Nt'], ent['Na'], ent['Nr'], 1, 1, batch=1, generator_mode='random', iterations=20,
                 alphabet=ent['alphabet'], channel_profile='uniform', channel_truncation='tail', device='cpu')
    ocfg = OracleConfig(ent['Nt'], ent['Na'], ent['Nr'], B=1, alphabet=ent['alphabet'], iterations=20, mode='random')
    diff = []
    for key, ref in sorted(ent['points'].items()):
        seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
        inp = _regen_inputs(cfg, seed, EbN0, svd=False)
        out = bamp_detect(inp['A'].numpy(), inp['y'].numpy()[..., 0], inp['SNR'], ocfg)
        got = loss_dict(out['xmap'], out['xmmse'], inp['x'].numpy()[..., 0], inp['sym'], inp['idx'], out['T'], ocfg)
        if float(got['ver']) != ref['ver'] or float(got['ser']) != ref['ser']:
            diff.append((key, float(got['ver']), ref['ver'], float(got['ser']), ref['ser']))
    assert len(diff) <= 1, diff


G9 = gio._group(np.load(os.path.join(gio.GOLDEN, 'g9_bamp_random_denoise.npz')))


@pytest.mark.parametrize('name', sorted(G9, key=lambda k: int(k[4:])))
def test_oracle_bamp_random_denoiser(name):
    """oracle.bamp_random_denoise against the reference's BAMPLayer.random_denoiser (g9)."""
    from oracle import bamp_random_denoise
    c = G9[name]
    cfg = OracleConfig(32, 4, 64, B=4, alphabet=str(c.alphabet), mode='random')
    xm, var = bamp_random_denoise(c.r, c.cov, cfg)
    np.testing.assert_allclose(xm, c.xmmse, rtol=1e-5, atol=1e-6, equal_nan=True)
    np.testing.assert_allclose(var, c.var, rtol=1e-5, atol=1e-6, equal_nan=True)
