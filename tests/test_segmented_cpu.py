"""generator_mode='segmented' (B = 1): the oracle's segmented_decision and metrics match the
reference's own Loss (g7: tests/golden/make_goldens.py g7), and the host Loss keeps the
reference's B > 1 failure (its reshape drops the batch axis, loss.py:232)."""
import json
import os

import numpy as np
import pytest

import golden_io as gio
from oracle import OracleConfig, loss_dict, segmented_decision

G7 = gio._group(np.load(os.path.join(gio.GOLDEN, 'g7_segmented.npz')))


def g7_cases():
    for c in G7.values():
        c['loss_ref'] = json.loads(str(c['loss']))
    return G7


@pytest.mark.parametrize('name', sorted(g7_cases()))
def test_g7_segmented_decision_metrics(name):
    c = G7[name]
    Nt, Na, Nr, B, Lin, Lh = (int(v) for v in c.dims)
    cfg = OracleConfig(Nt, Na, Nr, Lin=Lin, Lh=Lh, B=B, alphabet=str(c.alphabet), mode='segmented')
    xhat, shat, ihat = segmented_decision(c.xmap, cfg)
    np.testing.assert_array_equal(xhat, c.xhat)
    np.testing.assert_array_equal(shat, c.shat)
    np.testing.assert_array_equal(ihat, c.ihat)
    got = loss_dict(c.xmap, c.xmmse, c.x, c.sym, c.idx, 3, cfg)
    bad = gio.loss_close(got, c.loss_ref, count_tol=0.0, mse_rtol=1e-6)
    assert not bad, bad


def test_segmented_batch_gt_1_raises_like_reference():
    import torch
    from config import Config
    from loss import Loss
    cfg = Config(16, 2, 32, 1, 1, batch=2, generator_mode='segmented', alphabet='QPSK', device='cpu',
                 channel_profile='uniform', channel_truncation='tail')
    z = torch.zeros(2, 16, 1, dtype=torch.complex64)
    with pytest.raises(ValueError, match='cannot reshape'):
        Loss(cfg).device_counts(z, z, z, np.zeros(4, np.int64), np.zeros(4, np.int64))
