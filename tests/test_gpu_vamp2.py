"""GPU parity of the damped "Rangan" VAMP (vamp2.py) through amp_vamp2_run: the reference's own
traces (tests/golden/g12_vamp2.npz) and the numpy oracle on the same stored inputs.

The reference diverges in most of these cases (gamma -> inf at iteration 2, then NaN: SURVEY.md
§2 records VER = 1.0 for vamp2); the build has to diverge the same way: same T, same NaN pattern
and the same counting metrics, finite values within float32 GEMM-order noise.
"""
import numpy as np
import pytest
import torch

import golden_io as gio
from oracle import OracleConfig, loss_dict, vamp2_detect

pytestmark = pytest.mark.gpu

G12 = gio.g12_cases()


def _cfg(c, iters=None):
    from config import Config
    return Config(int(c.Nt), int(c.Na), int(c.Nr), 1, 1, batch=int(c.B), generator_mode='sparc',
                  iterations=int(iters or c.iters), alphabet=c.alphabet, channel_profile='uniform',
                  channel_truncation='tail', device='cuda')


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _close(a, b, rtol):
    a, b = np.asarray(a), np.asarray(b)
    assert np.array_equal(np.isnan(a), np.isnan(b)), (int(np.isnan(a).sum()), int(np.isnan(b).sum()))
    fin = np.isfinite(b) & np.isfinite(a)
    if fin.any():
        err = float(np.max(np.abs(a[fin] - b[fin]) / np.maximum(1.0, np.abs(b[fin]))))
        assert err <= rtol, err


@pytest.mark.parametrize('name', sorted(G12))
def test_vamp2_matches_reference(device, name):
    from vamp2 import VAMP
    c = G12[name]
    det = VAMP(_cfg(c), damping=float(c.damping))
    L = det(_t(c.U, device), _t(c.s, device), _t(c.Vh, device), _t(c.y, device), float(c.SNR), _t(c.x, device),
            c.sym, c.idx)
    got = {k: float(np.asarray(v)) for k, v in L.loss.items()}
    assert int(got['T']) == int(c.T), (got['T'], int(c.T))
    for k in gio.COUNT_KEYS:
        assert got[k] == float(c.loss_ref[k]), (k, got[k], c.loss_ref[k])
    t = int(c.T) - 1
    T = det.last
    _close(T.r.cpu().numpy()[..., 0], c[f'it{t}_r'], 2e-4)
    _close(T.xmmse.cpu().numpy()[..., 0], c[f'it{t}_xmmse'], 2e-4)
    _close(T.var.cpu().numpy()[..., 0], c[f'it{t}_var'], 2e-4)


@pytest.mark.parametrize('name', [n for n in sorted(G12) if '_16_' in n])
@pytest.mark.parametrize('iters', [1, 2])
def test_vamp2_first_iterations_match_oracle(device, name, iters):
    """The first iterations (before the reference's divergence) against the oracle: r, xmmse,
    var within float32 noise and gamma (status.last_scalar[0]) to float32 rounding."""
    from vamp2 import VAMP
    c = G12[name]
    det = VAMP(_cfg(c, iters), damping=float(c.damping))
    T = det.detect(_t(c.U, device), _t(c.s, device), _t(c.Vh, device), _t(c.y, device), float(c.SNR))
    torch.cuda.synchronize()
    ocfg = OracleConfig(int(c.Nt), int(c.Na), int(c.Nr), B=int(c.B), alphabet=c.alphabet, iterations=iters)
    tr = []
    out = vamp2_detect(c.U, c.s, c.Vh, c.y, float(c.SNR), ocfg, damping=float(c.damping), trace=tr)
    _close(T.r.cpu().numpy()[..., 0], out['r'], 2e-4)
    _close(T.xmmse.cpu().numpy()[..., 0], out['xmmse'], 2e-4)
    _close(T.var.cpu().numpy()[..., 0], out['var'], 2e-4)
    import amp_native as nat
    import ctypes as C
    raw = T.res.cpu().numpy().tobytes()
    s = nat.AmpStatus.from_buffer_copy(raw[:C.sizeof(nat.AmpStatus)])
    g_ref = float(tr[-1]['gamma'])
    g = float(s.last_scalar[0])
    assert (np.isinf(g_ref) and np.isinf(g)) or (np.isnan(g_ref) and np.isnan(g)) or abs(g - g_ref) <= 1e-5 * abs(g_ref), \
        (g, g_ref)
    assert s.T == out['T']


def test_vamp2_random_mode_raises(device):
    from config import Config
    from vamp2 import VAMP
    cfg = Config(16, 2, 32, 1, 1, batch=1, generator_mode='random', iterations=5, alphabet='QPSK',
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    z = torch.zeros(1, device=device)
    with pytest.raises(ValueError):
        VAMP(cfg)(z, z, z, z, 1.0, z, None, None)
