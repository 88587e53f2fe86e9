"""GPU parity of the Shrink kernels (csrc/amp_shrink.hip) through the C ABI.

g5: the reference's own Shrink outputs (bayes, shrinkOOK + dxdr, sw_shrinkOOK) on its inputs,
    NaN positions identical (e.g. the reciprocal of a denormal norm), values within
    rtol 2e-5 + atol 1e-6 (float32 exp/log ulp differences; see tests/test_shrink_cpu.py).
Full size: B=4096 x N=256 (cfg4's r) against the numpy oracle, plus ragged / empty inputs and
the non-power-of-two section path.
"""
import numpy as np
import pytest
import torch

from oracle import shrink_bayes, shrink_ook, shrink_sw_ook
from shrink_cases import compare, g5_cases

pytestmark = pytest.mark.gpu

CASES = g5_cases()
RTOL, ATOL = 2e-5, 1e-6


def _dev(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _shrink(c, fn, device):
    from shrink import Shrink
    c.cfg.device = str(device)
    return Shrink(c.cfg, fn)


@pytest.mark.parametrize('c', CASES, ids=[c.name for c in CASES])
def test_shrink_matches_reference(device, c):
    B, Na, Nt = int(c.dims[2]), int(c.dims[1]), int(c.dims[0])
    r = _dev(c.r, device).view(B, Nt, 1)
    cov = _dev(c.cov, device).view(B, Nt, 1) if c.cov.ndim else torch.tensor(c.cov, device=device)
    xb = _shrink(c, 'bayes', device)(r, cov)
    assert xb.shape == (B, Nt, 1)
    assert compare(xb.cpu().numpy()[..., 0], c.bayes, RTOL, ATOL) <= 0
    So = _shrink(c, 'shrinkOOK', device)
    xo, do = So(r, cov)
    assert xo.dtype == torch.float32 and do.shape == ()
    assert compare(xo.cpu().numpy()[..., 0], c.ook_x, RTOL, ATOL) <= 0
    assert abs(float(do) - float(c.ook_dxdr)) <= 1e-5 * abs(float(c.ook_dxdr)) + 1e-6
    xs, vs = So.sw_shrinkOOK(r, cov)
    assert xs.dtype == torch.complex64 and xs.shape == (B, Nt, 1)
    assert compare(xs.cpu().numpy()[..., 0], c.sw_x, RTOL, ATOL) <= 0
    assert compare(vs.cpu().numpy()[..., 0], c.sw_var, RTOL, ATOL) <= 0


def _cfg(Nt, Na, B, alphabet, device, is_complex=True):
    from config import Config
    return Config(Nt, Na, 2 * Nt, 1, 1, batch=B, generator_mode='sparc', alphabet=alphabet, is_complex=is_complex,
                  device=str(device), channel_profile='uniform', channel_truncation='tail')


@pytest.mark.parametrize('alphabet,is_complex,cov_kind', [('16QAM', True, 'scalar'), ('16QAM', True, 'vec'),
                                                         ('OOK', True, 'scalar'), ('4ASK', False, 'vec')])
def test_shrink_full_size_vs_oracle(device, alphabet, is_complex, cov_kind):
    from shrink import Shrink
    B, Nt, Na = 4096, 256, 8
    cfg = _cfg(Nt, Na, B, alphabet, device, is_complex)
    rng = np.random.default_rng(7)
    r = rng.standard_normal((B, Nt)) + (1j * rng.standard_normal((B, Nt)) if is_complex else 0)
    r = (0.6 * r).astype(np.complex64 if is_complex else np.float32)
    cov = (np.float32(0.15) if cov_kind == 'scalar'
           else ((np.abs(rng.standard_normal((B, Nt))) + 0.05) * 0.3).astype(np.float32))
    rt = _dev(r, device).view(B, Nt, 1)
    ct = torch.tensor(cov, device=device) if cov_kind == 'scalar' else _dev(cov, device).view(B, Nt, 1)
    sym = cfg.symbols.astype(np.complex64) if cfg.is_complex else cfg.symbols.astype(np.float32)
    xb = Shrink(cfg, 'bayes')(rt, ct).cpu().numpy()[..., 0]
    assert compare(xb, shrink_bayes(r, cov, sym, np.float32(cfg.P0), np.float32(cfg.Ps)), RTOL, ATOL) <= 0
    So = Shrink(cfg, 'shrinkOOK')
    xo, do = So(rt, ct)
    ro, rdo = shrink_ook(r, cov, So._theta)
    assert compare(xo.cpu().numpy()[..., 0], ro, RTOL, ATOL) <= 0
    assert abs(float(do) - float(rdo)) <= 1e-5 * abs(float(rdo)) + 1e-7
    xs, vs = So.sw_shrinkOOK(rt, ct)
    rs, rv = shrink_sw_ook(r, cov, B, Na, Nt // Na)
    assert compare(xs.cpu().numpy()[..., 0], rs, RTOL, ATOL) <= 0
    assert compare(vs.cpu().numpy()[..., 0], rv, RTOL, ATOL) <= 0


@pytest.mark.parametrize('Nt,Na,B', [(96, 1, 5), (640, 5, 3), (16, 16, 7), (2, 1, 1)])
def test_sw_shrink_ragged_sections(device, Nt, Na, B):
    """M = 96, 128 (wave-per-section kernel), M = 1 (leave-one-out of nothing: -log 0), tiny."""
    from shrink import Shrink
    cfg = _cfg(Nt, Na, B, 'OOK', device)
    rng = np.random.default_rng(Nt)
    r = (0.5 + 0.4 * rng.standard_normal((B, Nt))).astype(np.complex64)
    So = Shrink(cfg, 'shrinkOOK')
    xs, vs = So.sw_shrinkOOK(_dev(r, device).view(B, Nt, 1), torch.tensor(0.3, device=device))
    rs, rv = shrink_sw_ook(r, np.float32(0.3), B, Na, Nt // Na)
    assert compare(xs.cpu().numpy()[..., 0], rs, RTOL, ATOL) <= 0
    assert compare(vs.cpu().numpy()[..., 0], rv, RTOL, ATOL) <= 0


def test_shrink_empty_and_shape_errors(device):
    from shrink import Shrink
    import amp_native as nat
    cfg = _cfg(16, 2, 4, 'QPSK', device)
    S = Shrink(cfg, 'bayes')
    e = torch.empty(0, 16, 1, dtype=torch.complex64, device=device)
    assert S(e, torch.tensor(0.1, device=device)).shape == (0, 16, 1)
    with pytest.raises(RuntimeError):
        Shrink(cfg, 'shrinkOOK')(e, torch.tensor(0.1, device=device))
    with pytest.raises(RuntimeError, match='invalid for input'):
        Shrink(cfg, 'shrinkOOK').sw_shrinkOOK(torch.zeros(3, 16, 1, dtype=torch.complex64, device=device), 0.1)
    with pytest.raises(nat.AmpError):
        nat.check(nat.lib().amp_shrink_sw_ook(4, 0, 0, None, 0.1, None, None, None, None), 'sw')
