"""Shrink oracle (oracle/amp_oracle.py shrink_*) pinned against the reference's own outputs
(g5, tests/golden/make_goldens.py g5), plus the host class's exceptions (no GPU needed).

Tolerance: float32 element-wise work, so rtol 2e-5 relative plus atol 1e-6 absolute on outputs in
[0, 1.5] (exp / log implementations differ by an ulp between numpy, torch and ocml; a logit
of magnitude up to ~90 turns one ulp of the argument into ~1e-5 relative)."""
import numpy as np
import pytest
import torch

from oracle import shrink_bayes, shrink_ook, shrink_sw_ook
from shrink_cases import compare, g5_cases

CASES = g5_cases()
RTOL, ATOL = 2e-5, 1e-6


@pytest.mark.parametrize('c', CASES, ids=[c.name for c in CASES])
def test_oracle_matches_reference_shrink(c):
    B, Na = int(c.dims[2]), int(c.dims[1])
    xb = shrink_bayes(c.r, c.cov, c.sym, np.float32(c.cfg.P0), np.float32(c.cfg.Ps))
    assert compare(xb, c.bayes, RTOL, ATOL) <= 0
    xo, do = shrink_ook(c.r, c.cov, c.theta)
    assert compare(xo, c.ook_x, RTOL, ATOL) <= 0
    assert abs(float(do) - float(c.ook_dxdr)) <= 1e-5 * abs(float(c.ook_dxdr)) + 1e-6
    xs, vs = shrink_sw_ook(c.r, c.cov, B, Na, c.M)
    assert compare(xs, c.sw_x, RTOL, ATOL) <= 0
    assert compare(vs, c.sw_var, RTOL, ATOL) <= 0


def test_golden_covers_nan_and_overflow():
    assert sum(np.isnan(c.bayes).any() for c in CASES) >= 1      # reciprocal of a denormal norm
    assert sum('overflow' in c for c in CASES) >= 4
    assert {int(c.M) for c in CASES} >= {8, 12, 16, 128}


def test_host_class_surface_and_errors():
    from config import Config
    from shrink import Shrink
    cfg = Config(16, 2, 32, 1, 1, batch=4, generator_mode='sparc', alphabet='QPSK', device='cpu',
                 channel_profile='uniform', channel_truncation='tail')
    with pytest.raises(AssertionError):
        Shrink(cfg, 'nope')
    S = Shrink(cfg, 'bayes')
    assert S.Ps.dtype == torch.float32 and S.symbols.dtype == torch.complex64 and (S.M, S.L, S.B) == (8, 2, 4)
    r = torch.zeros(4, 16, 1, dtype=torch.complex64)
    with pytest.raises(NotImplementedError):
        Shrink(cfg, 'shrink')(r, torch.tensor(0.1))
    with pytest.raises(NotImplementedError):
        Shrink(cfg, 'lasso')(r, torch.tensor(0.1))
    rcfg = Config(16, 2, 32, 1, 1, batch=4, generator_mode='sparc', alphabet='BPSK', is_complex=False, device='cpu',
                  channel_profile='uniform', channel_truncation='tail')
    with pytest.raises(UnboundLocalError):
        Shrink(rcfg, 'shrink')(r.real.contiguous(), torch.tensor(0.1))
    with pytest.raises(AttributeError):
        Shrink(rcfg, 'lasso')(r.real.contiguous(), torch.tensor(0.1))
    # compute calls need a ROCm tensor: no CPU fallback
    with pytest.raises(ValueError, match='no CPU fallback'):
        S(r, torch.tensor(0.1))


@pytest.mark.parametrize('fn', ['bayes', 'shrinkOOK', 'sw_shrinkOOK'])
@pytest.mark.parametrize('dtype', [torch.float64, torch.complex128])
def test_shrink_refuses_double_inputs(fn, dtype):
    """The kernels compute in float32 / complex64; a float64 / complex128 r is refused instead of
    being returned downcast (the reference would keep float64)."""
    from config import Config
    from shrink import Shrink
    cfg = Config(16, 2, 32, 1, 1, batch=2, generator_mode='sparc', alphabet='QPSK', device='cpu')
    S = Shrink(cfg, 'shrinkOOK')
    r = torch.zeros(2, 16, 1, dtype=dtype)
    with pytest.raises(TypeError):
        getattr(S, fn)(r, 0.5)
