"""CPU: pin the numpy oracle against vectors produced by running the reference itself.

The oracle (oracle/amp_oracle.py) is the checker of every GPU parity test, so it is
validated first: per-iteration traces (g1), denoiser outputs (g2) and decisions +
metrics (g3) must match the reference's.
"""
import numpy as np
import pytest

import golden_io as gio
from oracle import (OracleConfig, bamp_detect, block_denoise, loss_dict, map_decision, scamp_denoise,
                    scamp_detect, vamp_detect)

G1 = gio.g1_cases()
G2 = gio.g2_cases()
G3 = gio.g3_cases()


def _cfg(c, **kw):
    return OracleConfig(int(c.Nt), int(c.Na), int(c.Nr), B=int(c.B), alphabet=str(c.alphabet), **kw)


@pytest.mark.parametrize('name', sorted(G1))
def test_g1_traces(name):
    c = G1[name]
    cfg = _cfg(c, iterations=int(c.iters))
    trace = []
    if c.algo == 'vamp':
        out = vamp_detect(c.U, c.s, c.Vh, c.y, float(c.SNR), cfg, trace=trace)
        dec, key = out['r'], 'r'
    elif c.algo == 'bamp':
        out = bamp_detect(c.A, c.y, float(c.SNR), cfg, trace=trace)
        dec, key = out['xmap'], 'xmap'
    else:
        out = scamp_detect(c.W, c.A, c.y, float(c.SNR), cfg, trace=trace)
        dec, key = out['xmap'], 'xmap'
    # same iteration count (early exit of vamp.py:185 / bamp.py:140 / scamp.py:105)
    assert out['T'] == int(c.T)
    # first iteration: same arithmetic, only BLAS summation order differs
    ref0 = c[f'it0_{key}']
    np.testing.assert_allclose(trace[0][key], ref0, rtol=0, atol=2e-6 * max(1.0, float(np.abs(ref0).max())))
    # NaN pattern of the whole trace identical (float64 underflow rule)
    for t in range(out['T']):
        assert np.array_equal(np.isnan(trace[t]['xmmse']), np.isnan(c[f'it{t}_xmmse'])), f'NaN pattern it{t}'
    got = loss_dict(dec, out['xmmse'], c.x, c.sym, c.idx, out['T'], cfg)
    bad = gio.loss_close(got, c.loss_ref, count_tol=0.0, mse_rtol=1e-2)
    assert not bad, bad


@pytest.mark.parametrize('name', sorted(k for k in G2))
def test_g2_denoiser(name):
    c = G2[name]
    cfg = OracleConfig(int(c.Nt), int(c.Na), 2 * int(c.Nt), B=int(c.B), alphabet=str(c.alphabet))
    xm, var = block_denoise(c.r, np.float32(c.tau), cfg)
    np.testing.assert_array_equal(np.isnan(xm), np.isnan(c.v_xmmse))
    np.testing.assert_allclose(xm, c.v_xmmse, rtol=0, atol=2e-6, equal_nan=True)
    np.testing.assert_allclose(var, c.v_var, rtol=2e-5, atol=1e-7, equal_nan=True)
    if 'b_xmmse' in c:
        xm, var = block_denoise(c.r, (c.cov / np.float32(2)).astype(np.float32), cfg)
        np.testing.assert_allclose(xm, c.b_xmmse, rtol=0, atol=2e-6, equal_nan=True)
        np.testing.assert_allclose(var, c.b_var, rtol=2e-5, atol=1e-7, equal_nan=True)
        xs = scamp_denoise(c.r, (c.tau_use / np.float32(2)).astype(np.float32), cfg)
        np.testing.assert_allclose(xs, c.s_xmmse, rtol=0, atol=2e-6, equal_nan=True)


@pytest.mark.parametrize('name', sorted(G3))
def test_g3_decision_metrics(name):
    c = G3[name]
    Nt, Na, Nr, B, Lin, Lh = (int(v) for v in c.dims)
    cfg = OracleConfig(Nt, Na, Nr, Lin=Lin, Lh=Lh, B=B, alphabet=str(c.alphabet))
    xhat, shat, ihat = map_decision(c.xmap, cfg)
    np.testing.assert_array_equal(xhat, c.xhat)
    np.testing.assert_array_equal(shat, c.shat)
    np.testing.assert_array_equal(ihat, c.ihat)
    got = loss_dict(c.xmap, c.xmmse, c.x, c.sym, c.idx, 3, cfg)
    bad = gio.loss_close(got, c.loss_ref, count_tol=0.0, mse_rtol=1e-6)
    assert not bad, bad
