"""CPU: the vamp2 oracle restatement (damped "Rangan" VAMP, vamp2.py:12-131) against the
reference's own traces (tests/golden/g12_vamp2.npz, make_goldens.py g12), and the C ABI
surface of amp_vamp2_run (no compute without a GPU)."""
import numpy as np
import pytest

import golden_io as gio
from oracle import OracleConfig, loss_dict, vamp2_detect

G12 = gio.g12_cases()


def _ocfg(c):
    return OracleConfig(int(c.Nt), int(c.Na), int(c.Nr), B=int(c.B), alphabet=c.alphabet, iterations=int(c.iters))


def _close(a, b, rtol):
    """Same NaN / inf pattern; finite entries within rtol of max(1, |b|)."""
    a, b = np.asarray(a), np.asarray(b)
    assert np.array_equal(np.isnan(a), np.isnan(b))
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin)
    if fin.any():
        err = np.max(np.abs(a[fin] - b[fin]) / np.maximum(1.0, np.abs(b[fin])))
        assert err <= rtol, err


@pytest.mark.parametrize('name', sorted(G12))
def test_vamp2_oracle_matches_reference(name):
    c = G12[name]
    cfg = _ocfg(c)
    tr = []
    out = vamp2_detect(c.U, c.s, c.Vh, c.y, float(c.SNR), cfg, damping=float(c.damping), trace=tr)
    assert out['T'] == int(c.T)
    for t in range(len(tr)):
        if f'it{t}_r' not in c:
            continue
        _close(tr[t]['r'], c[f'it{t}_r'], 1e-5)
        _close(tr[t]['xmmse'], c[f'it{t}_xmmse'], 1e-5)
        _close(tr[t]['var'], c[f'it{t}_var'], 1e-5)
        g, gr = float(tr[t]['gamma']), float(c[f'it{t}_gamma'])
        assert (np.isnan(g) and np.isnan(gr)) or g == gr or abs(g - gr) <= 1e-5 * abs(gr), (t, g, gr)
    ld = loss_dict(out['r'], out['xmmse'], c.x, c.sym, c.idx, out['T'], cfg)
    for k in gio.COUNT_KEYS:
        assert float(ld[k]) == float(c.loss_ref[k]), (k, float(ld[k]), c.loss_ref[k])


def test_vamp2_abi_exported():
    import amp_native as nat
    lib = nat.lib()
    for sym in ('amp_vamp2_run', 'amp_vamp2_workspace_bytes'):
        assert hasattr(lib, sym)
    from config import Config
    cfg = Config(16, 2, 32, 1, 1, batch=8, generator_mode='sparc', iterations=20, alphabet='QPSK',
                 channel_profile='uniform', channel_truncation='tail', device='cpu')
    import ctypes as C
    assert lib.amp_vamp2_workspace_bytes(C.byref(cfg.dims()), 16) > 0
    assert lib.amp_vamp2_workspace_bytes(C.byref(cfg.dims()), 0) == 0
