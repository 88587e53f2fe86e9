"""GPU parity for BAMP (bamp.py) and SCAMP (scamp.py) through the C ABI.

g1: the reference's stored inputs -> same iteration count and counting metrics.
g4: the reference's curves (BASELINE cfg1 BAMP and cfg3 SCAMP, 16-QAM and QPSK) ->
    VER / SER within 1e-3 at every point on the same seeds.
"""
import numpy as np
import pytest

import golden_io as gio
from test_gpu_vamp import _check_T, _config, _regen_inputs, _t

pytestmark = pytest.mark.gpu

G1 = gio.g1_cases()
CURVES = gio.g4_curves()


@pytest.mark.parametrize('name', sorted(k for k in G1 if k.startswith('bamp')))
def test_bamp_g1_reference_inputs(device, name):
    from bamp import BAMP
    c = G1[name]
    cfg = _config(int(c.Nt), int(c.Na), int(c.Nr), int(c.B), c.alphabet, iterations=int(c.iters))
    L = BAMP(cfg)(_t(c.A, device), _t(c.y, device), float(c.SNR), _t(c.x, device), c.sym, c.idx)
    assert L.loss['T'] == int(c.T)
    bad = gio.loss_close(L.loss, c.loss_ref, count_tol=0.0, mse_rtol=5e-2)
    assert not bad, bad


@pytest.mark.parametrize('name', sorted(k for k in G1 if k.startswith('scamp')))
def test_scamp_g1_reference_inputs(device, name):
    from scamp import SCAMP
    c = G1[name]
    cfg = _config(int(c.Nt), int(c.Na), int(c.Nr), int(c.B), c.alphabet, iterations=int(c.iters))
    det = SCAMP(cfg)
    L = det(_t(c.W, device), _t(c.A, device), _t(c.y, device), float(c.SNR), _t(c.x, device), c.sym, c.idx)
    assert L.loss['T'] == int(c.T)
    bad = gio.loss_close(L.loss, c.loss_ref, count_tol=0.0, mse_rtol=5e-2)
    assert not bad, bad
    last = int(c.T) - 1
    psi_ref = c[f'it{last}_psi']
    np.testing.assert_allclose(det.psi.cpu().numpy(), psi_ref.reshape(det.psi.shape), rtol=1e-3, atol=1e-4,
                               equal_nan=True)


def _points(name, every=1):
    ent = CURVES[name]
    keys = sorted(ent['points'], key=lambda k: (int(k.split('/')[0]), float(k.split('/')[1])))
    return [(name, k) for k in keys[::every]]


POINTS = (_points('cfg1_bamp_qpsk') + _points('cfg3_scamp_16qam') + _points('cfg3_scamp_qpsk'))


@pytest.mark.parametrize('name,key', POINTS)
def test_curve_point(device, name, key):
    from bamp import BAMP
    from scamp import SCAMP
    ent = CURVES[name]
    ref = ent['points'][key]
    seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
    cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'], iterations=ent['iterations'])
    inp = _regen_inputs(cfg, seed, EbN0, svd=False)
    if ent['algo'] == 'bamp':
        L = BAMP(cfg)(inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
    else:
        L = SCAMP(cfg)(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
    got = L.loss
    assert abs(float(got['ver']) - ref['ver']) <= 1e-3, (float(got['ver']), ref['ver'])
    assert abs(float(got['ser']) - ref['ser']) <= 1e-3, (float(got['ser']), ref['ser'])
    _check_T(int(got['T']), int(ref['T']), ent['iterations'])


@pytest.mark.parametrize('name', ['bamp_QPSK_0_0', 'bamp_QPSK_12_0', 'scamp_16QAM_8_0', 'scamp_QPSK_2_0'])
def test_layer_level_equals_forward(device, name):
    """Tracker + Layer.forward(T) per iteration (the reference's layer surface, bamp.py:12-64,
    scamp.py:8-59) == the detector's whole-loop launch sequence, bit for bit, with the same T."""
    import torch
    c = G1[name]
    cfg = _config(int(c.Nt), int(c.Na), int(c.Nr), int(c.B), c.alphabet, iterations=int(c.iters))
    if name.startswith('bamp'):
        from bamp import BAMP, Tracker
        det = BAMP(cfg)
        args = (_t(c.A, device), _t(c.y, device))
        T1 = det.detect(*args, float(c.SNR))
        ref = (T1.xmap.clone(), T1.var.clone(), T1.status().T)
        T = Tracker(*args, det.E / float(c.SNR), cfg)
        outs = lambda T: (T.xmap, T.var)  # noqa: E731
    else:
        from scamp import SCAMP, Tracker
        det = SCAMP(cfg)
        args = (_t(c.W, device), _t(c.A, device), _t(c.y, device))
        T1 = det.detect(*args, float(c.SNR))
        ref = (T1.xmap.clone(), T1.psi.clone(), T1.status().T)
        T = Tracker(*args, det.E / float(c.SNR), cfg)
        outs = lambda T: (T.xmap, T.psi)  # noqa: E731
    T.prepare()
    for layer in det.layers:
        layer(T)
    T.finalize()
    a, b = outs(T)
    assert T.status().T == ref[2] == int(c.T)
    assert gio.bits_equal(a, ref[0]) and gio.bits_equal(b, ref[1])

