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


# SCAMP variants: (engine, persistent GEMM arithmetic); 'persistent' is the product default
# (bf16x3 where it fits), 'persistent-f32' the f32-MFMA form.  The fp16x2 form is not SCAMP's
# default: one QPSK golden (1/7) misses the psi allclose exit with it (amp_scamp.hip), so it is
# checked against the f32 form (test_scamp_x3_matches_f32) rather than on every curve point.
SVARIANTS = {'launches': (1, 0), 'persistent': (2, 0), 'persistent-f32': (2, 1)}
POINTS = ([(n, k, 'bamp') for n, k in _points('cfg1_bamp_qpsk')] +
          [(n, k, e) for n, k in _points('cfg3_scamp_16qam') + _points('cfg3_scamp_qpsk') for e in sorted(SVARIANTS)])


@pytest.mark.parametrize('name,key,engine', POINTS)
def test_curve_point(device, name, key, engine):
    """VER / SER within 1e-3 of the reference on the same seeds; SCAMP on both of its engines
    (cfg3 is persistent-eligible) and both GEMM arithmetics of the persistent one."""
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
        eng, gemm = SVARIANTS[engine]
        L = SCAMP(cfg, engine=eng, gemm=gemm)(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'],
                                              inp['idx'])
    got = L.loss
    assert abs(float(got['ver']) - ref['ver']) <= 1e-3, (float(got['ver']), ref['ver'])
    assert abs(float(got['ser']) - ref['ser']) <= 1e-3, (float(got['ser']), ref['ser'])
    _check_T(int(got['T']), int(ref['T']), ent['iterations'], ref['ver'], ref.get('T_pert'))


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



@pytest.mark.parametrize('ebn0', [0.0, 8.0])
@pytest.mark.parametrize('alph', ['QPSK', '16QAM'])
@pytest.mark.parametrize('split', ['x3', 'h2'])
def test_scamp_x3_matches_f32(device, alph, ebn0, split):
    """The persistent SCAMP engine's split-precision GEMMs (bf16x3, fp16x2) against its f32-MFMA
    GEMMs at cfg3: after one and three iterations xmap agrees to float32 GEMM summation-order
    noise, the full detection to the same T and counting metrics within 1e-3."""
    import torch
    import amp_native as nat
    from scamp import SCAMP
    inp = None
    for iters in (1, 3):
        cfg = _config(128, 8, 256, 4096, alph, iterations=iters)
        if inp is None:
            inp = _regen_inputs(cfg, 0, ebn0, svd=False)
        xs = []
        sg = nat.GEMM_X3 if split == 'x3' else nat.GEMM_H2
        for gemm in (nat.GEMM_F32, sg):
            det = SCAMP(cfg, engine=nat.ENGINE_PERSISTENT, gemm=gemm)
            det.detect(inp['W'], inp['A'], inp['y'], inp['SNR'])
            xs.append(det.xmap.clone())
        scale = float(torch.nan_to_num(xs[0]).abs().max())
        assert torch.allclose(xs[0], xs[1], rtol=0, atol=4e-6 * scale, equal_nan=True), \
            (iters, float((xs[0] - xs[1]).abs().nan_to_num().max()), scale)
    cfg = _config(128, 8, 256, 4096, alph, iterations=20)
    outs = []
    for gemm in (nat.GEMM_F32, sg):
        L = SCAMP(cfg, engine=nat.ENGINE_PERSISTENT, gemm=gemm)(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'],
                                                                inp['sym'], inp['idx'])
        outs.append({k: float(np.asarray(v)) for k, v in L.loss.items()})
    a, b = outs
    assert abs(a['T'] - b['T']) <= 1, (a['T'], b['T'])
    for k in ('ver', 'ser', 'fer', 'ier'):
        assert abs(a[k] - b[k]) <= 1e-3, (k, a[k], b[k])


@pytest.mark.parametrize('ebn0', [0.0, 8.0])
@pytest.mark.parametrize('alph', ['QPSK', '16QAM'])
@pytest.mark.parametrize('split', ['x3', 'h2'])
def test_bamp_split_matches_f32(device, alph, ebn0, split):
    """BAMP's split-precision launch tiles (bf16x3 amp_gemm_x3.h, fp16x2 amp_gemm_h2.h) against
    its f32-MFMA tiles (N = 1024, n = 256, B = 1024): after one and three iterations xmap agrees
    to float32 GEMM summation-order noise, the full detection to T within one and the counting
    metrics within 1e-3."""
    import torch
    import amp_native as nat
    from bamp import BAMP
    sg = nat.GEMM_X3 if split == 'x3' else nat.GEMM_H2
    inp = None
    for iters in (1, 3):
        cfg = _config(128, 8, 256, 1024, alph, iterations=iters)
        if inp is None:
            inp = _regen_inputs(cfg, 0, ebn0, svd=False)
        xs = []
        for gemm in (nat.GEMM_F32, sg):
            T = BAMP(cfg, gemm=gemm).detect(inp['A'], inp['y'], inp['SNR'])
            xs.append(T.xmap.clone())
        scale = float(torch.nan_to_num(xs[0]).abs().max())
        assert torch.allclose(xs[0], xs[1], rtol=0, atol=4e-6 * scale, equal_nan=True), \
            (iters, float((xs[0] - xs[1]).abs().nan_to_num().max()), scale)
    cfg = _config(128, 8, 256, 1024, alph, iterations=20)
    outs = []
    for gemm in (nat.GEMM_F32, sg):
        L = BAMP(cfg, gemm=gemm)(inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        outs.append({k: float(np.asarray(v)) for k, v in L.loss.items()})
    a, b = outs
    assert abs(a['T'] - b['T']) <= 1, (a['T'], b['T'])
    for k in ('ver', 'ser', 'fer', 'ier'):
        assert abs(a[k] - b[k]) <= 1e-3, (k, a[k], b[k])


@pytest.mark.parametrize('ebn0', [0.0, 8.0])
@pytest.mark.parametrize('alph', ['QPSK', '16QAM'])
def test_scamp_launch_x3_matches_f32(device, alph, ebn0):
    """SCAMP's launch engine on bf16x3 tiles (amp_gemm_x3.h) against its f32-MFMA tiles at cfg3
    (N = 1024, n = 256): after one and three iterations xmap agrees to float32 GEMM summation-order
    noise, the full detection to T within one and the counting metrics within 1e-3."""
    import torch
    import amp_native as nat
    from scamp import SCAMP
    inp = None
    for iters in (1, 3):
        cfg = _config(128, 8, 256, 4096, alph, iterations=iters)
        if inp is None:
            inp = _regen_inputs(cfg, 0, ebn0, svd=False)
        xs = []
        for gemm in (nat.GEMM_F32, nat.GEMM_X3):
            det = SCAMP(cfg, engine=nat.ENGINE_LAUNCHES, gemm=gemm)
            det.detect(inp['W'], inp['A'], inp['y'], inp['SNR'])
            xs.append(det.xmap.clone())
        scale = float(torch.nan_to_num(xs[0]).abs().max())
        assert torch.allclose(xs[0], xs[1], rtol=0, atol=4e-6 * scale, equal_nan=True), \
            (iters, float((xs[0] - xs[1]).abs().nan_to_num().max()), scale)
    cfg = _config(128, 8, 256, 4096, alph, iterations=20)
    outs = []
    for gemm in (nat.GEMM_F32, nat.GEMM_X3):
        L = SCAMP(cfg, engine=nat.ENGINE_LAUNCHES, gemm=gemm)(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'],
                                                              inp['sym'], inp['idx'])
        outs.append({k: float(np.asarray(v)) for k, v in L.loss.items()})
    a, b = outs
    assert abs(a['T'] - b['T']) <= 1, (a['T'], b['T'])
    for k in ('ver', 'ser', 'fer', 'ier'):
        assert abs(a[k] - b[k]) <= 1e-3, (k, a[k], b[k])


@pytest.mark.parametrize('ebn0', [0.0, 4.0, 8.0, 20.0])
@pytest.mark.parametrize('alph', ['QPSK', '16QAM'])
def test_scamp_engines_agree(device, alph, ebn0):
    """The persistent SCAMP engine against the launch engine at cfg3 (incl. the NaN-onset regime
    of 16-QAM from 4 dB): same T and counting metrics; after one iteration xmap agrees to float32
    GEMM summation-order noise."""
    import torch
    from scamp import SCAMP
    cfg = _config(128, 8, 256, 4096, alph, iterations=20)
    inp = _regen_inputs(cfg, 0, ebn0, svd=False)
    outs = []
    for eng in (1, 2):
        L = SCAMP(cfg, engine=eng)(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        outs.append({k: float(np.asarray(v)) for k, v in L.loss.items()})
    a, b = outs
    assert a['T'] == b['T'], (a['T'], b['T'])
    for k in ('ver', 'ser', 'fer', 'ier'):
        assert abs(a[k] - b[k]) <= 1e-3, (k, a[k], b[k])
    cfg1 = _config(128, 8, 256, 4096, alph, iterations=1)
    xs = []
    for eng in (1, 2):
        det = SCAMP(cfg1, engine=eng)
        det.detect(inp['W'], inp['A'], inp['y'], inp['SNR'])
        xs.append(det.xmap.clone())
    scale = float(torch.nan_to_num(xs[0]).abs().max())
    assert torch.allclose(xs[0], xs[1], rtol=0, atol=2e-6 * scale, equal_nan=True), \
        float((xs[0] - xs[1]).abs().nan_to_num().max())


@pytest.mark.parametrize('B', [1, 17, 1000, 4097])
def test_scamp_ragged_batches_engines_agree(device, B):
    """Ragged batches on the persistent SCAMP engine (a partial last workgroup; B = 4097 falls back
    to the launch engine under AUTO): the same counting metrics as the launch engine."""
    import amp_native as nat
    from scamp import SCAMP
    cfg = _config(128, 8, 256, B, 'QPSK', iterations=20)
    inp = _regen_inputs(cfg, 5, 4.0, svd=False)
    ncu = torch_ncu()
    eng = nat.lib().amp_scamp_select_engine(cfg.dims(), nat.ENGINE_AUTO)
    assert eng == (nat.ENGINE_LAUNCHES if B > 16 * ncu else nat.ENGINE_PERSISTENT)
    outs = []
    for e in (nat.ENGINE_LAUNCHES, nat.ENGINE_AUTO):
        L = SCAMP(cfg, engine=e)(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        outs.append({k: float(np.asarray(v)) for k, v in L.loss.items()})
    a, b = outs
    # the allclose(psi) exit over only B psi values (B = 17: 17 numbers near a slow fixed point)
    # moves with float32 summation order by an iteration or two; the metrics must agree
    assert abs(a['T'] - b['T']) <= (1 if B >= 1000 else 3), (a['T'], b['T'])
    for k in ('ver', 'ser', 'fer', 'ier'):
        assert abs(a[k] - b[k]) <= max(1e-3, 2.0 / B), (k, a[k], b[k])
    # three iterations (no early exit yet): xmap of both engines within float32 GEMM-order noise
    import torch
    cfg3 = _config(128, 8, 256, B, 'QPSK', iterations=3)
    xs = []
    for e in (nat.ENGINE_LAUNCHES, nat.ENGINE_AUTO):
        det = SCAMP(cfg3, engine=e)
        det.detect(inp['W'], inp['A'], inp['y'], inp['SNR'])
        xs.append(det.xmap.clone())
    scale = float(xs[0].abs().max())
    assert torch.allclose(xs[0], xs[1], rtol=0, atol=1e-4 * scale), float((xs[0] - xs[1]).abs().max())


def torch_ncu():
    import torch
    return torch.cuda.get_device_properties(0).multi_processor_count


@pytest.mark.parametrize('alph,ebn0,B,shape', [('16QAM', 8.0, 4096, (128, 8, 256)), ('QPSK', 2.0, 4096, (128, 8, 256)),
                                               ('16QAM', 20.0, 4096, (128, 8, 256)), ('16QAM', 12.0, 1000, (128, 8, 256)),
                                               ('QPSK', 6.0, 17, (128, 8, 256)),
                                               # M = 1 and M = 2: 128 / 64 sections per row, whose labels
                                               # (17 B per section) exceed the free LDS region at
                                               # (2N, 2n) = (256, 256) and are then read from global memory
                                               ('16QAM', 8.0, 4096, (128, 128, 128)), ('QPSK', 4.0, 1000, (128, 64, 128)),
                                               ('16QAM', 10.0, 4096, (128, 128, 256))])
def test_scamp_fused_decision_equals_standalone(device, alph, ebn0, B, shape):
    """amp_scamp_detect_count (decision + counters inside the persistent SCAMP launch, from LDS;
    scamp.py:107 -> loss.py:67-179) gives the same amp_counts as amp_scamp_run followed by
    amp_map_decide_count on the same forward: integer counters exactly, the float64 squared-error
    sums to summation-order rounding; ragged batches (B = 1000, 17) and one-position sections
    (M = 1, 2: the label staging bound of amp_decide_fused.h) included."""
    import amp_native as nat
    from scamp import SCAMP
    from vamp import read_result
    Nt, Na, Nr = shape
    cfg = _config(Nt, Na, Nr, B, alph, iterations=20)
    inp = _regen_inputs(cfg, 0, ebn0, svd=False)
    det = SCAMP(cfg, engine=nat.ENGINE_PERSISTENT)
    L = det(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
    L.resolve()
    _, fused = read_result(det.last.res)
    T = det.detect(inp['W'], inp['A'], inp['y'], inp['SNR'])
    buf = det.L.device_counts(T.buf.xmap, T.buf.xmmse, inp['x'], inp['sym'], inp['idx'])
    sep = det.L.read_counts(buf)
    for f in ('ier', 'ser', 'iber', 'sber', 'ver', 'verf', 'verm', 'verL', 'fer'):
        assert getattr(fused, f) == getattr(sep, f), (f, getattr(fused, f), getattr(sep, f))
    for f in ('mse', 'msef', 'msem', 'mseL'):
        a, b = getattr(fused, f), getattr(sep, f)
        assert (a == b) or abs(a - b) <= 1e-12 * max(abs(a), abs(b)) or (a != a and b != b), (f, a, b)
    assert int(L.loss['T']) == int(T.status().T)


@pytest.mark.parametrize('name,alphabet', [('cfg3_scamp_16qam', None), ('cfg3_scamp_qpsk', None),
                                           ('cfg3_scamp_16qam', '16PSK')])
def test_scamp_persistent_reproducible(device, name, alphabet):
    """cfg3's shape runs the SCAMP engine with eight waves per workgroup (two per SIMD; 16-QAM
    keeps the packed product-grid denoiser there; 16PSK, not a grid, the scalar
    per-point form): five forwards of the same batch give the same T and every Loss value, bit for
    bit."""
    from scamp import SCAMP
    ent = CURVES[name]
    cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], alphabet or ent['alphabet'],
                  iterations=ent['iterations'])
    inp = _regen_inputs(cfg, 1, 8.0, svd=False)
    det = SCAMP(cfg, engine=2)
    first = None
    for rep in range(5):
        L = det(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        got = {k: float(np.asarray(v)) for k, v in L.loss.items() if np.asarray(v).ndim == 0}
        if first is None:
            first = got
        else:   # the same bits; a NaN metric (a collapsed batch) must stay NaN
            assert got.keys() == first.keys(), rep
            for k in got:
                assert np.array_equal(got[k], first[k], equal_nan=True), (rep, k, got[k], first[k])
