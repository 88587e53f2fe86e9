"""torch.ops.amp (TORCH_LIBRARY(amp), csrc/amp_torch_ops.cpp) on the GPU: each custom op runs the
same gfx950 entry point as the ctypes host classes, so its results equal theirs bit for bit, and
the VAMP op reproduces the reference's own Loss dict on a golden trace (g1)."""
import numpy as np
import pytest
import torch

import golden_io as gio

pytestmark = pytest.mark.gpu

G1 = gio.g1_cases()
G3 = gio.g3_cases()


def _cfg(Nt, Na, Nr, B, alph, iterations=20, Lin=1, Lh=1):
    from config import Config
    return Config(Nt, Na, Nr, Lin, Lh, batch=B, generator_mode='sparc', iterations=iterations, alphabet=alph,
                  channel_profile='uniform', channel_truncation='tail', device='cuda')


def _t(a, device):
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def _sym(cfg):
    return torch.tensor(np.asarray(cfg.symbols).astype(np.complex128))


@pytest.mark.parametrize('name', ['vamp_QPSK_6_0', 'vamp_16QAM_20_1', 'vamp_QPSK_0_0'])
def test_vamp_run_op_equals_host_class(device, name):
    import amp_native as nat
    from vamp import VAMP
    ops = nat.torch_ops()
    c = G1[name]
    cfg = _cfg(int(c.Nt), int(c.Na), int(c.Nr), int(c.B), c.alphabet, iterations=int(c.iters))
    U, s, Vh, y = _t(c.U, device), _t(c.s, device), _t(c.Vh, device), _t(c.y, device)
    det = VAMP(cfg)
    T = det.detect(U, s, Vh, y, float(c.SNR))
    r_ref, T_ref = T.r.clone(), T.status().T
    r, xm, var, st = ops.vamp_run(U, s, Vh, y, det.E / float(c.SNR), det.sparsity, cfg.Nt, cfg.Na, cfg.N_Layers,
                                  _sym(cfg), cfg.gray, 0)
    torch.cuda.synchronize()
    assert int(st[0]) == T_ref == int(c.T)
    assert gio.bits_equal(r.view_as(r_ref), r_ref)
    # the decision op on the op's r: the reference's counting metrics of this trace
    counts = ops.map_decide_count(r, xm, _t(c.x, device), _t(np.asarray(c.sym, np.int64), device),
                                  _t(np.asarray(c.idx, np.int64), device), cfg.Nt, cfg.Na, _sym(cfg), cfg.gray)
    from loss import Loss
    L = Loss(cfg)
    rates = dict(zip(L.keys, L.rates_from_vector(counts.cpu().numpy())))
    for k in ('ver', 'ser', 'fer', 'ier', 'iber', 'sber'):
        assert float(rates[k]) == pytest.approx(float(c.loss_ref[k]), abs=1e-12), k


@pytest.mark.parametrize('case', sorted(G3)[:12])
def test_map_decide_count_op_equals_loss(device, case):
    import amp_native as nat
    from config import Config
    from loss import Loss, counts_to_vector
    ops = nat.torch_ops()
    c = G3[case]
    Nt, Na, Nr, B, Lin, Lh = (int(v) for v in c.dims)
    cfg = Config(Nt, Na, Nr, Lin, Lh, batch=B, generator_mode='sparc', iterations=5, alphabet=str(c.alphabet),
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    args = [_t(c.xmap, device), _t(c.xmmse, device), _t(c.x, device)]
    sym, idx = _t(np.asarray(c.sym, np.int64), device), _t(np.asarray(c.idx, np.int64), device)
    got = ops.map_decide_count(*args, sym, idx, Nt, Na, _sym(cfg), cfg.gray).cpu().numpy()
    L = Loss(cfg)
    ref = counts_to_vector(L.read_counts(L.device_counts(*args, sym, idx)))
    assert np.array_equal(got[:9], ref[:9]), (got, ref)
    assert np.allclose(got[9:], ref[9:], rtol=1e-12, atol=0, equal_nan=True)


@pytest.mark.parametrize('mode', [0, 1, 2])
def test_block_denoise_op_equals_layer(device, mode):
    import amp_native as nat
    from vamp import block_denoise
    ops = nat.torch_ops()
    cfg = _cfg(64, 4, 128, 32, '16QAM')
    g = torch.Generator().manual_seed(mode)
    r = (torch.randn(32, 64, generator=g) + 1j * torch.randn(32, 64, generator=g)).to(torch.complex64).to(device)
    tau = torch.tensor(0.3) if mode == 0 else (torch.rand(32, 64, generator=g) + 0.1).to(device)
    xm, var = ops.block_denoise(r, tau.to(device) if mode else tau, mode, cfg.Nt, cfg.Na, _sym(cfg), cfg.gray)
    ref = block_denoise(cfg, r.view(32, 64, 1), tau.to(device) if mode else tau, mode)
    if mode == 2:
        assert gio.bits_equal(xm, ref.view(32, 64)) and var.numel() == 0
    else:
        assert gio.bits_equal(xm, ref[0].view(32, 64)) and gio.bits_equal(var, ref[1].view(32, 64))


def test_bamp_scamp_ops_equal_host_classes(device):
    import amp_native as nat
    from bamp import BAMP
    from scamp import SCAMP
    ops = nat.torch_ops()
    cb = G1['bamp_QPSK_6_0']
    cfg = _cfg(int(cb.Nt), int(cb.Na), int(cb.Nr), int(cb.B), 'QPSK', iterations=int(cb.iters))
    A, y = _t(cb.A, device), _t(cb.y, device)
    det = BAMP(cfg)
    det.detect(A, y, float(cb.SNR))
    xmap, xm, var, st = ops.bamp_run(A, y, det.E / float(cb.SNR), cfg.Nt, cfg.Na, cfg.N_Layers, _sym(cfg), cfg.gray)
    assert gio.bits_equal(xmap, det.xmap) and gio.bits_equal(var, det.var)
    cs = G1['scamp_16QAM_8_0']
    cfg = _cfg(int(cs.Nt), int(cs.Na), int(cs.Nr), int(cs.B), '16QAM', iterations=int(cs.iters))
    W, A, y = _t(cs.W, device), _t(cs.A, device), _t(cs.y, device)
    det = SCAMP(cfg)
    det.detect(W, A, y, float(cs.SNR))
    xmap, xm, psi, st = ops.scamp_run(W.reshape(cfg.Lout, cfg.Lin), A, y, det.E / float(cs.SNR), cfg.Nt, cfg.Na,
                                      cfg.N_Layers, _sym(cfg), cfg.gray)
    assert gio.bits_equal(xmap, det.xmap) and gio.bits_equal(psi, det.psi)


def test_ops_reject_bad_shapes(device):
    import amp_native as nat
    ops = nat.torch_ops()
    cfg = _cfg(64, 4, 128, 8, 'QPSK')
    r = torch.zeros(8, 60, dtype=torch.complex64, device=device)             # not a multiple of Nt
    with pytest.raises(RuntimeError):
        ops.block_denoise(r, torch.tensor(0.5), 0, cfg.Nt, cfg.Na, _sym(cfg), cfg.gray)
    r = torch.zeros(8, 64, dtype=torch.complex128, device=device)            # wrong dtype
    with pytest.raises(RuntimeError):
        ops.block_denoise(r, torch.tensor(0.5), 0, cfg.Nt, cfg.Na, _sym(cfg), cfg.gray)
