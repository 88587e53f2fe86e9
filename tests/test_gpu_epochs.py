"""GPU: side-by-side epochs (amp_vamp_detect_count_epochs, VAMP.forward_epochs).

E epochs that share one channel (one `res` block of Model.simulate, vamp_model.py:55-61) run
in ONE persistent launch, each with its own batch-global scalars and early exit.  The bar is
bit-identity with E sequential forwards: same T, same counters and the same r / xmmse / var
bits (the per-epoch granule sweep reduces in the same fixed order as a one-epoch launch).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cfg(Nt, Na, Nr, B, alphabet, device='cuda', iterations=20):
    from config import Config
    return Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=iterations, alphabet=alphabet,
                  channel_profile='uniform', channel_truncation='tail', device=device)


def _epochs(cfg, E, ebn0, seed, scales=None):
    """One channel and E epochs of messages + noise in the reference's call order (host replica)."""
    from channel import Channel
    from data import Data
    np.random.seed(seed)
    torch.manual_seed(seed)
    c = _cfg(cfg.Nt, cfg.Na, cfg.Nr, cfg.B, cfg.alphabet, device='cpu', iterations=cfg.N_Layers)
    ch, da = Channel(c), Data(c)
    _, A = ch.generate_as_sparc()
    U, s, Vh = torch.linalg.svd(A, full_matrices=False)
    SNR = c.snr(ebn0)
    eps = []
    for e in range(E):
        x, sym, idx = da.generate_message()
        y = A @ x + ch.awgn(SNR)
        if scales is not None:
            y = y * scales[e]
        eps.append((x, sym, idx, y))
    return (U, s, Vh), SNR, eps


def _two_per_cu(det, N):
    """Whether epoch groups may hold two workgroups per CU (diagnostic build with
    AMP_EPOCHS_TWO_PER_CU=1; the shipped library caps a group at one per CU since round 6)."""
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    return det.max_epochs(N) == 2 * ncu // ((det.config.B + 15) // 16)


def _run_both(cfg, chan, SNR, eps, device):
    from vamp import VAMP
    mv = lambda t: t.to(device).contiguous()  # noqa: E731
    U, s, Vh = (mv(t) for t in chan)
    det = VAMP(cfg)
    seq = []
    for x, sym, idx, y in eps:
        L = det(U, s, Vh, mv(y), SNR, mv(x), sym, idx)
        seq.append((dict(L.loss), L.last_status, det.last.r.clone(), det.last.xmmse.clone(), det.last.var.clone()))
    grp = det.forward_epochs(U, s, Vh, [mv(e[3]) for e in eps], SNR, [mv(e[0]) for e in eps],
                             [e[1] for e in eps], [e[2] for e in eps])
    return det, seq, grp


@pytest.mark.parametrize('alphabet,ebn0,E', [('16QAM', 8.0, 4), ('16QAM', 20.0, 4), ('QPSK', 4.0, 4),
                                             ('QPSK', 12.0, 4), ('QPSK', 6.0, 4), ('16QAM', 14.0, 2),
                                             ('QPSK', 6.0, 8), ('16QAM', 8.0, 8), ('QPSK', 2.0, 8),
                                             ('16QAM', 20.0, 8)])
def test_epochs_equal_sequential_cfg2(device, alphabet, ebn0, E):
    from vamp import VAMP
    cfg = _cfg(64, 4, 128, 1024, alphabet)
    # one workgroup of 16 trials per CU at N = 64: 4 epochs of 64 workgroups on 256 CUs (8 at two
    # per CU, diagnostic build only)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    m = VAMP(cfg).max_epochs(64)
    assert m in (ncu // 64, 2 * ncu // 64)
    if E > m:
        pytest.skip(f'{E} epochs need two workgroups per CU (diagnostic build, AMP_EPOCHS_TWO_PER_CU=1)')
    chan, SNR, eps = _epochs(cfg, E, ebn0, seed=3)
    det, seq, grp = _run_both(cfg, chan, SNR, eps, device)
    r, xm, var = det.last_epochs
    assert len(grp) == E
    for e, (ls, st, r0, x0, v0) in enumerate(seq):
        lg = grp[e].loss
        assert int(lg['T']) == int(ls['T']), (e, lg['T'], ls['T'])
        assert grp[e].last_status.nan_state == st.nan_state
        assert lg.keys() == ls.keys()
        for k in ls:
            assert np.array_equal(np.asarray(lg[k]), np.asarray(ls[k]), equal_nan=True), (e, k)
        assert torch.equal(r[e].view(torch.int32), r0.view(torch.int32)), e
        assert torch.equal(xm[e].view(torch.int32), x0.view(torch.int32)), e
        assert torch.equal(var[e].view(torch.int32), v0.view(torch.int32)), e
    # the same epochs as stacked [E, B, ...] tensors (used without a copy)
    mv = lambda t: t.to(device).contiguous()  # noqa: E731
    U, s, Vh = (mv(t) for t in chan)
    ys = torch.stack([mv(e[3]) for e in eps])
    xs = torch.stack([mv(e[0]) for e in eps])
    syms = torch.stack([torch.as_tensor(np.asarray(e[1], np.int64)) for e in eps]).to(device)
    idxs = torch.stack([torch.as_tensor(np.asarray(e[2], np.int64)) for e in eps]).to(device)
    grp2 = det.forward_epochs(U, s, Vh, ys, SNR, xs, syms, idxs)
    r2 = det.last_epochs[0]
    for e in range(E):
        assert int(grp2[e].loss['T']) == int(grp[e].loss['T']) and float(grp2[e].loss['ser']) == float(grp[e].loss['ser'])
        assert torch.equal(r2[e].view(torch.int32), r[e].view(torch.int32)), e


@pytest.mark.parametrize('alphabet,ebn0', [('16QAM', 8.0), ('16PSK', 10.0), ('QPSK', 4.0)])
def test_epochs_equal_sequential_n256(device, alphabet, ebn0):
    """The eight-wave N = 256 engine (two waves per SIMD; cfg4's shape at B = 1024, 64 workgroups
    per epoch): 4 epochs side by side equal 4 sequential forwards bit for bit, in three
    repetitions of the grouped launch."""
    cfg = _cfg(256, 8, 512, 1024, alphabet)
    chan, SNR, eps = _epochs(cfg, 4, ebn0, seed=7)
    det, seq, grp = _run_both(cfg, chan, SNR, eps, device)
    mv = lambda t: t.to(device).contiguous()  # noqa: E731
    U, s, Vh = (mv(t) for t in chan)
    for rep in range(3):
        if rep:
            grp = det.forward_epochs(U, s, Vh, [mv(e[3]) for e in eps], SNR, [mv(e[0]) for e in eps],
                                     [e[1] for e in eps], [e[2] for e in eps])
        r, xm, var = det.last_epochs
        for e, (ls, st, r0, x0, v0) in enumerate(seq):
            assert int(grp[e].loss['T']) == int(ls['T']), (rep, e)
            assert torch.equal(r[e].view(torch.int32), r0.view(torch.int32)), (rep, e)
            assert torch.equal(xm[e].view(torch.int32), x0.view(torch.int32)), (rep, e)
            assert torch.equal(var[e].view(torch.int32), v0.view(torch.int32)), (rep, e)


def _epochs_per_channel(cfg, E, ebn0, seed):
    """E epochs with a channel each, in the reference's call order at res = 1 (vamp_model.py:55-61:
    channel + SVD, then message + noise, every epoch)."""
    from channel import Channel
    from data import Data
    np.random.seed(seed)
    torch.manual_seed(seed)
    c = _cfg(cfg.Nt, cfg.Na, cfg.Nr, cfg.B, cfg.alphabet, device='cpu', iterations=cfg.N_Layers)
    ch, da = Channel(c), Data(c)
    SNR = c.snr(ebn0)
    out = []
    for e in range(E):
        _, A = ch.generate_as_sparc()
        U, s, Vh = torch.linalg.svd(A, full_matrices=False)
        x, sym, idx = da.generate_message()
        y = A @ x + ch.awgn(SNR)
        out.append(((U, s, Vh), (x, sym, idx, y)))
    return SNR, out


@pytest.mark.parametrize('Nt,Na,Nr,B,alphabet,ebn0,E', [(64, 4, 128, 1024, '16QAM', 8.0, 4),
                                                        (64, 4, 128, 1024, 'QPSK', 4.0, 4),
                                                        (256, 8, 512, 1024, '16QAM', 10.0, 4),
                                                        (256, 8, 512, 1024, 'QPSK', 2.0, 4)])
def test_epochs_per_channel_equal_sequential(device, Nt, Na, Nr, B, alphabet, ebn0, E):
    """One channel per epoch (the reference's default res = 1, vamp_model.py:45, 56-58) in ONE
    persistent launch (amp_vamp_detect_count_epochs_ch): every epoch equals its own sequential
    forward bit for bit — T, every Loss value, r / xmmse / var."""
    from vamp import VAMP
    cfg = _cfg(Nt, Na, Nr, B, alphabet)
    SNR, eps = _epochs_per_channel(cfg, E, ebn0, seed=13)
    mv = lambda t: t.to(device).contiguous()  # noqa: E731
    det = VAMP(cfg)
    assert det.max_epochs(Nt) >= E
    seq = []
    for (U, s, Vh), (x, sym, idx, y) in eps:
        L = det(mv(U), mv(s), mv(Vh), mv(y), SNR, mv(x), sym, idx)
        seq.append((dict(L.loss), det.last.r.clone(), det.last.xmmse.clone(), det.last.var.clone()))
    Us = [mv(e[0][0]) for e in eps]
    ss = [mv(e[0][1]) for e in eps]
    Vhs = [mv(e[0][2]) for e in eps]
    for rep in range(2):
        grp = det.forward_epochs(Us if rep == 0 else torch.stack(Us), ss if rep == 0 else torch.stack(ss),
                                 Vhs if rep == 0 else torch.stack(Vhs), [mv(e[1][3]) for e in eps], SNR,
                                 [mv(e[1][0]) for e in eps], [e[1][1] for e in eps], [e[1][2] for e in eps])
        r, xm, var = det.last_epochs
        for e, (ls, r0, x0, v0) in enumerate(seq):
            lg = grp[e].loss
            assert int(lg['T']) == int(ls['T']), (rep, e, lg['T'], ls['T'])
            for k in ls:
                assert np.array_equal(np.asarray(lg[k]), np.asarray(ls[k]), equal_nan=True), (rep, e, k)
            assert torch.equal(r[e].view(torch.int32), r0.view(torch.int32)), (rep, e)
            assert torch.equal(xm[e].view(torch.int32), x0.view(torch.int32)), (rep, e)
            assert torch.equal(var[e].view(torch.int32), v0.view(torch.int32)), (rep, e)


def test_simulate_group_epochs_res1_identical(device, tmp_path):
    """Model.simulate at the reference's default res = 1 with group_epochs=True (one channel per
    epoch, side by side) writes the same points as the per-epoch loop."""
    from model import Model
    cfg = _cfg(64, 4, 128, 1024, '16QAM')
    outs = []
    for grouped in (False, True):
        m = Model(cfg, 'vamp', path=str(tmp_path / f'r{int(grouped)}'), seed=5, group_epochs=grouped)
        outs.append(m.simulate(epochs=10, start=6.0, final=8.0, step=2.0, res=1))
    assert len(outs[0]) == len(outs[1])
    for a, b in zip(*outs):
        assert a.keys() == b.keys()
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), k


@pytest.mark.parametrize('gemm', ['f32', 'x3_n_ne_2k'])
def test_simulate_group_epochs_res1_shared_channel_only(device, tmp_path, gemm):
    """Where one launch cannot hold a channel per epoch (amp_vamp_epochs_ch_eligible: GEMM_F32, or
    n != 2 k), Model.simulate(group_epochs=True) at res = 1 sends runs of one channel and still writes
    the points of the per-epoch loop (round-5 advisor: these runs failed with AMP_E_ARG)."""
    import amp_native as nat
    from model import Model
    from vamp import VAMP
    if gemm == 'f32':
        cfg, g = _cfg(64, 4, 128, 1024, '16QAM'), nat.GEMM_F32
    else:
        cfg, g = _cfg(64, 4, 192, 1024, '16QAM'), nat.GEMM_AUTO   # n = 192 != 2 k = 128
    det = VAMP(cfg, gemm=g)
    assert not det.epochs_channels_eligible(64)
    outs = []
    for grouped in (False, True):
        m = Model(cfg, 'vamp', path=str(tmp_path / f'r{int(grouped)}'), amp=VAMP(cfg, gemm=g), seed=5,
                  group_epochs=grouped)
        if grouped:
            assert m.group_cap >= 1
        outs.append(m.simulate(epochs=6, start=6.0, final=8.0, step=2.0, res=1))
    assert len(outs[0]) == len(outs[1])
    for a, b in zip(*outs):
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), k


def test_epochs_independent_rare_path(device):
    """One epoch driven into the exact float64 rare path (its y scaled up: logits beyond the
    float64 range of the global shift) while the others are not: the per-epoch barrier counters
    keep the groups apart and every epoch still equals its sequential forward."""
    cfg = _cfg(64, 4, 128, 1024, '16QAM')
    chan, SNR, eps = _epochs(cfg, 3, 14.0, seed=5, scales=[1.0, 40.0, 1.0])
    det, seq, grp = _run_both(cfg, chan, SNR, eps, device)
    r, xm, var = det.last_epochs
    for e, (ls, st, r0, x0, v0) in enumerate(seq):
        assert int(grp[e].loss['T']) == int(ls['T']), e
        assert grp[e].last_status.nan_state == st.nan_state, e
        assert float(grp[e].loss['ser']) == float(ls['ser']), e
        assert torch.equal(var[e].view(torch.int32), v0.view(torch.int32)), e


def test_epochs_cfg4_two(device):
    """Two cfg4 epochs would need 512 workgroups > 256 CUs: refused (AMP_E_ARG), no fallback."""
    import amp_native as nat
    cfg = _cfg(256, 8, 512, 4096, '16QAM')
    from vamp import VAMP
    det = VAMP(cfg)
    assert not det.epochs_eligible(512, 256, 2)
    assert det.epochs_eligible(512, 256, 1) and det.max_epochs(256) == 1
    z = torch.zeros(4096, 256, dtype=torch.complex64, device=device)
    with pytest.raises(nat.AmpError):
        det.forward_epochs(torch.zeros(512, 256, dtype=torch.complex64, device=device),
                           torch.ones(256, device=device), torch.zeros(256, 256, dtype=torch.complex64, device=device),
                           [torch.zeros(4096, 512, dtype=torch.complex64, device=device)] * 2, 10.0, [z, z],
                           [np.zeros(4096 * 8, np.int64)] * 2, [np.zeros(4096 * 8, np.int64)] * 2)


def test_simulate_group_epochs_identical(device, tmp_path):
    """Model.simulate(res=4) with group_epochs=True writes the same points as the per-epoch loop."""
    from model import Model
    cfg = _cfg(64, 4, 128, 1024, 'QPSK')
    outs = []
    for grouped in (False, True):
        m = Model(cfg, 'vamp', path=str(tmp_path / f'g{int(grouped)}'), seed=11, group_epochs=grouped)
        if grouped:
            assert m.group_cap >= 4
        outs.append(m.simulate(epochs=8, start=2.0, final=4.0, step=2.0, res=4))
    assert len(outs[0]) == len(outs[1])
    for a, b in zip(*outs):
        assert a.keys() == b.keys()
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), k


@pytest.mark.parametrize('alphabet,ebn0', [('QPSK', 6.0), ('16QAM', 8.0)])
def test_epochs8_two_per_cu_reproducible(device, alphabet, ebn0):
    """8 cfg2 epochs in one launch (two workgroups per CU; diagnostic build only since round 6, when
    gpurun r6c49 saw such a launch differ once) three times over: every r / xmmse / var
    word equal to the sequential forwards in every repetition.  Round 2 saw these co-resident epochs
    change run to run; the cause was the packed-math variance sum of the denoiser (one half of a
    v_pk_fma_f32 result lost in lanes 48-63 with two waves per SIMD)."""
    from vamp import VAMP
    cfg = _cfg(64, 4, 128, 1024, alphabet)
    if not _two_per_cu(VAMP(cfg), 64):
        pytest.skip('two workgroups per CU: diagnostic build only (AMP_EPOCHS_TWO_PER_CU=1)')
    chan, SNR, eps = _epochs(cfg, 8, ebn0, seed=3)
    det, seq, grp = _run_both(cfg, chan, SNR, eps, device)
    mv = lambda t: t.to(device).contiguous()  # noqa: E731
    U, s, Vh = (mv(t) for t in chan)
    for rep in range(3):
        if rep:
            grp = det.forward_epochs(U, s, Vh, [mv(e[3]) for e in eps], SNR, [mv(e[0]) for e in eps],
                                     [e[1] for e in eps], [e[2] for e in eps])
        r, xm, var = det.last_epochs
        for e, (ls, st, r0, x0, v0) in enumerate(seq):
            assert int(grp[e].loss['T']) == int(ls['T']), (rep, e)
            assert torch.equal(r[e].view(torch.int32), r0.view(torch.int32)), (rep, e)
            assert torch.equal(xm[e].view(torch.int32), x0.view(torch.int32)), (rep, e)
            assert torch.equal(var[e].view(torch.int32), v0.view(torch.int32)), (rep, e)
