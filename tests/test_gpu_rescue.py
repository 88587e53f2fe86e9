"""GPU: a persistent launch whose grid exchange was lost (nan_state = -1: every spin is bounded,
the grid drains, the results are invalid) is re-run on the launch engine in the same process
(LazyResult._check_grid), and the event is counted in `grid_rescues`.

The loss is injected through the detectors' test-only status hook (LazyResult.status_hook: the
status record is reported as a timed-out grid exactly as the kernel writes it); the rescued Loss
must equal a plain
launch-engine forward of the same epoch exactly (same engine, same inputs, same arithmetic).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

KEYS = ('T', 'fer', 'ver', 'ser', 'ier', 'iber', 'sber', 'nMSE')


def _inputs(cfg, seed, ebn0, E=1):
    from channel import Channel
    from config import Config
    from data import Data
    np.random.seed(seed)
    torch.manual_seed(seed)
    c = Config(cfg.Nt, cfg.Na, cfg.Nr, 1, 1, batch=cfg.B, generator_mode='sparc', iterations=cfg.N_Layers,
               alphabet=cfg.alphabet, channel_profile='uniform', channel_truncation='tail', device='cpu')
    ch, da = Channel(c), Data(c)
    W, A = ch.generate_as_sparc()
    SNR = c.snr(ebn0)
    eps = []
    for _ in range(E):
        x, sym, idx = da.generate_message()
        eps.append((x, sym, idx, A @ x + ch.awgn(SNR)))
    return W, A, SNR, eps


def _lose_grids(n):
    """A status hook that reports the next `n` persistent results as lost grids (nan_state = -1,
    what a timed-out grid exchange writes)."""
    left = [n]

    def hook(status):
        if left[0] > 0:
            left[0] -= 1
            status.nan_state = -1
        return status
    return hook


def _same(a, b):
    for k in KEYS:
        va, vb = np.asarray(a[k], dtype=np.float64), np.asarray(b[k], dtype=np.float64)
        assert np.array_equal(va, vb, equal_nan=True), (k, va, vb)


@pytest.mark.parametrize('alphabet,ebn0', [('16QAM', 8.0), ('QPSK', 6.0)])
def test_vamp_lost_grid_rescued_on_launch_engine(device, alphabet, ebn0):
    import amp_native as nat
    import vamp as vm
    from config import Config
    cfg = Config(64, 4, 128, 1, 1, batch=1024, generator_mode='sparc', iterations=20, alphabet=alphabet,
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    _, A, SNR, eps = _inputs(cfg, 3, ebn0, E=2)
    U, s, Vh = (t.to(device) for t in torch.linalg.svd(A, full_matrices=False))
    mv = lambda t: t.to(device).contiguous()  # noqa: E731
    x, sym, idx, y = eps[0]
    ref = dict(vm.VAMP(cfg, engine=nat.ENGINE_LAUNCHES)(U, s, Vh, mv(y), SNR, mv(x), sym, idx).loss)
    det = vm.VAMP(cfg)
    assert det.max_epochs(64) >= 2        # the shape runs on the persistent engine
    det.status_hook = _lose_grids(1)
    try:
        got = dict(det(U, s, Vh, mv(y), SNR, mv(x), sym, idx).loss)
    finally:
        det.status_hook = None
    assert det.grid_rescues == 1
    _same(got, ref)
    # side-by-side epochs: epoch 0's grid lost, epoch 1 kept
    det.status_hook = _lose_grids(1)
    try:
        Ls = det.forward_epochs(U, s, Vh, [mv(e[3]) for e in eps], SNR, [mv(e[0]) for e in eps],
                                [e[1] for e in eps], [e[2] for e in eps])
        got0, got1 = dict(Ls[0].loss), dict(Ls[1].loss)
    finally:
        det.status_hook = None
    assert det.grid_rescues == 2
    _same(got0, ref)
    x1, sym1, idx1, y1 = eps[1]
    _same(got1, dict(vm.VAMP(cfg)(U, s, Vh, mv(y1), SNR, mv(x1), sym1, idx1).loss))


def test_scamp_lost_grid_rescued_on_launch_engine(device):
    import amp_native as nat
    import vamp as vm
    from config import Config
    from scamp import SCAMP
    cfg = Config(128, 8, 256, 1, 1, batch=512, generator_mode='sparc', iterations=20, alphabet='16QAM',
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    W, A, SNR, eps = _inputs(cfg, 5, 10.0)
    x, sym, idx, y = eps[0]
    mv = lambda t: t.to(device).contiguous()  # noqa: E731
    ref = dict(SCAMP(cfg, engine=nat.ENGINE_LAUNCHES)(mv(W), mv(A), mv(y), SNR, mv(x), sym, idx).loss)
    det = SCAMP(cfg)
    det.status_hook = _lose_grids(1)
    try:
        got = dict(det(mv(W), mv(A), mv(y), SNR, mv(x), sym, idx).loss)
    finally:
        det.status_hook = None
    assert det.grid_rescues == 1
    _same(got, ref)
