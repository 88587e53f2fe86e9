"""Monte-Carlo driver (model.py, reference vamp_model.py:45-69) on the CPU: the sweep,
averaging, JSON export and FER early stop with a stand-in detector, and the rank-sharded
sweep (world size 2, gloo) merging to the same averages."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from config import Config
from loss import Loss


def _cfg():
    return Config(16, 2, 32, 1, 1, batch=4, generator_mode='sparc', iterations=5, alphabet='QPSK',
                  channel_profile='uniform', channel_truncation='tail', device='cpu')


class FakeAmp:
    """Stands in for VAMP.forward: same call signature, fills its Loss like Loss.__call__."""

    def __init__(self, config, fer_until_snr=None):
        self.L = Loss(config)
        self.calls = 0
        self.fer_until_snr = fer_until_snr
        self.shapes = []

    def __call__(self, U, s, Vh, y, SNR, x, sym, idx):
        self.calls += 1
        self.shapes.append((tuple(U.shape), tuple(y.shape), len(sym)))
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        fer = 1.0 if (self.fer_until_snr is None or SNR < self.fer_until_snr) else 0.0
        rates = [fer] + [float(rank + 1)] * 13
        self.L.dump()
        self.L.loss = {'T': 0}
        self.L.record(rates, 3)
        return self.L


def test_simulate_export_and_early_stop(tmp_path):
    from model import Model
    cfg = _cfg()
    amp = FakeAmp(cfg, fer_until_snr=10 ** ((2 + 10 * np.log10(cfg.code_rate)) / 10))
    m = Model(cfg, 'vamp', path=str(tmp_path), amp=amp, seed=0)
    res = m.simulate(epochs=3, start=0, final=6.0, step=1)
    # EbN0 0, 1 have fer 1; EbN0 2 has fer 0 -> exported, then the sweep stops
    assert [r['EbN0dB'] for r in res] == [0.0, 1.0, 2.0]
    assert amp.calls == 9
    assert amp.shapes[0] == ((32, 16), (4, 32, 1), 4 * 2)
    for e in (0, 1, 2):
        with open(tmp_path / f'{float(e)}.json') as f:
            d = json.load(f)
        assert d['T'] == 3.0 and d['EbN0dB'] == float(e)
        assert set(['fer', 'ser', 'ver', 'nMSE', 'ber', 'SNRdB', 'rate', 'C', 'ShannonLimitdB']) <= set(d)
        assert d['ser'] == pytest.approx(1.0)
    assert not os.path.exists(tmp_path / '3.0.json')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    torch.distributed.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                                         world_size=world)
    try:
        from model import Model
        cfg = _cfg()
        amp = FakeAmp(cfg)
        m = Model(cfg, 'vamp', path=out, amp=amp, seed=3)
        res = m.simulate(epochs=6, start=0, final=1.0, step=1, res=2)
        with open(os.path.join(out, f'rank{rank}.json'), 'w') as f:
            json.dump({'calls': amp.calls, 'res': res}, f)
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.timeout(180)
def test_simulate_two_ranks_gloo(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method='spawn')
    r0 = json.load(open(tmp_path / 'rank0.json'))
    r1 = json.load(open(tmp_path / 'rank1.json'))
    # 6 epochs in blocks of res=2: rank 0 gets blocks {0, 2} (4 epochs), rank 1 block {1}
    assert r0['calls'] == 2 * 4 and r1['calls'] == 2 * 2
    for a, b in zip(r0['res'], r1['res']):
        assert a == b                        # every rank holds the merged average
        assert a['T'] == pytest.approx(3.0)
        assert a['ser'] == pytest.approx((4 * 1.0 + 2 * 2.0) / 6)
    # only rank 0 writes the JSON files
    assert sorted(p for p in os.listdir(tmp_path) if p.endswith('.json') and not p.startswith('rank')) == \
        ['0.0.json', '1.0.json']


class FakeShardedAmp(FakeAmp):
    """Stands in for ShardedVAMP: every rank returns the WHOLE batch's Loss (the same values on
    every rank), FER 1 below `fer_until_snr` and 0 from there on."""

    def __call__(self, U, s, Vh, y, SNR, x, sym, idx):
        self.calls += 1
        fer = 1.0 if SNR < self.fer_until_snr else 0.0
        self.L.dump()
        self.L.loss = {'T': 0}
        self.L.record([fer] + [0.5] * 13, 3)
        return self.L


def _worker_trials(rank, world, port, out):
    torch.distributed.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                                         world_size=world)
    try:
        from model import Model
        cfg = _cfg()
        amp = FakeShardedAmp(cfg, fer_until_snr=10 ** ((2 + 10 * np.log10(cfg.code_rate)) / 10))
        m = Model(cfg, 'vamp', path=out, amp=amp, seed=3, shard='trials')
        res = m.simulate(epochs=3, start=0, final=6.0, step=1)
        with open(os.path.join(out, f'rank{rank}.json'), 'w') as f:
            json.dump({'calls': amp.calls, 'res': res}, f)
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.timeout(180)
def test_simulate_trial_shard_two_ranks_gloo(tmp_path):
    """shard='trials' over several SNR points: every rank must clear its totals after each point
    (only rank 0 did, so the other ranks carried the previous point's averages into
    the next, their FER never reached the stop and their results differed from rank 0's)."""
    world = 2
    mp.start_processes(_worker_trials, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method='spawn')
    r0 = json.load(open(tmp_path / 'rank0.json'))
    r1 = json.load(open(tmp_path / 'rank1.json'))
    # every rank runs every epoch of every point (the detector splits each batch), 3 points, stop
    assert r0['calls'] == r1['calls'] == 3 * 3
    assert [p['EbN0dB'] for p in r0['res']] == [0.0, 1.0, 2.0]
    assert r0['res'] == r1['res']
    assert [p['fer'] for p in r0['res']] == [1.0, 1.0, 0.0]


class FakeGroupedAmp(FakeAmp):
    """Also stands in for VAMP.forward_epochs / max_epochs: records each grouped call's channels
    (one shared channel, or one per epoch) and returns one Loss per epoch, the values a function
    of the epoch's y, so grouped and sequential sweeps can be compared."""

    def __init__(self, config, cap, ch_ok=True):
        super().__init__(config)
        self.cap = cap
        self.ch_ok = ch_ok
        self.groups = []

    def max_epochs(self, k):
        return self.cap

    def epochs_channels_eligible(self, k):
        return self.ch_ok

    def _one(self, y):
        L = Loss(self.L.config) if hasattr(self.L, 'config') else Loss(_cfg())
        v = float(torch.view_as_real(y).double().abs().sum())
        L.dump()
        L.loss = {'T': 0}
        L.record([1.0] + [v] * 13, 3)
        return L

    def __call__(self, U, s, Vh, y, SNR, x, sym, idx):
        self.calls += 1
        self.seq_U = getattr(self, 'seq_U', []) + [U]
        return self._one(y)

    def forward_epochs(self, U, s, Vh, ys, SNR, xs, syms, idxs):
        per = isinstance(U, (list, tuple))
        self.groups.append((len(ys), per, U if per else [U] * len(ys)))
        return [self._one(y) for y in ys]


@pytest.mark.parametrize('res,cap,ch_ok', [(1, 4, True), (4, 3, True), (2, 8, True), (1, 4, False), (2, 8, False)])
def test_simulate_group_epochs_host_logic(tmp_path, res, cap, ch_ok):
    """Model.simulate(group_epochs=True) draws the epochs' inputs in the reference's call order
    (vamp_model.py:55-61: a channel when i % res == 0), hands chunks of at most max_epochs epochs to
    forward_epochs — one channel per epoch when the chunk spans channels (res = 1), the shared one
    otherwise — and writes the same points as the sequential sweep.  Where the detector takes one
    shared channel per launch only (ch_ok False: GEMM_F32 or n != 2k, amp_vamp_epochs_ch_eligible),
    every call holds epochs of one channel."""
    from model import Model
    cfg = _cfg()
    outs, amps = [], []
    for grouped in (False, True):
        amp = FakeGroupedAmp(cfg, cap, ch_ok)
        m = Model(cfg, 'vamp', path=str(tmp_path / f'g{int(grouped)}'), amp=amp, seed=3, group_epochs=grouped)
        outs.append(m.simulate(epochs=10, start=0, final=1.0, step=1, res=res))
        amps.append(amp)
    seq, grp = amps
    assert seq.groups == [] and grp.calls == 0
    assert sum(n for n, _, _ in grp.groups) == 20 and max(n for n, _, _ in grp.groups) <= cap
    for n, per, Us in grp.groups:
        distinct = len({id(u) for u in Us})
        assert per == (distinct > 1), (n, per, distinct)
        if not ch_ok:
            assert distinct == 1 and n <= res   # one channel per call
        elif res == 1:
            assert distinct == n          # a channel per epoch
    # the channels each epoch was detected with: the same matrices in both sweeps
    grouped_U = [u for _, _, Us in grp.groups for u in Us]
    assert len(grouped_U) == len(seq.seq_U) == 20
    for a, b in zip(grouped_U, seq.seq_U):
        assert torch.equal(a, b)
    for a, b in zip(*outs):
        assert a.keys() == b.keys()
        for k in a:
            assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), k
