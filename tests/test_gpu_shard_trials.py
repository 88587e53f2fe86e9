"""GPU: trial sharding across ranks (SURVEY §8(e) exact-compat mode; ShardedVAMP /
amp_vamp_run_sharded, ShardedBAMP / amp_bamp_run_sharded, ShardedSCAMP / amp_scamp_run_sharded,
incl. ISI shapes on the banded GEMMs).  2 and 3 rank processes on the one GPU, gloo process group (the hook
all-reduces the batch scalars through host memory; RCCL is the same hook on the device words).

Bar: every rank's Loss equals the single-process whole-batch forward's — T exact, VER / SER /
FER / IER within 1e-3 (the north star's parity bar; in practice equal) — and the ranks' r slices
match the whole batch's r (the GEMM rows are computed identically; only the float64 order of the
var.mean() sum differs).
"""
import json
import math
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from shard_trials_worker import case_inputs  # noqa: E402

CASES = ['16QAM:8:1024', 'QPSK:4:1024', '16QAM:20:1024', 'QPSK:12:1000', '16QAM:14:1024:40',
         'bamp:QPSK:6:1024', 'bamp:16QAM:12:1000', 'bamp:16QAM:20:1024', 'bampisi:QPSK:6:256',
         'scampisi:QPSK:6:256', 'scampisi:16QAM:12:500', 'scampisi:16QAM:24:256']


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_equals_whole_batch(device, tmp_path, world):
    import amp_native as nat
    from vamp import VAMP
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, 'shard_trials_worker.py'), str(r), str(world),
                               str(port), str(tmp_path)] + CASES, env=env) for r in range(world)]
    rcs = [p.wait(timeout=100) for p in procs]
    assert rcs == [0] * world, rcs
    outs = [json.load(open(tmp_path / f'rank{r}.json')) for r in range(world)]
    from bamp import BAMP
    from scamp import SCAMP
    for name in CASES:
        algo, cfg, args = case_inputs(name)
        mv = lambda t: t.to(device).contiguous() if isinstance(t, torch.Tensor) else t  # noqa: E731
        det = {'vamp': lambda: VAMP(cfg, engine=nat.ENGINE_LAUNCHES), 'bamp': lambda: BAMP(cfg),
               'scamp': lambda: SCAMP(cfg, engine=nat.ENGINE_LAUNCHES)}[algo]()
        L = det(*(mv(a) for a in args))
        whole = dict(L.loss)
        r_whole = (det.last.r if algo == 'vamp' else det.last.xmap).cpu().numpy()
        for r in range(world):
            o = outs[r][name]
            assert int(o['T']) == int(whole['T']), (name, r, o['T'], whole['T'])
            for k in ('ver', 'ser', 'fer', 'ier'):
                a, b = float(o[k]), float(whole[k])
                assert abs(a - b) <= 1e-3 or (np.isnan(a) and np.isnan(b)), (name, r, k, a, b)
        rs = np.concatenate([np.load(tmp_path / f'{name.replace(":", "_")}_r{r}.npy') for r in range(world)])
        fin = np.isfinite(r_whole)
        assert np.array_equal(np.isfinite(rs), fin), name
        if fin.any():
            frac = float(np.mean(np.abs(rs[fin] - r_whole[fin]) > 1e-4 * max(1.0, float(np.abs(r_whole[fin]).max()))))
            assert frac <= 0.01, (name, frac)


@pytest.mark.parametrize('name', ['16QAM:8:1024', 'bamp:QPSK:6:1024', 'scampisi:16QAM:12:500'])
def test_sharded_single_process_is_whole_batch(device, name):
    """Without torch.distributed the sharded detectors hold the whole batch and the hook is the
    identity: the Loss equals the plain forward's exactly."""
    import amp_native as nat
    from bamp import BAMP, ShardedBAMP
    from scamp import SCAMP, ShardedSCAMP
    from vamp import VAMP, ShardedVAMP
    assert not (torch.distributed.is_available() and torch.distributed.is_initialized())
    algo, cfg, args = case_inputs(name)
    mv = lambda t: t.to(device).contiguous() if isinstance(t, torch.Tensor) else t  # noqa: E731
    plain = {'vamp': lambda: VAMP(cfg, engine=nat.ENGINE_LAUNCHES), 'bamp': lambda: BAMP(cfg),
             'scamp': lambda: SCAMP(cfg, engine=nat.ENGINE_LAUNCHES)}[algo]()
    shard = {'vamp': ShardedVAMP, 'bamp': ShardedBAMP, 'scamp': ShardedSCAMP}[algo](cfg)
    a = dict(plain(*(mv(x) for x in args)).loss)
    b = dict(shard(*(mv(x) for x in args)).loss)
    assert a.keys() == b.keys()
    for k in a:
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k]), equal_nan=True), (k, a[k], b[k])


# ---- persistent engine: several grids sharing one exchange buffer (amp_vamp_detect_count_shard) ----
@pytest.mark.parametrize('Nt,Na,Nr,B,alphabet,ebn0,R', [(256, 8, 512, 4096, '16QAM', 8.0, 2),
                                                        (256, 8, 512, 4096, 'QPSK', 2.0, 2),
                                                        (256, 8, 512, 2048, '16QAM', 20.0, 4),
                                                        (64, 4, 128, 1024, '16QAM', 10.0, 4),
                                                        (64, 4, 128, 1000, 'QPSK', 6.0, 2)])
def test_persistent_shards_equal_whole_batch(device, Nt, Na, Nr, B, alphabet, ebn0, R):
    """R persistent grids on one GPU, each on its own CUs (a CU-masked stream), each detecting a
    contiguous slice of ONE batch
    and exchanging the per-iteration batch partials through one shared buffer (SURVEY §8(e)
    exact-compat on the persistent engine): every shard's T and status equal the whole-batch
    persistent forward's, its rows of r / xmmse / var are the same bits, and the shards' counters
    sum to the whole batch's (the reduction runs over every workgroup of the batch in the same
    order, so nothing differs, not even the float64 order of var.mean())."""
    from test_gpu_vamp import _config, _regen_inputs
    from vamp import VAMP, PersistentShard, read_result
    cfg = _config(Nt, Na, Nr, B, alphabet, iterations=20)
    inp = _regen_inputs(cfg, 3, ebn0)
    det = VAMP(cfg, engine=2)
    L = det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
    whole = {k: float(np.asarray(v)) for k, v in L.loss.items()}
    wst, wct = L.last_status, L.last_counts
    wr, wx, wv = det.last.r.clone(), det.last.xmmse.clone(), det.last.var.clone()
    # co-resident grids: every shard's workgroups on the CUs at once (16 trials per workgroup)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    assert (B + 15) // 16 <= (2 if Nt == 64 else 1) * ncu
    per = ((B + R - 1) // R + 15) // 16 * 16
    bounds = [(r0, min(B, r0 + per)) for r0 in range(0, B, per)]
    xbuf = PersistentShard.xbuf(cfg, device)
    import ctypes as C
    import amp_native as nat
    nat.check(nat.lib().amp_vamp_shard_reset(nat.dptr(xbuf), nat.stream_ptr(device)), 'reset')
    torch.cuda.synchronize()
    L_ = cfg.L
    sym = torch.as_tensor(np.asarray(inp['sym'], np.int64)).reshape(B, L_)
    idx = torch.as_tensor(np.asarray(inp['idx'], np.int64)).reshape(B, L_)
    # each shard's grid on its own CUs and hardware queue (co-resident by construction)
    per_cu = 2 if Nt == 64 else 1
    cuts = [ncu * i // len(bounds) for i in range(len(bounds) + 1)]
    for (b0, b1), c0, c1 in zip(bounds, cuts[:-1], cuts[1:]):
        assert (b1 - b0 + 15) // 16 <= per_cu * (c1 - c0), (b0, b1, c0, c1)
    streams = [nat.cu_range_stream(c0, c1, device) for c0, c1 in zip(cuts[:-1], cuts[1:])]
    shards, results = [], []
    for (b0, b1), st in zip(bounds, streams):
        sh = PersistentShard(cfg, b0, b1 - b0)
        with torch.cuda.stream(st):
            results.append(sh.launch(inp['U'], inp['s'], inp['Vh'], inp['y'][b0:b1], inp['SNR'], inp['x'][b0:b1],
                                     sym[b0:b1], idx[b0:b1], xbuf, gen=0x51A2D000 + 16 * B + 4 * R + (alphabet == 'QPSK')))
        shards.append(sh)
    torch.cuda.synchronize()
    tot = {f: 0 for f, _ in nat.AmpCounts._fields_}
    for (b0, b1), sh, res in zip(bounds, shards, results):
        st, ct = read_result(res)
        assert st.nan_state >= 0, 'a shard lost its grid (exchange timed out)'
        assert (st.T, st.nan_state, st.stopped) == (wst.T, wst.nan_state, wst.stopped), (b0, st.T, wst.T)
        # the same bits (NaN where the reference's scalar is NaN: a noiseless point's 0/0)
        assert np.array_equal(np.asarray(list(st.last_scalar), np.float64), np.asarray(list(wst.last_scalar), np.float64),
                              equal_nan=True), b0
        for f, _ in nat.AmpCounts._fields_:
            tot[f] += getattr(ct, f)
        for a, w in ((sh.r, wr), (sh.xmmse, wx), (sh.var, wv)):
            assert torch.equal(a.reshape(b1 - b0, -1).view(torch.int32), w.reshape(B, -1)[b0:b1].view(torch.int32)), b0
    for f, ty in nat.AmpCounts._fields_:
        if ty is C.c_int64:
            assert tot[f] == getattr(wct, f), f
        elif math.isnan(getattr(wct, f)):
            assert math.isnan(tot[f]), f   # the whole batch's sum is NaN (a noiseless point's 0/0)
        else:
            assert abs(tot[f] - getattr(wct, f)) <= 1e-12 * max(1.0, abs(getattr(wct, f))), f
    assert whole['T'] == wst.T


def test_persistent_shard_stream_checks(device):
    """amp_vamp_detect_count_shard refuses, before launching, every launch whose grid could fail to
    be co-resident with its partners: a plain stream (two of them may share a
    hardware queue: gpurun r5c7's lost grid), a CU range its workgroups do not fit, and a range
    overlapping another shard of the same generation; then the valid pair runs to the whole batch's T."""
    import amp_native as nat
    from test_gpu_vamp import _config, _regen_inputs
    from vamp import VAMP, PersistentShard, read_result
    B = 4096
    cfg = _config(256, 8, 512, B, '16QAM', iterations=20)
    inp = _regen_inputs(cfg, 3, 8.0)
    det = VAMP(cfg, engine=2)
    L = det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
    T_whole = int(L.loss['T'])
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    half = ncu // 2
    xbuf = PersistentShard.xbuf(cfg, device)
    nat.check(nat.lib().amp_vamp_shard_reset(nat.dptr(xbuf), nat.stream_ptr(device)), 'reset')
    torch.cuda.synchronize()
    sym = torch.as_tensor(np.asarray(inp['sym'], np.int64)).reshape(B, cfg.L)
    idx = torch.as_tensor(np.asarray(inp['idx'], np.int64)).reshape(B, cfg.L)
    rows = B // 2
    gen = 0x5EED0000 + ncu

    def launch(b0, stream):
        sh = PersistentShard(cfg, b0, rows)
        with torch.cuda.stream(stream):
            return sh.launch(inp['U'], inp['s'], inp['Vh'], inp['y'][b0:b0 + rows], inp['SNR'],
                             inp['x'][b0:b0 + rows], sym[b0:b0 + rows], idx[b0:b0 + rows], xbuf, gen=gen)

    with pytest.raises(nat.AmpError, match='amp_stream_create_cu_range'):
        launch(0, torch.cuda.Stream(device))
    with pytest.raises(nat.AmpError, match='do not fit'):
        launch(0, nat.cu_range_stream(0, half // 2, device))
    r0 = launch(0, nat.cu_range_stream(0, half, device))
    with pytest.raises(nat.AmpError, match='overlap'):
        launch(rows, nat.cu_range_stream(half // 2, half + half // 2, device))
    r1 = launch(rows, nat.cu_range_stream(half, ncu, device))
    torch.cuda.synchronize()
    for res in (r0, r1):
        st, _ = read_result(res)
        assert st.nan_state >= 0 and st.T == T_whole, (st.nan_state, st.T, T_whole)
