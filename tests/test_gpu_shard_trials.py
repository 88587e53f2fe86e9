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
