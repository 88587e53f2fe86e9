"""Trial-sharded Monte-Carlo epochs across ranks (one process per GPU; gloo on the CPU here):
the real Loss counter merge that bench.py and Model use (one all-reduce of amp_counts), and
distinct random streams per rank when no seed is given."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from config import Config


def _cfg(B=64):
    return Config(32, 4, 64, 1, 1, batch=B, generator_mode='sparc', iterations=5, alphabet='16QAM',
                  channel_profile='uniform', channel_truncation='tail', device='cpu')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _counts_for(rank, epoch, cfg):
    """Plausible amp_counts of one epoch (every counter within its range)."""
    import amp_native as nat
    rng = np.random.default_rng(1000 * rank + epoch)
    S = cfg.B * cfg.Na * cfg.Lin
    c = nat.AmpCounts()
    c.ier, c.ser = int(rng.integers(0, S)), int(rng.integers(0, S))
    c.iber, c.sber = int(rng.integers(0, 3 * S)), int(rng.integers(0, 4 * S))
    c.ver = int(rng.integers(0, cfg.B * cfg.Lin))
    c.verf = c.verm = c.verL = c.fer = int(rng.integers(0, cfg.B))
    c.mse, c.msef, c.msem, c.mseL = (float(v) for v in rng.random(4) * S)
    return c


def _merge_worker(rank, world, port, out, epochs):
    torch.distributed.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                                         world_size=world)
    try:
        from loss import Loss, allreduce_counts, counts_to_vector
        cfg = _cfg()
        acc = np.zeros(13)
        for e in range(epochs):
            acc += counts_to_vector(_counts_for(rank, e, cfg))
        merged = allreduce_counts(acc)
        L = Loss(cfg)
        rates = L.rates_from_vector(merged, epochs=world * epochs)
        with open(os.path.join(out, f'merge{rank}.json'), 'w') as f:
            json.dump({'rates': [float(r) for r in rates], 'keys': L.keys}, f)
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.timeout(180)
def test_counter_merge_two_ranks_equals_epoch_average(tmp_path):
    """Summed counters of 2 ranks x 3 epochs, one all-reduce, then the metrics: equal to
    Loss.accumulate + Loss.average over the six per-epoch Loss dicts (loss.py:325-346)."""
    world, epochs = 2, 3
    mp.start_processes(_merge_worker, args=(world, _free_port(), str(tmp_path), epochs), nprocs=world, join=True,
                       start_method='spawn')
    got = [json.load(open(tmp_path / f'merge{r}.json')) for r in range(world)]
    assert got[0] == got[1]
    from loss import Loss
    cfg = _cfg()
    tot = Loss(cfg)
    for r in range(world):
        for e in range(epochs):
            L = Loss(cfg)
            L.dump()
            L.loss = {'T': 0}
            L.record(L.rates_from_counts(_counts_for(r, e, cfg)), 3)
            tot.accumulate(L)
    tot.average(world * epochs)
    for k, v in zip(got[0]['keys'], got[0]['rates']):
        assert v == pytest.approx(float(tot.loss[k]), rel=1e-6, abs=1e-12), k


def _seed_worker(rank, world, port, out):
    torch.distributed.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                                         world_size=world)
    try:
        from model import Model
        m = Model(_cfg(4), 'vamp', path=out, amp=object(), seed=None)
        draws = {'np': np.random.normal(size=4).tolist(), 'torch': torch.randn(4).tolist(), 'seed': m.seed}
        with open(os.path.join(out, f'seed{rank}.json'), 'w') as f:
            json.dump(draws, f)
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.timeout(180)
def test_unseeded_ranks_draw_distinct_streams(tmp_path):
    world = 2
    mp.start_processes(_seed_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method='spawn')
    a, b = (json.load(open(tmp_path / f'seed{r}.json')) for r in range(world))
    assert a['seed'] == b['seed'] and a['seed'] is not None      # one broadcast base seed
    assert a['np'] != b['np'] and a['torch'] != b['torch']        # per-rank streams differ
