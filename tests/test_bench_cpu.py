"""bench.py's measured region (timed_epochs: warmup, timed steps, counter merge, max over ranks)
driven on gloo CPU ranks, world size 2, in both shard modes, with the numpy oracle standing in
for the GPU detector (test infrastructure only; bench.py itself never imports it):

* --shard trials: ONE batch split over the ranks (vamp_detect_sharded: the batch scalars of every
  iteration all-reduced, as ShardedVAMP's hook does), each rank deciding its slice with the
  whole-batch flat indices, the slice counters summed by the detector's own all-reduce and
  timed_epochs' merge the identity -> every rank's merged counters equal the single-rank
  (whole-batch) run's exactly;
* --shard epochs: each rank its own epoch, timed_epochs' merge = loss.allreduce_counts -> the sum
  of the per-rank counters.
"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import golden_io as gio

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = ['vamp_QPSK_6_0', 'vamp_16QAM_20_0', 'vamp_QPSK_0_1']


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _slice_counts(r, xmmse, x, sym, idx, b0, ocfg):
    """amp_counts (loss.COUNT_FIELDS order) of rows [b0, b0 + len(r)) of a batch, with the
    whole-batch flat indices (loss.py:105-179; amp_map_decide_count_rows)."""
    from oracle.amp_oracle import _de2bi_count, map_decision
    Bl = r.shape[0]
    L, M, Nt = ocfg.L, ocfg.M, ocfg.Nt
    xhat, shat, ihat = map_decision(r, ocfg)
    ihat = ihat + b0 * L * M
    sym = np.asarray(sym).reshape(-1)[b0 * L:(b0 + Bl) * L]
    idx = np.asarray(idx).reshape(-1)[b0 * L:(b0 + Bl) * L]
    xs = np.asarray(x).reshape(-1, Nt)[b0:b0 + Bl]
    cu = (np.count_nonzero(xhat.reshape(-1, Nt) - xs, axis=-1) > 0)          # Lin = 1: one channel use per trial
    se = np.abs(np.asarray(xmmse).reshape(-1, Nt).astype(np.complex128) - xs) ** 2
    v = [np.count_nonzero(ihat - idx), np.count_nonzero(shat - sym),
         _de2bi_count(np.bitwise_xor(ihat, idx), ocfg._ibits), _de2bi_count(np.bitwise_xor(shat, sym), ocfg.symbol_bits),
         cu.sum(), cu.sum(), cu.sum(), cu.sum(), cu.sum(),
         se.sum(), se.sum(), se.sum(), se.sum()]
    return np.array(v, dtype=np.float64)


def _worker(rank, world, port, out, mode):
    torch.distributed.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                                         world_size=world)
    try:
        sys.path.insert(0, REPO)
        import bench
        from loss import allreduce_counts
        from oracle import OracleConfig, vamp_detect_sharded

        def allreduce(v, op):
            t = torch.as_tensor(np.asarray(v, dtype=np.float64))
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM if op == 'sum'
                                         else torch.distributed.ReduceOp.MAX)
            return t.numpy()

        res = {}
        for name in CASES:
            c = gio.g1_cases()[name]
            B = int(c.B)
            ocfg = OracleConfig(int(c.Nt), int(c.Na), int(c.Nr), B=B, alphabet=str(c.alphabet), iterations=int(c.iters))
            y = np.asarray(c.y).reshape(B, -1)
            if mode == 'trials':
                b0, b1 = rank * B // world, (rank + 1) * B // world
            else:                          # epochs: the whole batch on every rank (its own epoch)
                b0, b1 = 0, B
            calls = []

            def step():
                o = vamp_detect_sharded(c.U, c.s, c.Vh, y[b0:b1], float(c.SNR), ocfg, B if mode == 'trials' else b1 - b0,
                                        allreduce if mode == 'trials' else (lambda v, op: np.asarray(v)))
                cnt = _slice_counts(o['r'], o['xmmse'], c.x, c.sym, c.idx, b0, ocfg)
                if mode == 'trials':
                    cnt = allreduce(cnt, 'sum')        # the detector's own counter all-reduce
                calls.append(int(o['T']))
                return cnt

            el, merged, _, npre = bench.timed_epochs(
                step, lambda h: h, steps=2, warmup=1,
                merge=(lambda v: v) if mode == 'trials' else allreduce_counts,
                barrier=torch.distributed.barrier,
                max_over_ranks=lambda e: float(allreduce([e], 'max')[0]))
            res[name] = {'merged': merged.tolist(), 'steps_run': len(calls), 'T': calls[-1], 'el': el}
        with open(os.path.join(out, f'{mode}{rank}.json'), 'w') as f:
            json.dump(res, f)
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize('mode', ['trials', 'epochs'])
def test_bench_timed_region_two_ranks_gloo(tmp_path, mode):
    from oracle import OracleConfig, vamp_detect
    cases = [n for n in CASES if n in gio.g1_cases()]
    assert len(cases) >= 2
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world, join=True)
    got = [json.load(open(tmp_path / f'{mode}{r}.json')) for r in range(world)]
    for name in cases:
        c = gio.g1_cases()[name]
        B = int(c.B)
        ocfg = OracleConfig(int(c.Nt), int(c.Na), int(c.Nr), B=B, alphabet=str(c.alphabet), iterations=int(c.iters))
        whole = vamp_detect(c.U, c.s, c.Vh, np.asarray(c.y).reshape(B, -1), float(c.SNR), ocfg)
        one = _slice_counts(whole['r'], whole['xmmse'], c.x, c.sym, c.idx, 0, ocfg)
        # warmup 1 + timed 2 steps; the timed region's counters are those of the 2 timed steps
        want = 2 * one * (1 if mode == 'trials' else world)
        for r in range(world):
            g = got[r][name]
            assert g['steps_run'] == 3 and g['T'] == int(whole['T']), (name, r, g)
            m = np.array(g['merged'])
            assert np.array_equal(m[:9], want[:9]), (name, r, m[:9], want[:9])      # integer counters: exact
            assert np.allclose(m[9:], want[9:], rtol=1e-12, atol=0, equal_nan=True), (name, r, m[9:], want[9:])
        assert got[0][name]['el'] == got[1][name]['el']                          # max over ranks on every rank
