#!/usr/bin/env python3
"""Diagnostic (GPU): why a trial-sharded persistent forward on two PLAIN streams can lose its grid
(gpurun r5c7).  Two shards of one cfg4 batch (2048 trials, 128 workgroups each: the
pair fills the 256 CUs exactly) are launched on plain torch streams s[0] and s[j], j = 1 .. K - 1,
one pair at a time.  Per pair: each shard's status (nan_state -1 = its grid exchange timed out),
its wall span between HIP events recorded around its launch sequence, and when shard B's launch
began relative to shard A's.  If two plain streams are served by one hardware queue (HIP maps
streams onto GPU_MAX_HW_QUEUES = 4 queues), B's grid cannot be dispatched until A's grid — which
spins on B's partials — has given up after its bounded 2 s wait: B then starts ~2 s after A and
both report a lost grid; on separate queues both finish in about one forward.

Needs the diagnostic library (the shipped one refuses plain streams for this entry point):
  make -C amp-sparc-spatialmodulation_amd/csrc DIAG=1
  AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_diag.so AMP_SHARD_ANY_STREAM=1 \\
      python tools/shard_queue_probe.py [K]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    assert os.environ.get('AMP_SHARD_ANY_STREAM') and os.environ.get('AMP_LIB_PATH'), __doc__
    import amp_native as nat
    from test_gpu_vamp import _config, _regen_inputs
    from vamp import PersistentShard, read_result
    dev = torch.device('cuda:0')
    B = 4096
    cfg = _config(256, 8, 512, B, '16QAM', iterations=20)
    inp = _regen_inputs(cfg, 3, 8.0)
    sym = torch.as_tensor(np.asarray(inp['sym'], np.int64)).reshape(B, cfg.L)
    idx = torch.as_tensor(np.asarray(inp['idx'], np.int64)).reshape(B, cfg.L)
    xbuf = PersistentShard.xbuf(cfg, dev)
    streams = [torch.cuda.Stream(dev) for _ in range(K)]
    rows = B // 2
    print(f'{K} plain streams; shard A on s[0], shard B on s[j]; cfg4 16-QAM, 2 x {rows} trials', flush=True)
    for npair, j in enumerate(list(range(1, K)) + [1]):
        gen = 0x0DE50000 + npair   # one generation per forward: the same for both shards of the pair
        nat.check(nat.lib().amp_vamp_shard_reset(nat.dptr(xbuf), nat.stream_ptr(dev)), 'reset')
        torch.cuda.synchronize()
        res, ev = [], []
        for b0, st in ((0, streams[0]), (rows, streams[j])):
            sh = PersistentShard(cfg, b0, rows)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(st):
                e0.record(st)
                res.append(sh.launch(inp['U'], inp['s'], inp['Vh'], inp['y'][b0:b0 + rows], inp['SNR'],
                                     inp['x'][b0:b0 + rows], sym[b0:b0 + rows], idx[b0:b0 + rows], xbuf,
                                     gen=gen))
                e1.record(st)
            ev.append((e0, e1))
        torch.cuda.synchronize()
        stA, _ = read_result(res[0])
        stB, _ = read_result(res[1])
        spanA = ev[0][0].elapsed_time(ev[0][1])
        spanB = ev[1][0].elapsed_time(ev[1][1])
        startB = ev[0][0].elapsed_time(ev[1][0])
        endB = ev[0][0].elapsed_time(ev[1][1])
        print(f'j={j}: A nan_state {stA.nan_state:2d} T {stA.T:2d} span {spanA:8.2f} ms | '
              f'B nan_state {stB.nan_state:2d} T {stB.T:2d} span {spanB:8.2f} ms, B began {startB:8.2f} ms and '
              f'ended {endB:8.2f} ms after A began', flush=True)


if __name__ == '__main__':
    main()
