"""Failure semantics of the trial-sharded all-reduce hook (amp_sparc.h amp_set_allreduce_hook,
vamp.ShardHook): a rank whose hook fails locally still takes part in every
collective (NaN words), the driver keeps calling it, and EVERY rank raises at the end — no rank
waits on a peer that left the collective sequence.  Two gloo ranks on the CPU; the C driver's
call sequence is played by a Python stand-in (the hook is host code)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


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
        import amp_native as nat
        from config import Config
        from vamp import ShardedVAMP
        cfg = Config(16, 2, 32, 1, 1, batch=8, generator_mode='sparc', iterations=3, alphabet='QPSK',
                     channel_profile='uniform', channel_truncation='tail', device='cpu')
        det = ShardedVAMP(cfg)
        det._ws = torch.zeros(4096, dtype=torch.uint8)
        words = det._ws[:64].view(torch.float64)
        words[:] = float(rank + 1)

        def driver():   # the C driver's call pattern: every call is made, failure reported at the end
            failed = False
            for i in range(4):
                buf = det._ws.data_ptr() + 16 * i
                if rank == 1 and i == 1:
                    buf = det._ws.data_ptr() + 10 ** 6          # outside the workspace: a local error
                failed |= det._allreduce(buf, 2, nat.ALLREDUCE_SUM, None, None) != 0
            return -3 if failed else 0          # AMP_E_LAUNCH

        try:
            det._run_hooked(driver, 'stand-in driver')
            msg = 'no error'
        except RuntimeError as e:
            msg = str(e)
        with open(os.path.join(out, f'rank{rank}.txt'), 'w') as f:
            f.write(msg + '\n' + ' '.join(repr(float(v)) for v in words[:8].tolist()))
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.timeout(180)
def test_hook_failure_fails_every_rank(tmp_path):
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method='spawn')
    r0 = open(tmp_path / 'rank0.txt').read().splitlines()
    r1 = open(tmp_path / 'rank1.txt').read().splitlines()
    assert 'failed on another rank' in r0[0]
    assert 'all-reduce hook failed' in r1[0]
    w0 = [float(v) for v in r0[1].split()]
    # call 0 summed 1 + 2; call 1: rank 1 sent NaN; calls 2 and 3 went on normally
    assert w0[0] == w0[1] == 3.0
    assert w0[2] != w0[2] and w0[3] != w0[3]
    assert w0[4] == w0[5] == w0[6] == w0[7] == 3.0
