"""One rank of the trial-sharded GPU test (tests/test_gpu_shard_trials.py): ShardedVAMP on this
rank's slice of each case's batch, gloo process group (every rank on cuda:0), results to JSON /
npy in the output directory.  Usage: shard_trials_worker.py RANK WORLD PORT OUTDIR CASE..."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, '..'), os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def case_inputs(name):
    """CASE = [bamp:|bampisi:|scampisi:]alphabet:EbN0:B[:yscale] — VAMP / BAMP at the cfg2 shape
    (Nt=64 Na=4 Nr=128), or BAMP / SCAMP at a small ISI shape (Nt=32 Na=4 Nr=32 Lin=4 Lh=2:
    banded GEMMs); host
    replica, seed 7.  Returns (detector, cfg, forward arguments)."""
    from channel import Channel
    from config import Config
    from data import Data
    f = name.split(':')
    algo = f.pop(0) if f[0] in ('bamp', 'bampisi', 'scampisi') else 'vamp'
    alph, ebn0, B = f[0], float(f[1]), int(f[2])
    scale = float(f[3]) if len(f) > 3 else 1.0
    shape = (32, 4, 32, 4, 2) if algo in ('bampisi', 'scampisi') else (64, 4, 128, 1, 1)
    cfg = Config(*shape, batch=B, generator_mode='sparc', iterations=20, alphabet=alph,
                 channel_profile='uniform', channel_truncation='tail', device='cpu')
    np.random.seed(7)
    torch.manual_seed(7)
    ch, da = Channel(cfg), Data(cfg)
    Wc, A = ch.generate_as_sparc()
    x, sym, idx = da.generate_message()
    SNR = cfg.snr(ebn0)
    y = (A @ x + ch.awgn(SNR)) * scale
    cfg.device = 'cuda'
    if algo == 'vamp':
        U, s, Vh = torch.linalg.svd(A, full_matrices=False)
        return 'vamp', cfg, (U, s, Vh, y, SNR, x, sym, idx)
    if algo == 'scampisi':
        return 'scamp', cfg, (Wc, A, y, SNR, x, sym, idx)
    return 'bamp', cfg, (A, y, SNR, x, sym, idx)


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    torch.distributed.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank,
                                         world_size=world)
    try:
        from bamp import ShardedBAMP
        from scamp import ShardedSCAMP
        from vamp import ShardedVAMP
        dev = torch.device('cuda:0')
        res = {}
        for name in sys.argv[5:]:
            algo, cfg, args = case_inputs(name)
            det = {'vamp': ShardedVAMP, 'bamp': ShardedBAMP, 'scamp': ShardedSCAMP}[algo](cfg)
            mv = lambda t: t.to(dev).contiguous() if isinstance(t, torch.Tensor) else t  # noqa: E731
            L = det(*(mv(a) for a in args))
            res[name] = {k: (float(v) if np.ndim(v) == 0 else np.asarray(v).tolist()) for k, v in L.loss.items()}
            res[name]['slice'] = list(det.shard())
            np.save(os.path.join(out, f'{name.replace(":", "_")}_r{rank}.npy'), det.last_shard[0].cpu().numpy())
        with open(os.path.join(out, f'rank{rank}.json'), 'w') as fh:
            json.dump(res, fh)
    finally:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
