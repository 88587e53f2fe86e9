#!/usr/bin/env python3
"""time(oracle) / time(reference) on the same cores, same inputs (build container only: the
reference never travels to the GPU box).  SURVEY.md §8(d): the CPU baseline that bench.py times
on the GPU box is the numpy oracle; this records how its speed relates to the reference's own
CPU path so the reported baseline can be read as "the reference's CPU path".

Both run VAMP.forward + Loss (detection, decision and metrics) at cfg4 (Nt=256 Nr=512 Na=8
16-QAM, 20 iterations) on `--trials` trials, one warm-up then the median of `--repeats`.

  python tools/cpu_ratio.py [--trials 4096] [--threads 8] [--repeats 3]
"""
import argparse
import json
import os
import sys
import time

sys.dont_write_bytecode = True
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get('AMP_REFERENCE', '/root/reference')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--trials', type=int, default=4096)
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--repeats', type=int, default=3)
    ap.add_argument('--ebn0', type=float, default=8.0)
    args = ap.parse_args()
    import numpy as np
    import torch
    from threadpoolctl import threadpool_limits
    torch.set_num_threads(args.threads)
    sys.path.insert(0, REF)
    from config import Config            # reference modules (flat import, as its drivers do)
    from channel import Channel
    from data import Data
    import vamp as ref_vamp
    sys.path.remove(REF)
    sys.path.insert(0, REPO)
    from oracle import OracleConfig, vamp_detect, loss_dict

    cfg = Config(256, 8, 512, 1, 1, batch=args.trials, generator_mode='sparc', iterations=20, alphabet='16QAM',
                 channel_profile='uniform', channel_truncation='tail', device='cpu')
    np.random.seed(0)
    torch.manual_seed(0)
    ch, da = Channel(cfg), Data(cfg)
    _, A = ch.generate_as_sparc()
    U, s, Vh = torch.linalg.svd(A, full_matrices=False)
    x, sym, idx = da.generate_message()
    SNR = 10 ** ((args.ebn0 + 10 * np.log10(cfg.code_rate)) / 10)
    y = A @ x + ch.awgn(SNR)

    def run_ref():
        L = ref_vamp.VAMP(cfg)(U, s, Vh, y, SNR, x, sym, idx)
        return int(L.loss['T'])

    ocfg = OracleConfig(256, 8, 512, B=args.trials, alphabet='16QAM', iterations=20)
    xs, ys = x.numpy()[..., 0], y.numpy()[..., 0]

    def run_oracle():
        out = vamp_detect(U.numpy(), s.numpy(), Vh.numpy(), ys, SNR, ocfg)
        loss_dict(out['r'], out['xmmse'], xs, sym, idx, out['T'], ocfg)
        return int(out['T'])

    res = {}
    with threadpool_limits(limits=args.threads):
        for name, fn in (('reference', run_ref), ('oracle', run_oracle)):
            fn()
            ts = []
            for _ in range(args.repeats):
                t0 = time.perf_counter()
                T = fn()
                ts.append(time.perf_counter() - t0)
            res[name] = dict(median_s=float(np.median(ts)), runs_s=ts, T=T,
                             symbol_vectors_per_s=args.trials / float(np.median(ts)))
    res['oracle_over_reference_time'] = res['oracle']['median_s'] / res['reference']['median_s']
    res['threads'] = args.threads
    res['trials'] = args.trials
    print(json.dumps(res))


if __name__ == '__main__':
    main()
