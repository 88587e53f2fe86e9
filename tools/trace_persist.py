#!/usr/bin/env python3
"""Phase timing of the persistent engines (amp_vamp_persist_trace / amp_scamp_persist_trace): per
iteration and workgroup s_memtime stamps -> median cycles per phase, barrier skew across workgroups.

  python tools/trace_persist.py [--config cfg4] [--ebn0 8] [--gemm auto|x3|f32|h2|i8]
  python tools/trace_persist.py --config cfg3        (SCAMP, tools/configs_bench.py's cfg3 inputs)
"""
import argparse
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd'))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch        # noqa: E402

PHASES = ['r~ build', 'GEMM1', 'w store', 'GEMM2 + r', 'denoiser', 'partial publish', 'partial gather', 'scalars']
STRIDE = 10   # stamps per (workgroup, iteration): amp_vamp_persist.hip AMP_TRACE_STRIDE
ORDER = [0, 1, 2, 3, 4, 8, 5, 6, 7]   # stamp slots in time order
SPHASES = ['scalars + x planes', 'GEMM1', 's store', 'GEMM2 + xmap', 'denoiser', 'psi + publish',
           'partial gather', 'danger / exit']
SORDER = [0, 1, 2, 3, 4, 5, 6, 7, 8]


def scamp_trace(cfgname, ebn0):
    """cfg3-like SCAMP inputs (tools/configs_bench.py), one traced persistent forward."""
    import amp_native as nat
    from channel import Channel
    from config import Config
    from data import Data
    from scamp import SCAMP
    sys.path.insert(0, os.path.join(REPO, 'tools'))
    import configs_bench
    algo, Nt, Na, Nr, B, alph, iters, e0 = configs_bench.CFGS[cfgname]
    assert algo == 'scamp', cfgname
    cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=iters, alphabet=alph,
                 channel_profile='uniform', channel_truncation='tail', device='cpu')
    np.random.seed(0)
    torch.manual_seed(0)
    ch, da = Channel(cfg), Data(cfg)
    W, A = ch.generate_as_sparc()
    x, _, _ = da.generate_message()
    SNR = cfg.snr(ebn0 if ebn0 is not None else e0)
    y = A @ x + ch.awgn(SNR)
    cfg.device = 'cuda'
    dev = torch.device('cuda', 0)
    W, A, y = (t.to(dev).contiguous() for t in (W, A, y))
    det = SCAMP(cfg, engine=nat.ENGINE_PERSISTENT)
    for _ in range(3):
        det.detect(W, A, y, SNR)
    T = det.detect(W, A, y, SNR)
    nwg = (B + 15) // 16
    tr = torch.zeros(nwg * iters * STRIDE + 2 * nwg, dtype=torch.int64, device=dev)
    nat.check(nat.lib().amp_scamp_persist_trace(C.byref(T.dims), C.byref(T.const), C.byref(T.args), nat.dptr(tr),
                                                T.stream), 'trace')
    torch.cuda.synchronize()
    Tn = int(T.status().T)
    st = tr.cpu().numpy()[:nwg * iters * STRIDE].reshape(nwg, iters, STRIDE).astype(np.int64)[:, :Tn, SORDER]
    d = np.diff(st, axis=2)
    per_it = np.median(st[:, 1:, 0] - st[:, :-1, 0]) if Tn > 1 else 0
    print(f'SCAMP {cfgname}: T={Tn}  nwg={nwg}  median cycles per iteration {per_it:.0f}')
    for i, name in enumerate(SPHASES):
        v = d[:, 1:, i] if Tn > 1 else d[:, :, i]
        print(f'  {name:22s} median {np.median(v):9.0f}  p10 {np.percentile(v, 10):9.0f}  p90 {np.percentile(v, 90):9.0f}'
              f'  ({100 * np.median(v) / per_it:5.1f} %)' if per_it else '')


def main():
    import bench
    import amp_native as nat
    from config import Config
    from vamp import VAMP
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='cfg4')
    ap.add_argument('--ebn0', type=float, default=None)
    ap.add_argument('--gemm', default='auto', choices=['auto', 'x3', 'f32', 'h2', 'i8'])
    args = ap.parse_args()
    if args.config.startswith('cfg3'):
        return scamp_trace(args.config, args.ebn0)
    if args.ebn0 is None:
        args.ebn0 = 8.0
    Nt, Na, Nr, B, alph, iters = bench.CONFIGS[args.config]
    cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=iters, alphabet=alph,
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    dev = torch.device('cuda', 0)
    inp = bench.make_inputs(cfg, 0, args.ebn0, dev)
    gemm = {'auto': nat.GEMM_AUTO, 'x3': nat.GEMM_X3, 'f32': nat.GEMM_F32, 'h2': nat.GEMM_H2,
            'i8': nat.GEMM_I8}[args.gemm]
    det = VAMP(cfg, engine=nat.ENGINE_PERSISTENT, gemm=gemm)
    for _ in range(3):
        det.detect(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])
    T = det.detect(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])
    nwg = (B + 15) // 16
    tr = torch.zeros(nwg * iters * STRIDE + 4 * nwg, dtype=torch.int64, device=dev)
    s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    nat.check(nat.lib().amp_vamp_persist_trace(C.byref(T.dims), C.byref(T.const), C.byref(T.args), nat.dptr(tr),
                                               T.stream), 'trace')
    e0.record()
    torch.cuda.synchronize()
    ms = s0.elapsed_time(e0)
    a = tr.cpu().numpy()
    st = a[:nwg * iters * STRIDE].reshape(nwg, iters, STRIDE).astype(np.int64)[:, :, ORDER]
    Tn = int(T.status().T)
    st = st[:, :Tn]
    d = np.diff(st, axis=2)                       # [nwg, T, 8]
    total_cyc = np.median(st[:, -1, -1] - st[:, 0, 0])
    print(f'T={Tn}  nwg={nwg}  kernel+prepare {ms:.3f} ms (events)  median loop cycles {total_cyc:.0f}')
    per_it = np.median(st[:, 1:, 0] - st[:, :-1, 0]) if Tn > 1 else 0
    print(f'median cycles per iteration {per_it:.0f}')
    for i, name in enumerate(PHASES):
        v = d[:, 1:, i] if Tn > 1 else d[:, :, i]
        print(f'  {name:22s} median {np.median(v):9.0f}  p10 {np.percentile(v, 10):9.0f}  p90 {np.percentile(v, 90):9.0f}'
              f'  ({100 * np.median(v) / per_it:5.1f} %)' if per_it else '')
    raw = a[:nwg * iters * STRIDE].reshape(nwg, iters, STRIDE).astype(np.int64)[:, 1:Tn]
    if Tn > 1 and np.all(raw[:, :, 9] > 0):   # slot 9: the start of vamp_advance (the scalars' own work)
        print(f'  scalars: gather end -> advance start median {np.median(raw[:, :, 9] - raw[:, :, 6]):.0f}, '
              f'vamp_advance median {np.median(raw[:, :, 7] - raw[:, :, 9]):.0f} cycles')
    arrival_spread(a, st, nwg, iters, Tn)


def arrival_spread(a, st, nwg, iters, Tn):
    """Spread of the workgroups' arrival at the batch exchange (the stamp after the partial publish)
    per iteration, in cycles.  s_memtime counts each XCD's own clock (its own origin), so stamps
    are put on one time base with the per-workgroup (s_memtime, s_memrealtime) pairs taken at
    kernel start and end: rate = d memtime / d realtime (cycles per 10 ns tick), and
    t = realtime_start + (memtime - memtime_start) / rate.  (Raw s_memtime values are never compared
    across workgroups: their origins differ, even within one XCD.)"""
    base = nwg * iters * STRIDE
    m0, r0 = a[base:base + 2 * nwg:2].astype(np.float64), a[base + 1:base + 2 * nwg:2].astype(np.float64)
    m1, r1 = a[base + 2 * nwg::2].astype(np.float64), a[base + 2 * nwg + 1::2].astype(np.float64)
    if Tn < 2 or not (np.all(r1 > r0) and np.all(m1 > m0)):
        print('  barrier arrival spread: no valid end stamps (old library?) '
              f'm0 {m0[:3]} m1 {m1[:3]} r0 {r0[:3]} r1 {r1[:3]}')
        return
    rate = (m1 - m0) / (r1 - r0)                          # cycles per realtime tick, per workgroup
    arr = st[:, 1:, 6].astype(np.float64)                 # [nwg, T-1]: publish done
    g = r0[:, None] + (arr - m0[:, None]) / rate[:, None]  # realtime ticks
    cyc = np.median(rate)
    spread = (g.max(0) - g.min(0)) * cyc
    lag = (g - g.min(0)) * cyc                            # [nwg, T-1] cycles behind the first arrival
    late = np.argsort(-lag.mean(1))[:4]
    # per XCD (workgroup wg runs on XCD wg % 8: round-robin dispatch): mean lag and clock
    xl = [float(lag[x::8].mean()) for x in range(8)]
    xc = [float(np.median(rate[x::8]) * 100) for x in range(8)]
    print(f'  clock: {cyc * 100:.0f} MHz median (min {rate.min() * 100:.0f}, max {rate.max() * 100:.0f})')
    print(f'  barrier arrival spread, all workgroups (realtime-aligned, cycles): median {np.median(spread):.0f} '
          f'p10 {np.percentile(spread, 10):.0f} p90 {np.percentile(spread, 90):.0f}')
    print('  mean arrival lag per XCD (cycles): ' + ' '.join(f'{v:.0f}' for v in xl))
    print('  clock per XCD (MHz, median of its workgroups): ' + ' '.join(f'{v:.0f}' for v in xc))
    print(f'  latest workgroups on average: {list(map(int, late))} '
          f'(mean lag {[round(float((g[w] - g.min(0)).mean() * cyc)) for w in late]} cycles)')

if __name__ == '__main__':
    main()
