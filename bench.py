#!/usr/bin/env python3
"""Benchmark: detected symbol-vectors/s of the VAMP detector at BASELINE.json's config
(Nt=256, Nr=512, Na=8, 16-QAM, batch 4096, T <= 20), one process per GPU.

A step = one Monte-Carlo epoch of the hot path on inputs already resident in HBM:
VAMP.forward (all iterations, early exit, MAP decision and every error counter on the
GPU) + the one 128-byte result read-back — exactly what Model.simulate calls per epoch
(vamp_model.py:61).  The read-back of step k is waited for after step k+1's launches are
queued (Loss resolves lazily), so the GPU does not idle on the host between steps.  Input generation and the SVD are outside the timed region
(SURVEY.md §8(d)).  Each rank runs its own independent epoch (its own seed): Monte-Carlo
epochs are independent, so the path shards with no data-path collective ("weak").
`--shard trials` instead splits ONE batch over the ranks (ShardedVAMP, exact-compat: the
batch-global scalars of every iteration all-reduced through amp_set_allreduce_hook; "strong").

  python bench.py [--gpus N --steps K --warmup W] [--shard epochs|trials]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'amp-sparc-spatialmodulation_amd'))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch        # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense f32 MFMA (= f32 vector peak)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA
HBM_PEAK_GBS = 8000.0
# time(oracle) / time(reference) on the same 8 cores of the build container, same cfg4 workload
# (tools/cpu_ratio.py; the reference cannot travel to the GPU box): the port's CPU speed relative
# to the reference's CPU path: the two take the same time.
PORT_OVER_REFERENCE = 1.004   # profiles/r02_cpu_ratio.json (cfg4, 1024 trials, 8 threads, median of 3)

CONFIGS = {
    # name: (Nt, Na, Nr, B, alphabet, iterations)
    'cfg4': (256, 8, 512, 4096, '16QAM', 20),
    'cfg2': (64, 4, 128, 1024, '16QAM', 20),
}


def make_inputs(cfg, seed, EbN0, device):
    """Reference call order on the host RNG replica (CPU), then moved to the GPU."""
    from channel import Channel
    from data import Data
    dev = cfg.device
    cfg.device = 'cpu'
    np.random.seed(seed)
    torch.manual_seed(seed)
    ch, da = Channel(cfg), Data(cfg)
    _, A = ch.generate_as_sparc()
    U, s, Vh = torch.linalg.svd(A, full_matrices=False)
    x, sym, idx = da.generate_message()
    SNR = cfg.snr(EbN0)
    y = A @ x + ch.awgn(SNR)
    cfg.device = dev
    to = lambda t: t.to(device).contiguous()  # noqa: E731
    return dict(A=A, U=to(U), s=to(s), Vh=to(Vh), y=to(y), x=to(x), SNR=SNR,
                sym=torch.from_numpy(np.asarray(sym, np.int64)).to(device),
                idx=torch.from_numpy(np.asarray(idx, np.int64)).to(device),
                cpu=dict(U=U.numpy(), s=s.numpy(), Vh=Vh.numpy(), y=y.numpy()[..., 0], x=x.numpy()[..., 0],
                         sym=sym, idx=idx))


def cpu_baseline(cfgname, EbN0, seed, sample_trials, repeats=3):
    """The oracle (numpy restatement of the reference path, oracle/) timed on this host's
    cores on a bounded sample of the same workload: `sample_trials` trials of the config, one
    warm-up run, then the median of `repeats` timed runs."""
    from threadpoolctl import threadpool_limits
    from oracle import OracleConfig, vamp_detect, loss_dict
    from config import Config
    Nt, Na, Nr, B, alph, iters = CONFIGS[cfgname]
    cores = min(16, os.cpu_count() or 1)
    cfg = Config(Nt, Na, Nr, 1, 1, batch=sample_trials, generator_mode='sparc', iterations=iters, alphabet=alph,
                 channel_profile='uniform', channel_truncation='tail', device='cpu')
    inp = make_inputs(cfg, seed, EbN0, 'cpu')['cpu']
    ocfg = OracleConfig(Nt, Na, Nr, B=sample_trials, alphabet=alph, iterations=iters)
    times = []
    with threadpool_limits(limits=cores):
        for rep in range(repeats + 1):
            t0 = time.perf_counter()
            out = vamp_detect(inp['U'], inp['s'], inp['Vh'], inp['y'], cfg.snr(EbN0), ocfg)
            loss_dict(out['r'], out['xmmse'], inp['x'], inp['sym'], inp['idx'], out['T'], ocfg)
            if rep > 0:                       # run 0 is the warm-up
                times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    return dict(value=sample_trials / dt, unit='symbol-vectors/s', cores=cores, kind='port',
                sample=f'{sample_trials} trials of {cfgname} (Nt={Nt} Nr={Nr} Na={Na} {alph}), EbN0={EbN0} dB, '
                       f'T={out["T"]}, numpy oracle incl. decision+metrics, median of {repeats} runs '
                       f'({", ".join(f"{t:.1f}" for t in times)} s) after one warm-up',
                port_over_reference_time=PORT_OVER_REFERENCE)


# The PMC summary (tools/profile.sh -> tools/prof_summary.py) of THIS build's default command, per
# GEMM arithmetic; `roofline.traffic` names it (`traffic_source`).  The counters cannot be read by
# the timed run itself (rocprofv3 --pmc replays the launch), so the file is the measurement.
TRAFFIC_PROFILE = {'bf16x3': 'profiles/r06_cfg4_vamp_x3.txt', 'fp16x2': 'profiles/r03_cfg4_vamp_swz.txt'}


def traffic_from_profile(persistent, gname):
    """HBM bytes per launch of the dominant kernel from the committed PMC summary of the same
    command: FETCH_SIZE x 2 (gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md) +
    WRITE_SIZE.  Returns (bytes or None, the profile file it came from or None)."""
    import re
    name = 'amp::vamp_persist' if persistent else 'amp::vamp_k2'
    rel = TRAFFIC_PROFILE.get(gname) if persistent else None
    if not rel or not os.path.exists(os.path.join(REPO, rel)):
        return None, None
    for line in open(os.path.join(REPO, rel)):
        if line.startswith(name) and 'FETCH_SIZE' in line and 'WRITE_SIZE' in line:
            fe = re.search(r'FETCH_SIZE=(\d+)KB', line)
            wr = re.search(r'WRITE_SIZE=(\d+)KB', line)
            if fe and wr:
                return (2 * int(fe.group(1)) + int(wr.group(1))) * 1024, rel
    return None, None


def timed_epochs(step, counts_of, steps, warmup, merge, sync=lambda: None, barrier=lambda: None,
                 max_over_ranks=lambda el: el, prewarm_s=0.0):
    """The measured region of every mode (the driver contract), on any device:

    * untimed: first `prewarm_s` seconds of steps (the chip's clocks ramp over the first ~25 ms of
      back-to-back epochs, DESIGN.md §3.3: a short `--warmup` would time the ramp), then EXACTLY
      `warmup` steps;
    * barrier + sync, then EXACTLY `steps` timed steps. step() queues one epoch and returns its
      handle; counts_of(handle) -> float64[13] counters of that epoch (for the GPU detector it
      resolves the lazy read-back, so step k's counters are read while step k+1's launches run);
    * merge(sum of the counters) inside the timed region: ONE all-reduce over the ranks for
      independent epochs, the identity for trial sharding (the detector already merged them);
    * sync, barrier, elapsed time max over ranks.
    Returns (elapsed seconds, merged float64[13], last handle, prewarm steps run)."""
    npre = 0
    if prewarm_s > 0:
        t_end = time.perf_counter() + prewarm_s
        while time.perf_counter() < t_end:
            h = step()
            npre += 1
        counts_of(h)
    for _ in range(warmup):
        h = step()
    if warmup:
        counts_of(h)
    barrier()
    sync()
    t0 = time.perf_counter()
    acc = np.zeros(13)
    h = None
    for _ in range(steps):
        prev = h
        h = step()
        if prev is not None:
            acc += counts_of(prev)
    acc += counts_of(h)          # the last step's counters inside the timed region too
    merged = merge(acc)
    sync()
    el = time.perf_counter() - t0
    barrier()
    return max_over_ranks(el), merged, h, npre


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher: start N fresh child processes, one per
    GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them), wait for
    all of them and return the worst exit status.  The parent makes no GPU call (it never
    initialises HIP, and never re-execs itself)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return (bad[0] if bad[0] > 0 else 1) if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    # the chip's clocks ramp over the first ~25 ms of back-to-back epochs (vamp_persist 1.22 ms
    # -> 1.05 ms over 20 steps on the box, r01): the default warmup covers the ramp
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=30)
    ap.add_argument('--config', default='cfg4', choices=sorted(CONFIGS))
    ap.add_argument('--ebn0', type=float, default=8.0)
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--cpu-sample', type=int, default=4096)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--engine', default='auto', choices=['auto', 'launches', 'persistent'])
    # the persistent engine's GEMM arithmetic: auto = bf16x3 (three bf16 pieces per f32 operand,
    # 24 bits, dropped product terms < 2^-24: the reference's c64 operand precision); h2 = the
    # opt-in fp16x2 form (22-bit operands, narrower than the reference: a second, labelled line)
    ap.add_argument('--gemm', default='auto', choices=['auto', 'x3', 'f32', 'h2', 'i8'])
    # independent epochs per rank (weak scaling, the default) or ONE batch of B trials split over
    # the ranks (strong scaling: ShardedVAMP, the batch scalars all-reduced every iteration)
    ap.add_argument('--shard', default='epochs', choices=['epochs', 'trials'])
    ap.add_argument('--prewarm-ms', type=float, default=300.0,
                    help='untimed steps for this long before the --warmup steps (clock ramp)')
    args = ap.parse_args()

    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}')
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(local)
        tdist.init_process_group('nccl', device_id=torch.device('cuda', local))
    device = torch.device('cuda', local)

    from config import Config
    from vamp import VAMP, ShardedVAMP
    from loss import allreduce_counts, counts_to_vector
    import ctypes as C
    import amp_native as nat
    nat.lib()

    Nt, Na, Nr, B, alph, iters = CONFIGS[args.config]
    cfg = Config(Nt, Na, Nr, 1, 1, batch=B, generator_mode='sparc', iterations=iters, alphabet=alph,
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    trials = args.shard == 'trials'
    # epochs: every rank detects its own independent Monte-Carlo epoch (its own channel, messages
    # and noise: seed + rank); trials: every rank draws the SAME epoch and detects its slice
    inp = make_inputs(cfg, args.seed + (0 if trials else rank), args.ebn0, device)
    engine = {'auto': nat.ENGINE_AUTO, 'launches': nat.ENGINE_LAUNCHES, 'persistent': nat.ENGINE_PERSISTENT}[args.engine]
    gemm = {'auto': nat.GEMM_AUTO, 'x3': nat.GEMM_X3, 'f32': nat.GEMM_F32, 'h2': nat.GEMM_H2, 'i8': nat.GEMM_I8}[args.gemm]
    det = ShardedVAMP(cfg) if trials else VAMP(cfg, engine=engine, gemm=gemm)
    seq = [0]

    def step():
        det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        seq[0] += 1
        return seq[0]

    def counts_of(h):
        # step() resolved the previous forward's read-back; only the newest one is waited for here
        if h == seq[0]:
            det.L.resolve()
        return counts_to_vector(det.L.last_counts)

    def max_over_ranks(el):
        if not dist:
            return el
        t = torch.tensor([el], dtype=torch.float64, device=device)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        return t.item()

    el, merged, _, npre = timed_epochs(
        step, counts_of, args.steps, args.warmup,
        merge=(lambda v: v) if trials else allreduce_counts,    # ONE all-reduce (RCCL) of the counters
        sync=lambda: torch.cuda.synchronize(device), barrier=(tdist.barrier if dist else (lambda: None)),
        max_over_ranks=max_over_ranks, prewarm_s=args.prewarm_ms * 1e-3)
    L = det.L
    T = int(L.loss['T'])
    n_epochs = args.steps * (1 if trials else world)     # epochs whose counters `merged` holds
    rates = dict(zip(L.keys, L.rates_from_vector(merged, epochs=n_epochs)))
    ver, ser = float(rates['ver']), float(rates['ser'])

    # dominant kernel timed with HIP events on the stream it runs on: the persistent engine's
    # single vamp_persist launch (T iterations: 2 complex mat-vecs per trial-iteration), or the
    # launch engine's GEMM2 + fused denoiser kernel (one complex mat-vec per trial); trial
    # sharding profiles the launch engine on this rank's slice (what it runs per iteration)
    if trials:
        b0, b1 = det.shard()
        Bp = b1 - b0
        pcfg = Config(Nt, Na, Nr, 1, 1, batch=Bp, generator_mode='sparc', iterations=iters, alphabet=alph,
                      channel_profile='uniform', channel_truncation='tail', device='cuda')
        prof = VAMP(pcfg, engine=nat.ENGINE_LAUNCHES)
        Tr = prof.detect(inp['U'], inp['s'], inp['Vh'], inp['y'][b0:b1].contiguous(), inp['SNR'])
    else:
        Bp = B
        Tr = det.detect(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])
    persistent = nat.lib().amp_vamp_select_engine(C.byref(Tr.dims), Tr.k, Tr.args.engine) == nat.ENGINE_PERSISTENT
    ms = (C.c_float * 4)()
    nat.check(nat.lib().amp_vamp_profile(C.byref(Tr.dims), C.byref(Tr.const), C.byref(Tr.args), ms, Tr.stream),
              'amp_vamp_profile')
    N, k = Nt, min(Nt, Nr)
    flops_mv = 8.0 * Bp * N * k                    # complex [N x k] . [k] per trial = 8 real flop / CMAC
    gmode = nat.lib().amp_vamp_select_gemm(C.byref(Tr.dims), Tr.k, Tr.args.gemm) if persistent else nat.GEMM_F32
    gname = {nat.GEMM_X3: 'bf16x3', nat.GEMM_H2: 'fp16x2', nat.GEMM_I8: 'int8x4'}.get(gmode, 'f32')
    arith = {'bf16x3': 'GEMMs: every f32 operand split into three bf16 pieces (24 significant bits), six '
                       'products per f32 product (dropped terms < 2^-24 relative), f32 accumulation on '
                       'v_mfma_f32_16x16x32_bf16; denoiser f32, scalars f32/f64 as the reference',
             'fp16x2': 'OPT-IN, narrower than the reference: GEMM operands split into two fp16 pieces (22 '
                       'significant bits), the 2^-22 lo.lo term dropped, f32 accumulation',
             'int8x4': 'GEMMs in block fixed point: every A row and operator column scaled by its own power of '
                       'two, each value a 31-bit integer in four balanced int8 digits, the ten digit products '
                       'of levels 0-3 exact in int32 on v_mfma_i32_16x16x64_i8, levels combined in f32 '
                       '(>= 24 significant bits down to 2^-7 of the row/column max; dropped terms < 2^-30 of '
                       'row max . column max); denoiser f32, scalars f32/f64 as the reference',
             'f32': 'GEMMs on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32)'}[gname]
    # the fp16x2 engine forms y~ = (s Uh) y in its prologue when n == 2N (amp_vamp.hip): those
    # 8 B n k flops per trial belong to the launch then
    ytil_in = persistent and gname == 'fp16x2' and Nr == 2 * Nt and os.environ.get('AMP_YTIL_IN_KERNEL') != '0'
    if persistent:
        kern, flops_launch = 'vamp_persist (whole iteration loop: 2 GEMMs + LMMSE + Onsager + denoiser per iteration' + \
            (', y~ GEMM in the prologue)' if ytil_in else ')'), 2.0 * flops_mv * T + (8.0 * Bp * Nr * k if ytil_in else 0.0)
        kms = {'prepare': ms[0], 'vamp_persist': ms[1], 'forward': ms[3]}
    else:
        kern, flops_launch = 'vamp_k2 (GEMM2 + Onsager update + section denoiser)', flops_mv
        kms = {'gemm1': ms[0], 'gemm2_denoise': ms[1], 'reduce': ms[2], 'forward': ms[3]}
    achieved_alone = flops_launch / (ms[1] * 1e-3) / 1e12
    # the same kernel timed inside a loop of forwards, as the timed region runs it (the standalone
    # launch above runs ~2-3 % faster: no neighbouring launches): HIP event pairs
    # the library records around every vamp_persist launch (amp_debug_persist_timing)
    ms_loop = None
    if persistent and not trials:
        nat.check(nat.lib().amp_debug_persist_timing(1), 'amp_debug_persist_timing')
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(device)
        nat.check(nat.lib().amp_debug_persist_timing(0), 'amp_debug_persist_timing')
        n_t, m_t = C.c_int32(0), C.c_float(0.0)
        nat.check(nat.lib().amp_debug_persist_time(C.byref(n_t), C.byref(m_t)), 'amp_debug_persist_time')
        if n_t.value == args.steps:
            ms_loop = float(m_t.value)
            kms['vamp_persist_in_loop'] = ms_loop
    achieved = flops_launch / ((ms_loop if ms_loop else ms[1]) * 1e-3) / 1e12
    traffic, traffic_src = traffic_from_profile(persistent, gname)
    if rank != 0:
        if dist:
            tdist.destroy_process_group()
        nat.unload()
        return
    ms_step = el / args.steps * 1e3
    gb = B if trials else world * B                # trials detected per step, all ranks together
    value = gb / (el / args.steps)
    if trials:
        par = (f'trial-shard x{world} of ONE batch (exact-compat: rank r detects trials [r B/{world}, (r+1) B/{world}), '
               'the batch scalars all-reduced 4x per iteration, one counter all-reduce)')
    else:
        par = f'epoch-shard x{world} (independent epochs, one all-reduce of the error counters)'
    out = {
        'metric': 'detected symbol-vectors/sec, VAMP Nt=256 Nr=512 16-QAM; SER match vs ref',
        'value': value, 'unit': 'symbol-vectors/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': ms_step, 'higher_is_better': True, 'scaling': 'strong' if trials else 'weak',
        'vs_baseline': None, 'dtype': gname,
        'data': 'synthetic (reference generators replayed: sparc channel, segmented 16-QAM messages, AWGN)',
        'config': {'workload': f'{args.config}: VAMP Nt={Nt} Nr={Nr} Na={Na} {alph} batch={B} iterations<={iters} '
                               f'EbN0={args.ebn0} dB, one channel per batch',
                   'global_batch': gb, 'shard': args.shard, 'parallelism': par},
        'detail': {'T': T, 'ver': ver, 'ser': ser, 'epochs': n_epochs,
                   'trial_iterations_per_s': gb * T / (el / args.steps),
                   'engine': 'persistent' if persistent else 'launches', 'kernel_ms': kms,
                   'arithmetic': arith,
                   'grid_rescues': int(getattr(det, 'grid_rescues', 0)),
                   'prewarm': {'ms': args.prewarm_ms, 'steps': npre,
                               'why': 'untimed steps before --warmup: the clocks ramp over the first ~25 ms'}},
        'roofline': {'bound': 'mfma', 'achieved': achieved, 'peak': FP32_MFMA_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                     'frac': achieved / FP32_MFMA_PEAK_TFLOPS,
                     'timing': 'in-loop (HIP events around every vamp_persist launch of a loop of forwards)'
                               if ms_loop else 'standalone launch (HIP events)',
                     'frac_standalone': achieved_alone / FP32_MFMA_PEAK_TFLOPS, 'traffic': traffic,
                     'traffic_source': traffic_src,
                     'kernel': kern, 'flop_per_launch': flops_launch,
                     'gemm': gname},
    }
    if gname != 'f32':
        # the f32 products run as six bf16 (bf16x3) or three fp16 (fp16x2) MFMA products each
        # (amp_persist.h gemm_x3 / gemm_h2): the matrix cores' own rate against the dense peak of
        # that input type (bf16 and fp16 have the same dense peak on gfx950)
        mult = 6 if gname == 'bf16x3' else 3
        out['roofline'][gname[:4] + '_issued'] = {'achieved': mult * achieved, 'peak': BF16_MFMA_PEAK_TFLOPS,
                                                 'frac': mult * achieved / BF16_MFMA_PEAK_TFLOPS}
    if not args.no_cpu_baseline and world == 1:
        out['cpu_baseline'] = cpu_baseline(args.config, args.ebn0, args.seed, args.cpu_sample)
    print(json.dumps(out), flush=True)
    if dist:
        tdist.destroy_process_group()
    nat.unload()


if __name__ == '__main__':
    main()
