"""Monte-Carlo driver — drop-in for the reference's ``Model`` (vamp_model.py:17-69,
bamp_model.py:16-68, scamp_model.py:16-67): the EbN0 sweep that calls the detector once
per epoch, accumulates its ``Loss``, averages, writes ``{EbN0dB}.json`` and stops early
once FER < 1e-3.

One process per GPU: with ``torch.distributed`` initialised, the epochs of an SNR point
are split over the ranks in blocks of ``res`` (one channel realisation per block, as
``i % res == 0`` regenerates it in the reference), every rank runs its blocks on its own
GPU with its own random stream, and one all-reduce of the accumulated metrics per SNR
point merges them before the average (the only exchange: Monte-Carlo epochs are
independent).  With one process the epoch loop and the random-call order are exactly the
reference's.
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch import nn

from channel import Channel
from config import Config
from data import Data
from loss import Loss

_DIRS = {'vamp': 'VAMP', 'bamp': 'BAMPfinal', 'scamp': 'SCAMP'}   # vamp_model.py:29 etc.


def _detector(name: str, config: Config):
    if name == 'vamp':
        from vamp import VAMP
        return VAMP(config)
    if name == 'bamp':
        from bamp import BAMP
        return BAMP(config)
    if name == 'scamp':
        from scamp import SCAMP
        return SCAMP(config)
    raise ValueError(f'unknown detector {name!r}')


def _dist():
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        return torch.distributed.get_rank(), torch.distributed.get_world_size()
    return 0, 1


def _comm_device():
    """Where a collective's tensor must live: the rank's GPU for RCCL ('nccl'), host for gloo."""
    if torch.distributed.get_backend() == 'nccl':
        return torch.device('cuda', torch.cuda.current_device())
    return torch.device('cpu')


def _broadcast_seed() -> int:
    """A fresh base seed drawn on rank 0 (OS entropy) and broadcast to every rank."""
    base = torch.tensor([int(np.random.SeedSequence().entropy % (2 ** 31))], dtype=torch.int64)
    base = base.to(_comm_device())
    torch.distributed.broadcast(base, src=0)
    return int(base.cpu().item())


def svd_gram(A: torch.Tensor, max_cond: float = 20.0):
    """Thin SVD of a full-rank matrix through the Hermitian eigendecomposition of its Gram matrix
    (the smaller of A^H A / A A^H; torch.linalg.eigh), for Model(rng='device'): on MI355X 6.8 ms
    per cfg4 channel (512 x 256 c64) against 28.9 ms for torch.linalg.svd, and closer to exact
    (max |U S Vh - A| / max |A| 1.5e-6 vs 4.8e-5, max |Vh Vh^H - I| 1.0e-6 vs 5.5e-5;
    tools/svd_bench.py).  Squaring the matrix squares its condition number (the
    factors' orthogonality error grows as eps kappa^2: 4e-6 at kappa 6), so a channel with
    s_max / s_min above `max_cond` falls back to torch.linalg.svd; a random SPARC channel with
    n = 2N (cfg2, cfg4) sits near kappa = 6, a square one near N.  Returns (U, s, Vh) as torch.linalg.svd(A,
    full_matrices=False): s descending, U [n, k], Vh [k, N], k = min(n, N)."""
    n, N = A.shape[-2], A.shape[-1]
    tall = n >= N
    G = A.mH @ A if tall else A @ A.mH
    w, E = torch.linalg.eigh(G)                    # ascending
    w, E = w.flip(-1), E.flip(-1)
    s = w.clamp_min(0).sqrt()
    if not bool((s[..., -1] * max_cond > s[..., 0]).all()):
        return torch.linalg.svd(A, full_matrices=False)
    sd = s.to(A.dtype)
    if tall:                                       # E = V:  U = A V / s
        return (A @ E) / sd.unsqueeze(-2), s, E.mH
    return E, s, (E.mH @ A) / sd.unsqueeze(-1)     # E = U:  Vh = U^H A / s


class Model(nn.Module):
    def __init__(self, config: Config, detector: str = 'vamp', path: str | None = None, amp=None,
                 seed: int | None = None, rng: str = 'host', group_epochs: bool = False,
                 shard: str = 'epochs') -> None:
        """rng='host' (default): the reference's numpy / torch-CPU random streams, bit for bit
        (parity mode).  rng='device': channel, messages and noise drawn on the GPU and the SVD
        on the GPU through the Gram matrix's eigendecomposition (svd_gram; throughput mode: same
        distributions, different streams).
        group_epochs: VAMP detects up to max_epochs of its epochs side by side in one persistent
        launch (VAMP.forward_epochs: one channel per epoch, or one per `res` block; same results,
        fills the GPU at small B).
        shard (with torch.distributed): 'epochs' (default) gives each rank whole epochs with its
        own random stream and merges the metrics once per SNR point; 'trials' (SURVEY §8(e)
        exact-compat, VAMP / BAMP / SCAMP) gives every rank the SAME epochs (one seed) and splits each batch's
        trials over the ranks with the batch scalars all-reduced every iteration (ShardedVAMP),
        so the sweep equals the single-process sweep."""
        super().__init__()
        self.config = config
        self.detector = detector
        self.rate = config.code_rate
        self.shannon_limit = config.shannon_limit_dB
        self.min_snr = self.shannon_limit
        if shard not in ('epochs', 'trials'):
            raise ValueError(f"shard must be 'epochs' or 'trials', got {shard!r}")
        self.shard = shard
        if amp is None and shard == 'trials':
            if detector == 'vamp':
                from vamp import ShardedVAMP
                amp = ShardedVAMP(config)
            elif detector == 'bamp':
                from bamp import ShardedBAMP
                amp = ShardedBAMP(config)
            else:
                from scamp import ShardedSCAMP
                amp = ShardedSCAMP(config)
        self.amp = amp if amp is not None else _detector(detector, config)
        self.loss = Loss(config)
        self.rng = rng
        self.channel = Channel(config, rng=rng)
        self.data = Data(config, rng=rng)
        self.path = path if path is not None else f'Simulations/{_DIRS[detector]}/{config.name}'
        self.rank, self.world = _dist()
        # trial sharding: every rank draws the same epochs (rank-independent seeding), the
        # detector splits each batch; epoch sharding: one stream per rank
        self._stream_rank = 0 if shard == 'trials' else self.rank
        self._epoch_world = 1 if shard == 'trials' else self.world
        if seed is None and self.world > 1:
            # unseeded multi-rank sweep: every rank would start torch's and numpy's generators
            # from the same default state and draw the same epochs; rank 0 draws a base seed
            # and broadcasts it, so the ranks' streams are distinct
            seed = _broadcast_seed()
        self.seed = seed
        if seed is not None:
            # one independent stream per rank (rank 0 of a 1-process run = the plain seed)
            np.random.seed((seed + 7919 * self._stream_rank) % 2 ** 32)
            torch.manual_seed(seed + 7919 * self._stream_rank)
        if self.rank == 0:
            os.makedirs(self.path, exist_ok=True)
        self.group_cap = 0
        self._ch_ok = None
        if group_epochs:
            if detector != 'vamp' or not hasattr(self.amp, 'forward_epochs'):
                raise ValueError('group_epochs: side-by-side epochs are built for the VAMP detector')
            N, n = config.Nt * config.Lin, config.Nr * config.Lout
            self.group_cap = self.amp.max_epochs(min(n, N))

    # one epoch, in the reference's random-call order (vamp_model.py:55-61)
    def _epoch(self, SNR: float, new_channel: bool):
        x, sym, idx, y = self._inputs(SNR, new_channel)
        if self.detector == 'vamp':
            U, s, Vh = self._svd
            return self.amp(U, s, Vh, y, SNR, x, sym, idx)
        if self.detector == 'bamp':
            return self.amp(self._A, y, SNR, x, sym, idx)
        return self.amp(self._W, self._A, y, SNR, x, sym, idx)

    def _group(self, SNR: float, ids: list, res: int) -> list:
        """The epochs `ids` (this rank's, in order) detected side by side with VAMP's persistent
        launch (VAMP.forward_epochs): every epoch's inputs are drawn in the reference's call order
        (the channel first when i % res == 0, then message + noise), then the epochs are
        detected in chunks that fit one persistent grid — with one channel per epoch where the
        chunk spans several channels (the reference's default res = 1 redraws it every epoch).
        Results equal the sequential _epoch calls."""
        cap = max(1, self.group_cap)
        out = []
        for c0 in range(0, len(ids), cap):
            chunk = []
            for i in ids[c0:c0 + cap]:
                x, sym, idx, y = self._inputs(SNR, i % res == 0)
                chunk.append((x, sym, idx, y, self._svd))
            chans = [v[4] for v in chunk]
            if all(c is chans[0] for c in chans):
                runs = [chunk]
            elif self._per_epoch_channels():
                runs = [chunk]
            else:
                # this arithmetic / shape takes one shared channel per launch only (e.g. GEMM_F32, or
                # n != 2k): the chunk goes as runs of epochs that share a channel (single epochs at res = 1)
                runs, cur = [], [chunk[0]]
                for v in chunk[1:]:
                    if v[4] is cur[-1][4]:
                        cur.append(v)
                    else:
                        runs.append(cur)
                        cur = [v]
                runs.append(cur)
            for run in runs:
                cs = [v[4] for v in run]
                if all(c is cs[0] for c in cs):
                    U, s, Vh = cs[0]
                else:
                    U, s, Vh = [c[0] for c in cs], [c[1] for c in cs], [c[2] for c in cs]
                out += self.amp.forward_epochs(U, s, Vh, [v[3] for v in run], SNR, [v[0] for v in run],
                                               [v[1] for v in run], [v[2] for v in run])
        return out

    def _per_epoch_channels(self) -> bool:
        """Whether one launch may hold epochs with different channels (VAMP.epochs_channels_eligible)."""
        if self._ch_ok is None:
            n, N = self.config.Nr * self.config.Lout, self.config.Nt * self.config.Lin
            self._ch_ok = self.amp.epochs_channels_eligible(min(n, N))
        return self._ch_ok

    def _inputs(self, SNR: float, new_channel: bool):
        if new_channel:
            W, A = self.channel.generate_as_sparc()
            self._A = A
            self._W = W
            if self.detector == 'vamp':
                if self.rng == 'device':
                    self._svd = svd_gram(A)
                else:   # LAPACK on the host, as the reference's CPU path (vamp_model.py:58)
                    U, s, Vh = torch.linalg.svd(A.cpu(), full_matrices=False)
                    self._svd = (U.to(A.device), s.to(A.device), Vh.to(A.device))
        x, sym, idx = self.data.generate_message()
        if self.rng == 'device':
            # one [B, N] x [N, n] GEMM (torch's batched A @ x over [B, N, 1] runs as B GEMVs:
            # 2.5 ms at cfg4 on the box, r01)
            B = x.shape[0]
            y = (x.reshape(B, -1) @ self._A.transpose(0, 1)).reshape(B, -1, 1) + self.channel.awgn(SNR)
        else:
            # y = A x + n on the host as the reference's CPU path forms it (vamp_model.py:60)
            A_h = self._A if self._A.device.type == 'cpu' else self._A.cpu()
            y = (A_h @ x.cpu() + self.channel.awgn(SNR).cpu()).to(x.device)
        return x, sym, idx, y

    @torch.no_grad()
    def run(self, SNR: float) -> Loss:
        loss = self._epoch(SNR, True)
        print(loss.loss)
        return loss

    def _merge(self) -> None:
        """Sum the per-rank accumulated metrics (one all-reduce per SNR point).  Trial sharding
        needs none: every rank's Loss already holds the whole batch's counters."""
        if self.world == 1 or self.shard == 'trials':
            return
        keys = ['T'] + [k for k in self.loss.keys if k in self.loss.loss]
        vals = torch.tensor([float(np.asarray(self.loss.loss.get(k, 0.0), dtype=np.float64)) for k in keys],
                            dtype=torch.float64).to(_comm_device())
        torch.distributed.all_reduce(vals)
        vals = vals.cpu().numpy()
        self.loss.loss['T'] = float(vals[0])
        for k, v in zip(keys[1:], vals[1:]):
            self.loss.loss[k] = np.float64(v)

    @torch.no_grad()
    def simulate(self, epochs: int, final=None, start=None, step: float = 1, res: int = 1):
        if start is None:
            start = int(np.ceil(self.min_snr))
        if final is None:
            final = start + 20.0
        EbN0dB_range = np.arange(start, final + step, step)
        SNRdB_range = EbN0dB_range + 10 * np.log10(self.rate)
        results = []
        for SNRdB, EbN0dB in zip(SNRdB_range, EbN0dB_range):
            if self.rank == 0:
                print(f'EbN0dB={EbN0dB}')
            SNR = 10 ** (SNRdB / 10)
            # blocks of `res` epochs share a channel and go to one rank
            mine = [i for i in range(epochs) if (i // res) % self._epoch_world == self.rank % self._epoch_world]
            if self.group_cap > 1:
                for loss in self._group(SNR, mine, res):      # side by side, chunks of group_cap epochs
                    self.loss.accumulate(loss)
            else:
                for i in mine:
                    loss = self._epoch(SNR, i % res == 0)
                    self.loss.accumulate(loss)
            if 'fer' not in self.loss.loss:                   # a rank without epochs at this point
                for k in self.loss.keys:
                    self.loss.loss[k] = np.float64(0.0)
            self._merge()
            self.loss.average(epochs)
            fer = self.loss.loss['fer']
            it = self.loss.loss['T']
            point = {k: (float(v) if np.ndim(v) == 0 else v) for k, v in self.loss.loss.items()}
            point.update(EbN0dB=float(EbN0dB), SNRdB=float(SNRdB))
            results.append(point)
            if self.rank == 0:
                print(f'FER={fer}, iter={it}')
                self.loss.export(SNRdB, EbN0dB, self.path)   # also clears the totals (loss.py:323)
            else:
                # every other rank clears its totals too (both shard modes): its next point must
                # start from zero, or its FER (and with it the stop decision below, which every
                # rank takes on the same merged / whole-batch values) would drift from rank 0's
                self.loss.loss = {'T': 0}
            if fer < 1e-3:
                break
        return results
