"""BAMP detector — drop-in for the reference's ``BAMP`` / ``BAMPLayer`` / ``Tracker``
(bamp.py:12-143), running on the gfx950 kernels of libampsparc.so.

``BAMP.forward(H, y, SNR, x, symbols, indices) -> Loss`` keeps the reference's signature and
returns its own reused ``Loss`` (bamp.py:116-143): the iteration loop (amp_bamp_run), the
allclose early exit and the decision / counters run on the device; the Loss resolves its
counters lazily, so consecutive epochs queue without a host stall.  The layer-level surface of
the reference is kept too: ``Tracker(H, y, sigma2, config)`` + ``BAMPLayer.forward(T)``
(amp_bamp_prepare / amp_bamp_iterate / amp_bamp_finalize).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
from torch import nn

import amp_native as nat
from config import Config
from loss import Loss
from vamp import LazyResult, ShardHook, _c64, block_denoise


class _Buffers:
    """Per-shape device buffers reused across forwards (no allocation in steady state)."""

    def __init__(self):
        self.key = None

    def get(self, device, B, N, ws_bytes):
        key = (str(device), B, N, ws_bytes)
        if key != self.key:
            self.xmap = torch.empty(B, N, dtype=torch.complex64, device=device)
            self.xmmse = torch.empty(B, N, dtype=torch.complex64, device=device)
            self.var = torch.empty(B, N, dtype=torch.float32, device=device)
            self.res = torch.zeros(256, dtype=torch.uint8, device=device)     # amp_status @0, amp_counts @64
            self.ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=device)
            self.key = key
        return self


class Tracker:
    """Device state of one BAMP forward (bamp.py:12-25): xmap, xmmse, var and the workspace holding
    the H, H^H, |H|^2, |H|^2^T operators and z, u, cov of the running iteration."""

    def __init__(self, H, y, sigma2: float, config: Config, bufs: _Buffers | None = None, gemm: int = nat.GEMM_AUTO):
        self.config = config
        B = config.B
        n, N = H.shape[-2], H.shape[-1]
        self.H = _c64(H, (n, N))
        self.y = _c64(y, (B, n))
        self.noise_var = sigma2
        self.dims = config.dims()
        self.const = config.constellation()
        lib = nat.lib()
        wsb = lib.amp_bamp_workspace_bytes(C.byref(self.dims), config.N_Layers)
        if wsb == 0:
            raise ValueError('amp_bamp_workspace_bytes: invalid dimensions')
        self.buf = (bufs or _Buffers()).get(self.y.device, B, N, wsb)
        a = nat.AmpBampArgs()
        a.H, a.y = nat.dptr(self.H, name='H'), nat.dptr(self.y, name='y')
        a.max_iter = config.N_Layers
        a.noise_var = float(sigma2)                                       # bamp.py:124
        # bamp.py:38-41: 'random' mode denoises element-wise (random_denoiser, bamp.py:79-88)
        a.denoiser = 1 if config.mode == 'random' else 0
        a.P0, a.Ps = float(np.float32(config.P0)), float(np.float32(config.Ps))
        a.gemm = gemm                                                     # amp_bamp_args.gemm
        a.xmap, a.xmmse, a.var = nat.dptr(self.buf.xmap), nat.dptr(self.buf.xmmse), nat.dptr(self.buf.var)
        a.status = nat.dptr(self.buf.res)
        a.ws, a.ws_bytes = nat.dptr(self.buf.ws), self.buf.ws.numel()
        self.args = a
        self.stream = nat.stream_ptr(self.y.device)

    @property
    def xmap(self):
        return self.buf.xmap.view(self.config.B, -1, 1)

    @property
    def xmmse(self):
        return self.buf.xmmse.view(self.config.B, -1, 1)

    @property
    def var(self):
        return self.buf.var.view(self.config.B, -1, 1)

    def _call(self, fn, *extra):
        nat.check(getattr(nat.lib(), fn)(C.byref(self.dims), C.byref(self.const), C.byref(self.args), *extra,
                                         self.stream), fn)

    def prepare(self):
        self._call('amp_bamp_prepare')

    def finalize(self):
        self._call('amp_bamp_finalize')

    def status(self) -> nat.AmpStatus:
        res = getattr(self, 'res', None)
        res = self.buf.res if res is None else res
        return nat.AmpStatus.from_buffer_copy(res[:C.sizeof(nat.AmpStatus)].cpu().numpy().tobytes())


class BAMPLayer(nn.Module):
    """BAMPLayer (bamp.py:27-64): forward(T) is one iteration on the device (a no-op once the
    early exit of bamp.py:140 has fired); its denoiser is the per-element-tau block denoiser."""

    def __init__(self, config: Config, index: int = 0) -> None:
        super().__init__()
        self.config = config
        self.index = index
        self.Nt, self.Na, self.Lin, self.B = config.Nt, config.Na, config.Lin, config.B
        self.K = config.K
        self.M = self.Nt // self.Na
        self.L = self.Na * self.Lin
        self.LM = self.L * self.M

    def forward(self, T: Tracker) -> None:
        T._call('amp_bamp_iterate', self.index)

    def segmented_denoiser(self, s: torch.Tensor, tau: torch.Tensor):
        """bamp.py:66-77: tau is cov, halved inside (tau = cov/2)."""
        return block_denoise(self.config, s, tau, mode=1)

    def random_denoiser(self, r: torch.Tensor, cov: torch.Tensor):
        """bamp.py:79-88 (generator_mode 'random'): element-wise float64 Bayes posterior under the
        P0 / Ps prior; (xmmse complex64, var float32) shaped like r."""
        cfg = self.config
        rr = _c64(r, (-1,))
        cv = cov.to(device=rr.device, dtype=torch.float32).expand(r.shape).reshape(-1).contiguous()
        xm = torch.empty_like(rr)
        var = torch.empty(rr.shape, dtype=torch.float32, device=rr.device)
        nat.check(nat.lib().amp_bamp_random_denoise(
            cfg.constellation(), rr.numel(), nat.dptr(rr, name='r'), nat.dptr(cv, name='cov'),
            float(np.float32(cfg.P0)), float(np.float32(cfg.Ps)), nat.dptr(xm), nat.dptr(var),
            nat.stream_ptr(rr.device)), 'amp_bamp_random_denoise')
        return xm.view(r.shape), var.view(r.shape)

    @property
    def denoiser(self):
        """The mode's denoiser (bamp.py:38-41)."""
        return self.random_denoiser if self.config.mode == 'random' else self.segmented_denoiser


class BAMP(LazyResult, nn.Module):
    """``gemm``: the GEMM arithmetic (amp_sparc.h amp_bamp_args.gemm): nat.GEMM_AUTO (f32 MFMA),
    GEMM_F32, GEMM_X3 (bf16x3 tiles, 24-bit operands) or GEMM_H2 (fp16x2 tiles, 22-bit operands,
    opt-in).  The arithmetic that ran is reported in ``self.L.arithmetic``."""

    def __init__(self, config: Config, gemm: int = nat.GEMM_AUTO) -> None:
        super().__init__()
        self.config = config
        self.gemm = gemm
        self.E = config.Na / config.Nr                                    # bamp.py:102
        self.layers = nn.ModuleList([BAMPLayer(config, i) for i in range(config.N_Layers)])
        self.L = Loss(config)
        self._bufs = _Buffers()
        self.last = None

    # buffers of the last forward (the Tracker's), for callers that read them directly
    @property
    def xmap(self):
        return self._bufs.xmap

    @property
    def xmmse(self):
        return self._bufs.xmmse

    @property
    def var(self):
        return self._bufs.var

    def detect(self, H: torch.Tensor, y: torch.Tensor, SNR: float) -> Tracker:
        """All iterations on the device, asynchronous (no host sync)."""
        with torch.cuda.device(y.device):
            T = Tracker(H, y, self.E / SNR, self.config, self._bufs, self.gemm)
            T._call('amp_bamp_run')
        self._keep = T
        return T

    def forward(self, H: torch.Tensor, y: torch.Tensor, SNR: float, x: torch.Tensor, symbols, indices) -> Loss:
        """bamp.py:116-143; the counters resolve lazily (see LazyResult)."""
        with torch.cuda.device(y.device):
            T = Tracker(H, y, self.E / SNR, self.config, self._bufs, self.gemm)
            res, host = self._result_slot(T.y.device)
            T.res = res
            T.args.status = nat.dptr(res)
            T._call('amp_bamp_run')
            # decision on T.xmap (bamp.py:142); counters next to the status record
            self.L.device_counts(T.buf.xmap, T.buf.xmmse, x, symbols, indices, out=res[64:])
            self._arm(self.L, res, host, 'amp_bamp_run')                  # + L.dump(), bamp.py:125
        self._keep = T
        self.last = T
        return self.L


class ShardedBAMP(ShardHook, BAMP):
    """SURVEY §8(e) exact-compat mode for BAMP: ONE batch split over the ranks of
    torch.distributed (rank r detects trials [r B / P, (r + 1) B / P)).  ``forward`` keeps
    BAMP.forward's signature and takes the whole batch's inputs (replicated from one seed); the
    rank runs its slice through amp_bamp_run_sharded, whose hook all-reduces the batch-global
    values of every iteration (max |xi| of the denoiser's shift, bamp.py:70; the allclose count,
    bamp.py:140; the rare path's exact values), decides its rows on xmap (bamp.py:142) and merges
    the counters with ONE all-reduce: the returned Loss equals the whole-batch forward's."""

    def __init__(self, config: Config, group=None) -> None:
        super().__init__(config)
        self._shard_init(group)

    def forward(self, H: torch.Tensor, y: torch.Tensor, SNR: float, x: torch.Tensor, symbols, indices) -> Loss:
        if self.config.mode == 'random':
            raise NotImplementedError("trial sharding needs the batch (generator_mode 'random' runs at B = 1)")
        with torch.cuda.device(y.device):
            return self._forward_sharded(H, y, SNR, x, symbols, indices)

    def _forward_sharded(self, H, y, SNR, x, symbols, indices) -> Loss:
        cfg = self.config
        B = cfg.B
        b0, b1 = self.shard()
        Bl = b1 - b0
        n, N = H.shape[-2], H.shape[-1]
        dev = y.device
        Hc = _c64(H, (n, N))
        yl = _c64(y, (B, n))[b0:b1].contiguous()
        d, cst = cfg.dims(batch=Bl), cfg.constellation()
        lib = nat.lib()
        wsb = lib.amp_bamp_workspace_bytes(C.byref(d), cfg.N_Layers)
        if wsb == 0:
            raise ValueError('amp_bamp_workspace_bytes: invalid dimensions')
        self._ws = nat.WORKSPACE.get(dev, 'bamp_sharded', wsb)
        xmap = torch.empty(Bl, N, dtype=torch.complex64, device=dev)
        xm = torch.empty_like(xmap)
        var = torch.empty(Bl, N, dtype=torch.float32, device=dev)
        res = torch.zeros(256, dtype=torch.uint8, device=dev)      # amp_status @0, amp_counts @64
        a = nat.AmpBampArgs()
        a.H, a.y = nat.dptr(Hc, name='H'), nat.dptr(yl, name='y')
        a.max_iter = cfg.N_Layers
        a.denoiser = 0
        a.noise_var = float(self.E / SNR)                                  # bamp.py:124
        a.P0, a.Ps = float(np.float32(cfg.P0)), float(np.float32(cfg.Ps))
        a.xmap, a.xmmse, a.var = nat.dptr(xmap), nat.dptr(xm), nat.dptr(var)
        a.status = nat.dptr(res)
        a.ws, a.ws_bytes = nat.dptr(self._ws), self._ws.numel()
        st = nat.stream_ptr(dev)
        self._run_hooked(lib.amp_bamp_run_sharded, 'amp_bamp_run_sharded', C.byref(d), C.byref(cst), C.byref(a), B,
                         st)
        L = self._decide_merge(d, cst, xmap, xm, x, symbols, indices, b0, b1, res, st)
        self.last_shard = (xmap.view(Bl, N, 1), xm.view(Bl, N, 1), var.view(Bl, N, 1))
        return L
