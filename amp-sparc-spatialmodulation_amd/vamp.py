"""VAMP detector (SVD form) — drop-in for the reference's ``VAMP`` / ``VAMPLayer`` /
``Tracker`` (vamp.py:12-191), running on the gfx950 kernels of libampsparc.so.

``VAMP.forward(U, s, Vh, y, SNR, x, symbols, indices) -> Loss`` keeps the reference's
signature and returns its own reused ``Loss`` (vamp.py:187-191).  The whole
iteration loop, the allclose early exit and the decision/counting run on the device;
the host reads back one 128-byte record per forward.
"""
from __future__ import annotations

import ctypes as C
import warnings
import os

import numpy as np
import torch
from torch import nn

import amp_native as nat
from config import Config
from loss import Loss


def _c64(t: torch.Tensor, shape) -> torch.Tensor:
    """Contiguous complex64 view/copy with torch's lazy conjugate / negative bits materialised
    (torch.linalg.svd on the GPU returns such views: the raw memory is NOT the value)."""
    t = t.reshape(shape)
    if t.dtype != torch.complex64:
        t = t.to(torch.complex64)
    return t.resolve_conj().resolve_neg().contiguous()


_FUSED_DECIDE = os.environ.get('AMP_FUSED_DECIDE', '1') != '0'


class _Buffers:
    """Per-shape device buffers reused across forwards (no allocation in steady state)."""

    def __init__(self):
        self.key = None

    def get(self, device, B, N, k, iters, ws_bytes):
        key = (str(device), B, N, k, iters, ws_bytes)
        if key != self.key:
            self.r = torch.empty(B, N, dtype=torch.complex64, device=device)
            self.xmmse = torch.empty(B, N, dtype=torch.complex64, device=device)
            self.var = torch.empty(B, N, dtype=torch.float32, device=device)
            self.res = torch.zeros(256, dtype=torch.uint8, device=device)     # amp_status @0, amp_counts @64
            self.ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=device)
            self.key = key
        return self


class Tracker:
    """Device state of one VAMP forward (vamp.py:12-28): r, xmmse, var and the workspace
    holding the expanded V/Vh/U weights, y~ and the per-iteration scalar record."""

    def __init__(self, U, s, Vh, y, x, sigma2: float, sparsity: float, config: Config, bufs: _Buffers | None = None):
        self.config = config
        B = config.B
        n, k = U.shape[0], U.shape[1]
        N = Vh.shape[1]
        self.U = _c64(U, (n, k))
        self.s = s.reshape(k).to(torch.float32).resolve_neg().contiguous()
        self.Vh = _c64(Vh, (k, N))
        self.y = _c64(y, (B, n))
        self.noise_var = sigma2
        self.sparsity = sparsity
        self.k = k
        self.t = 0
        self.dims = config.dims()
        self.const = config.constellation()
        lib = nat.lib()
        wsb = lib.amp_vamp_workspace_bytes(C.byref(self.dims), k, config.N_Layers)
        if wsb == 0:
            raise ValueError('amp_vamp_workspace_bytes: invalid dimensions')
        self.buf = (bufs or _Buffers()).get(self.y.device, B, N, k, config.N_Layers, wsb)
        a = nat.AmpVampArgs()
        a.U, a.s, a.Vh, a.y = (nat.dptr(self.U, name='U'), nat.dptr(self.s, torch.float32, 's'),
                               nat.dptr(self.Vh, name='Vh'), nat.dptr(self.y, name='y'))
        a.k, a.max_iter = k, config.N_Layers
        a.noise_var, a.sparsity = float(sigma2), float(sparsity)
        a.r, a.xmmse, a.var = nat.dptr(self.buf.r), nat.dptr(self.buf.xmmse), nat.dptr(self.buf.var)
        a.status = nat.dptr(self.buf.res)
        a.ws, a.ws_bytes = nat.dptr(self.buf.ws), self.buf.ws.numel()
        self.args = a
        self.stream = nat.stream_ptr(self.y.device)

    @property
    def r(self):
        return self.buf.r.view(self.config.B, -1, 1)

    @property
    def xmmse(self):
        return self.buf.xmmse.view(self.config.B, -1, 1)

    @property
    def var(self):
        return self.buf.var.view(self.config.B, -1, 1)

    def prepare(self):
        nat.check(nat.lib().amp_vamp_prepare(C.byref(self.dims), C.byref(self.const), C.byref(self.args),
                                             self.stream), 'amp_vamp_prepare')

    def finalize(self):
        nat.check(nat.lib().amp_vamp_finalize(C.byref(self.dims), C.byref(self.const), C.byref(self.args),
                                              self.stream), 'amp_vamp_finalize')

    def status(self) -> nat.AmpStatus:
        res = getattr(self, 'res', None)
        res = self.buf.res if res is None else res
        return nat.AmpStatus.from_buffer_copy(res[:C.sizeof(nat.AmpStatus)].cpu().numpy().tobytes())


class VAMPLayer(nn.Module):
    """One VAMP iteration (vamp.py:56-94) as a device launch pair; a no-op once the
    early exit of vamp.py:185 has fired."""

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
        nat.check(nat.lib().amp_vamp_iterate(C.byref(T.dims), C.byref(T.const), C.byref(T.args), self.index,
                                             T.stream), 'amp_vamp_iterate')

    def segmented_denoiser(self, s: torch.Tensor, tau) -> tuple[torch.Tensor, torch.Tensor]:
        """vamp.py:96-119 on the device: (xmmse c64 [B, LM, 1], var f32 [B, LM, 1])."""
        return block_denoise(self.config, s, tau, mode=0)


def block_denoise(config: Config, s: torch.Tensor, tau, mode: int):
    """amp_block_denoise: mode 0 scalar tau (VAMP), 1 per-element cov (BAMP, tau = cov/2),
    2 per-element tau_use, mean only (SCAMP)."""
    B = config.B
    r = _c64(s, (B, -1))
    d = config.dims()
    cst = config.constellation()
    xm = torch.empty_like(r)
    var = torch.empty(r.shape, dtype=torch.float32, device=r.device) if mode != 2 else None
    tau_s = 0.0
    tau_p = None
    if mode == 0:
        tau_s = float(tau.item() if isinstance(tau, torch.Tensor) else tau)
    else:
        tv = tau.reshape(B, -1).to(torch.float32).resolve_neg().contiguous()
        tau_p = nat.dptr(tv, torch.float32, 'tau')
    lib = nat.lib()
    wsb = lib.amp_block_denoise_workspace_bytes(C.byref(d))
    ws = nat.WORKSPACE.get(r.device, 'denoise', wsb)
    nat.check(lib.amp_block_denoise(C.byref(d), C.byref(cst), nat.dptr(r, name='r'), mode, tau_s, tau_p,
                                    nat.dptr(xm), nat.dptr(var) if var is not None else None, nat.dptr(ws), wsb,
                                    nat.stream_ptr(r.device)), 'amp_block_denoise')
    if mode == 2:
        return xm.view(B, -1, 1)
    return xm.view(B, -1, 1), var.view(B, -1, 1)


class LazyResult:
    """A detector's result read-back without a host stall: a forward leaves its status + counter
    record in one of two (device, pinned host) 256-byte slots, copies it to the host
    asynchronously and arms Loss._pending; the record is resolved (and the metrics recorded)
    on the Loss's first access or at the next forward, so the launches of the next epoch are
    queued before this one's results are waited for (Model.simulate's loop)."""

    _ring = None
    _slot = 1

    def _result_slot(self, device):
        """One of two (device, pinned host) 256-byte result buffers, alternating per forward, so
        a forward's status / counters stay readable while the next forward runs."""
        if self._ring is None or self._ring[0][0].device != device:
            self._ring = [(torch.zeros(256, dtype=torch.uint8, device=device),
                           torch.zeros(256, dtype=torch.uint8, pin_memory=True)) for _ in range(2)]
        self._slot ^= 1
        return self._ring[self._slot]

    def _arm(self, L: Loss, res: torch.Tensor, host: torch.Tensor, what: str, rescue=None,
             written: bool = False) -> None:
        """Queue the copy of `res` to `host` on the device's current stream and make L resolve it
        lazily; the previous forward's record is resolved first.

        A persistent launch whose grid exchange timed out reports nan_state = -1 (every spin is
        bounded; the grid drains and the results are invalid).  `rescue()` then re-runs that
        forward on the launch engine in this process (no exec, no co-residency needed) and
        returns its (status, counts); the event is counted in self.grid_rescues.  Without a
        rescue (or if it fails too) the resolve raises.  The rescue re-reads the forward's input
        tensors when the Loss resolves (at the latest inside the next forward call), so they must
        not be overwritten in place before then — the reference's own contract for the returned
        Loss (read it before the next call, vamp_model.py:61-62).
        written: the forward's last kernel wrote the record into `host` itself
        (amp_vamp_decide_args.host_record), so no copy is queued."""
        if not written:
            host.copy_(res, non_blocking=True)
        done = torch.cuda.Event()
        done.record(torch.cuda.current_stream(res.device))   # the stream the launches and the copy ran on
        L.resolve()                 # the previous forward's counters (it has finished by now)
        L.dump()

        def finish(L=L):
            done.synchronize()
            raw = host.numpy().tobytes()
            status = nat.AmpStatus.from_buffer_copy(raw[:C.sizeof(nat.AmpStatus)])
            counts = nat.AmpCounts.from_buffer_copy(raw[64:64 + C.sizeof(nat.AmpCounts)])
            status, counts = self._check_grid(status, counts, rescue, what)
            L.last_counts = counts
            L.last_status = status
            L.record(L.rates_from_counts(counts), int(status.T))
        L._pending = finish

    grid_rescues = 0         # rescues of this detector
    rescues_total = 0        # every rescue in this process (LazyResult.rescues_total; tests/conftest.py)
    # Test-only hook (tests/test_gpu_rescue.py): a callable that may rewrite a resolved persistent
    # status record (e.g. report the grid as lost) before it is checked; None in production.
    status_hook = None

    def _check_grid(self, status, counts, rescue, what):
        if self.status_hook is not None and rescue is not None:
            status = self.status_hook(status)
        if status.nan_state >= 0:
            return status, counts
        if rescue is not None:
            self.grid_rescues += 1
            LazyResult.rescues_total += 1
            warnings.warn(f'{what}: persistent grid lost (a grid exchange timed out); the forward is re-run '
                          'on the launch engine', RuntimeWarning, stacklevel=2)
            status, counts = rescue()
            if status.nan_state >= 0:
                return status, counts
        raise RuntimeError(f'{what}: persistent engine grid barrier timed out (results invalid)')



class VAMP(LazyResult, nn.Module):
    """``engine``: nat.ENGINE_AUTO (persistent single-launch engine when the shape allows it,
    else three launches per iteration), ENGINE_LAUNCHES or ENGINE_PERSISTENT (amp_sparc.h).
    ``gemm``: the persistent engine's GEMM arithmetic, nat.GEMM_AUTO (split-precision bf16x3
    where it fits: 24-bit operands, the reference's; else f32 MFMA), GEMM_F32, GEMM_X3, or the
    opt-in GEMM_H2 (fp16x2, 22-bit operands: narrower than the reference) (amp_sparc.h)."""

    def __init__(self, config: Config, engine: int = nat.ENGINE_AUTO, gemm: int = nat.GEMM_AUTO) -> None:
        super().__init__()
        self.config = config
        self.engine = engine
        self.gemm = gemm
        self.E = config.Na / config.Nr                                   # vamp.py:154
        self.sparsity = config.Na / config.Nt                            # vamp.py:155
        self.layers = nn.ModuleList([VAMPLayer(config, i) for i in range(config.N_Layers)])
        self.L = Loss(config)
        self._bufs = _Buffers()
        self.last = None

    def detect(self, U, s, Vh, y, SNR: float) -> Tracker:
        """All iterations on the device, asynchronous (no host sync)."""
        with torch.cuda.device(y.device):
            T = Tracker(U, s, Vh, y, None, self.E / SNR, self.sparsity, self.config, self._bufs)
            T.args.engine = self.engine
            T.args.gemm = self.gemm
            nat.check(nat.lib().amp_vamp_run(C.byref(T.dims), C.byref(T.const), C.byref(T.args), T.stream),
                      'amp_vamp_run')
        return T

    def forward(self, U: torch.Tensor, s: torch.Tensor, Vh: torch.Tensor, y: torch.Tensor, SNR: float,
                x: torch.Tensor, symbols: np.ndarray, indices: np.ndarray) -> Loss:
        """vamp.py:159-187.  Everything runs on the device; the returned Loss resolves its
        counters on first access (the forward's one host synchronisation), so the launches of
        the next forward can be queued before this one's results are read back."""
        if self.config.mode == 'random':
            # vamp.py:45-48 picks Shrink('bayes') for 'random', which returns one tensor; the
            # layer's two-value unpacking then fails (recorded in tests/golden/g8_random_curves.json)
            raise ValueError('not enough values to unpack (expected 2, got 1)')
        with torch.cuda.device(y.device):   # the C ABI sizes and launches on the current device
            return self._forward(U, s, Vh, y, SNR, x, symbols, indices)

    def _forward(self, U, s, Vh, y, SNR, x, symbols, indices) -> Loss:
        T = Tracker(U, s, Vh, y, None, self.E / SNR, self.sparsity, self.config, self._bufs)
        T.args.engine = self.engine
        T.args.gemm = self.gemm
        res, host = self._result_slot(T.y.device)
        T.res = res
        T.args.status = nat.dptr(res)
        lib = nat.lib()
        fused = (_FUSED_DECIDE and self.L.decision_mode == 'sparc' and
                 lib.amp_vamp_select_engine(C.byref(T.dims), T.k, self.engine) == nat.ENGINE_PERSISTENT)
        if fused:
            # forward + decision on T.r (vamp.py:187) + counters in one launch sequence
            dec = self.L.decide_args(x, symbols, indices, out=res[64:])
            dec.host_record = None if nat.fold_launch() else host.data_ptr()   # status + counters written there
            nat.check(lib.amp_vamp_detect_count(C.byref(T.dims), C.byref(T.const), C.byref(T.args), C.byref(dec),
                                                 T.stream), 'amp_vamp_detect_count')
        else:
            nat.check(lib.amp_vamp_run(C.byref(T.dims), C.byref(T.const), C.byref(T.args), T.stream), 'amp_vamp_run')
            # decision on T.r (vamp.py:187); counters land next to the status record
            self.L.device_counts(T.buf.r, T.buf.xmmse, x, symbols, indices, out=res[64:])
        persistent = lib.amp_vamp_select_engine(C.byref(T.dims), T.k, self.engine) == nat.ENGINE_PERSISTENT
        rescue = (lambda: self._rescue_forward(U, s, Vh, y, SNR, x, symbols, indices)) if persistent else None
        self._arm(self.L, res, host, 'amp_vamp_run', rescue, written=fused and not nat.fold_launch())   # + L.dump()
        self.last = T
        return self.L

    def _rescue_forward(self, U, s, Vh, y, SNR, x, symbols, indices):
        """One forward on the launch engine (three launches per iteration: no grid-wide
        exchange inside a kernel), synchronously, into buffers of its own: the rescue of a
        persistent launch whose grid was lost (LazyResult._check_grid).  Returns (status, counts)."""
        with torch.cuda.device(y.device):
            if getattr(self, '_rescue_bufs', None) is None:
                self._rescue_bufs = _Buffers()
            T = Tracker(U, s, Vh, y, None, self.E / SNR, self.sparsity, self.config, self._rescue_bufs)
            T.args.engine = nat.ENGINE_LAUNCHES
            T.args.gemm = nat.GEMM_AUTO
            res = torch.zeros(256, dtype=torch.uint8, device=T.y.device)
            T.args.status = nat.dptr(res)
            nat.check(nat.lib().amp_vamp_run(C.byref(T.dims), C.byref(T.const), C.byref(T.args), T.stream),
                      'amp_vamp_run (rescue)')
            self.L.device_counts(T.buf.r, T.buf.xmmse, x, symbols, indices, out=res[64:])
            return read_result(res)

    def max_epochs(self, k: int) -> int:
        """The most epochs of this config ONE persistent launch holds (amp_vamp_max_epochs:
        one workgroup of 16 trials per CU, two at N = 64; 0 when not persistent-eligible)."""
        if self.config.mode != 'sparc':
            return 0
        d = self.config.dims()
        if nat.lib().amp_vamp_select_engine(C.byref(d), k, self.engine) != nat.ENGINE_PERSISTENT:
            return 0
        return int(nat.lib().amp_vamp_max_epochs_gemm(C.byref(d), k, self.gemm))

    def epochs_channels_eligible(self, k: int) -> bool:
        """Whether forward_epochs takes one channel per epoch for this config and GEMM arithmetic
        (amp_vamp_epochs_ch_eligible: the bf16x3 / int8x4 engine and n == 2 k); otherwise a call
        must share one channel across its epochs."""
        if self.max_epochs(k) < 1:
            return False
        d = self.config.dims()
        return bool(nat.lib().amp_vamp_epochs_ch_eligible(C.byref(d), k, self.gemm))

    def epochs_eligible(self, n: int, k: int, epochs: int) -> bool:
        """Whether `epochs` forwards of this config fit ONE persistent launch
        (amp_vamp_detect_count_epochs)."""
        return 1 <= epochs <= self.max_epochs(k)

    def forward_epochs(self, U, s, Vh, ys, SNR: float, xs, symbols, indices) -> list:
        """E epochs detected side by side in one persistent launch (amp_vamp_detect_count_epochs_ch).
        (U, s, Vh) is either ONE channel shared by every epoch — the epochs of one `res` block of
        Model.simulate (vamp_model.py:55-61 redraws the channel only when i % res == 0) — or one
        channel per epoch (sequences of E tensors, or stacked [E, ...] tensors: the reference's
        default res = 1 redraws it every epoch).  Every epoch keeps its own batch-global scalars
        and early exit (vamp.py:85, 112, 185), so the returned Loss objects (one per epoch, in
        order) equal E sequential forward() calls.
        ys / xs: sequences of the epochs' y [B, n, 1] and x [B, N, 1], or stacked [E, B, ...]
        tensors (used without a copy); symbols / indices: sequences of their label arrays or
        stacked label tensors.  The Losses resolve lazily (no host stall inside the call)."""
        if self.config.mode != 'sparc':
            raise NotImplementedError("side-by-side epochs decide in generator_mode='sparc' only")
        E = len(ys)
        if not (E == len(xs) == len(symbols) == len(indices)) or E < 1:
            raise ValueError('forward_epochs: ys, xs, symbols and indices must hold the same number (>= 1) of epochs')
        dev = ys[0].device
        with torch.cuda.device(dev):
            return self._forward_epochs(U, s, Vh, ys, SNR, xs, symbols, indices, E, dev)

    @staticmethod
    def _epoch_channels(U, s, Vh, E):
        """(U [n, k], s [k], Vh [k, N]) of one shared channel, or per-epoch channels stacked into
        contiguous [E, n, k] / [E, k] / [E, k, N]; returns (Uc, sc, Vhc, per_epoch)."""
        seq = lambda v: isinstance(v, (list, tuple))   # noqa: E731
        per = seq(U) or (isinstance(U, torch.Tensor) and U.dim() == 3 and U.shape[0] == E and E > 1)
        if not per:
            n, k = U.shape[-2], U.shape[-1]
            N = Vh.shape[-1]
            return (_c64(U, (n, k)), s.reshape(k).to(torch.float32).resolve_neg().contiguous(), _c64(Vh, (k, N)),
                    False)
        Us = list(U) if seq(U) else [U[e] for e in range(E)]
        ss = list(s) if seq(s) else [s[e] for e in range(E)]
        Vhs = list(Vh) if seq(Vh) else [Vh[e] for e in range(E)]
        if not (len(Us) == len(ss) == len(Vhs) == E):
            raise ValueError(f'forward_epochs: {E} epochs need {E} channels (U, s, Vh), got '
                             f'{len(Us)}, {len(ss)}, {len(Vhs)}')
        n, k = Us[0].shape[-2], Us[0].shape[-1]
        N = Vhs[0].shape[-1]
        Uc = torch.stack([_c64(u, (n, k)) for u in Us]).contiguous()
        sc = torch.stack([v.reshape(k).to(torch.float32).resolve_neg() for v in ss]).contiguous()
        Vhc = torch.stack([_c64(v, (k, N)) for v in Vhs]).contiguous()
        return Uc, sc, Vhc, True

    def _forward_epochs(self, U, s, Vh, ys, SNR, xs, symbols, indices, E, dev):
        from loss import _as_device_labels, _flat_c64
        cfg = self.config
        B = cfg.B
        Uc, sc, Vhc, per = self._epoch_channels(U, s, Vh, E)
        n, k, N = Uc.shape[-2], Uc.shape[-1], Vhc.shape[-1]
        # a stacked [E, B, ...] tensor is used as it lies (no copy); a sequence is concatenated
        stack = lambda v, f: (f(v, E) if isinstance(v, torch.Tensor) else torch.cat([f(u, 1) for u in v]))  # noqa: E731
        y = stack(ys, lambda v, e: _c64(v, (e * B, n))).contiguous()
        x = stack(xs, lambda v, e: _flat_c64(v, e * B, 'x')).contiguous()
        sym = stack(symbols, lambda v, e: _as_device_labels(v, dev).reshape(-1)).contiguous()
        idx = stack(indices, lambda v, e: _as_device_labels(v, dev).reshape(-1)).contiguous()
        if sym.numel() != E * B * cfg.L or idx.numel() != E * B * cfg.L:
            raise ValueError(f'expected {E * B * cfg.L} labels/indices, got {sym.numel()}/{idx.numel()}')
        d, cst = cfg.dims(), cfg.constellation()
        lib = nat.lib()
        wsb = lib.amp_vamp_epochs_workspace_bytes(C.byref(d), k, cfg.N_Layers, E)
        if wsb == 0:
            raise ValueError('amp_vamp_epochs_workspace_bytes: invalid dimensions')
        ws = nat.WORKSPACE.get(dev, 'vamp_epochs', wsb)
        r = torch.empty(E * B, N, dtype=torch.complex64, device=dev)
        xm = torch.empty_like(r)
        var = torch.empty(E * B, N, dtype=torch.float32, device=dev)
        st_sz, ct_sz = C.sizeof(nat.AmpStatus), C.sizeof(nat.AmpCounts)
        res, host = self._epochs_slot(dev, E * (st_sz + ct_sz))
        a = nat.AmpVampArgs()
        a.U, a.s, a.Vh, a.y = nat.dptr(Uc, name='U'), nat.dptr(sc, torch.float32, 's'), nat.dptr(Vhc, name='Vh'), \
            nat.dptr(y, name='y')
        a.k, a.max_iter, a.engine, a.gemm = k, cfg.N_Layers, self.engine, self.gemm
        a.noise_var, a.sparsity = float(self.E / SNR), float(self.sparsity)
        a.r, a.xmmse, a.var = nat.dptr(r), nat.dptr(xm), nat.dptr(var)
        a.status = nat.dptr(res)
        a.ws, a.ws_bytes = nat.dptr(ws), ws.numel()
        dec = nat.AmpVampDecideArgs()
        dec.x, dec.sym, dec.idx = nat.dptr(x, name='x'), nat.dptr(sym, name='symbols'), nat.dptr(idx, name='indices')
        dec.ibits_trunc = self.L._ibits
        dec.counts = nat.dptr(res) + E * st_sz
        if per:
            strides = (n * k, k, k * N)     # elements between epochs' channels
            nat.check(lib.amp_vamp_detect_count_epochs_ch(C.byref(d), C.byref(cst), C.byref(a), C.byref(dec), E,
                                                          *strides, nat.stream_ptr(dev)), 'amp_vamp_detect_count_epochs_ch')
        else:
            nat.check(lib.amp_vamp_detect_count_epochs(C.byref(d), C.byref(cst), C.byref(a), C.byref(dec), E,
                                                       nat.stream_ptr(dev)), 'amp_vamp_detect_count_epochs')
        # the records come back asynchronously: each Loss resolves on first access, and the
        # previous call's Losses are resolved here, after this call's launches are queued
        host[:res.numel()].copy_(res, non_blocking=True)
        done = torch.cuda.Event()
        done.record(torch.cuda.current_stream(dev))
        for L in self._epochs_prev:
            L.resolve()
        out = []

        def finish(L, e):
            done.synchronize()
            raw = host.numpy()
            status = nat.AmpStatus.from_buffer_copy(raw[e * st_sz:(e + 1) * st_sz].tobytes())
            counts = nat.AmpCounts.from_buffer_copy(raw[E * st_sz + e * ct_sz:E * st_sz + (e + 1) * ct_sz].tobytes())
            ch = (Uc[e], sc[e], Vhc[e]) if per else (Uc, sc, Vhc)
            status, counts = self._check_grid(
                status, counts, lambda: self._rescue_forward(ch[0], ch[1], ch[2], y[e * B:(e + 1) * B], SNR,
                                                             x[e * B:(e + 1) * B], sym[e * B * cfg.L:(e + 1) * B * cfg.L],
                                                             idx[e * B * cfg.L:(e + 1) * B * cfg.L]),
                'amp_vamp_detect_count_epochs')
            L.last_counts, L.last_status = counts, status
            L.record(L.rates_from_counts(counts), int(status.T))

        for e in range(E):
            L = Loss(cfg)
            L._pending = (lambda L=L, e=e: finish(L, e))
            out.append(L)
        self._epochs_prev = out
        self._epochs_keep = (y, x, sym, idx, Uc, Vhc, sc)   # alive until the kernels have read them
        self.last_epochs = (r.view(E, B, N, 1), xm.view(E, B, N, 1), var.view(E, B, N, 1))
        return out

    _epochs_prev = ()
    _epochs_ring = None
    _epochs_i = 1

    def _epochs_slot(self, device, nbytes):
        """One of two (device, pinned host) result buffers for forward_epochs, alternating per
        call, so a call's records stay readable while the next call runs.  Not cleared: the
        engine writes every epoch's status and counter record whole."""
        if self._epochs_ring is None or self._epochs_ring[0][0].device != device or \
                self._epochs_ring[0][0].numel() < nbytes:
            self._epochs_ring = [(torch.zeros(nbytes, dtype=torch.uint8, device=device),
                                  torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True)) for _ in range(2)]
        self._epochs_i ^= 1
        d, h = self._epochs_ring[self._epochs_i]
        return d[:nbytes], h[:nbytes]


class ShardHook:
    """Shared host side of the trial-sharded detectors (SURVEY §8(e) exact-compat mode): the rank's
    slice of the batch, the all-reduce hook the C drivers call between launches
    (amp_set_allreduce_hook), and the slice's decision + the ONE counter all-reduce that gives
    every rank the whole batch's Loss."""

    def _shard_init(self, group) -> None:
        self.group = group
        self._ws = None
        self._hook_error = None
        self._hook = nat.ALLREDUCE_FN(self._allreduce)     # kept alive with the detector

    def _allreduce(self, buf, count, op, stream, ctx) -> int:
        """amp_allreduce_fn: `count` float64 words at device address `buf` (inside this
        detector's workspace), in place, ordered on the current stream.

        Failure semantics (amp_sparc.h): a local error (a buffer outside the workspace) still
        takes part in the collective, with NaN words, so the other ranks never wait on a missing
        peer; the error is kept, the C driver makes every later call too and returns
        AMP_E_LAUNCH, and _run_hooked raises on EVERY rank (one flag all-reduce per forward)."""
        dist = torch.distributed
        if not (dist.is_available() and dist.is_initialized()):
            return 0                       # one process: the reduction over one rank is the identity
        try:
            ws = self._ws
            off = int(buf) - ws.data_ptr()
            if off < 0 or off + 8 * count > ws.numel():
                raise ValueError(f'hook buffer outside the workspace (offset {off})')
            view = ws[off:off + 8 * count].view(torch.float64)
        except Exception as e:   # noqa: BLE001 — the collective below still runs, on poison
            if self._hook_error is None:
                self._hook_error = e
            view = torch.full((int(count),), float('nan'), dtype=torch.float64, device=self._ws.device)
        try:
            rop = dist.ReduceOp.SUM if op == nat.ALLREDUCE_SUM else dist.ReduceOp.MAX
            if view.device.type == 'cuda' and dist.get_backend(self.group) == 'nccl':
                dist.all_reduce(view, op=rop, group=self.group)
            else:
                h = view.cpu()
                dist.all_reduce(h, op=rop, group=self.group)
                view.copy_(h)
        except Exception as e:   # noqa: BLE001 — the group itself failed: surfaced as AMP_E_LAUNCH
            if self._hook_error is None:
                self._hook_error = e
        return 0 if self._hook_error is None else 1

    def shard(self):
        dist = torch.distributed
        rank, world = (dist.get_rank(self.group), dist.get_world_size(self.group)) if dist.is_initialized() else (0, 1)
        B = self.config.B
        return rank * B // world, (rank + 1) * B // world

    def _run_hooked(self, fn, what, *args) -> None:
        """Runs a trial-sharded C driver with this detector's hook; if the hook failed on ANY
        rank, every rank raises (the failed rank's poisoned words made the others' results
        meaningless too)."""
        lib = nat.lib()
        self._hook_error = None
        nat.check(lib.amp_set_allreduce_hook(C.cast(self._hook, C.c_void_p), None), 'amp_set_allreduce_hook')
        rc = fn(*args)
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized():
            flag = torch.tensor([1.0 if self._hook_error is not None else 0.0], dtype=torch.float64)
            if dist.get_backend(self.group) == 'nccl':
                flag = flag.to(self._ws.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
            if float(flag.item()) != 0.0 and self._hook_error is None:
                raise RuntimeError(f'{what}: the all-reduce hook failed on another rank')
        if self._hook_error is not None:
            raise RuntimeError(f'{what}: all-reduce hook failed') from self._hook_error
        nat.check(rc, what)

    def _decide_merge(self, d, cst, xmap, xm, x, symbols, indices, b0, b1, res, st) -> Loss:
        """Decision on this slice (flat indices of the whole batch), ONE all-reduce of the
        counters, the whole batch's metrics recorded on self.L."""
        from loss import _as_device_labels, _flat_c64, allreduce_counts, counts_to_vector, vector_to_counts
        cfg = self.config
        B, L = cfg.B, cfg.L
        dev = xmap.device
        xl = _flat_c64(x, B, 'x')[b0:b1].contiguous()
        syml = _as_device_labels(symbols, dev).reshape(-1)[b0 * L:b1 * L].contiguous()
        idxl = _as_device_labels(indices, dev).reshape(-1)[b0 * L:b1 * L].contiguous()
        lib = nat.lib()
        dwsb = lib.amp_map_decide_workspace_bytes(C.byref(d))
        dws = nat.WORKSPACE.get(dev, 'decide_sharded', dwsb)
        nat.check(lib.amp_map_decide_count_rows(C.byref(d), C.byref(cst), nat.dptr(xmap), nat.dptr(xm), nat.dptr(xl),
                                                nat.dptr(syml), nat.dptr(idxl), self.L._ibits, b0,
                                                nat.dptr(res) + 64, None, nat.dptr(dws), dwsb, st),
                  'amp_map_decide_count_rows')
        raw = res.cpu().numpy().tobytes()
        status = nat.AmpStatus.from_buffer_copy(raw[:C.sizeof(nat.AmpStatus)])
        counts = nat.AmpCounts.from_buffer_copy(raw[64:64 + C.sizeof(nat.AmpCounts)])
        merged = vector_to_counts(allreduce_counts(counts_to_vector(counts), self.group))   # the ONE counter all-reduce
        self.L.resolve()
        self.L.dump()
        self.L.last_counts, self.L.last_status = merged, status
        self.L.record(self.L.rates_from_counts(merged), int(status.T))
        return self.L


class ShardedVAMP(ShardHook, VAMP):
    """SURVEY §8(e) exact-compat mode: ONE batch of config.B trials split over the ranks of
    torch.distributed, rank r detecting trials [r B / P, (r + 1) B / P).

    ``forward`` keeps VAMP.forward's signature and takes the WHOLE batch's inputs (every rank
    draws the same epoch from the same seed: channel, messages and noise are replicated with no
    communication); the rank runs its slice through amp_vamp_run_sharded, whose
    registered hook all-reduces the batch-global scalars of every iteration (var.mean(),
    max |xi|, allclose; vamp.py:85, 112, 185) four times per iteration, decides its rows with
    amp_map_decide_count_rows and merges the error counters with ONE all-reduce.  The returned
    Loss equals the whole-batch forward's, up to the float64 summation order of var.mean().
    The hook runs torch.distributed.all_reduce on the device words for RCCL ('nccl') and
    through host memory for gloo."""

    def __init__(self, config: Config, group=None) -> None:
        super().__init__(config, engine=nat.ENGINE_LAUNCHES)
        self._shard_init(group)

    def _forward(self, U, s, Vh, y, SNR, x, symbols, indices) -> Loss:
        cfg = self.config
        B = cfg.B
        b0, b1 = self.shard()
        Bl = b1 - b0
        n, k = U.shape[0], U.shape[1]
        N = Vh.shape[1]
        dev = y.device
        Uc, Vhc = _c64(U, (n, k)), _c64(Vh, (k, N))
        sc = s.reshape(k).to(torch.float32).resolve_neg().contiguous()
        yl = _c64(y, (B, n))[b0:b1].contiguous()
        d, cst = cfg.dims(batch=Bl), cfg.constellation()
        lib = nat.lib()
        wsb = lib.amp_vamp_workspace_bytes(C.byref(d), k, cfg.N_Layers)
        if wsb == 0:
            raise ValueError('amp_vamp_workspace_bytes: invalid dimensions')
        self._ws = nat.WORKSPACE.get(dev, 'vamp_sharded', wsb)
        r = torch.empty(Bl, N, dtype=torch.complex64, device=dev)
        xm = torch.empty_like(r)
        var = torch.empty(Bl, N, dtype=torch.float32, device=dev)
        res = torch.zeros(256, dtype=torch.uint8, device=dev)      # amp_status @0, amp_counts @64
        a = nat.AmpVampArgs()
        a.U, a.s, a.Vh, a.y = nat.dptr(Uc, name='U'), nat.dptr(sc, torch.float32, 's'), nat.dptr(Vhc, name='Vh'), \
            nat.dptr(yl, name='y')
        a.k, a.max_iter, a.engine, a.gemm = k, cfg.N_Layers, nat.ENGINE_LAUNCHES, nat.GEMM_AUTO
        a.noise_var, a.sparsity = float(self.E / SNR), float(self.sparsity)
        a.r, a.xmmse, a.var = nat.dptr(r), nat.dptr(xm), nat.dptr(var)
        a.status = nat.dptr(res)
        a.ws, a.ws_bytes = nat.dptr(self._ws), self._ws.numel()
        st = nat.stream_ptr(dev)
        self._run_hooked(lib.amp_vamp_run_sharded, 'amp_vamp_run_sharded', C.byref(d), C.byref(cst), C.byref(a), B,
                         st)
        # decision on T.r (vamp.py:187) over this slice
        L = self._decide_merge(d, cst, r, xm, x, symbols, indices, b0, b1, res, st)
        self.last_shard = (r.view(Bl, N, 1), xm.view(Bl, N, 1), var.view(Bl, N, 1))
        return L


class PersistentShard:
    """One grid of a batch whose trials are split over several PERSISTENT grids that share one
    exchange buffer (amp_vamp_detect_count_shard, SURVEY §8(e) exact-compat): this shard detects
    trials [row_offset, row_offset + rows) of the batch `config` describes, publishes its
    per-iteration partials at its workgroups' global indices and reduces every shard's, so its
    scalars, T and rows of r / xmmse / var equal the whole-batch forward's bit for bit.  All
    shards of one forward run concurrently (different streams; on one GPU they must fit on the CUs
    together) with the same `gen`, after amp_vamp_shard_reset of the buffer; each returns its rows'
    counters (sum them).  Inputs are this shard's rows (y, x, labels) and the whole channel."""

    def __init__(self, config: Config, row_offset: int, rows: int, gemm: int = nat.GEMM_AUTO) -> None:
        from loss import Loss
        self.config, self.row_offset, self.rows, self.gemm = config, row_offset, rows, gemm
        self.E = config.Na / config.Nr
        self.sparsity = config.Na / config.Nt
        self._whole = Loss(config)          # the batch's ibits (flat indices of the whole batch)
        self._bufs = None

    @staticmethod
    def xbuf(config: Config, device) -> torch.Tensor:
        nbytes = nat.lib().amp_vamp_shard_xbuf_bytes(config.B, config.N_Layers)
        return torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=device)

    def launch(self, U, s, Vh, y, SNR: float, x, symbols, indices, xbuf: torch.Tensor, gen: int) -> torch.Tensor:
        """Queue this shard's forward on the current stream; returns its 256-byte result buffer
        (amp_status @0, amp_counts @64; read it after the stream has finished: read_result)."""
        from loss import _as_device_labels, _flat_c64
        cfg, Bl = self.config, self.rows
        n, k = U.shape[0], U.shape[1]
        N = Vh.shape[1]
        dev = y.device
        Uc, Vhc = _c64(U, (n, k)), _c64(Vh, (k, N))
        sc = s.reshape(k).to(torch.float32).resolve_neg().contiguous()
        yl = _c64(y, (Bl, n)).contiguous()
        d, cst = cfg.dims(batch=Bl), cfg.constellation()
        lib = nat.lib()
        wsb = lib.amp_vamp_workspace_bytes(C.byref(d), k, cfg.N_Layers)
        if wsb == 0:
            raise ValueError('amp_vamp_workspace_bytes: invalid dimensions')
        self.ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        self.r = torch.empty(Bl, N, dtype=torch.complex64, device=dev)
        self.xmmse = torch.empty_like(self.r)
        self.var = torch.empty(Bl, N, dtype=torch.float32, device=dev)
        res = torch.zeros(256, dtype=torch.uint8, device=dev)
        a = nat.AmpVampArgs()
        a.U, a.s, a.Vh, a.y = nat.dptr(Uc, name='U'), nat.dptr(sc, torch.float32, 's'), nat.dptr(Vhc, name='Vh'), \
            nat.dptr(yl, name='y')
        a.k, a.max_iter, a.engine, a.gemm = k, cfg.N_Layers, nat.ENGINE_PERSISTENT, self.gemm
        a.noise_var, a.sparsity = float(self.E / SNR), float(self.sparsity)
        a.r, a.xmmse, a.var = nat.dptr(self.r), nat.dptr(self.xmmse), nat.dptr(self.var)
        a.status = nat.dptr(res)
        a.ws, a.ws_bytes = nat.dptr(self.ws), self.ws.numel()
        xt = _flat_c64(x, Bl, 'x')
        sym = _as_device_labels(symbols, dev).reshape(-1)
        idx = _as_device_labels(indices, dev).reshape(-1)
        if sym.numel() != Bl * cfg.L or idx.numel() != Bl * cfg.L:
            raise ValueError(f'expected {Bl * cfg.L} labels/indices for the shard, got {sym.numel()}/{idx.numel()}')
        dec = nat.AmpVampDecideArgs()
        dec.x, dec.sym, dec.idx = nat.dptr(xt, name='x'), nat.dptr(sym, name='symbols'), nat.dptr(idx, name='indices')
        dec.ibits_trunc = self._whole._ibits
        dec.counts = nat.dptr(res) + 64
        sh = nat.AmpVampShard()
        sh.xbuf, sh.xbuf_bytes = nat.dptr(xbuf), xbuf.numel()
        sh.B_global, sh.row_offset, sh.gen = cfg.B, self.row_offset, gen
        nat.check(lib.amp_vamp_detect_count_shard(C.byref(d), C.byref(cst), C.byref(a), C.byref(dec), C.byref(sh),
                                                  nat.stream_ptr(dev)), 'amp_vamp_detect_count_shard')
        self._keep = (Uc, sc, Vhc, yl, xt, sym, idx, res)
        return res


def read_result(res: torch.Tensor):
    """(amp_status, amp_counts) from the 256-byte result buffer (status @0, counts @64)."""
    raw = res.cpu().numpy().tobytes()
    return (nat.AmpStatus.from_buffer_copy(raw[:C.sizeof(nat.AmpStatus)]),
            nat.AmpCounts.from_buffer_copy(raw[64:64 + C.sizeof(nat.AmpCounts)]))

