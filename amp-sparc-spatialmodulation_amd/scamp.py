"""SCAMP (spatially coupled SPARC AMP) — drop-in for the reference's ``SCAMP`` / ``SCAMPLayer`` /
``Tracker`` (scamp.py:8-108), running on the gfx950 kernels of libampsparc.so.

``SCAMP.forward(W, A, y, SNR, x, symbol, index) -> Loss`` keeps the reference's signature and
returns its own reused ``Loss`` (scamp.py:77-107); the loop (amp_scamp_run), the allclose(psi)
early exit and the decision run on the device, and the counters resolve lazily.  Layer level:
``Tracker(W, A, y, sigma2, config)`` + ``SCAMPLayer.forward(T)`` (amp_scamp_prepare /
amp_scamp_iterate / amp_scamp_finalize).
"""
from __future__ import annotations

import ctypes as C

import torch
from torch import nn

import amp_native as nat
from config import Config
from loss import Loss
from vamp import _FUSED_DECIDE, LazyResult, ShardHook, _c64, block_denoise


class _Buffers:
    """Per-shape device buffers reused across forwards (no allocation in steady state)."""

    def __init__(self):
        self.key = None

    def get(self, device, B, N, Lin, ws_bytes):
        key = (str(device), B, N, Lin, ws_bytes)
        if key != self.key:
            self.xmap = torch.empty(B, N, dtype=torch.complex64, device=device)
            self.xmmse = torch.empty(B, N, dtype=torch.complex64, device=device)
            self.psi = torch.empty(B, Lin, dtype=torch.float32, device=device)
            self.res = torch.zeros(256, dtype=torch.uint8, device=device)
            self.ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=device)
            self.key = key
        return self


class Tracker:
    """Device state of one SCAMP forward (scamp.py:8-25): xmap, xmmse, psi and the workspace holding
    the A / A^H operators and z, phi, tau of the running iteration."""

    def __init__(self, W, A, y, sigma2: float, config: Config, bufs: _Buffers | None = None):
        self.config = config
        B = config.B
        n, N = A.shape[-2], A.shape[-1]
        self.A = _c64(A, (n, N))
        self.y = _c64(y, (B, n))
        self.W = W.reshape(config.Lout, config.Lin).to(device=self.y.device, dtype=torch.float32).resolve_neg()
        self.W = self.W.contiguous()
        self.noise_var = sigma2
        self.dims = config.dims()
        self.const = config.constellation()
        lib = nat.lib()
        wsb = lib.amp_scamp_workspace_bytes(C.byref(self.dims), config.N_Layers)
        if wsb == 0:
            raise ValueError('amp_scamp_workspace_bytes: invalid dimensions')
        self.buf = (bufs or _Buffers()).get(self.y.device, B, N, config.Lin, wsb)
        a = nat.AmpScampArgs()
        a.W, a.A, a.y = nat.dptr(self.W, torch.float32, 'W'), nat.dptr(self.A, name='A'), nat.dptr(self.y, name='y')
        a.max_iter = config.N_Layers
        a.noise_var = float(sigma2)                                       # scamp.py:98
        a.xmap, a.xmmse, a.psi = nat.dptr(self.buf.xmap), nat.dptr(self.buf.xmmse), nat.dptr(self.buf.psi)
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
    def psi(self):
        return self.buf.psi.view(self.config.B, -1, 1)

    def _call(self, fn, *extra):
        nat.check(getattr(nat.lib(), fn)(C.byref(self.dims), C.byref(self.const), C.byref(self.args), *extra,
                                         self.stream), fn)

    def prepare(self):
        self._call('amp_scamp_prepare')

    def finalize(self):
        self._call('amp_scamp_finalize')

    def status(self) -> nat.AmpStatus:
        res = getattr(self, 'res', None)
        res = self.buf.res if res is None else res
        return nat.AmpStatus.from_buffer_copy(res[:C.sizeof(nat.AmpStatus)].cpu().numpy().tobytes())


class SCAMPLayer(nn.Module):
    """SCAMPLayer (scamp.py:27-68): forward(T) is one iteration on the device (a no-op once the
    early exit of scamp.py:105 has fired); its denoiser is the mean-only block denoiser."""

    def __init__(self, config: Config, index: int = 0) -> None:
        super().__init__()
        self.config = config
        self.index = index
        self.B, self.Na = config.B, config.Na
        self.M = config.Nt // config.Na
        self.Mc, self.Mr = config.Nt, config.Nr
        self.L = config.Na * config.Lin
        self.Lc, self.Lr = config.Lin, config.Lout
        self.n = self.Mr * self.Lr
        self.LM = self.Mc * self.Lc
        self.K = config.K

    def forward(self, T: Tracker) -> None:
        T._call('amp_scamp_iterate', self.index)

    def denoiser(self, s: torch.Tensor, tau: torch.Tensor) -> torch.Tensor:
        """scamp.py:61-68: tau is tau_use, halved inside."""
        return block_denoise(self.config, s, tau, mode=2)


class SCAMP(LazyResult, nn.Module):
    """``engine``: nat.ENGINE_AUTO (the persistent single-launch engine when the shape allows it,
    else seven launches per iteration), ENGINE_LAUNCHES or ENGINE_PERSISTENT (amp_sparc.h).
    ``gemm``: the persistent engine's GEMM arithmetic, nat.GEMM_AUTO (split-precision bf16x3 where
    it fits, else f32 MFMA), GEMM_F32 or GEMM_X3 (amp_sparc.h)."""

    def __init__(self, config: Config, engine: int = nat.ENGINE_AUTO, gemm: int = nat.GEMM_AUTO) -> None:
        super().__init__()
        self.config = config
        self.engine = engine
        self.gemm = gemm
        self.E = config.Na / config.Nr                                    # scamp.py:72
        self.layers = nn.ModuleList([SCAMPLayer(config, i) for i in range(config.N_Layers)])
        self.L = Loss(config)
        self._bufs = _Buffers()
        self.last = None

    @property
    def xmap(self):
        return self._bufs.xmap

    @property
    def xmmse(self):
        return self._bufs.xmmse

    @property
    def psi(self):
        return self._bufs.psi

    def detect(self, W: torch.Tensor, A: torch.Tensor, y: torch.Tensor, SNR: float) -> Tracker:
        """All iterations on the device, asynchronous (no host sync)."""
        with torch.cuda.device(y.device):
            T = Tracker(W, A, y, self.E / SNR, self.config, self._bufs)
            T.args.engine = self.engine
            T.args.gemm = self.gemm
            T._call('amp_scamp_run')
        self._keep = T
        return T

    def forward(self, W: torch.Tensor, A: torch.Tensor, y: torch.Tensor, SNR: float, x: torch.Tensor, symbol,
                index) -> Loss:
        """scamp.py:77-107; the counters resolve lazily (see LazyResult)."""
        with torch.cuda.device(y.device):
            T = Tracker(W, A, y, self.E / SNR, self.config, self._bufs)
            T.args.engine = self.engine
            T.args.gemm = self.gemm
            res, host = self._result_slot(T.y.device)
            T.res = res
            T.args.status = nat.dptr(res)
            persistent = nat.lib().amp_scamp_select_engine(C.byref(T.dims), self.engine) == nat.ENGINE_PERSISTENT
            if persistent and _FUSED_DECIDE and self.L.decision_mode == 'sparc':
                # forward + decision on T.xmap (scamp.py:107) + counters in one launch sequence
                dec = self.L.decide_args(x, symbol, index, out=res[64:])
                dec.host_record = None if nat.fold_launch() else host.data_ptr()   # status + counters written there
                T._call('amp_scamp_detect_count', C.byref(dec))
                written = not nat.fold_launch()
            else:
                T._call('amp_scamp_run')
                # decision on T.xmap (scamp.py:107); counters next to the status record
                self.L.device_counts(T.buf.xmap, T.buf.xmmse, x, symbol, index, out=res[64:])
                written = False
            rescue = (lambda: self._rescue_forward(W, A, y, SNR, x, symbol, index)) if persistent else None
            self._arm(self.L, res, host, 'amp_scamp_run', rescue, written=written)   # + L.dump(), scamp.py:99
        self._keep = T
        self.last = T
        return self.L

    def _rescue_forward(self, W, A, y, SNR, x, symbol, index):
        """One forward on the launch engine, synchronously, into buffers of its own: the rescue
        of a persistent launch whose grid was lost (vamp.LazyResult._check_grid)."""
        from vamp import read_result
        with torch.cuda.device(y.device):
            if getattr(self, '_rescue_bufs', None) is None:
                self._rescue_bufs = _Buffers()
            T = Tracker(W, A, y, self.E / SNR, self.config, self._rescue_bufs)
            T.args.engine = nat.ENGINE_LAUNCHES
            T.args.gemm = nat.GEMM_AUTO
            res = torch.zeros(256, dtype=torch.uint8, device=T.y.device)
            T.args.status = nat.dptr(res)
            T._call('amp_scamp_run')
            self.L.device_counts(T.buf.xmap, T.buf.xmmse, x, symbol, index, out=res[64:])
            return read_result(res)


class ShardedSCAMP(ShardHook, SCAMP):
    """SURVEY §8(e) exact-compat mode for SCAMP: ONE batch split over the ranks of
    torch.distributed (rank r detects trials [r B / P, (r + 1) B / P)).  ``forward`` keeps
    SCAMP.forward's signature and takes the whole batch's inputs (replicated from one seed); the
    rank runs its slice through amp_scamp_run_sharded (launch engine), whose hook all-reduces the
    batch-global values of every iteration (the denoiser's max |xi| shift, scamp.py:64; the psi
    allclose count, scamp.py:105; the rare path's exact values), decides its rows on xmap
    (scamp.py:107) and merges the counters with ONE all-reduce."""

    def __init__(self, config: Config, group=None) -> None:
        super().__init__(config)
        self._shard_init(group)

    def forward(self, W: torch.Tensor, A: torch.Tensor, y: torch.Tensor, SNR: float, x: torch.Tensor, symbol,
                index) -> Loss:
        with torch.cuda.device(y.device):
            return self._forward_sharded(W, A, y, SNR, x, symbol, index)

    def _forward_sharded(self, W, A, y, SNR, x, symbol, index) -> Loss:
        cfg = self.config
        B = cfg.B
        b0, b1 = self.shard()
        Bl = b1 - b0
        n, N = A.shape[-2], A.shape[-1]
        dev = y.device
        Ac = _c64(A, (n, N))
        yl = _c64(y, (B, n))[b0:b1].contiguous()
        Wc = W.reshape(cfg.Lout, cfg.Lin).to(device=dev, dtype=torch.float32).resolve_neg().contiguous()
        d, cst = cfg.dims(batch=Bl), cfg.constellation()
        lib = nat.lib()
        wsb = lib.amp_scamp_workspace_bytes(C.byref(d), cfg.N_Layers)
        if wsb == 0:
            raise ValueError('amp_scamp_workspace_bytes: invalid dimensions')
        self._ws = nat.WORKSPACE.get(dev, 'scamp_sharded', wsb)
        xmap = torch.empty(Bl, N, dtype=torch.complex64, device=dev)
        xm = torch.empty_like(xmap)
        psi = torch.empty(Bl, cfg.Lin, dtype=torch.float32, device=dev)
        res = torch.zeros(256, dtype=torch.uint8, device=dev)      # amp_status @0, amp_counts @64
        a = nat.AmpScampArgs()
        a.W, a.A, a.y = nat.dptr(Wc, torch.float32, 'W'), nat.dptr(Ac, name='A'), nat.dptr(yl, name='y')
        a.max_iter = cfg.N_Layers
        a.engine = nat.ENGINE_LAUNCHES
        a.noise_var = float(self.E / SNR)                                  # scamp.py:98
        a.xmap, a.xmmse, a.psi = nat.dptr(xmap), nat.dptr(xm), nat.dptr(psi)
        a.status = nat.dptr(res)
        a.ws, a.ws_bytes = nat.dptr(self._ws), self._ws.numel()
        st = nat.stream_ptr(dev)
        self._run_hooked(lib.amp_scamp_run_sharded, 'amp_scamp_run_sharded', C.byref(d), C.byref(cst), C.byref(a), B,
                         st)
        L = self._decide_merge(d, cst, xmap, xm, x, symbol, index, b0, b1, res, st)
        self.last_shard = (xmap.view(Bl, N, 1), xm.view(Bl, N, 1), psi.view(Bl, cfg.Lin, 1))
        return L
