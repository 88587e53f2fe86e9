"""SCAMP (spatially coupled SPARC AMP) — drop-in for the reference's ``SCAMP`` /
``SCAMPLayer`` (scamp.py:8-108), running on the gfx950 kernels of libampsparc.so
(amp_scamp_run)."""
from __future__ import annotations

import ctypes as C

import torch
from torch import nn

import amp_native as nat
from config import Config
from loss import Loss
from vamp import _c64, block_denoise, read_result


class SCAMPLayer(nn.Module):
    """SCAMPLayer (scamp.py:27-68); its denoiser is the mean-only block denoiser."""

    def __init__(self, config: Config) -> None:
        super().__init__()
        self.config = config
        self.B, self.Na = config.B, config.Na
        self.M = config.Nt // config.Na
        self.Mc, self.Mr = config.Nt, config.Nr
        self.L = config.Na * config.Lin
        self.Lc, self.Lr = config.Lin, config.Lout
        self.n = self.Mr * self.Lr
        self.LM = self.Mc * self.Lc
        self.K = config.K

    def denoiser(self, s: torch.Tensor, tau: torch.Tensor) -> torch.Tensor:
        """scamp.py:61-68: tau is tau_use, halved inside."""
        return block_denoise(self.config, s, tau, mode=2)


class SCAMP(nn.Module):
    def __init__(self, config: Config) -> None:
        super().__init__()
        self.config = config
        self.E = config.Na / config.Nr                                    # scamp.py:72
        self.layers = nn.ModuleList([SCAMPLayer(config) for _ in range(config.N_Layers)])
        self.L = Loss(config)
        self._key = None
        self.last = None

    def _ensure_buffers(self, dev, B, N, Lin, wsb):
        key = (str(dev), B, N, Lin, wsb)
        if key != self._key:
            self.xmap = torch.empty(B, N, dtype=torch.complex64, device=dev)
            self.xmmse = torch.empty(B, N, dtype=torch.complex64, device=dev)
            self.psi = torch.empty(B, Lin, dtype=torch.float32, device=dev)
            self.res = torch.zeros(256, dtype=torch.uint8, device=dev)
            self.ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
            self._key = key

    def detect(self, W: torch.Tensor, A: torch.Tensor, y: torch.Tensor, SNR: float):
        cfg = self.config
        B = cfg.B
        n, N = A.shape[-2], A.shape[-1]
        A = _c64(A, (n, N))
        y = _c64(y, (B, n))
        W = W.reshape(cfg.Lout, cfg.Lin).to(device=y.device, dtype=torch.float32).resolve_neg().contiguous()
        d, c = cfg.dims(), cfg.constellation()
        lib = nat.lib()
        wsb = lib.amp_scamp_workspace_bytes(C.byref(d), cfg.N_Layers)
        self._ensure_buffers(y.device, B, N, cfg.Lin, wsb)
        a = nat.AmpScampArgs()
        a.W, a.A, a.y = nat.dptr(W, torch.float32, 'W'), nat.dptr(A, name='A'), nat.dptr(y, name='y')
        a.max_iter = cfg.N_Layers
        a.noise_var = float(self.E / SNR)                                 # scamp.py:98
        a.xmap, a.xmmse, a.psi = nat.dptr(self.xmap), nat.dptr(self.xmmse), nat.dptr(self.psi)
        a.status = nat.dptr(self.res)
        a.ws, a.ws_bytes = nat.dptr(self.ws), self.ws.numel()
        self._keep = (W, A, y)
        nat.check(lib.amp_scamp_run(C.byref(d), C.byref(c), C.byref(a), nat.stream_ptr(y.device)), 'amp_scamp_run')

    def forward(self, W: torch.Tensor, A: torch.Tensor, y: torch.Tensor, SNR: float, x: torch.Tensor, symbol,
                index) -> Loss:
        self.detect(W, A, y, SNR)
        self.L.dump()                                                     # scamp.py:99
        self.L.device_counts(self.xmap, self.xmmse, x, symbol, index, out=self.res[64:])   # scamp.py:107
        status, counts = read_result(self.res)
        self.L.record(self.L.rates_from_counts(counts), int(status.T))
        self.last = status
        return self.L
