"""BAMP detector — drop-in for the reference's ``BAMP`` / ``BAMPLayer`` (bamp.py:12-143),
running on the gfx950 kernels of libampsparc.so (amp_bamp_run)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
from torch import nn

import amp_native as nat
from config import Config
from loss import Loss
from vamp import _c64, block_denoise, read_result


class BAMPLayer(nn.Module):
    """BAMPLayer (bamp.py:27-64); its denoiser is the per-element-tau block denoiser."""

    def __init__(self, config: Config) -> None:
        super().__init__()
        self.config = config
        self.Nt, self.Na, self.Lin, self.B = config.Nt, config.Na, config.Lin, config.B
        self.K = config.K
        self.M = self.Nt // self.Na
        self.L = self.Na * self.Lin
        self.LM = self.L * self.M

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


class BAMP(nn.Module):
    def __init__(self, config: Config) -> None:
        super().__init__()
        self.config = config
        self.E = config.Na / config.Nr                                    # bamp.py:102
        self.layers = nn.ModuleList([BAMPLayer(config) for _ in range(config.N_Layers)])
        self.L = Loss(config)
        self._key = None
        self.last = None

    def _ensure_buffers(self, dev, B, N, wsb):
        key = (str(dev), B, N, wsb)
        if key != self._key:
            self.xmap = torch.empty(B, N, dtype=torch.complex64, device=dev)
            self.xmmse = torch.empty(B, N, dtype=torch.complex64, device=dev)
            self.var = torch.empty(B, N, dtype=torch.float32, device=dev)
            self.res = torch.zeros(256, dtype=torch.uint8, device=dev)
            self.ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
            self._key = key

    def detect(self, H: torch.Tensor, y: torch.Tensor, SNR: float):
        cfg = self.config
        B = cfg.B
        n, N = H.shape[-2], H.shape[-1]
        H = _c64(H, (n, N))
        y = _c64(y, (B, n))
        d, c = cfg.dims(), cfg.constellation()
        lib = nat.lib()
        wsb = lib.amp_bamp_workspace_bytes(C.byref(d), cfg.N_Layers)
        self._ensure_buffers(y.device, B, N, wsb)
        a = nat.AmpBampArgs()
        a.H, a.y = nat.dptr(H, name='H'), nat.dptr(y, name='y')
        a.max_iter = cfg.N_Layers
        a.noise_var = float(self.E / SNR)                                 # bamp.py:124
        # bamp.py:38-41: 'random' mode denoises element-wise (random_denoiser, bamp.py:79-88)
        a.denoiser = 1 if cfg.mode == 'random' else 0
        a.P0, a.Ps = float(np.float32(cfg.P0)), float(np.float32(cfg.Ps))
        a.xmap, a.xmmse, a.var = nat.dptr(self.xmap), nat.dptr(self.xmmse), nat.dptr(self.var)
        a.status = nat.dptr(self.res)
        a.ws, a.ws_bytes = nat.dptr(self.ws), self.ws.numel()
        self._keep = (H, y)
        nat.check(lib.amp_bamp_run(C.byref(d), C.byref(c), C.byref(a), nat.stream_ptr(y.device)), 'amp_bamp_run')

    def forward(self, H: torch.Tensor, y: torch.Tensor, SNR: float, x: torch.Tensor, symbols, indices) -> Loss:
        self.detect(H, y, SNR)
        self.L.dump()                                                     # bamp.py:125
        self.L.device_counts(self.xmap, self.xmmse, x, symbols, indices, out=self.res[64:])   # bamp.py:142
        status, counts = read_result(self.res)
        self.L.record(self.L.rates_from_counts(counts), int(status.T))
        self.last = status
        return self.L
