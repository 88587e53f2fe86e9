"""Damped "Rangan" VAMP — drop-in for the reference's ``vamp2.py`` (``Tracker``, ``VAMPLayer``,
``VAMP``; vamp2.py:12-135), running on the gfx950 kernels of libampsparc.so
(``amp_vamp2_run``, csrc/amp_vamp2.hip).

``VAMP(config, damping=1.0).forward(U, s, Vh, y, SNR, x, symbols, indices) -> Loss`` keeps the
reference's signature: the whole iteration loop (denoiser at tau = gamma, damping, the
gamma / d updates and the allclose early exit on var, vamp2.py:62-77, 123-131) runs on the
device, then the MAP decision and the counters of ``Loss`` on T.r (vamp2.py:131).  Like the
reference, sparc mode only: its 'random' mode builds a Shrink denoiser whose single return
value the layer cannot unpack, and its 'segmented' decision reshapes B > 1 batches wrongly.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
from torch import nn

import amp_native as nat
from config import Config
from loss import Loss
from vamp import LazyResult, _c64, block_denoise


class Tracker:
    """Device state of one damped-VAMP forward (vamp2.py:12-26): r, xmmse, var, gamma and the
    workspace holding the expanded Uh / Vh / eta V operators, y~ and the scalar record."""

    def __init__(self, U, s, Vh, y, x, sigma2: float, config: Config, damping: float = 1.0):
        self.config = config
        B = config.B
        n, k = U.shape[0], U.shape[1]
        N = Vh.shape[1]
        self.U = _c64(U, (n, k))
        self.s = s.reshape(k).to(torch.float32).resolve_neg().contiguous()
        self.Vh = _c64(Vh, (k, N))
        self.y = _c64(y, (B, n))
        self.sigma2 = sigma2
        self.eta = N / k                                                  # vamp2.py:26
        self.k = k
        self.dims = config.dims()
        self.const = config.constellation()
        dev = self.y.device
        wsb = nat.lib().amp_vamp2_workspace_bytes(C.byref(self.dims), k)
        if wsb == 0:
            raise ValueError('amp_vamp2_workspace_bytes: invalid dimensions')
        self._r = torch.empty(B, N, dtype=torch.complex64, device=dev)
        self._xmmse = torch.empty(B, N, dtype=torch.complex64, device=dev)
        self._var = torch.empty(B, N, dtype=torch.float32, device=dev)
        self.ws = nat.WORKSPACE.get(dev, 'vamp2', wsb)
        a = nat.AmpVamp2Args()
        a.U, a.s, a.Vh, a.y = (nat.dptr(self.U, name='U'), nat.dptr(self.s, torch.float32, 's'),
                               nat.dptr(self.Vh, name='Vh'), nat.dptr(self.y, name='y'))
        a.k, a.max_iter = k, config.N_Layers
        a.sigma2, a.damping = float(sigma2), float(damping)
        a.r, a.xmmse, a.var = nat.dptr(self._r), nat.dptr(self._xmmse), nat.dptr(self._var)
        a.ws, a.ws_bytes = nat.dptr(self.ws), self.ws.numel()
        self.args = a
        self.stream = nat.stream_ptr(dev)

    @property
    def r(self):
        return self._r.view(self.config.B, -1, 1)

    @property
    def xmmse(self):
        return self._xmmse.view(self.config.B, -1, 1)

    @property
    def var(self):
        return self._var.view(self.config.B, -1, 1)


class VAMPLayer(nn.Module):
    """vamp2.py:28-93.  The iteration itself runs inside ``amp_vamp2_run``; the layer keeps the
    reference's attributes and its denoiser as a standalone device op."""

    def __init__(self, config: Config, damping: float = 0.97) -> None:
        super().__init__()
        self.config = config
        self.Nt, self.Na, self.Lin, self.B = config.Nt, config.Na, config.Lin, config.B
        self.K = config.K
        self.M = self.Nt // self.Na
        self.L = self.Na * self.Lin
        self.LM = self.L * self.M
        self.rho = damping
        self.var_min = torch.tensor(1.0e-11)
        self.var_max = torch.tensor(1.0e11)

    def segmented_denoiser(self, s: torch.Tensor, tau) -> tuple[torch.Tensor, torch.Tensor]:
        """vamp2.py:79-88 on the device (the same float64-shift softmax as vamp.py; its variance
        E|a|^2 - |xmmse|^2 equals vamp.py's var0 + vars)."""
        return block_denoise(self.config, s, tau, mode=0)


class VAMP(LazyResult, nn.Module):
    """vamp2.py:95-135 with the loop on the device."""

    def __init__(self, config: Config, damping: float = 1.0) -> None:
        super().__init__()
        self.config = config
        self.damping = damping
        self.E = config.Na / config.Nr                                   # vamp2.py:98
        self.sparsity = config.Na / config.Nt
        self.layers = nn.ModuleList([VAMPLayer(config, damping) for _ in range(config.N_Layers)])
        self.L = Loss(config)
        self.last = None

    def detect(self, U, s, Vh, y, SNR: float) -> Tracker:
        """All iterations on the device, asynchronous (no host sync)."""
        with torch.cuda.device(y.device):
            T = Tracker(U, s, Vh, y, None, self.E / SNR, self.config, self.damping)
            res, _ = self._result_slot(T.y.device)
            T.res = res
            T.args.status = nat.dptr(res)
            nat.check(nat.lib().amp_vamp2_run(C.byref(T.dims), C.byref(T.const), C.byref(T.args), T.stream),
                      'amp_vamp2_run')
        self.last = T
        return T

    def forward(self, U: torch.Tensor, s: torch.Tensor, Vh: torch.Tensor, y: torch.Tensor, SNR: float,
                x: torch.Tensor, symbols: np.ndarray, indices: np.ndarray) -> Loss:
        if self.config.mode == 'random':
            # vamp2.py:45-46 picks Shrink('bayes'), which returns one tensor; vamp2.py:62 then fails
            raise ValueError('not enough values to unpack (expected 2, got 1)')
        with torch.cuda.device(y.device):
            T = Tracker(U, s, Vh, y, None, self.E / SNR, self.config, self.damping)
            res, host = self._result_slot(T.y.device)
            T.res = res
            T.args.status = nat.dptr(res)
            nat.check(nat.lib().amp_vamp2_run(C.byref(T.dims), C.byref(T.const), C.byref(T.args), T.stream),
                      'amp_vamp2_run')
            self.L.device_counts(T.r, T.xmmse, x, symbols, indices, out=res[64:])   # vamp2.py:131
            self._arm(self.L, res, host, 'amp_vamp2_run')
        self.last = T
        return self.L
