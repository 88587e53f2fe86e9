"""Element-wise shrinkage denoisers — drop-in for the reference's ``Shrink`` (shrink.py:8-166),
running on the gfx950 kernels of libampsparc.so (csrc/amp_shrink.hip).

Same constructor, method names, argument meaning, output dtypes/shapes and exceptions:

* ``bayes(r, cov) -> x``               posterior mean under the P0/Ps sparse prior
  (shrink.py:78-96); one tensor, like the reference (its ``var`` line is commented out).
* ``shrinkOOK(r, cov) -> (x, dxdr)``   OOK posterior mean and the batch-mean derivative
  (shrink.py:139-157); ``dxdr`` is a 0-dim float32 device tensor.
* ``sw_shrinkOOK(r, cov) -> (x, var)`` section-wise leave-one-out OOK denoiser
  (shrink.py:58-76), x complex64 [B, L*M, 1], var float32.
* ``shrink`` / ``lasso`` raise for every input in the reference (shrink.py:98-137: torch.sign
  of a complex tensor, an unbound local ``d0``, the missing attribute ``lmda``); they raise the
  same exception types here.

``cov`` is a python float, a 0-dim tensor or a tensor broadcastable to ``r``.  Every compute
call runs on the device through the C ABI; there is no CPU fallback.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch
from torch import nn

import amp_native as nat
from config import Config

_SIGN_COMPLEX_MSG = ('Unlike NumPy, torch.sign is not intended to support complex numbers. '
                     'Please use torch.sgn instead.')


class Shrink(nn.Module):
    def __init__(self, config: Config, shrink_fn: str) -> None:
        super().__init__()
        assert shrink_fn in ["bayes", "shrink", "lasso", "shrinkOOK"], "shrink_fn needs to be ..."   # shrink.py:17
        self.config = config
        self.Ps, self.P0 = torch.tensor(config.Ps), torch.tensor(config.P0)                      # float32, :19
        self.dtype = torch.complex64 if config.is_complex else torch.float32                    # :21-24
        self.symbols = torch.tensor(config.symbols, device=config.device, dtype=self.dtype)     # :26
        self.symbols2 = torch.abs(self.symbols) ** 2
        self.tol = torch.tensor(1.0e-9)
        self.M = config.Nt // config.Na
        self.L = config.Na * config.Lin
        self.B = config.B
        self.shrink_fn = shrink_fn
        self.shrinkage = {'bayes': self.bayes, 'shrink': self.shrink, 'lasso': self.lasso,
                          'shrinkOOK': self.shrinkOOK}[shrink_fn]
        # theta = log(P0 / Ps) with the reference's float32 tensor ops (shrink.py:152)
        self._theta = float(torch.log(self.P0 / self.Ps))
        self._const = None

    def forward(self, r: torch.Tensor, cov):
        return self.shrinkage(r, cov)

    # -- helpers ------------------------------------------------------------------------------
    def _constellation(self):
        if self._const is None:
            c = self.config
            sym = np.asarray(c.symbols)
            if self.dtype == torch.float32:
                sym = sym.real.astype(np.float64)
            self._const = nat.make_constellation(sym, c.gray, c.symbol_bits)
        return self._const

    @staticmethod
    def _cov_args(cov, shape, device):
        """(cov_scalar, cov_vec tensor or None) for the C ABI."""
        if not isinstance(cov, torch.Tensor):
            return float(np.float32(cov)), None
        if cov.numel() == 1:
            return float(cov.reshape(()).to(torch.float32).item()), None
        v = cov.to(device=device, dtype=torch.float32).expand(shape).contiguous()
        return 0.0, v

    @staticmethod
    def _single(r: torch.Tensor, what: str) -> None:
        """The kernels compute in float32 / complex64 (the dtypes every reference caller hands
        over).  For float64 / complex128 r the reference's outputs would be float64 / complex128;
        rather than silently returning a downcast result, such inputs are refused."""
        if r.dtype in (torch.float64, torch.complex128):
            raise TypeError(f'Shrink.{what}: {r.dtype} input is not supported by the gfx950 kernels '
                            '(float32 / complex64 only; no silent downcast)')

    @staticmethod
    def _real_part(r: torch.Tensor):
        """(tensor, is_complex) whose real part the kernels read (r.real, shrink.py:68/:153):
        complex64 r is handed over as it lies (the kernel reads the real lanes), no copy."""
        if r.is_complex():
            return r.to(torch.complex64).resolve_conj().resolve_neg().contiguous(), 1
        return r.to(torch.float32).contiguous(), 0

    # -- denoisers ----------------------------------------------------------------------------
    def bayes(self, r: torch.Tensor, cov) -> torch.Tensor:
        """shrink.py:78-96.  Output dtype = promote(r, symbols) as in the reference."""
        self._single(r, 'bayes')
        cplx = r.is_complex() or self.dtype == torch.complex64
        rr = r.to(torch.complex64 if cplx else torch.float32).resolve_conj().resolve_neg().contiguous()
        out = torch.empty_like(rr)
        cs, cv = self._cov_args(cov, rr.shape, rr.device)
        nat.check(nat.lib().amp_shrink_bayes(
            self._constellation(), rr.numel(), int(cplx), nat.dptr(rr, name='r'), cs,
            None if cv is None else nat.dptr(cv, name='cov'), float(self.P0), float(self.Ps),
            nat.dptr(out, name='out'), nat.stream_ptr(rr.device)), 'amp_shrink_bayes')
        return out

    def shrinkOOK(self, r: torch.Tensor, cov) -> Tuple[torch.Tensor, torch.Tensor]:
        """shrink.py:139-157: (exp float32 shaped like r, dxdr = der.mean() 0-dim float32)."""
        self._single(r, 'shrinkOOK')
        re, cplx = self._real_part(r)
        if re.numel() == 0:
            raise RuntimeError('shrinkOOK: empty input (the reference returns a NaN mean)')
        out = torch.empty(re.shape, dtype=torch.float32, device=re.device)
        dxdr = torch.empty((), dtype=torch.float32, device=re.device)
        cs, cv = self._cov_args(cov, re.shape, re.device)
        L = nat.lib()
        wsb = L.amp_shrink_ook_workspace_bytes(re.numel())
        ws = nat.WORKSPACE.get(re.device, 'shrink_ook', wsb)
        nat.check(L.amp_shrink_ook(
            re.numel(), cplx, nat.dptr(re, name='r'), cs, None if cv is None else nat.dptr(cv, name='cov'),
            self._theta, nat.dptr(out, name='exp'), nat.dptr(dxdr, name='dxdr'), nat.dptr(ws), wsb,
            nat.stream_ptr(re.device)), 'amp_shrink_ook')
        return out, dxdr

    def sw_shrinkOOK(self, r: torch.Tensor, cov) -> Tuple[torch.Tensor, torch.Tensor]:
        """shrink.py:58-76: sections of M along the flattened (B, L, M) view."""
        self._single(r, 'sw_shrinkOOK')
        re, cplx = self._real_part(r)
        if re.numel() != self.B * self.L * self.M:
            raise RuntimeError(f"shape '[{self.B}, {self.L}, {self.M}]' is invalid for input of size {re.numel()}")
        S = self.B * self.L
        x = torch.empty(self.B, self.L * self.M, 1, dtype=torch.complex64, device=re.device)
        var = torch.empty(self.B, self.L * self.M, 1, dtype=torch.float32, device=re.device)
        cs, cv = self._cov_args(cov, re.shape, re.device)
        nat.check(nat.lib().amp_shrink_sw_ook(
            S, self.M, cplx, nat.dptr(re, name='r'), cs, None if cv is None else nat.dptr(cv, name='cov'),
            nat.dptr(x, name='exp'), nat.dptr(var, name='var'), nat.stream_ptr(re.device)), 'amp_shrink_sw_ook')
        return x, var

    def shrink(self, r: torch.Tensor, cov):
        """shrink.py:98-119 raises for every input: torch.sign of the complex difference, or,
        for real inputs, ``d0`` used in the same tuple assignment that defines it (:113)."""
        if r.is_complex() or self.dtype == torch.complex64:
            raise NotImplementedError(_SIGN_COMPLEX_MSG)
        raise UnboundLocalError("local variable 'd0' referenced before assignment")

    def lasso(self, r: torch.Tensor, cov):
        """shrink.py:121-137 raises for every input: torch.sign of complex r, or the attribute
        ``lmda`` that no code path defines."""
        if r.is_complex():
            raise NotImplementedError(_SIGN_COMPLEX_MSG)
        raise AttributeError("'Shrink' object has no attribute 'lmda'")

    # -- reference helpers (shrink.py:159-166), in-place like the reference ------------------
    def regularize_zero(self, a):
        a[a == 0.] = self.tol.to(a.device)
        return a

    def regularize_exp(self, a: torch.Tensor):
        mx = np.log(torch.finfo(a.dtype).max)
        a[a >= mx] = mx - 1
        return a
