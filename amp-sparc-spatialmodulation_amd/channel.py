"""Channel model — drop-in for the reference's ``Channel`` (channel.py:8-116).

Input generation, not the hot path.  It reproduces the reference's random streams
exactly so that the same seeds give the same (W, A, noise):
  * ``generate_as_sparc`` draws ``normal(size=(Nr, Nt, Lh))`` twice from numpy's global
    legacy RNG (channel.py:85-86) and places ``sqrt(W[o,i]) * h_l`` on the block
    (o, i) with o - i = l (the nonzero blocks of channel.py:90's kron sum, same
    float64 products and complex64 accumulation order);
  * ``awgn`` draws two ``torch.normal`` tensors from torch's CPU generator
    (channel.py:113-114) and only then moves the result to ``config.device``, so a
    GPU run sees the noise the reference's CPU path sees (``rng='device'`` draws on
    the GPU generator instead, for throughput runs that do not need parity).
"""
from __future__ import annotations

import numpy as np
import torch

from config import Config


class Channel:
    def __init__(self, config: Config, rng: str = 'host') -> None:
        self.device = config.device
        self.B, self.Lin = config.B, config.Lin
        self.Nt, self.Na, self.Nr = config.Nt, config.Na, config.Nr
        self.Lh = config.Lh
        self.trunc = config.trunc
        self.Lout = config.Lout
        self.sparsity = config.sparsity
        self.is_complex = config.is_complex
        self.rng = rng
        if config.profile == 'exponential':          # channel.py:22-26
            pdp = np.exp(-np.arange(self.Lh))
        elif config.profile == 'uniform':
            pdp = np.ones(self.Lh)
        else:
            raise ValueError("channel_profile 'random' has no power-delay profile in the reference "
                             "(channel.py:22-26 leaves pdp undefined)")
        self.pdp = pdp / np.sum(pdp)
        self.dtype = torch.complex64 if self.is_complex else torch.float32
        self.npdtype = np.complex64 if self.is_complex else np.float32

    # ------------------------------------------------------------------
    def _base_matrix(self) -> np.ndarray:
        """Spatial-coupling base matrix W (channel.py:80-83)."""
        W = np.zeros((self.Lout, self.Lin))
        for l in range(self.Lh):
            W += np.eye(self.Lout, self.Lin, -l) * self.pdp[l]
        return W / W.mean() * self.Na / self.Nr

    def generate_as_sparc(self):
        """(W float32 [Lout,Lin], A complex64 [Nr*Lout, Nt*Lin]) — channel.py:75-95."""
        if self.rng == 'device':
            return self._generate_as_sparc_device()
        W = self._base_matrix()
        hr = np.random.normal(size=(self.Nr, self.Nt, self.Lh))
        hj = np.random.normal(size=(self.Nr, self.Nt, self.Lh))
        h = (hr + 1j * hj) / np.sqrt(2 * self.Na * self.Lin)
        A = np.zeros((self.Nr * self.Lout, self.Nt * self.Lin), dtype=self.npdtype)
        sw = np.sqrt(W)
        for l in range(self.Lh):
            hl = h[:, :, l]
            for i in range(self.Lin):
                o = i + l
                if o >= self.Lout:
                    continue
                blk = A[o * self.Nr:(o + 1) * self.Nr, i * self.Nt:(i + 1) * self.Nt]
                blk += sw[o, i] * hl
        Wt = torch.tensor(W, dtype=torch.float32, device=self.device)
        At = torch.tensor(A, dtype=self.dtype, device=self.device)
        return Wt, At

    def _generate_as_sparc_device(self):
        """Throughput mode: the same block structure and distribution as generate_as_sparc,
        h ~ CN(0, 1/(Na Lin)) drawn by the device generator (a different random stream from the
        reference's numpy one: statistical, not bitwise, parity)."""
        W = self._base_matrix()
        shape = (self.Nr, self.Nt, self.Lh)
        hr = torch.randn(shape, device=self.device, dtype=torch.float32)
        hj = torch.randn(shape, device=self.device, dtype=torch.float32)
        h = torch.complex(hr, hj) * float(1.0 / np.sqrt(2 * self.Na * self.Lin))
        sw = np.sqrt(W)
        A = torch.zeros((self.Nr * self.Lout, self.Nt * self.Lin), dtype=torch.complex64, device=self.device)
        for l in range(self.Lh):
            for i in range(self.Lin):
                o = i + l
                if o >= self.Lout:
                    continue
                A[o * self.Nr:(o + 1) * self.Nr, i * self.Nt:(i + 1) * self.Nt] += float(sw[o, i]) * h[:, :, l]
        Wt = torch.tensor(W, dtype=torch.float32, device=self.device)
        return Wt, A.to(self.dtype)

    def generate_correlated(self, rho: float = 0.5) -> torch.Tensor:
        """Kronecker exponentially-correlated Rayleigh channel A = L_r G L_t^T, [Nr, Nt] complex64.

        Not in the reference (its 'random' profile has no pdp and crashes, channel.py:27-31, and
        there is no correlated model); BASELINE cfg5 names it, so this build defines it:
        G ~ CN(0, 1/Nr) i.i.d. (the reference's entry variance for Lin = Lh = 1, channel.py:85-91),
        R_r[i,j] = R_t[i,j] = rho^|i-j|, and L the Cholesky factor of R, which for the exponential
        model is the AR(1) filter x_0 = g_0, x_i = rho x_{i-1} + sqrt(1 - rho^2) g_i.  Applied as
        elementwise recursions in float64 (no BLAS: bit-reproducible on every host).  Draws
        np.random.normal twice (real, imaginary parts), like generate_as_sparc."""
        assert self.Lin == 1 and self.Lh == 1, 'correlated channel: Lin = Lh = 1 only'
        gr = np.random.normal(size=(self.Nr, self.Nt))
        gi = np.random.normal(size=(self.Nr, self.Nt))
        A = (gr + 1j * gi) / np.sqrt(2 * self.Nr)
        c = np.sqrt(1.0 - rho * rho)
        for i in range(1, self.Nr):                    # receive side: rows
            A[i] = rho * A[i - 1] + c * A[i]
        for j in range(1, self.Nt):                    # transmit side: columns
            A[:, j] = rho * A[:, j - 1] + c * A[:, j]
        return torch.tensor(A.astype(np.complex64), dtype=self.dtype, device=self.device)

    def generate_channel(self) -> torch.Tensor:
        """Block-Toeplitz MIMO-ISI channel with trunc/tail/cyclic edges (channel.py:40-73)."""
        hr = np.random.normal(size=(self.Nr, self.Nt, self.Lh))
        hi = np.random.normal(size=(self.Nr, self.Nt, self.Lh))
        h = (hr + 1j * hi) * np.sqrt(self.pdp * self.Lout / self.Nr / self.Lin / 2)
        Nr, Nt, Lh, Lin = self.Nr, self.Nt, self.Lh, self.Lin
        H = np.zeros((Lin * Nr, Lin * Nt), dtype=self.npdtype)
        for l in range(Lh):
            for i in range(Lin - l):
                o = i + l
                H[o * Nr:(o + 1) * Nr, i * Nt:(i + 1) * Nt] += h[:, :, l]
        if self.trunc != 'trunc' and Lh > 1:
            tail = H[-Nr:, -Nt * Lh:-Nt]
            if self.trunc == 'tail':
                extra = np.zeros((Nr * (Lh - 1), Nt * Lin), dtype=self.npdtype)
                for l in range(Lh - 1):
                    w = Nt * (Lh - l - 1)
                    extra[l * Nr:(l + 1) * Nr, -w:] = tail[:, :w]
                H = np.block([[H], [extra]])
            else:  # cyclic
                for l in range(Lh - 1):
                    w = Nt * (Lh - l - 1)
                    H[l * Nr:(l + 1) * Nr, -w:] = tail[:, :w]
        return torch.tensor(H, dtype=self.dtype, device=self.device)

    def generate_as_random(self) -> torch.Tensor:
        """i.i.d. CN(0, 1/(Lin Nr)) channel on the device generator (channel.py:97-101)."""
        shape = (self.Nr * self.Lout, self.Nt * self.Lin)
        H = torch.normal(mean=0, std=1, size=shape, device=self.device)
        H = H + 1j * torch.normal(mean=0, std=1, size=shape, device=self.device)
        return (H / np.sqrt(2 * self.Lin * self.Nr)).to(self.dtype)

    def awgn(self, SNR) -> torch.Tensor:
        """CN(0, Na/Nr/SNR) noise [B, Nr*Lout, 1] (channel.py:103-116)."""
        size = (self.B, self.Nr * self.Lout, 1)
        gen_dev = 'cpu' if self.rng == 'host' else self.device
        nr = torch.normal(mean=0., std=1., size=size, device=gen_dev)
        ni = torch.normal(mean=0., std=1., size=size, device=gen_dev)
        noise = (nr + 1j * ni) * np.sqrt(self.Na / self.Nr / SNR / 2)
        return noise.to(self.device)
