"""Message generator — drop-in for the reference's ``Data`` (data.py:7-91).

``segmented`` (used by 'sparc' and 'segmented' modes) places one constellation point
per section of M = Nt/Na entries at a uniform position.  The reference draws
``np.random.choice(M)`` then ``np.random.choice(K)`` for every (trial, section) in a
Python loop (data.py:82-87).  Legacy ``choice(n)`` consumes one 32-bit MT19937 output
and masks it when n is a power of two (no rejection) and consumes nothing when n == 1,
so for power-of-two M and K the same stream is drawn here in one vectorised call;
other sizes fall back to the reference's per-draw order.  Either way the returned
(x, gray labels, flat indices) are bit-identical for the same numpy seed.
"""
from __future__ import annotations

import numpy as np
import torch

from config import Config


def _pow2(v: int) -> bool:
    return v > 0 and (v & (v - 1)) == 0


class Data:
    def __init__(self, config: Config, rng: str = 'host') -> None:
        self.rng = rng
        self.B = config.B
        self.Lin = config.Lin
        self.Nt = config.Nt
        self.Na = config.Na
        self.Ns = config.Na
        self.device = config.device
        self.symbols = config.symbols
        self.gray = config.gray
        self.cardinality = len(self.symbols)
        self.dtype = torch.complex64 if config.is_complex else torch.float32
        self.npdtype = np.complex64 if config.is_complex else np.float32
        if config.mode == 'random':
            self._generator = self.random
        else:
            assert self.Nt % self.Na == 0, 'Na must divide Nt'
            self.L = self.Na * self.Lin
            self.M = self.Nt // self.Na
            self._generator = self.segmented

    def generate_message(self):
        """(x [B, Nt*Lin, 1] on config.device, gray labels, flat nonzero indices) — data.py:45-53."""
        if self.rng == 'device':
            return self._segmented_device()
        x, z, i = self._generator()
        return torch.tensor(x, device=self.device, dtype=self.dtype), z, i

    def random(self):
        """Na active antennas per channel use, one symbol (data.py:55-72)."""
        x = np.zeros((self.B, self.Lin, self.Nt), dtype=self.npdtype)
        xgray = np.zeros((self.B, self.Lin, self.Nt), dtype=int)
        for b in range(self.B):
            for j in range(self.Lin):
                pos = np.random.choice(self.Nt, size=self.Na, replace=False)
                k = np.random.choice(self.cardinality)
                x[b, j, pos] = self.symbols[k]
                xgray[b, j, pos] = self.gray[k]
        x = np.reshape(x, (self.B, -1, 1))
        index = x.ravel().nonzero()[0]
        return x, xgray.ravel()[index], index

    def _draw_sections(self, S: int):
        M, K = self.M, self.cardinality
        if _pow2(M) and _pow2(K):
            per = int(M > 1) + int(K > 1)
            raw = (np.random.randint(0, 2 ** 32, size=S * per, dtype=np.uint32).reshape(S, per)
                   if per else np.zeros((S, 0), np.uint32))
            pos = (raw[:, 0] & np.uint32(M - 1)).astype(np.int64) if M > 1 else np.zeros(S, np.int64)
            k = (raw[:, per - 1] & np.uint32(K - 1)).astype(np.int64) if K > 1 else np.zeros(S, np.int64)
            return pos, k
        pos = np.empty(S, np.int64)
        k = np.empty(S, np.int64)
        for s in range(S):
            pos[s] = np.random.choice(M)
            k[s] = np.random.choice(K)
        return pos, k

    def segmented(self):
        """One point per section at a uniform position (data.py:74-91)."""
        S = self.B * self.L
        pos, k = self._draw_sections(S)
        x = np.zeros((S, self.M), dtype=self.npdtype)
        xgray = np.zeros((S, self.M), dtype=int)
        rows = np.arange(S)
        x[rows, pos] = np.asarray(self.symbols)[k]
        xgray[rows, pos] = np.asarray(self.gray)[k]
        x = np.reshape(x, (self.B, -1, 1))
        index = x.ravel().nonzero()[0]
        return x, xgray.ravel()[index], index

    def _segmented_device(self):
        """Throughput mode of ``segmented``: positions and symbols drawn by the device generator
        (uniform, as data.py:82-87), x scattered on the device; labels and indices returned as
        int64 device tensors (the decision consumes them there)."""
        if self._generator != self.segmented:
            raise NotImplementedError("rng='device' implements the 'sparc' / 'segmented' generator")
        S, M, K = self.B * self.L, self.M, self.cardinality
        pos = torch.randint(0, M, (S,), device=self.device)
        k = torch.randint(0, K, (S,), device=self.device)
        sym = torch.as_tensor(np.asarray(self.symbols), dtype=torch.complex128, device=self.device).to(self.dtype)
        gray = torch.as_tensor(np.asarray(self.gray), dtype=torch.int64, device=self.device)
        x = torch.zeros((S, M), dtype=self.dtype, device=self.device)
        x[torch.arange(S, device=self.device), pos] = sym[k]
        index = torch.arange(S, device=self.device, dtype=torch.int64) * M + pos
        return x.reshape(self.B, -1, 1), gray[k], index
