"""System parameters — drop-in for the reference's ``Config`` (config.py:4-157).

Same constructor, same attribute names and values (the detectors, drivers and Loss
read them), plus two additions for the native path: ``dims()`` and
``constellation()`` produce the C structs of include/amp_sparc.h.
"""
from __future__ import annotations

import numpy as np

_ALPHABET_TABLE = {
    # alphabet: (points, gray labels, Ps divisor, forces complex)          config.py:78-116
    'OOK': ([1], [1], 1, False),
    'BPSK': ([-1, 1], [0, 1], 2, False),
    '4ASK': ([-3, -1, 1, 3], [0, 1, 3, 2], 4, False),
    'QPSK': ([1 + 0j, 0 + 1j, -1 + 0j, 0 - 1j], [0, 1, 3, 2], 4, True),
    '8PSK': ([np.exp((2 * np.pi * 1j / 8) * n) for n in range(8)], [0, 1, 3, 2, 6, 7, 5, 4], 8, True),
    '16PSK': ([np.exp((2 * np.pi * 1j / 16) * n) for n in range(16)],
              [0, 1, 3, 2, 6, 7, 5, 4, 12, 13, 15, 14, 10, 11, 9, 8], 16, True),
    # the reference's table, including its duplicated -1+3j / missing 1-3j (config.py:112):
    # parity means reproducing it
    '16QAM': ([1 + 1j, 1 - 1j, -1 + 1j, -1 - 1j, 3 + 1j, 3 - 1j, -3 + 1j, -3 - 1j,
               3 + 3j, 3 - 3j, -3 + 3j, -3 - 3j, 1 + 3j, -1 + 3j, -1 + 3j, -1 - 3j],
              [0, 1, 13, 7, 8, 9, 2, 15, 12, 11, 5, 10, 14, 3, 6, 4], 16, True),
}


class Config:
    def __init__(self,
                 N_transmit_antenna: int,
                 N_active_antenna: int,
                 N_receive_antenna: int,
                 block_length: int,
                 channel_length: int,
                 batch: int = 100,
                 generator_mode: str = 'random',
                 iterations: int = 20,
                 alphabet: str = 'OOK',
                 channel_profile: str = 'exponential',
                 channel_truncation: bool = 'trunc',
                 is_complex: bool = True,
                 device: str = 'cuda') -> None:
        # same argument checks and messages as config.py:40-44
        assert channel_profile in ['exponential', 'uniform', 'random'], \
            "channel_profile has to be 'exponential' or 'uniform'"
        assert channel_truncation in ['trunc', 'tail', 'cyclic'], \
            "channel_truncation has to be 'trunc', 'tail' or 'cyclic'"
        assert channel_length > 0, "channel_length needs to be at least 1"
        assert generator_mode in ['segmented', 'random', 'sparc'], \
            "generator_mode needs to be 'segmented' or 'random' or 'sparc'"
        assert alphabet in _ALPHABET_TABLE, \
            "alphabet has to be 'OOK','BPSK','4ASK','QPSK','8PSK','16PSK' or'16QAM'"

        self.device = device
        self.B, self.Lin = batch, block_length
        self.Nt, self.Na, self.Nr = N_transmit_antenna, N_active_antenna, N_receive_antenna
        self.sparsity = self.Na / self.Nt
        self.mode = generator_mode

        self.is_complex = is_complex
        self.Lh = channel_length
        self.profile = channel_profile
        self.trunc = channel_truncation
        self.Lout = self.Lin + self.Lh - 1 if channel_truncation == 'tail' else self.Lin
        self.ISI = self.Lh > 1

        self.Ns = self.B * self.Lin * self.Na
        self.N0 = self.B * self.Lin * (self.Nt - self.Na)
        self.alphabet = alphabet
        points, gray, ps_div, forces_complex = _ALPHABET_TABLE[alphabet]
        self.modulated = alphabet != 'OOK'
        self.Ps = self.sparsity / ps_div
        self.P0 = 1 - self.sparsity
        if forces_complex:
            self.is_complex = True
        # unit mean power (config.py:117); float64 for real alphabets, complex128 otherwise
        self.symbols = np.array(points) / np.sqrt(np.mean(np.abs(points) ** 2))
        self.gray = list(gray)
        self.K = len(self.symbols)
        self.symbol_bits = int(np.log2(self.K))

        if self.mode == 'random':
            self.index_bits = np.log2(np.prod([1 + (self.Nt - self.Na) / j for j in range(1, self.Na + 1)]))
            self.info_bits = self.symbol_bits + self.index_bits
            self.code_rate = self.Lin * self.info_bits / self.Nr / self.Lout
        elif self.mode == 'segmented':
            assert self.Nt % self.Na == 0, 'Na must divide Nt'
            self.index_bits = self.Na * np.log2(self.Nt / self.Na)
            self.info_bits = self.symbol_bits + self.index_bits
            self.code_rate = self.Lin * self.info_bits / self.Nr / self.Lout
        else:  # 'sparc'
            assert self.Nt % self.Na == 0, 'Na must divide Nt'
            self.M = self.Nt // self.Na
            self.Mc, self.Mr = self.Nt, self.Nr
            self.L = self.Na * self.Lin
            self.Lc, self.Lr = self.Lin, self.Lout
            self.n = self.Nr * self.Lout
            self.index_bits = self.Na * np.log2(self.M)
            self.inner_code_rate = self.Na * np.log2(self.M * self.K) / self.Mr
            self.code_rate = self.Lc * self.inner_code_rate / self.Lr

        self.N_Layers = iterations
        self.kappa = self.Lout / self.Lin
        with np.errstate(divide='ignore'):
            self.min_amp_snr = 1 / (self.kappa * (1 / (np.exp(2 * self.code_rate) - 1) - 1 / self.Lh))
        self.min_snr = 2 ** self.code_rate - 1
        self.min_snr_dB = 10 * np.log10(self.min_snr)
        self.shannon_limit_dB = self.min_snr_dB - 10 * np.log10(self.code_rate)
        self.name = (f'{self.alphabet},{self.mode}/{self.profile},{self.trunc}/'
                     f'Nt={self.Nt},Na={self.Na},Nr={self.Nr},Lh={self.Lh},Lin={self.Lin}')

    # ---- native-path helpers (not in the reference) ----
    def dims(self, batch: int | None = None):
        from amp_native import AmpDims
        d = AmpDims()
        d.B = self.B if batch is None else batch
        d.Nt, d.Na, d.Nr, d.Lin, d.Lout = self.Nt, self.Na, self.Nr, self.Lin, self.Lout
        d.N, d.n = self.Nt * self.Lin, self.Nr * self.Lout
        d.L, d.M = self.Na * self.Lin, self.Nt // self.Na
        return d

    def constellation(self):
        """The amp_constellation struct of the current alphabet (memoised on its contents, so
        an alphabet injected after construction is picked up)."""
        from amp_native import make_constellation
        key = (np.asarray(self.symbols).tobytes(), tuple(self.gray), self.symbol_bits)
        memo = getattr(self, '_const_memo', None)
        if memo is None or memo[0] != key:
            memo = (key, make_constellation(self.symbols, self.gray, self.symbol_bits))
            self._const_memo = memo
        return memo[1]

    def inject_square_qam(self, K: int = 64) -> 'Config':
        """Square K-QAM (unit mean power, per-axis binary-reflected gray code) in place of the
        constructed alphabet — BASELINE cfg5's 64-QAM, which the reference's Config rejects
        (config.py:44).  Same injection as tests/golden/make_goldens.py applies to the reference's
        Config: every attribute the constellation feeds is re-derived as
        config.py:117-157 would.  Call it before building Data / Loss / detectors."""
        m = int(round(np.sqrt(K)))
        if m * m != K or m & (m - 1):
            raise ValueError(f'square QAM needs K = 4^j, got {K}')
        b = int(np.log2(m))
        levels = np.arange(-(m - 1), m, 2)
        g1 = [i ^ (i >> 1) for i in range(m)]
        pts = [complex(levels[i], levels[q]) for i in range(m) for q in range(m)]
        self.symbols = np.array(pts) / np.sqrt(np.mean(np.abs(pts) ** 2))
        self.gray = [(g1[i] << b) | g1[q] for i in range(m) for q in range(m)]
        self.alphabet = f'{K}QAM'
        self.K = K
        self.symbol_bits = int(np.log2(K))
        self.Ps = self.sparsity / K
        self.is_complex = True
        if self.mode == 'sparc':
            self.inner_code_rate = self.Na * np.log2(self.M * self.K) / self.Mr
            self.code_rate = self.Lc * self.inner_code_rate / self.Lr
        else:
            self.info_bits = self.symbol_bits + self.index_bits
            self.code_rate = self.Lin * self.info_bits / self.Nr / self.Lout
        with np.errstate(divide='ignore'):
            self.min_amp_snr = 1 / (self.kappa * (1 / (np.exp(2 * self.code_rate) - 1) - 1 / self.Lh))
        self.min_snr = 2 ** self.code_rate - 1
        self.min_snr_dB = 10 * np.log10(self.min_snr)
        self.shannon_limit_dB = self.min_snr_dB - 10 * np.log10(self.code_rate)
        self.name = (f'{self.alphabet},{self.mode}/{self.profile},{self.trunc}/'
                     f'Nt={self.Nt},Na={self.Na},Nr={self.Nr},Lh={self.Lh},Lin={self.Lin}')
        return self

    def snr(self, EbN0dB: float) -> float:
        """Linear SNR of an EbN0 point as the drivers compute it (vamp_model.py:50-54)."""
        return 10 ** ((EbN0dB + 10 * np.log10(self.code_rate)) / 10)
