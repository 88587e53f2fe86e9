"""ORACLE (test infrastructure only) — numpy restatement of the reference
detector path of AhmedKishki/AMP-SPARC-SpatialModulation.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this file, and only as the checker: the
product (``amp-sparc-spatialmodulation_amd/``) never routes through it.

Every function cites the reference file:line it restates.  The restatement
keeps the reference's dtype flow, because parity depends on it:

* GEMMs in complex64 (the reference's torch c64 matmuls),
* batch scalars (sigma2, alpha, dxdr, ...) as float32 0-dim values, except in
  the first VAMP iteration where ``sigma2_tilde`` is a Python float
  (``vamp.py:26``),
* ``c64 / real`` as multiplication by the float32 reciprocal (measured: torch
  and numpy both divide complex by real this way),
* ``python_float / tensor`` as ``reciprocal(tensor) * python_float``
  (torch's ``Tensor.__rtruediv__``),
* the block-sparse denoiser in float64 with the batch-global ``max |xi|``
  shift, so the float64 underflow -> 0/0 -> NaN behaviour is reproduced
  (``vamp.py:111-112``),
* ``torch.allclose`` semantics evaluated in float32 for the early exit.

Pinning: ``tests/test_oracle_goldens.py`` checks this file against vectors
produced by running the reference itself (``tests/golden/make_goldens.py``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

F32 = np.float32
C64 = np.complex64

# vamp.py:51-54 — torch.tensor(...) makes these float32 0-dim tensors.
VAR_RATIO_MIN = F32(1.0e-5)
VAR_RATIO_MAX = F32(1.0) - F32(1.0e-5)
VAR_MIN = F32(1.0e-9)
VAR_MAX = F32(1.0e5)
# torch.allclose defaults (vamp.py:185, bamp.py:140, scamp.py:105)
ALLCLOSE_RTOL = F32(1.0e-5)
ALLCLOSE_ATOL = F32(1.0e-8)

# config.py:78-116 — constellation lists (16QAM keeps the reference's
# duplicate -1+3j / missing 1-3j) and gray labels.
_ALPHABETS = {
    'OOK': ([1], [1]),
    'BPSK': ([-1, 1], [0, 1]),
    '4ASK': ([-3, -1, 1, 3], [0, 1, 3, 2]),
    'QPSK': ([1 + 0j, 0 + 1j, -1 + 0j, 0 - 1j], [0, 1, 3, 2]),
    '8PSK': ([np.exp((2 * np.pi * 1j / 8) * n) for n in range(8)], [0, 1, 3, 2, 6, 7, 5, 4]),
    '16PSK': ([np.exp((2 * np.pi * 1j / 16) * n) for n in range(16)],
              [0, 1, 3, 2, 6, 7, 5, 4, 12, 13, 15, 14, 10, 11, 9, 8]),
    '16QAM': ([1 + 1j, 1 - 1j, -1 + 1j, -1 - 1j, 3 + 1j, 3 - 1j, -3 + 1j, -3 - 1j,
               3 + 3j, 3 - 3j, -3 + 3j, -3 - 3j, 1 + 3j, -1 + 3j, -1 + 3j, -1 - 3j],
              [0, 1, 13, 7, 8, 9, 2, 15, 12, 11, 5, 10, 14, 3, 6, 4]),
}
_PS_DIV = {'OOK': 1, 'BPSK': 2, '4ASK': 4, 'QPSK': 4, '8PSK': 8, '16PSK': 16, '16QAM': 16}


def constellation(alphabet: str):
    """config.py:78-118: unit-mean-power points (float64 or complex128) and gray labels."""
    pts, gray = _ALPHABETS[alphabet]
    sym = np.array(pts) / np.sqrt(np.mean(np.abs(pts) ** 2))
    return sym, list(gray)


@dataclass
class OracleConfig:
    """Restates the constants of ``Config`` (config.py:4-157) the path needs."""
    Nt: int
    Na: int
    Nr: int
    Lin: int = 1
    Lh: int = 1
    B: int = 100
    alphabet: str = 'QPSK'
    mode: str = 'sparc'
    trunc: str = 'tail'
    iterations: int = 20
    # derived
    Lout: int = field(init=False)
    symbols: np.ndarray = field(init=False)
    gray: list = field(init=False)

    def __post_init__(self):
        self.Lout = self.Lin + self.Lh - 1 if self.trunc == 'tail' else self.Lin   # config.py:60-63
        self.symbols, self.gray = constellation(self.alphabet)
        self.K = len(self.symbols)
        self.symbol_bits = int(np.log2(self.K))                                  # config.py:119
        self.sparsity = self.Na / self.Nt
        self.Ps = self.sparsity / _PS_DIV[self.alphabet]
        self.P0 = 1 - self.sparsity
        self.Ns = self.B * self.Lin * self.Na                                    # config.py:71
        self.M = self.Nt // self.Na
        self.L = self.Na * self.Lin
        self.N = self.Nt * self.Lin
        self.n = self.Nr * self.Lout
        if self.mode == 'random':                                                # config.py:121-124
            self.index_bits = np.log2(np.prod([1 + (self.Nt - self.Na) / j for j in range(1, self.Na + 1)]))
            self.code_rate = self.Lin * (self.symbol_bits + self.index_bits) / self.Nr / self.Lout
        elif self.mode == 'segmented':                                           # config.py:126-130
            self.index_bits = self.Na * np.log2(self.Nt / self.Na)
            self.code_rate = self.Lin * (self.symbol_bits + self.index_bits) / self.Nr / self.Lout
        else:                                                                    # config.py:132-144
            self.index_bits = self.Na * np.log2(self.M)
            self.code_rate = self.Lin * (self.Na * np.log2(self.M * self.K) / self.Nr) / self.Lout
        self.N_Layers = self.iterations
        self.min_snr_dB = 10 * np.log10(2 ** self.code_rate - 1)                 # config.py:152-154
        self.shannon_limit_dB = self.min_snr_dB - 10 * np.log10(self.code_rate)
        self._ibits = int(np.ceil(np.log2(self.Lin * self.B * self.Na)))         # loss.py:20

    def snr(self, EbN0dB: float) -> float:
        """vamp_model.py:50-54: SNR (linear) of an EbN0 point."""
        return 10 ** ((EbN0dB + 10 * np.log10(self.code_rate)) / 10)


# ----------------------------------------------------------------------------
# small helpers with torch semantics
# ----------------------------------------------------------------------------
def _clamp(v, lo, hi):
    """torch.max(v, lo) then torch.min(v, hi): NaN-propagating (vamp.py:76-77)."""
    return np.minimum(np.maximum(v, lo), hi)


def _recip(v):
    """torch.reciprocal / ``1 / tensor`` in float32."""
    return F32(1.0) / F32(v) if np.ndim(v) == 0 else (F32(1.0) / v.astype(F32))


def allclose_f32(nxt: np.ndarray, prev: np.ndarray) -> bool:
    """torch.allclose(nxt, prev) (rtol 1e-5, atol 1e-8) evaluated in float32."""
    nxt = nxt.astype(F32, copy=False)
    prev = prev.astype(F32, copy=False)
    with np.errstate(invalid='ignore', over='ignore'):
        actual = np.abs(nxt - prev)
        allowed = ALLCLOSE_ATOL + np.abs(ALLCLOSE_RTOL * prev)
        close = (nxt == prev) | (np.isfinite(actual) & (actual <= allowed))
    return bool(np.all(close))


def _torch_abs(z: np.ndarray) -> np.ndarray:
    """torch.abs of complex64 on CPU = correctly rounded hypot (measured)."""
    return np.sqrt(z.real.astype(np.float64) ** 2 + z.imag.astype(np.float64) ** 2).astype(F32)


def _div_real(z: np.ndarray, d) -> np.ndarray:
    """complex64 / float32 as the reference computes it: z * (1/d)."""
    return (z * _recip(d)).astype(C64, copy=False)


# ----------------------------------------------------------------------------
# block-sparse denoisers
# ----------------------------------------------------------------------------
def _logits(r: np.ndarray, tau, cfg: OracleConfig, B: int) -> np.ndarray:
    """xi[b,l,m,k] = Re((r/tau) * conj(a_k)) in float64 (vamp.py:111, bamp.py:69, scamp.py:64)."""
    s = r.reshape(B, cfg.L, cfg.M)
    if np.ndim(tau) == 0:
        u = _div_real(s, tau)
    else:
        u = _div_real(s, tau.reshape(B, cfg.L, cfg.M))
    sym = cfg.symbols.astype(np.complex128)
    return (u.astype(np.complex128)[..., None] * np.conj(sym)[None, None, None, :]).real


def block_denoise(r: np.ndarray, tau, cfg: OracleConfig, G=None):
    """Posterior mean and variance of the section-sparse prior.

    VAMP ``segmented_denoiser`` (vamp.py:96-119): ``tau`` is the 0-dim sigma2.
    BAMP ``segmented_denoiser`` (bamp.py:66-77): pass ``tau = cov/2`` (per element).
    Float64 with the batch-global ``max |xi|`` shift (vamp.py:112); ``G`` overrides the shift
    (a trial-sharded batch: the max over every rank's slice).
    Returns (xmmse complex64 [B,N], var float32 [B,N]).
    """
    B = r.shape[0]
    # keep the symbols' dtype: float64 for OOK/BPSK/4ASK (real division by Z), complex128
    # otherwise (c128 / f64 = multiply by 1/Z, which overflows once Z is denormal)
    sym = cfg.symbols
    xi = _logits(r, tau, cfg, B)
    with np.errstate(under='ignore', invalid='ignore', divide='ignore', over='ignore'):
        eta = np.exp(xi - (np.abs(xi).max() if G is None else G))
        zm = eta.sum(axis=-1)                          # [B,L,M]
        z = zm.sum(axis=2, keepdims=True)              # [B,L,1]
        xm = (sym * eta).sum(axis=-1) / z              # vamp.py:114
        var0 = np.abs(xm) ** 2 * (1 - zm / z)          # vamp.py:116
        vars_ = (np.abs(xm[..., None] - sym[None, None, None, :]) ** 2 * eta).sum(axis=-1) / z   # vamp.py:117
        var = var0 + vars_
    return xm.astype(C64).reshape(B, -1), var.astype(F32).reshape(B, -1)


def scamp_denoise(r: np.ndarray, tau_half: np.ndarray, cfg: OracleConfig) -> np.ndarray:
    """SCAMPLayer.denoiser (scamp.py:61-68): posterior mean only, tau = tau_use/2."""
    B = r.shape[0]
    sym = cfg.symbols
    xi = _logits(r, tau_half, cfg, B)
    with np.errstate(under='ignore', invalid='ignore', divide='ignore', over='ignore'):
        eta = np.exp(xi - np.abs(xi).max())
        xm = (sym * eta).sum(axis=-1) / eta.sum(axis=-1).sum(axis=2, keepdims=True)
    return xm.astype(C64).reshape(B, -1)


# ----------------------------------------------------------------------------
# detectors
# ----------------------------------------------------------------------------
def vamp_detect(U, s, Vh, y, SNR: float, cfg: OracleConfig, trace: list | None = None, mm=None, mm_y=None):
    """VAMP (SVD form): Tracker (vamp.py:12-28), VAMPLayer.forward (vamp.py:56-94),
    VAMP.forward loop + early exit (vamp.py:159-187).

    U [n,k] c64, s [k] f32, Vh [k,N] c64, y [B,n] c64.
    Returns dict(r, xmmse, var, T) where ``r`` is the decision input (vamp.py:187).
    mm / mm_y: the c64 matrix product of the two per-iteration GEMMs (vamp.py:67, 72) / of y~
    (vamp.py:22), default numpy's (BLAS); diagnostics pass other summation orders
    (tools/gemm_order_probe.py).
    """
    mm = mm or (lambda a, b: a @ b)
    mm_y = mm_y or (lambda a, b: a @ b)                          # the y~ product (vamp.py:22)
    U = np.asarray(U, C64); Vh = np.asarray(Vh, C64); y = np.asarray(y, C64)
    s = np.asarray(s, F32)
    B = y.shape[0]
    E = cfg.Na / cfg.Nr                                           # vamp.py:154
    p = cfg.Na / cfg.Nt                                           # vamp.py:155
    noise_var = E / SNR                                           # vamp.py:179 (Python float)
    Uh = np.conj(U).T
    Vt = np.conj(Vh)                                              # x @ V.T with V = Vh^H
    s2 = (s * s).astype(F32)
    ytil = mm_y(y, ((s[:, None] * Uh).astype(C64)).T).astype(C64)  # vamp.py:22
    r = np.zeros((B, Vh.shape[1]), C64)
    var = np.ones((B, Vh.shape[1]), F32)
    rt = np.full((B, Vh.shape[1]), F32(p), dtype=C64)
    s2t = p ** 2 * (1 - p) + (1 - p) ** 2 * p                     # vamp.py:26 (Python float)
    eta = s.shape[0] / Vh.shape[1]                                # vamp.py:28
    xm = None
    t = 0
    for t in range(cfg.N_Layers):
        prev = var
        first = isinstance(s2t, float)
        # vamp.py:66 — python/python at t=0, else reciprocal(tensor)*python
        vr = F32(noise_var / s2t) if first else F32(_recip(s2t) * F32(noise_var))
        q = mm(rt, Vh.T).astype(C64)                              # vamp.py:67
        scale = _recip(s2 + vr)                                   # vamp.py:68
        xt = (scale * (ytil + vr * q)).astype(C64)                # vamp.py:70
        varL = F32(F32(np.sum(scale, dtype=np.float64) / scale.size) * F32(noise_var))   # vamp.py:71
        xt = (mm((xt - q).astype(C64), Vt) + rt).astype(C64)      # vamp.py:72
        if first:                                                 # vamp.py:73
            xtv = F32(F32(eta) * varL + F32((1 - eta) * s2t))
            alpha = F32(xtv / F32(s2t))                           # vamp.py:75
            s2t32 = F32(s2t)
        else:
            xtv = F32(F32(eta) * varL + F32(F32(1 - eta) * s2t))
            alpha = F32(xtv / s2t)
            s2t32 = s2t
        alpha = _clamp(alpha, VAR_RATIO_MIN, VAR_RATIO_MAX)       # vamp.py:76-77
        r = _div_real(xt - alpha * rt, F32(1) - alpha)            # vamp.py:79
        sigma2 = F32(F32(alpha / (F32(1) - alpha)) * s2t32)       # vamp.py:80
        sigma2 = _clamp(sigma2, VAR_MIN, VAR_MAX)                 # vamp.py:81-82
        xm, var = block_denoise(r, sigma2, cfg)                  # vamp.py:84
        mean_var = F32(np.sum(var, dtype=np.float64) / var.size)
        dxdr = _clamp(F32(mean_var / sigma2), VAR_RATIO_MIN, VAR_RATIO_MAX)   # vamp.py:85-87
        ns = _recip(F32(1) - dxdr)                                # vamp.py:89
        rt = ((xm - dxdr * r) * ns).astype(C64)                   # vamp.py:91
        s2t = _clamp(F32(F32(sigma2 * dxdr) * ns), VAR_MIN, VAR_MAX)          # vamp.py:92-94
        if trace is not None:
            trace.append(dict(r=r.copy(), xmmse=xm.copy(), var=var.copy(), alpha=alpha,
                              sigma2=sigma2, dxdr=dxdr, sigma2_tilde=s2t, r_tilde=rt.copy()))
        if allclose_f32(var, prev):                               # vamp.py:185
            break
    return dict(r=r, xmmse=xm, var=var, T=t + 1)


def vamp_detect_sharded(U, s, Vh, y_local, SNR: float, cfg: OracleConfig, B_global: int, allreduce):
    """vamp_detect on ONE rank's slice of a trial-sharded batch (SURVEY §8(e) exact-compat
    mode; the build's amp_vamp_run_sharded): the batch-global values of vamp.py:85
    (var.mean()), vamp.py:112 (max |xi|) and vamp.py:185 (allclose) come from
    ``allreduce(np.float64 array, 'sum' | 'max')`` over the ranks, so every rank follows the
    whole-batch trajectory (up to the float64 summation order of the mean).  A NaN max |xi| is
    sent as +inf: exp(xi - inf) makes every section 0/0 = NaN, as the NaN shift does."""
    U = np.asarray(U, C64); Vh = np.asarray(Vh, C64); y = np.asarray(y_local, C64)
    s = np.asarray(s, F32)
    B = y.shape[0]
    E = cfg.Na / cfg.Nr
    p = cfg.Na / cfg.Nt
    noise_var = E / SNR
    Uh = np.conj(U).T
    Vt = np.conj(Vh)
    s2 = (s * s).astype(F32)
    ytil = (y @ ((s[:, None] * Uh).astype(C64)).T).astype(C64)
    N = Vh.shape[1]
    r = np.zeros((B, N), C64)
    var = np.ones((B, N), F32)
    rt = np.full((B, N), F32(p), dtype=C64)
    s2t = p ** 2 * (1 - p) + (1 - p) ** 2 * p
    eta = s.shape[0] / N
    xm = None
    t = 0
    for t in range(cfg.N_Layers):
        prev = var
        first = isinstance(s2t, float)
        vr = F32(noise_var / s2t) if first else F32(_recip(s2t) * F32(noise_var))
        q = (rt @ Vh.T).astype(C64)
        scale = _recip(s2 + vr)
        xt = (scale * (ytil + vr * q)).astype(C64)
        varL = F32(F32(np.sum(scale, dtype=np.float64) / scale.size) * F32(noise_var))
        xt = ((xt - q) @ Vt + rt).astype(C64)
        if first:
            xtv = F32(F32(eta) * varL + F32((1 - eta) * s2t))
            alpha = F32(xtv / F32(s2t))
            s2t32 = F32(s2t)
        else:
            xtv = F32(F32(eta) * varL + F32(F32(1 - eta) * s2t))
            alpha = F32(xtv / s2t)
            s2t32 = s2t
        alpha = _clamp(alpha, VAR_RATIO_MIN, VAR_RATIO_MAX)
        r = _div_real(xt - alpha * rt, F32(1) - alpha)
        sigma2 = _clamp(F32(F32(alpha / (F32(1) - alpha)) * s2t32), VAR_MIN, VAR_MAX)
        with np.errstate(invalid='ignore'):
            g = np.abs(_logits(r, sigma2, cfg, B)).max()
        g = np.float64(np.inf) if not np.isfinite(g) else g
        G = allreduce(np.array([g]), 'max')[0]
        xm, var = block_denoise(r, sigma2, cfg, G=G)
        # torch.allclose over the whole batch (vamp.py:185): the count of not-close elements
        with np.errstate(invalid='ignore', over='ignore'):
            nxt, prv = var.astype(F32), prev.astype(F32)
            actual = np.abs(nxt - prv)
            close = (nxt == prv) | (np.isfinite(actual) & (actual <= ALLCLOSE_ATOL + np.abs(ALLCLOSE_RTOL * prv)))
        tot = allreduce(np.array([np.sum(var, dtype=np.float64), float(np.sum(~close))]), 'sum')
        mean_var = F32(tot[0] / (B_global * N))
        dxdr = _clamp(F32(mean_var / sigma2), VAR_RATIO_MIN, VAR_RATIO_MAX)
        ns = _recip(F32(1) - dxdr)
        rt = ((xm - dxdr * r) * ns).astype(C64)
        s2t = _clamp(F32(F32(sigma2 * dxdr) * ns), VAR_MIN, VAR_MAX)
        if tot[1] == 0:
            break
    return dict(r=r, xmmse=xm, var=var, T=t + 1)


# vamp2.py:48-49 — torch.tensor(...) float32 0-dim clamps of the damped VAMP
V2_VAR_MIN = F32(1.0e-11)
V2_VAR_MAX = F32(1.0e11)


def vamp2_denoise(r: np.ndarray, tau, cfg: OracleConfig):
    """vamp2 ``VAMPLayer.segmented_denoiser`` (vamp2.py:79-88): the same float64 logits and
    batch-global shift as vamp.py, variance as E|a|^2 - |xmmse|^2 (vamp2.py:85-87)."""
    B = r.shape[0]
    sym = cfg.symbols
    xi = _logits(r, tau, cfg, B)
    with np.errstate(under='ignore', invalid='ignore', divide='ignore', over='ignore'):
        eta = np.exp(xi - np.abs(xi).max())                                    # vamp2.py:83
        z = eta.sum(axis=-1).sum(axis=2, keepdims=True)
        xm = (sym * eta).sum(axis=-1) / z                                      # vamp2.py:86
        var = (np.abs(sym) ** 2 * eta).sum(axis=-1) / z - np.abs(xm) ** 2       # vamp2.py:85, 87
    return xm.astype(C64).reshape(B, -1), var.astype(F32).reshape(B, -1)


def vamp2_detect(U, s, Vh, y, SNR: float, cfg: OracleConfig, damping: float = 1.0,
                 trace: list | None = None):
    """Damped "Rangan" VAMP: Tracker (vamp2.py:12-26), VAMPLayer.forward (vamp2.py:52-77),
    VAMP.forward loop + early exit on var (vamp2.py:123-131).

    U [n,k] c64, s [k] f32, Vh [k,N] c64, y [B,n] c64.  Returns dict(r, xmmse, var, T).
    """
    U = np.asarray(U, C64); Vh = np.asarray(Vh, C64); y = np.asarray(y, C64)
    s = np.asarray(s, F32)
    B, N = y.shape[0], Vh.shape[1]
    sigma2 = cfg.Na / cfg.Nr / SNR                                # vamp2.py:98, 123 (Python float)
    Uh = np.conj(U).T
    s2 = (s * s).astype(F32)                                      # vamp2.py:17
    ytil = _div_real((y @ Uh.T).astype(C64), s[None, :])          # vamp2.py:22
    eta = Vh.shape[1] / s.shape[0]                                # vamp2.py:26
    Vt_eta = (F32(eta) * np.conj(Vh)).astype(C64)                 # (eta * V)^T, V = Vh^H: vamp2.py:77
    rho = F32(damping)
    gamma = F32(1.0)                                              # vamp2.py:21
    r = np.zeros((B, N), C64)
    var = np.ones((B, N), F32)
    xm_state = np.zeros((B, N), C64)
    t = 0
    with np.errstate(invalid='ignore', over='ignore', divide='ignore'):
        for t in range(cfg.N_Layers):
            prev = var
            xm, var = vamp2_denoise(r, gamma, cfg)                                # vamp2.py:62
            xm_state = (rho * xm + F32(1 - damping) * xm_state).astype(C64)       # vamp2.py:63
            alpha = F32(F32(np.sum(var, dtype=np.float64) / var.size) * gamma)    # vamp2.py:64
            rt = _div_real(xm_state - alpha * r, F32(1) - alpha)                  # vamp2.py:66
            gt = F32(F32(gamma * F32(F32(1) - alpha)) / alpha)                    # vamp2.py:67
            gt = _clamp(gt, V2_VAR_MIN, V2_VAR_MAX)                               # vamp2.py:68-69
            d = (s2 / (s2 + F32(F32(sigma2) * gt))).astype(F32)                   # vamp2.py:71
            dm = F32(np.sum(d, dtype=np.float64) / d.size)
            g = F32(F32(gt * dm) / F32(F32(eta) - dm))                            # vamp2.py:72
            gamma = F32(rho * g + F32(1 - damping) * gamma)                       # vamp2.py:73
            z = ((d / dm).astype(F32) * (ytil - (rt @ Vh.T).astype(C64))).astype(C64)
            r = (rt + (z @ Vt_eta).astype(C64)).astype(C64)                       # vamp2.py:77
            if trace is not None:
                trace.append(dict(r=r.copy(), xmmse=xm_state.copy(), var=var.copy(), gamma=gamma,
                                  alpha=alpha, r_tilde=rt.copy()))
            if allclose_f32(var, prev):                                           # vamp2.py:129
                break
    return dict(r=r, xmmse=xm_state, var=var, T=t + 1)


def bamp_random_denoise(r, cov, cfg: OracleConfig):
    """BAMPLayer.random_denoiser (bamp.py:79-88): element-wise Bayes posterior under the P0/Ps
    prior.  G(0) in float32 (r - 0 stays complex64); G(a_k) in float64 (complex64 - complex128:
    torch.tensor(config.symbols) keeps numpy's complex128, bamp.py:37); float32 prior scalars
    promoted to float64; complex128 / float64 as a reciprocal multiply."""
    r = np.asarray(r, C64)
    cov = np.asarray(cov, F32)
    sym = cfg.symbols.astype(np.complex128)
    P0, Ps = F32(cfg.P0), F32(cfg.Ps)
    with np.errstate(all='ignore'):
        G0 = np.exp(-(_torch_abs(r) ** 2) / cov).astype(F32)
        Gs = np.exp(-(np.abs(r.astype(np.complex128)[..., None] - sym) ** 2) / cov[..., None].astype(np.float64))
        norm = (P0 * G0).astype(np.float64) + np.float64(Ps) * Gs.sum(axis=-1)
        norm[norm == 0.] = 1e-9
        ex = (np.float64(Ps) * (sym * Gs).sum(axis=-1)) * (1.0 / norm)
        var = np.float64(Ps) * ((np.abs(sym) ** 2) * Gs).sum(axis=-1) / norm - np.abs(ex) ** 2
    return ex.astype(C64), var.astype(F32)


def bamp_detect(H, y, SNR: float, cfg: OracleConfig, trace: list | None = None):
    """BAMP: Tracker (bamp.py:12-25), BAMPLayer.forward (bamp.py:48-64),
    denoiser with tau = cov/2 (bamp.py:66-77), BAMP.forward (bamp.py:116-143).
    H [n,N] c64, y [B,n] c64. Returns dict(xmap, xmmse, var, T)."""
    H = np.asarray(H, C64); y = np.asarray(y, C64)
    B = y.shape[0]
    N = H.shape[1]
    sigma2 = (cfg.Na / cfg.Nr) / SNR                              # bamp.py:124 (Python float)
    Hc = np.conj(H)
    abs2 = (_torch_abs(H) ** 2).astype(F32)                        # bamp.py:18
    xm = np.zeros((B, N), C64)
    var = np.ones((B, N), F32)
    z = y.copy()
    u = None                                                      # bamp.py:25: c64 (sigma2 + 0j) at t=0
    xmap = None
    t = 0
    for t in range(cfg.N_Layers):
        prev = var
        v = (var @ abs2.T).astype(F32)                            # bamp.py:59
        res = (y - z).astype(C64)
        ud = F32(sigma2) if u is None else u
        z = (xm @ H.T - _div_real((v * res).astype(C64), ud)).astype(C64)     # bamp.py:60
        u = (v + F32(sigma2)).astype(F32)                         # bamp.py:61
        cov = _recip(((_recip(u)) @ abs2).astype(F32))            # bamp.py:62
        g = (_div_real((y - z).astype(C64), u) @ Hc).astype(C64)  # bamp.py:63
        xmap = (xm + cov * g).astype(C64)
        if cfg.mode == 'random':                                  # bamp.py:38-41
            xm, var = bamp_random_denoise(xmap, cov, cfg)
        else:
            tau = (cov / F32(2)).astype(F32)                      # bamp.py:68
            xm, var = block_denoise(xmap, tau, cfg)               # bamp.py:64
        if trace is not None:
            trace.append(dict(xmap=xmap.copy(), xmmse=xm.copy(), var=var.copy(), z=z.copy(), u=u.copy()))
        if allclose_f32(var, prev):                               # bamp.py:140
            break
    return dict(xmap=xmap, xmmse=xm, var=var, T=t + 1)


def scamp_detect(W, A, y, SNR: float, cfg: OracleConfig, trace: list | None = None):
    """SCAMP: Tracker (scamp.py:8-25), SCAMPLayer.forward (scamp.py:43-59),
    denoiser (scamp.py:61-68), SCAMP.forward (scamp.py:77-107).
    W [Lout,Lin] f32, A [n,N] c64, y [B,n] c64. Returns dict(xmap, xmmse, psi, T)."""
    W = np.asarray(W, F32); A = np.asarray(A, C64); y = np.asarray(y, C64)
    B = y.shape[0]
    Lout, Lin = W.shape
    N = A.shape[1]
    Mr, Mc, Lc, L = cfg.Nr, cfg.Nt, cfg.Lin, cfg.Na * cfg.Lin
    sigma2 = (cfg.Na / cfg.Nr) / SNR                              # scamp.py:98
    Ac = np.conj(A)
    z = y.copy()
    psi = np.ones((B, Lin), F32)
    phi = np.full((B, Lout), np.inf, F32)
    xm = np.zeros((B, N), C64)
    xmap = None
    t = 0
    for t in range(cfg.N_Layers):
        psi_prev = psi
        gma = ((psi @ W.T).astype(F32) / F32(Lc)).astype(F32)     # scamp.py:45
        b = (gma / phi).astype(F32)                               # scamp.py:47
        z = (y - (xm @ A.T).astype(C64) + np.repeat(b, Mr, axis=1) * z).astype(C64)   # scamp.py:49
        phi = (F32(sigma2) + gma).astype(F32)                     # scamp.py:51
        tau = ((_recip((_recip(phi) @ W).astype(F32)) * F32(L)) / F32(Mr)).astype(F32)   # scamp.py:53
        tau_use = np.repeat(tau, Mc, axis=1)                      # scamp.py:54
        phi_use = np.repeat(phi, Mr, axis=1)                      # scamp.py:55
        g = (_div_real(z, phi_use) @ Ac).astype(C64)
        xmap = (xm + tau_use * g).astype(C64)                     # scamp.py:57
        xm = scamp_denoise(xmap, (tau_use / F32(2)).astype(F32), cfg)   # scamp.py:58
        psi = (F32(1) - (_torch_abs(xm) ** 2).reshape(B, Lc, Mc).sum(axis=-1) / F32(cfg.Na)).astype(F32)  # scamp.py:59
        if trace is not None:
            trace.append(dict(xmap=xmap.copy(), xmmse=xm.copy(), psi=psi.copy(), z=z.copy()))
        if allclose_f32(psi, psi_prev):                           # scamp.py:105
            break
    return dict(xmap=xmap, xmmse=xm, psi=psi, T=t + 1)


# ----------------------------------------------------------------------------
# decision + metrics (Loss)
# ----------------------------------------------------------------------------
def map_decision(xmap: np.ndarray, cfg: OracleConfig):
    """Loss.MAP_decision (loss.py:282-302), vectorised over sections.

    Per section: argmax over the flattened (M, K) grid of Re(x_m * conj(a_k)),
    computed with numpy's complex multiply (same ufunc loop as np.outer);
    first index wins on ties, an all-NaN row gives index 0.
    Returns (xhat c64 [S*M], gray labels [S], flat indices [S]).
    """
    xa = np.asarray(xmap).reshape(-1, cfg.M)
    sym = cfg.symbols.astype(np.complex128)
    tmp = (xa.astype(np.complex128)[:, :, None] * np.conj(sym)[None, None, :]).real
    flat = tmp.reshape(xa.shape[0], -1).argmax(axis=1)
    m_hat, k_hat = np.divmod(flat, cfg.K)
    xhat = np.zeros_like(xa)
    rows = np.arange(xa.shape[0])
    xhat[rows, m_hat] = sym[k_hat]
    gray = np.asarray(cfg.gray)[k_hat]
    index = rows * cfg.M + m_hat
    return xhat.ravel(), gray, index


def segmented_decision(xmap: np.ndarray, cfg: OracleConfig):
    """Loss.segmented_decision (loss.py:222-250): per section of M, the position of the largest
    |x| (np.argsort()[-1] on float32 magnitudes: NaN sorts last), then the nearest constellation point (float64 |x - a_k|, first minimum).
    Returns (xhat c64 [S*M], gray labels, flat indices) like map_decision."""
    xa = np.asarray(xmap).reshape(-1, cfg.M)
    sym = cfg.symbols.astype(np.complex128)
    S = xa.shape[0]
    mag = np.abs(xa.astype(np.complex64))
    # numpy's own argsort, as loss.py:236: among exactly equal magnitudes its (SIMD quicksort)
    # order is implementation-defined, so the oracle defers to it rather than restating it
    m_hat = np.array([row.argsort()[-1] for row in mag], dtype=np.int64)
    xs = xa[np.arange(S), m_hat].astype(np.complex128)
    k_hat = np.abs(xs[:, None] - sym[None, :]).argmin(axis=1)
    xhat = np.zeros_like(xa)
    xhat[np.arange(S), m_hat] = sym[k_hat]
    return xhat.ravel(), np.asarray(cfg.gray)[k_hat], np.arange(S) * cfg.M + m_hat


def random_decision(xmap: np.ndarray, cfg: OracleConfig):
    """Loss.random_decision (loss.py:252-280): per channel use (row of Nt) the Na largest |x|
    (numpy's own argsort()[-Na:], as the reference), each decided to its nearest point (float64,
    first minimum); returns (xhat c64 [R*Nt], gray labels and flat indices in ascending order)."""
    xa = np.asarray(xmap).reshape(-1, cfg.Nt)
    sym = cfg.symbols.astype(np.complex128)
    xhat = np.zeros_like(xa)
    xgray = np.zeros(xa.shape, dtype=int)
    for j, x in enumerate(xa):
        for k in np.abs(x).argsort()[-cfg.Na:]:
            i = int(np.abs(x[k].astype(np.complex128) - sym).argmin())
            xhat[j, k] = sym[i]
            xgray[j, k] = cfg.gray[i]
    xhat = xhat.ravel()
    index = np.sort(xhat.nonzero()[0])
    return xhat, xgray.ravel()[index], index


def _de2bi_count(v: np.ndarray, bits: int) -> int:
    """count_nonzero(de2bi(v, bits)) (loss.py:181-196): set bits among the low `bits` bits."""
    v = v.astype(np.int64) & ((1 << bits) - 1)
    return int(sum(int(np.count_nonzero((v >> i) & 1)) for i in range(bits)))


def error_rates(xmap, xmmse, x, symbols, indices, cfg: OracleConfig):
    """Loss.error_rate (loss.py:67-103) with the sub-metrics of loss.py:105-179.
    Returns the 14 values in Loss.keys order (loss.py:27)."""
    B, Lin, Nt, Na = cfg.B, cfg.Lin, cfg.Nt, cfg.Na
    xmap = np.asarray(xmap).reshape(-1, Lin, Nt)
    xmmse = np.asarray(xmmse).reshape(-1, Lin, Nt)
    x = np.asarray(x).reshape(-1, Lin, Nt)
    decide = {'segmented': segmented_decision, 'random': random_decision}.get(cfg.mode, map_decision)   # loss.py:38-43
    xhat, shat, ihat = decide(xmap, cfg)
    xhat = xhat.reshape((-1, Lin, Nt))
    # loss.py:116-119
    nMSE = np.sum(np.abs(xmmse - x) ** 2) / cfg.Ns
    nMSEf = np.sum(np.abs(xmmse[:, 0] - x[:, 0]) ** 2) / Na / B
    nMSEm = np.sum(np.abs(xmmse[:, Lin // 2] - x[:, Lin // 2]) ** 2) / Na / B
    nMSEL = np.sum(np.abs(xmmse[:, -1] - x[:, -1]) ** 2) / Na / B
    # loss.py:133-136
    ver = (np.count_nonzero(xhat.reshape((-1, Nt)) - x.reshape((-1, Nt)), axis=-1) > 0).sum() / Lin / B
    verf = (np.count_nonzero(xhat[:, 0] - x[:, 0], axis=-1) > 0).sum() / B
    verm = (np.count_nonzero(xhat[:, Lin // 2] - x[:, Lin // 2], axis=-1) > 0).sum() / B
    verL = (np.count_nonzero(xhat[:, -1] - x[:, -1], axis=-1) > 0).sum() / B
    # loss.py:150
    fer = (np.count_nonzero(xhat.reshape(B, -1) - x.reshape(B, -1), axis=-1) > 0).sum() / B
    # loss.py:165-178
    symbols = np.asarray(symbols); indices = np.asarray(indices)
    ier = np.count_nonzero(ihat - indices) / cfg.Ns
    ser = np.count_nonzero(shat - symbols) / cfg.Ns
    iber_ = _de2bi_count(np.bitwise_xor(ihat, indices), cfg._ibits) / Lin / B
    iber = iber_ / cfg.index_bits
    if cfg.symbol_bits != 0:
        sber_ = _de2bi_count(np.bitwise_xor(shat, symbols), cfg.symbol_bits) / Lin / B
        sber = sber_ / cfg.symbol_bits / Na
    else:
        sber, sber_ = 0., 0.
    ber = (iber_ + sber_) / (Na * cfg.symbol_bits + cfg.index_bits)
    return fer, nMSE, nMSEf, nMSEm, nMSEL, ver, verf, verm, verL, ber, iber, sber, ier, ser


LOSS_KEYS = ['fer', 'nMSE', 'nMSEf', 'nMSEm', 'nMSEL', 'ver', 'verf', 'verm', 'verL',
             'ber', 'iber', 'sber', 'ier', 'ser']


def loss_dict(xmap, xmmse, x, symbols, indices, T: int, cfg: OracleConfig) -> dict:
    """Loss.__call__ after dump() (loss.py:43-65): {'T': T, key: value}."""
    out = {'T': T}
    for k, v in zip(LOSS_KEYS, error_rates(xmap, xmmse, x, symbols, indices, cfg)):
        out[k] = np.array(v)
    return out




# ---------------------------------------------------------------------------
# Shrink (shrink.py:8-166): element-wise prior-based denoisers.  float32 arithmetic in the
# reference's op order; regularize_exp (shrink.py:163-166) compares against
# float32(log(FLT_MAX)) and writes float32(log(FLT_MAX) - 1); regularize_zero (:159-161)
# replaces exact zeros by float32(1e-9).
SHR_REG_MAX = F32(np.log(np.finfo(np.float32).max))
SHR_REG_SET = F32(np.log(np.finfo(np.float32).max) - 1)
SHR_TOL = F32(1.0e-9)


def _shr_reg_exp(a):
    a = np.array(a, dtype=F32, copy=True)
    a[a >= SHR_REG_MAX] = SHR_REG_SET
    return a


def _shr_abs(z):
    """torch.abs: |z| of complex64 as float32 (correctly rounded hypot), |x| for float32."""
    if np.iscomplexobj(z):
        return np.hypot(z.real.astype(np.float64), z.imag.astype(np.float64)).astype(F32)
    return np.abs(z).astype(F32)


def shrink_bayes(r, cov, symbols, P0, Ps):
    """Shrink.bayes (shrink.py:91-96) on r [..] (complex64 or float32), cov scalar or like r.
    symbols: complex64 or float32 [K] (shrink.py:26); P0, Ps float32 (shrink.py:19)."""
    r = np.asarray(r)
    cov = np.asarray(cov, dtype=F32)
    sym = np.asarray(symbols)
    cplx = np.iscomplexobj(r) or np.iscomplexobj(sym)
    if cplx:
        r = r.astype(C64)
        sym = sym.astype(C64)
    else:
        r = r.astype(F32)
        sym = sym.astype(F32)
    with np.errstate(all='ignore'):
        covK = cov[..., None] if cov.ndim else cov
        G0 = np.exp(-(_shr_abs(r) ** 2) / cov).astype(F32)
        Gs = np.exp(-(_shr_abs(r[..., None] - sym) ** 2) / covK).astype(F32)   # [.., K]
        norm = (F32(P0) * G0 + F32(Ps) * Gs.sum(axis=-1, dtype=F32)).astype(F32)
        norm[norm == 0] = SHR_TOL
        num = F32(Ps) * (sym * Gs).sum(axis=-1)
        if cplx:
            return (num.astype(C64) * (F32(1) / norm)).astype(C64)
        return (num / norm).astype(F32)


def shrink_ook(r, cov, theta):
    """Shrink.shrinkOOK (shrink.py:152-157): (exp float32, dxdr float32 = der.mean())."""
    rr = np.real(np.asarray(r)).astype(F32)
    cov = np.asarray(cov, dtype=F32)
    with np.errstate(all='ignore'):
        eta = np.exp(_shr_reg_exp(F32(theta) + (F32(1) - F32(2) * rr) / cov)).astype(F32)
        x = (F32(1) / ((F32(1) + eta) + SHR_TOL)).astype(F32)
        der = ((F32(2) * eta) * (x * x) / cov).astype(F32)
    der = np.nan_to_num(der, nan=0.0)
    return x, F32(der.astype(np.float64).mean())


def shrink_sw_ook(r, cov, B, L, M):
    """Shrink.sw_shrinkOOK (shrink.py:68-76): leave-one-out OOK softmax per section of M.
    Returns (exp complex64 [B, L*M], var float32 [B, L*M])."""
    rr = np.real(np.asarray(r)).astype(F32)
    cov = np.broadcast_to(np.asarray(cov, dtype=F32), rr.shape)
    with np.errstate(all='ignore'):
        Lr = _shr_reg_exp(((F32(2) * rr - F32(1)) / cov).reshape(B, L, M))   # in place in the reference
        e = np.exp(Lr).astype(F32)
        S = e.sum(axis=-1, keepdims=True, dtype=F32)
        Le = (-np.log(S - e)).astype(F32)
        eta = np.exp(_shr_reg_exp(Lr + Le)).astype(F32)
        x = (eta / (F32(1) + eta)).astype(F32)
        var = (x * (F32(1) - x)).astype(F32)
    return x.reshape(B, L * M).astype(C64), var.reshape(B, L * M)


__all__ = ['OracleConfig', 'constellation', 'block_denoise', 'scamp_denoise', 'vamp_detect', 'vamp_detect_sharded', 'vamp2_detect',
           'vamp2_denoise',
           'bamp_detect', 'scamp_detect', 'map_decision', 'error_rates', 'loss_dict', 'allclose_f32',
           'LOSS_KEYS', 'VAR_RATIO_MIN', 'VAR_RATIO_MAX', 'VAR_MIN', 'VAR_MAX',
           'shrink_bayes', 'shrink_ook', 'shrink_sw_ook', 'segmented_decision',
           'random_decision', 'bamp_random_denoise']
