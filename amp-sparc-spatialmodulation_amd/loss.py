"""Decision + error metrics — drop-in for the reference's ``Loss`` (loss.py:8-349).

``__call__`` / ``error_rate`` run the MAP decision and every counter on the GPU
(``amp_map_decide_count``, include/amp_sparc.h) and copy back one small struct;
the reference copies the whole batch to the host and loops over sections in Python
(loss.py:85-88, 291-302).  The resulting dict has the reference's keys, order and
numpy dtypes, so ``accumulate`` / ``average`` / ``export`` behave the same.
"""
from __future__ import annotations

import ctypes as C
import json
import os

import numpy as np
import torch

import amp_native as nat
from config import Config

KEYS = ['fer', 'nMSE', 'nMSEf', 'nMSEm', 'nMSEL', 'ver', 'verf', 'verm', 'verL', 'ber', 'iber', 'sber', 'ier', 'ser']
# amp_counts (include/amp_sparc.h) fields in struct order
COUNT_FIELDS = ('ier', 'ser', 'iber', 'sber', 'ver', 'verf', 'verm', 'verL', 'fer', 'mse', 'msef', 'msem', 'mseL')


def counts_to_vector(c) -> np.ndarray:
    """amp_counts -> float64[13] (the integer counters are exact in float64 below 2^53), the
    payload of the one all-reduce that merges trial-sharded epochs."""
    return np.array([float(getattr(c, f)) for f in COUNT_FIELDS], dtype=np.float64)


def vector_to_counts(v):
    c = nat.AmpCounts()
    for i, f in enumerate(COUNT_FIELDS):
        setattr(c, f, int(round(float(v[i]))) if i < 9 else float(v[i]))
    return c


def allreduce_counts(vec: np.ndarray, group=None) -> np.ndarray:
    """Sum the per-rank counter vectors with ONE all-reduce (RCCL on the rank's GPU for the
    'nccl' backend, host memory for gloo) over `group` (default: the world); identity without
    torch.distributed."""
    dist = torch.distributed
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return np.asarray(vec, dtype=np.float64)
    dev = (torch.device('cuda', torch.cuda.current_device()) if dist.get_backend(group) == 'nccl'
           else torch.device('cpu'))
    t = torch.as_tensor(np.asarray(vec, dtype=np.float64)).to(dev)
    dist.all_reduce(t, group=group)
    return t.cpu().numpy()


def _as_device_labels(a, device) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        t = a.to(device=device, dtype=torch.int64)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int64))).to(device, non_blocking=True)
    return t.contiguous()


def _flat_c64(t: torch.Tensor, B: int, name: str) -> torch.Tensor:
    t = t.reshape(B, -1)
    if t.dtype != torch.complex64:
        t = t.to(torch.complex64)
    return t.resolve_conj().resolve_neg().contiguous()


class Loss:
    def __init__(self, config: Config) -> None:
        self.config = config
        self.B, self.Nt, self.Na, self.Nr, self.Lin = config.B, config.Nt, config.Na, config.Nr, config.Lin
        self.Ns, self.sparsity = config.Ns, config.sparsity
        self.gray = config.gray
        self.symbols = config.symbols
        self._ibits = int(np.ceil(np.log2(self.Lin * self.B * self.Na)))      # loss.py:20
        self.ibits = config.index_bits
        self.sbits = config.symbol_bits
        self.rate = config.code_rate
        self.shannon_limt_dB = config.shannon_limit_dB
        self._pending = None
        self.loss = {'T': 0}
        self.keys = list(KEYS)
        self.dtype = torch.complex64 if config.is_complex else torch.float32
        # loss.py:38-43: 'sparc' -> MAP_decision, 'segmented' -> segmented_decision,
        # 'random' -> random_decision (all three on the GPU)
        self.decision_mode = config.mode
        self._const = None
        self._dims = None

    # ------------------------------------------------------------------
    # The metrics dict.  A detector may leave its last forward's counters in flight on the
    # device (``_pending``: a callable that waits for them and records them here); the first
    # access resolves them, so callers see the reference's eager semantics.
    @property
    def loss(self) -> dict:
        if self._pending is not None:
            self.resolve()
        return self._loss

    @loss.setter
    def loss(self, value: dict) -> None:
        self._loss = value

    @property
    def arithmetic(self):
        """The GEMM arithmetic of the last forward recorded here, as the engine reported it
        (amp_status.gemm: 'bf16x3', 'f32', 'fp16x2' or 'int8x4'; None before any forward)."""
        if self._pending is not None:
            self.resolve()
        st = getattr(self, 'last_status', None)
        if st is None:
            return None
        from amp_native import ARITH_NAMES
        return ARITH_NAMES.get(int(st.gemm))

    def resolve(self) -> None:
        """Wait for and record the counters of the forward still in flight (if any)."""
        p, self._pending = self._pending, None
        if p is not None:
            p()

    def _native(self):
        if self._const is None:
            self._const = self.config.constellation()
            self._dims = self.config.dims()
        return self._dims, self._const

    def device_counts(self, xmap, xmmse, x, symbols, indices, decisions: torch.Tensor | None = None,
                      out: torch.Tensor | None = None, rule: str | None = None):
        """Launch the decision/count kernels; returns the device amp_counts buffer (async).
        ``out``: optional uint8 device buffer (>= sizeof(amp_counts)) to write the counters to."""
        rule = rule or self.decision_mode
        if rule not in ('sparc', 'segmented', 'random'):
            raise ValueError(f'unknown decision rule {rule!r}')
        d, c = self._native()
        dev = xmap.device
        B = self.B
        L = self.Na * self.Lin
        M = self.Nt // self.Na
        if rule == 'segmented' and B != 1:
            # loss.py:232 reshapes the whole batch to (Na*Lin, M): numpy raises for B > 1
            raise ValueError(f'cannot reshape array of size {B * L * M} into shape ({L},{M})')
        if rule == 'random' and B != 1:
            # loss.py:262 reshapes the whole batch to (Lin, Nt)
            raise ValueError(f'cannot reshape array of size {B * self.Lin * self.Nt} into shape ({self.Lin},{self.Nt})')
        xmap = _flat_c64(xmap, B, 'xmap')
        xmmse = _flat_c64(xmmse, B, 'xmmse')
        x = _flat_c64(x, B, 'x')
        sym = _as_device_labels(symbols, dev)
        idx = _as_device_labels(indices, dev)
        S = B * L
        if sym.numel() != S or idx.numel() != S:
            raise ValueError(f'expected {S} labels/indices, got {sym.numel()}/{idx.numel()}')
        lib = nat.lib()
        wsb = lib.amp_map_decide_workspace_bytes(C.byref(d))
        ws = nat.WORKSPACE.get(dev, 'decide', wsb)
        counts = out if out is not None else nat.WORKSPACE.get(dev, 'counts', C.sizeof(nat.AmpCounts))
        dec_ptr = nat.dptr(decisions, torch.int32, 'decisions') if decisions is not None else None
        fn = {'sparc': lib.amp_map_decide_count, 'segmented': lib.amp_segmented_decide_count,
              'random': lib.amp_random_decide_count}[rule]
        nat.check(fn(C.byref(d), C.byref(c), nat.dptr(xmap, name='xmap'), nat.dptr(xmmse, name='xmmse'),
                     nat.dptr(x, name='x'), nat.dptr(sym, name='symbols'), nat.dptr(idx, name='indices'),
                     self._ibits, nat.dptr(counts), dec_ptr, nat.dptr(ws), wsb, nat.stream_ptr(dev)),
                  f'{rule} decide_count')
        return counts

    def decide_args(self, x, symbols, indices, out: torch.Tensor) -> nat.AmpVampDecideArgs:
        """amp_vamp_decide_args for a fused forward + decision (amp_vamp_detect_count): the
        truth tensors on the device, kept alive on this Loss until the next call."""
        if self.decision_mode != 'sparc':
            raise NotImplementedError("native decision implements generator_mode='sparc' (loss.py:282-302)")
        dev = out.device
        B = self.B
        xt = _flat_c64(x, B, 'x')
        sym = _as_device_labels(symbols, dev)
        idx = _as_device_labels(indices, dev)
        S = B * self.config.L
        if sym.numel() != S or idx.numel() != S:
            raise ValueError(f'expected {S} labels/indices, got {sym.numel()}/{idx.numel()}')
        self._keep = (xt, sym, idx)
        a = nat.AmpVampDecideArgs()
        a.x, a.sym, a.idx = nat.dptr(xt, name='x'), nat.dptr(sym, name='symbols'), nat.dptr(idx, name='indices')
        a.ibits_trunc = self._ibits
        a.counts = nat.dptr(out)
        return a

    @staticmethod
    def read_counts(buf: torch.Tensor) -> nat.AmpCounts:
        raw = buf[:C.sizeof(nat.AmpCounts)].cpu().numpy().tobytes()
        return nat.AmpCounts.from_buffer_copy(raw)

    def rates_from_counts(self, c: nat.AmpCounts):
        """The 14 metrics with the reference's arithmetic and dtypes (loss.py:105-179)."""
        B, Lin, Na, Ns = self.B, self.Lin, self.Na, self.Ns
        nMSE = np.float32(c.mse) / Ns
        nMSEf = np.float32(c.msef) / Na / B
        nMSEm = np.float32(c.msem) / Na / B
        nMSEL = np.float32(c.mseL) / Na / B
        ver = np.int64(c.ver) / Lin / B
        verf = np.int64(c.verf) / B
        verm = np.int64(c.verm) / B
        verL = np.int64(c.verL) / B
        fer = np.int64(c.fer) / B
        ier = int(c.ier) / Ns
        ser = int(c.ser) / Ns
        iber_ = int(c.iber) / Lin / B
        iber = iber_ / self.ibits
        if self.sbits != 0:
            sber_ = int(c.sber) / Lin / B
            sber = sber_ / self.sbits / Na
        else:
            sber, sber_ = 0., 0.
        ber = (iber_ + sber_) / (Na * self.sbits + self.ibits)
        return fer, nMSE, nMSEf, nMSEm, nMSEL, ver, verf, verm, verL, ber, iber, sber, ier, ser

    def rates_from_vector(self, vec: np.ndarray, epochs: int = 1):
        """The 14 metrics averaged over `epochs` epochs of B trials whose counters were summed
        into `vec` (counts_to_vector): every metric is linear in the counters, so this is the
        mean of the per-epoch metrics (Loss.accumulate + Loss.average, loss.py:325-346)."""
        return tuple(np.float64(r) / epochs for r in self.rates_from_counts(vector_to_counts(vec)))

    def record(self, rates, iterations: int) -> None:
        """Loss.__call__'s bookkeeping (loss.py:60-65)."""
        self.loss['T'] = iterations
        for key, value in zip(self.keys, rates):
            try:
                self.loss[key] = np.append(self.loss[key], value)
            except KeyError:
                self.loss[key] = np.array(value)

    # ------------------------------------------------------------------ reference surface
    def __call__(self, xmap, xmmse, x, symbols, indices, iterations: int) -> None:
        self.record(self.error_rate(xmap, xmmse, x, symbols, indices), iterations)

    def error_rate(self, xmap, xmmse, x, symbols=None, indices=None):
        counts = self.device_counts(xmap, xmmse, x, symbols, indices)
        return self.rates_from_counts(self.read_counts(counts))

    def MAP_decision(self, xamp: torch.Tensor):
        """(xhat, gray labels, flat indices) of loss.py:282-302, decided on the GPU."""
        return self._decide(xamp, 'sparc')

    def segmented_decision(self, xamp: torch.Tensor):
        """(xhat, gray labels, flat indices) of loss.py:222-250, decided on the GPU (B = 1)."""
        return self._decide(xamp, 'segmented')

    def random_decision(self, xamp: torch.Tensor):
        """(xhat, gray labels, flat indices) of loss.py:252-280, decided on the GPU (B = 1)."""
        return self._decide(xamp, 'random')

    def decision(self, xamp: torch.Tensor):
        """The mode's decision (loss.py:38-43)."""
        return self._decide(xamp, self.decision_mode)

    def _decide(self, xamp: torch.Tensor, rule: str):
        d, c = self._native()
        B = self.B
        xamp = _flat_c64(xamp, B, 'xamp')
        S = B * self.Na * self.Lin
        dec = torch.empty(S, dtype=torch.int32, device=xamp.device)
        zeros = torch.zeros(S, dtype=torch.int64, device=xamp.device)
        self.device_counts(xamp, xamp, xamp, zeros, zeros, decisions=dec, rule=rule)
        f = dec.cpu().numpy().astype(np.int64)
        m_hat, k_hat = np.divmod(f, self.config.K)
        if rule == 'random':                      # Na decided positions per row of Nt
            R = B * self.Lin
            xhat = np.zeros((R, self.Nt), dtype=np.complex64)
            rows = np.repeat(np.arange(R), self.Na)
            xhat[rows, m_hat] = np.asarray(self.symbols)[k_hat]
            return xhat.ravel(), np.asarray(self.gray)[k_hat], rows * self.Nt + m_hat
        M = self.Nt // self.Na
        xhat = np.zeros((S, M), dtype=np.complex64)
        xhat[np.arange(S), m_hat] = np.asarray(self.symbols)[k_hat]
        index = np.arange(S) * M + m_hat
        return xhat.ravel(), np.asarray(self.gray)[k_hat], index

    def export(self, SNRdB: float, EbN0dB: float, save_location: str) -> None:
        """Write {EbN0dB}.json (loss.py:304-323) and reset."""
        self.loss['EbN0dB'] = float(EbN0dB)
        self.loss['SNRdB'] = float(SNRdB)
        self.loss['rate'] = float(self.rate)
        self.loss['C'] = float(np.log2(1 + 10 ** (SNRdB / 10)))
        self.loss['ShannonLimitdB'] = float(self.shannon_limt_dB)
        out = {k: (v.item() if isinstance(v, (np.ndarray, np.generic)) and np.ndim(v) == 0 else
                   (v.tolist() if isinstance(v, np.ndarray) else v)) for k, v in self.loss.items()}
        with open(os.path.join(save_location, f'{EbN0dB}.json'), 'w', encoding='utf-8') as f:
            json.dump(out, f, ensure_ascii=False, indent=6, skipkeys=True)
        self.loss = {'T': 0}

    def accumulate(self, other) -> None:
        """loss.py:325-336."""
        self.loss['T'] += other.loss['T']
        for key in self.keys:
            try:
                self.loss[key] += other.loss[key]
            except KeyError:
                self.loss[key] = other.loss[key]

    def average(self, epochs: int) -> None:
        """loss.py:338-346."""
        self.loss['T'] = self.loss['T'] / epochs
        for key in self.keys:
            self.loss[key] = np.array(self.loss[key]) / epochs

    def dump(self) -> None:
        self.loss = {}
