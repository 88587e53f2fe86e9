"""Readers for the reference-generated golden fixtures in tests/golden/ (data only)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


class Case(dict):
    def __getattr__(self, k):
        return self[k]


def _group(npz):
    out = {}
    for k in npz.files:
        if '/' not in k:
            continue
        key, field = k.split('/', 1)
        out.setdefault(key, Case())[field] = npz[k]
    return out


def g1_cases():
    """{name: Case} — per-iteration reference traces with their stored inputs."""
    cases = _group(np.load(os.path.join(GOLDEN, 'g1_traces.npz')))
    for name, c in cases.items():
        algo, alph, ebn0, seed = name.split('_')
        c['algo'], c['alphabet'], c['EbN0'], c['seed'] = algo, alph, float(ebn0), int(seed)
        c['loss_ref'] = json.loads(str(c['loss']))
    return cases


def g12_cases():
    """{name: Case} — vamp2.py (damped VAMP) reference traces with their stored inputs."""
    cases = _group(np.load(os.path.join(GOLDEN, 'g12_vamp2.npz')))
    for name, c in cases.items():
        _, alph, nt, ebn0, seed, damp = name.split('_')
        c['alphabet'], c['EbN0'], c['seed'] = alph, float(ebn0), int(seed)
        c['loss_ref'] = json.loads(str(c['loss']))
    return cases


def g2_cases():
    return _group(np.load(os.path.join(GOLDEN, 'g2_denoiser.npz')))


def g3_cases():
    cases = _group(np.load(os.path.join(GOLDEN, 'g3_decision.npz')))
    for c in cases.values():
        c['loss_ref'] = json.loads(str(c['loss']))
    return cases


def g4_curves():
    with open(os.path.join(GOLDEN, 'g4_curves.json')) as f:
        return json.load(f)


LOSS_KEYS = ['fer', 'nMSE', 'nMSEf', 'nMSEm', 'nMSEL', 'ver', 'verf', 'verm', 'verL', 'ber', 'iber', 'sber',
             'ier', 'ser']
COUNT_KEYS = ['fer', 'ver', 'verf', 'verm', 'verL', 'ber', 'iber', 'sber', 'ier', 'ser']


def loss_close(got: dict, ref: dict, count_tol=0.0, mse_rtol=1e-3):
    """Compare Loss dicts: counting metrics within `count_tol` absolute, nMSE* within mse_rtol."""
    bad = {}
    for k in LOSS_KEYS:
        g, r = float(np.asarray(got[k])), float(ref[k])
        if np.isnan(r) or np.isnan(g):
            if not (np.isnan(r) and np.isnan(g)):
                bad[k] = (g, r)
            continue
        if k.startswith('nMSE'):
            if abs(g - r) > mse_rtol * max(abs(r), 1e-12) + 1e-9:
                bad[k] = (g, r)
        elif abs(g - r) > count_tol + 1e-12:
            bad[k] = (g, r)
    return bad


def bits_equal(a, b) -> bool:
    """Bitwise equality of two device tensors (NaN payloads included): the NaN-onset iterations
    must agree too, which torch.equal (NaN != NaN) cannot check."""
    import torch
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.is_complex():
        a, b = torch.view_as_real(a), torch.view_as_real(b)
    w = torch.int64 if a.element_size() == 8 else torch.int32
    return torch.equal(a.contiguous().view(w), b.contiguous().view(w))
