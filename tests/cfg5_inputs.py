"""Inputs of the g6 goldens (BASELINE cfg5 shape on the correlated channel), regenerated with the
build's host RNG replica in the reference's call order: seed -> channel -> message -> y."""
import json
import os

import numpy as np
import torch

import golden_io as gio


def g6_curves():
    with open(os.path.join(gio.GOLDEN, 'g6_cfg5_corr.json')) as f:
        return json.load(f)


def g6_points():
    out = []
    for name, ent in sorted(g6_curves().items()):
        for key in sorted(ent['points'], key=lambda k: float(k.split('/')[1])):
            out.append((name, key))
    return out


def cfg5_config(ent, device='cpu', B=None):
    """The entry's Config; 64-QAM (BASELINE cfg5's alphabet, which Config rejects like the
    reference) is injected after construction exactly as make_goldens.py injected it into the
    reference's Config, and checked against the table the golden recorded."""
    from config import Config
    qam64 = ent['alphabet'] == '64QAM'
    cfg = Config(ent['Nt'], ent['Na'], ent['Nr'], 1, 1, batch=B or ent['B'], generator_mode='sparc',
                 iterations=ent['iterations'], alphabet='16QAM' if qam64 else ent['alphabet'],
                 channel_profile='uniform', channel_truncation='tail', device=device)
    if qam64:
        cfg.inject_square_qam(64)
        assert np.array_equal(np.real(cfg.symbols), np.array(ent['symbols_re']))
        assert np.array_equal(np.imag(cfg.symbols), np.array(ent['symbols_im']))
        assert list(cfg.gray) == list(ent['gray']) and cfg.code_rate == ent['code_rate']
    return cfg


def cfg5_inputs(ent, seed, EbN0):
    """CPU tensors (A, x, y, sym, idx, SNR) exactly as tests/golden/make_goldens.py g6 built them."""
    from channel import Channel
    from data import Data
    cfg = cfg5_config(ent)
    np.random.seed(seed)
    torch.manual_seed(seed)
    ch, da = Channel(cfg), Data(cfg)
    A = ch.generate_correlated(ent['rho'])
    x, sym, idx = da.generate_message()
    SNR = cfg.snr(EbN0)
    y = A @ x + ch.awgn(SNR)
    return dict(A=A, x=x, y=y, sym=sym, idx=idx, SNR=SNR)


def cfg5_inputs_b(ent, seed, EbN0, B):
    """cfg5_inputs with the batch taken from the caller (entries recorded at another B)."""
    e = dict(ent)
    e['B'] = B
    return cfg5_inputs(e, seed, EbN0)
