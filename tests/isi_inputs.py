"""Inputs of the g11 goldens (ISI / spatial coupling: Lin > 1, Lh > 1, tail) and the g10 driver
runs, regenerated with the build's host RNG replica in the reference's call order."""
import json
import os

import numpy as np
import torch

import golden_io as gio


def g11():
    with open(os.path.join(gio.GOLDEN, 'g11_isi.json')) as f:
        return json.load(f)


def g10():
    with open(os.path.join(gio.GOLDEN, 'g10_simulate.json')) as f:
        return {k: v for k, v in json.load(f).items() if not k.startswith('_')}


def g11_points():
    out = []
    for name, ent in sorted(g11().items()):
        for key in sorted(ent['points'], key=lambda k: (int(k.split('/')[0]), float(k.split('/')[1]))):
            out.append((name, key))
    return out


def isi_config(ent, device='cpu'):
    from config import Config
    return Config(ent['Nt'], ent['Na'], ent['Nr'], ent['Lin'], ent['Lh'], batch=ent['B'], generator_mode='sparc',
                  iterations=ent['iterations'], alphabet=ent['alphabet'], channel_profile='uniform',
                  channel_truncation='tail', device=device)


def isi_inputs(ent, seed, EbN0, svd):
    """CPU tensors exactly as make_goldens.gen_inputs drew them for the reference."""
    from channel import Channel
    from data import Data
    cfg = isi_config(ent)
    np.random.seed(seed)
    torch.manual_seed(seed)
    ch, da = Channel(cfg), Data(cfg)
    W, A = ch.generate_as_sparc()
    U = s = Vh = None
    if svd:
        U, s, Vh = torch.linalg.svd(A, full_matrices=False)
    x, sym, idx = da.generate_message()
    SNR = cfg.snr(EbN0)
    y = A @ x + ch.awgn(SNR)
    return dict(W=W, A=A, U=U, s=s, Vh=Vh, x=x, y=y, sym=sym, idx=idx, SNR=SNR)
