"""g5 Shrink golden cases (tests/golden/g5_shrink.npz) with the inputs the kernels need."""
import numpy as np
import torch

import golden_io as gio
from config import Config


def g5_cases():
    z = gio._group(np.load(gio.GOLDEN + '/g5_shrink.npz'))
    out = []
    for name, c in sorted(z.items(), key=lambda kv: int(kv[0][4:])):
        Nt, Na, B = (int(v) for v in c.dims)
        cfg = Config(Nt, Na, 2 * Nt, 1, 1, batch=B, generator_mode='sparc', alphabet=str(c.alphabet),
                     is_complex=bool(c.is_complex), channel_profile='uniform', channel_truncation='tail',
                     device='cpu')
        c['name'] = name
        c['cfg'] = cfg
        c['M'] = Nt // Na
        c['sym'] = cfg.symbols.astype(np.complex64) if cfg.is_complex else cfg.symbols.astype(np.float32)
        c['theta'] = float(torch.log(torch.tensor(cfg.P0) / torch.tensor(cfg.Ps)))   # shrink.py:152
        out.append(c)
    return out


def compare(got, ref, rtol, atol):
    """NaN positions identical; elsewhere |got - ref| <= atol + rtol |ref|.  Returns the worst excess."""
    got, ref = np.asarray(got), np.asarray(ref)
    assert got.shape == ref.shape and got.dtype == ref.dtype, (got.shape, ref.shape, got.dtype, ref.dtype)
    nan_g, nan_r = np.isnan(got), np.isnan(ref)
    assert np.array_equal(nan_g, nan_r), f'NaN pattern differs at {np.argwhere(nan_g != nan_r)[:5].tolist()}'
    m = ~nan_r
    inf_r = np.isinf(ref) & m
    assert np.array_equal(got[inf_r], ref[inf_r]), 'inf values differ'
    m &= ~inf_r
    d = np.abs(got[m].astype(np.complex128) - ref[m].astype(np.complex128)) - (atol + rtol * np.abs(ref[m]))
    return float(d.max(initial=-np.inf))
