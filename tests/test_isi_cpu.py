"""ISI / spatial coupling (Lin > 1, Lh > 1, tail; g11): the build's input replica reproduces the
reference's block-Toeplitz A and base matrix W bit for bit (SHA-256) and y to float32 rounding,
and the numpy oracle reproduces the reference's Loss dicts there (VER / SER within 1e-3, T as in
the GPU curve tests).  g10: the reference driver's files are well formed."""
import hashlib

import numpy as np
import pytest

from isi_inputs import g10, g11, g11_points, isi_inputs
from oracle import OracleConfig, bamp_detect, loss_dict, scamp_detect, vamp_detect


def _sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.numpy()).tobytes()).hexdigest()


@pytest.mark.parametrize('name,key', g11_points())
def test_isi_inputs_replica_and_oracle(name, key):
    ent = g11()[name]
    ref = ent['points'][key]
    seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
    inp = isi_inputs(ent, seed, EbN0, svd=ent['algo'] == 'vamp')
    assert _sha(inp['A']) == ref['sha_A'] and _sha(inp['W']) == ref['sha_W'] and _sha(inp['x']) == ref['sha_x']
    y2 = float(np.sum(np.abs(inp['y'].numpy().astype(np.complex128)) ** 2))
    assert abs(y2 - ref['y_abs2_sum']) <= 1e-5 * ref['y_abs2_sum']
    cfg = OracleConfig(ent['Nt'], ent['Na'], ent['Nr'], Lin=ent['Lin'], Lh=ent['Lh'], B=ent['B'],
                       alphabet=ent['alphabet'], iterations=ent['iterations'])
    c = lambda t: t.numpy()[..., 0] if t.dim() == 3 else t.numpy()  # noqa: E731
    if ent['algo'] == 'vamp':
        out = vamp_detect(inp['U'].numpy(), inp['s'].numpy(), inp['Vh'].numpy(), c(inp['y']), inp['SNR'], cfg)
        dec = out['r']
    elif ent['algo'] == 'bamp':
        out = bamp_detect(inp['A'].numpy(), c(inp['y']), inp['SNR'], cfg)
        dec = out['xmap']
    else:
        out = scamp_detect(inp['W'].numpy(), inp['A'].numpy(), c(inp['y']), inp['SNR'], cfg)
        dec = out['xmap']
    got = loss_dict(dec, out['xmmse'], c(inp['x']), inp['sym'], inp['idx'], out['T'], cfg)
    for k in ('ver', 'ser'):
        assert abs(float(got[k]) - ref[k]) <= 1e-3, (k, got[k], ref[k])


def test_g10_driver_files_well_formed():
    runs = g10()
    assert set(runs) == {'vamp_cfg2_qpsk', 'bamp_cfg1_qpsk', 'scamp_qpsk'}
    for name, run in runs.items():
        kw = run['simulate']
        grid = np.arange(kw['start'], kw['final'] + kw['step'], kw['step'])
        names = [f'{float(e)}.json' for e in grid]
        got = sorted(run['files'], key=lambda f: float(f[:-5]))
        assert got == names[:len(got)], (name, got)          # a prefix: the FER < 1e-3 early stop
        last = run['files'][got[-1]]
        assert len(got) == len(names) or last['fer'] < 1e-3
        for f in got[:-1]:
            assert run['files'][f]['fer'] >= 1e-3
