"""generator_mode='segmented' on the GPU (amp_segmented_decide_count), B = 1 as in the reference.

g7 decision cases: decisions and all 14 metrics equal the reference's.  In the crafted 'ties'
cases several positions of a section share the largest |x| exactly; numpy's argsort orders such
ties in an implementation-defined way (SIMD quicksort), so there the kernel's choice must be
one of the tied maxima and the rest of the section's decision must agree.
g7 curves: VAMP and BAMP end to end at B = 1 on the reference's inputs (6 seeds x 5 EbN0 per
curve).  One trial per point makes VER/SER 0/1-valued; at most one point per curve may differ
(a single trial flipped by float32 summation order near a decision boundary)."""
import json
import os

import numpy as np
import pytest
import torch

import golden_io as gio
from test_gpu_vamp import _regen_inputs
from test_segmented_cpu import g7_cases

pytestmark = pytest.mark.gpu

G7 = g7_cases()
with open(os.path.join(gio.GOLDEN, 'g7_segmented_curves.json')) as f:
    CURVES = json.load(f)


def _cfg(Nt, Na, Nr, Lin, Lh, B, alphabet, iterations=5, device='cuda'):
    from config import Config
    return Config(Nt, Na, Nr, Lin, Lh, batch=B, generator_mode='segmented', iterations=iterations,
                  alphabet=alphabet, channel_profile='uniform', channel_truncation='tail', device=device)


@pytest.mark.parametrize('name', sorted(G7, key=lambda k: int(k[4:])))
def test_segmented_decision_matches_reference(device, name):
    from loss import Loss
    c = G7[name]
    Nt, Na, Nr, B, Lin, Lh = (int(v) for v in c.dims)
    cfg = _cfg(Nt, Na, Nr, Lin, Lh, B, str(c.alphabet))
    L = Loss(cfg)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device).view(B, -1, 1)  # noqa: E731
    xhat, shat, ihat = L.segmented_decision(t(c.xmap))
    ties = int(name[4:]) % 4 == 1
    if not ties:
        np.testing.assert_array_equal(xhat, c.xhat)
        np.testing.assert_array_equal(shat, c.shat)
        np.testing.assert_array_equal(ihat, c.ihat)
        L.dump()
        L(t(c.xmap), t(c.xmmse), t(c.x), c.sym, c.idx, 3)
        bad = gio.loss_close(L.loss, c.loss_ref, count_tol=0.0, mse_rtol=1e-5)
        assert not bad, bad
    else:
        M = Nt // Na
        mag = np.abs(c.xmap.reshape(-1, M))
        for j in range(mag.shape[0]):
            m = ihat[j] % M
            assert mag[j, m] == mag[j].max()
            if ihat[j] == c.ihat[j]:
                assert shat[j] == c.shat[j]


@pytest.mark.parametrize('name', sorted(CURVES))
def test_segmented_detectors_b1(device, name):
    from bamp import BAMP
    from vamp import VAMP
    ent = CURVES[name]
    cfg = _cfg(ent['Nt'], ent['Na'], ent['Nr'], 1, 1, 1, ent['alphabet'], iterations=ent['iterations'])
    det = VAMP(cfg) if ent['algo'] == 'vamp' else BAMP(cfg)
    diff = []
    for key, ref in sorted(ent['points'].items()):
        seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
        inp = _regen_inputs(cfg, seed, EbN0, svd=(ent['algo'] == 'vamp'))
        if ent['algo'] == 'vamp':
            L = det(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        else:
            L = det(inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
        if float(L.loss['ver']) != ref['ver'] or float(L.loss['ser']) != ref['ser']:
            diff.append((key, float(L.loss['ver']), ref['ver'], float(L.loss['ser']), ref['ser']))
    assert len(diff) <= 1, diff
