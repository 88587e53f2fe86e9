"""GPU parity at the reference's "long-sequence" axis and through its driver:

* g11 — ISI / spatial coupling (Lin > 1, Lh > 1, tail): VAMP (both engines), BAMP and SCAMP on
  the block-Toeplitz channel, VER / SER within 1e-3 of the reference on the same seeds, T as in
  the other curve tests;
* g10 — the reference's own Model.simulate (vamp/bamp/scamp_model.py:45-69) run end to end: the
  build's model.Model with the same seed writes the same {EbN0}.json files (names, keys, the
  early stop), VER / SER / FER within 1e-3, the SNR bookkeeping exact.
"""
import json
import os

import numpy as np
import pytest

from isi_inputs import g10, g11, g11_points, isi_config, isi_inputs
from test_gpu_vamp import _check_T

pytestmark = pytest.mark.gpu

def _engines(ent):
    """VAMP: both engines; BAMP and SCAMP: the default GEMM and, where the shape tiles
    (N % 64 == 0 and n % 64 == 0), the bf16x3 launch tiles on the block-banded operator ('x3')."""
    if ent['algo'] == 'vamp':
        return (1, 2)
    N, n = ent['Nt'] * ent['Lin'], ent['Nr'] * (ent['Lin'] + ent['Lh'] - 1)
    return (0, 'x3') if N % 64 == 0 and n % 64 == 0 else (0,)


ISI_CASES = [(n, k, e) for (n, k) in g11_points() for e in _engines(g11()[n])]


@pytest.mark.parametrize('name,key,engine', ISI_CASES)
def test_isi_curve_point(device, name, key, engine):
    from bamp import BAMP
    from scamp import SCAMP
    from vamp import VAMP
    ent = g11()[name]
    ref = ent['points'][key]
    seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
    inp = {k: (v.to(device) if hasattr(v, 'to') else v) for k, v in isi_inputs(ent, seed, EbN0,
                                                                                 ent['algo'] == 'vamp').items()}
    cfg = isi_config(ent, device='cuda')
    if ent['algo'] == 'vamp':
        L = VAMP(cfg, engine=engine)(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'], inp['x'], inp['sym'],
                                     inp['idx'])
    elif ent['algo'] == 'bamp':
        import amp_native as nat
        gemm = nat.GEMM_X3 if engine == 'x3' else nat.GEMM_AUTO
        L = BAMP(cfg, gemm=gemm)(inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
    else:
        import amp_native as nat
        gemm = nat.GEMM_X3 if engine == 'x3' else nat.GEMM_AUTO
        L = SCAMP(cfg, gemm=gemm)(inp['W'], inp['A'], inp['y'], inp['SNR'], inp['x'], inp['sym'], inp['idx'])
    got = L.loss
    for k in ('ver', 'ser'):                       # the north-star bar
        assert abs(float(got[k]) - ref[k]) <= 1e-3, (k, float(got[k]), ref[k])
    # beyond the bar: the index error rate and FER, within 1e-3 or a handful of the B*L sections /
    # B trials these small batches count (float32 vs the reference's float64 rounding can flip a
    # near-tied section, as in the 16-QAM points where the decision rule of loss.py:295 leaves
    # only corner points decodable)
    S = ent['B'] * ent['Na'] * ent['Lin']
    for k, tol in (('ier', max(1e-3, 5.0 / S)), ('fer', max(1e-3, 2.0 / ent['B']))):
        # ... or within the spread of the reference's own one-ulp rerun: in a diverging regime
        # (e.g. isi_vamp_16qam at 12 dB, nMSE 0.76) the reference's ier moves 0.19 -> 0.14 under
        # a rounding-sized change of y, and the GPU lands inside that span
        lo, hi = min(ref[k], ref[f'{k}_pert']), max(ref[k], ref[f'{k}_pert'])
        if hi - lo > tol:
            # the reference itself is not reproducible here (its ier moved by more than the
            # tolerance under a one-ulp change of y): any value within a few such spreads is
            # rounding, not a defect (sampled: 0.1875 / 0.1475 / 0.1631 / 0.1445 for 8, 1 and 3
            # threads and the perturbed y at isi_vamp_16qam 0/12)
            lo, hi = lo - 3 * (hi - lo), hi + 3 * (hi - lo)
        assert lo - tol <= float(got[k]) <= hi + tol, (k, float(got[k]), ref[k], ref[f'{k}_pert'])
    _check_T(int(got['T']), int(ref['T']), ent['iterations'], ref['ver'], ref['T_pert'])


@pytest.mark.parametrize('name', sorted(g10()))
def test_simulate_matches_reference_driver(device, name, tmp_path, monkeypatch):
    from config import Config
    from model import Model
    run = g10()[name]
    cfg = Config(run['Nt'], run['Na'], run['Nr'], 1, 1, batch=run['B'], generator_mode='sparc',
                 iterations=run['iterations'], alphabet=run['alphabet'], channel_profile='uniform',
                 channel_truncation='tail', device='cuda')
    algo = run['driver'].split('_')[0]
    m = Model(cfg, algo, path=str(tmp_path), seed=run['seed'])
    assert m.path == str(tmp_path)
    m.simulate(**run['simulate'])
    files = sorted(f for f in os.listdir(tmp_path) if f.endswith('.json'))
    assert files == sorted(run['files']), (files, sorted(run['files']))
    for f in files:
        got = json.load(open(tmp_path / f))
        ref = run['files'][f]
        assert sorted(got) == sorted(ref), (f, sorted(got), sorted(ref))   # the same keys
        for k in ('EbN0dB', 'SNRdB', 'rate', 'C', 'ShannonLimitdB'):
            assert got[k] == pytest.approx(ref[k], rel=1e-12), (f, k)
        for k in ('ver', 'ser', 'fer', 'ier'):
            assert abs(got[k] - ref[k]) <= 1e-3, (f, k, got[k], ref[k])
        # T is the mean over the point's epochs (loss.py:338-346)
        assert abs(got['T'] - ref['T']) <= 1.0 or ref['ver'] > 0.5, (f, got['T'], ref['T'])
    # the reference's own path naming (vamp_model.py:29, bamp_model.py:28, scamp_model.py:28),
    # created relative to the working directory as the drivers do
    monkeypatch.chdir(tmp_path)
    assert Model(cfg, algo, amp=object()).path == run['path']
    assert os.path.isdir(tmp_path / run['path'])
