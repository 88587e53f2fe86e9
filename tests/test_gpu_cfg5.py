"""BASELINE cfg5 shape on the GPU: BAMP Nt=512 Nr=1024 Na=16 on the Kronecker exponentially-
correlated channel (rho = 0.5), B = 1024, QPSK and 16-QAM twins of cfg5's 64-QAM (Config
rejects 64-QAM, config.py:44).  Reference: its own BAMP run on the same injected inputs
(tests/golden/make_goldens.py g6).  Bar: VER and SER within 1e-3 at every point, T as in the
other curve tests."""
import pytest

from cfg5_inputs import cfg5_config, cfg5_inputs, g6_curves, g6_points
from test_gpu_vamp import _check_T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('name,key', g6_points())
def test_cfg5_correlated_curve_point(device, name, key):
    from bamp import BAMP
    ent = g6_curves()[name]
    ref = ent['points'][key]
    seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
    inp = cfg5_inputs(ent, seed, EbN0)
    cfg = cfg5_config(ent, device='cuda')
    mv = lambda t: t.to(device)  # noqa: E731
    L = BAMP(cfg)(mv(inp['A']), mv(inp['y']), inp['SNR'], mv(inp['x']), inp['sym'], inp['idx'])
    got = L.loss
    assert abs(float(got['ver']) - ref['ver']) <= 1e-3, (float(got['ver']), ref['ver'])
    assert abs(float(got['ser']) - ref['ser']) <= 1e-3, (float(got['ser']), ref['ser'])
    _check_T(int(got['T']), int(ref['T']), ent['iterations'], ref['ver'])
