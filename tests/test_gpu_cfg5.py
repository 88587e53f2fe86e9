"""BASELINE cfg5 on the GPU: BAMP Nt=512 Nr=1024 Na=16 on the Kronecker exponentially-correlated
channel (rho = 0.5): 64-QAM (cfg5's own alphabet, injected into Config, which rejects it like the
reference's, config.py:44) at B = 1024 over 6 EbN0 points and at the named B = 8192, plus the
QPSK and 16-QAM twins at B = 1024.  Reference: its own BAMP run on the same injected inputs and
alphabet (tests/golden/make_goldens.py g6).  Bar: VER and SER within 1e-3 at every point, T as
in the other curve tests."""
import numpy as np
import pytest

from cfg5_inputs import cfg5_config, cfg5_inputs, g6_curves, g6_points
from test_gpu_vamp import _check_T

pytestmark = pytest.mark.gpu


GEMMS = {'auto': 0, 'h2': 3, 'x3': 2}   # amp_native GEMM_AUTO / GEMM_H2 / GEMM_X3


@pytest.mark.parametrize('gemm', sorted(GEMMS))
@pytest.mark.parametrize('name,key', g6_points())
def test_cfg5_correlated_curve_point(device, name, key, gemm):
    """Every GEMM arithmetic of BAMP's launch engine: 'auto' is the f32 MFMA GEMM (the reference's
    operand precision), 'x3' the bf16x3 tile GEMM (amp_gemm_x3.h, 24-bit operands), 'h2' the opt-in
    fp16x2 tile GEMM (amp_gemm_h2.h, 22-bit operands)."""
    import amp_native as nat
    from bamp import BAMP
    ent = g6_curves()[name]
    ref = ent['points'][key]
    seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
    inp = cfg5_inputs(ent, seed, EbN0)
    cfg = cfg5_config(ent, device='cuda')
    if 'SNR' in ref:
        assert inp['SNR'] == pytest.approx(ref['SNR'], rel=1e-12)
    mv = lambda t: t.to(device)  # noqa: E731
    assert (nat.GEMM_AUTO, nat.GEMM_H2, nat.GEMM_X3) == (GEMMS['auto'], GEMMS['h2'], GEMMS['x3'])
    L = BAMP(cfg, gemm=GEMMS[gemm])(mv(inp['A']), mv(inp['y']), inp['SNR'], mv(inp['x']), inp['sym'], inp['idx'])
    got = L.loss
    assert abs(float(got['ver']) - ref['ver']) <= 1e-3, (float(got['ver']), ref['ver'])
    assert abs(float(got['ser']) - ref['ser']) <= 1e-3, (float(got['ser']), ref['ser'])
    # The reference's QAM decision has no -|a|^2/2 term (loss.py:295), so for 64-QAM SER saturates
    # near 15/16 and VER at 1 at every SNR; the index error rate and the nMSE of xmmse still
    # follow the detector's quality (0.29 -> 0.11 over 0-9 dB) and NaN onset (>= 10 dB): checked too.
    assert abs(float(got['ier']) - ref['ier']) <= 1e-3, (float(got['ier']), ref['ier'])
    g, r = float(got['nMSE']), ref['nMSE']
    assert (np.isnan(g) and np.isnan(r)) or abs(g - r) <= 1e-2 * abs(r) + 1e-6, (g, r)
    _check_T(int(got['T']), int(ref['T']), ent['iterations'], ref['ver'])
