#!/usr/bin/env python3
"""Diagnostic (GPU): accuracy of one VAMP iteration's linear algebra on every engine against a
float64 evaluation of the same iteration, beside the numpy (BLAS complex64) restatement's.

After ONE iteration (vamp.py:66-79 with the Tracker's r~ = sparsity) r depends only on the inputs
and the float32 scalars of iteration 0, so r_exact = (V (scale (y~ + vr q) - q) + r~ - alpha r~) /
(1 - alpha) with y~ = (s Uh) y and q = Vh r~ evaluated in float64 is the reference value; the
printed statistics are |r - r_exact| / max|r_exact| (max, rms) per engine.  At a golden point whose
allclose exit is decided by rounding this says whether an engine's GEMMs are noisier than the
CPU path's.

  python tools/gemm_accuracy.py [--point cfg4_vamp_qpsk:1/0]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_io as gio  # noqa: E402
import oracle.amp_oracle as O  # noqa: E402
from test_gpu_vamp import VARIANTS, _config, _regen_inputs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--point', default='cfg4_vamp_qpsk:1/0')
    ap.add_argument('--variants', default='launches,persistent,persistent-f32,persistent-h2,persistent-i8')
    a = ap.parse_args()
    from vamp import VAMP
    name, key = a.point.split(':')
    ent = gio.g4_curves()[name]
    seed, ebn0 = int(key.split('/')[0]), float(key.split('/')[1])
    cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'], iterations=1)
    inp = _regen_inputs(cfg, seed, ebn0)
    c = lambda t: t.cpu().numpy()[..., 0] if t.dim() == 3 else t.cpu().numpy()   # noqa: E731
    U, s, Vh, y = c(inp['U']), c(inp['s']), c(inp['Vh']), c(inp['y'])
    ocfg = O.OracleConfig(ent['Nt'], ent['Na'], ent['Nr'], B=ent['B'], alphabet=ent['alphabet'], iterations=1)
    tr = []
    o = O.vamp_detect(U, s, Vh, y, inp['SNR'], ocfg, trace=tr)
    alpha = np.float64(tr[0]['alpha'])
    # float64 evaluation of the same iteration with the oracle's float32 scalars
    p = ocfg.Na / ocfg.Nt
    E = ocfg.Na / ocfg.Nr
    noise_var = E / inp['SNR']
    s2t = p ** 2 * (1 - p) + (1 - p) ** 2 * p
    vr = np.float64(np.float32(noise_var / s2t))
    s64 = s.astype(np.float64)
    Uh = np.conj(U.astype(np.complex128)).T
    ytil = y.astype(np.complex128) @ (s64[:, None] * Uh).T
    rt = np.full((y.shape[0], Vh.shape[1]), p, dtype=np.complex128)
    q = rt @ Vh.astype(np.complex128).T
    scale = 1.0 / (s64 * s64 + vr)
    w = scale * (ytil + vr * q) - q
    xt = w @ np.conj(Vh.astype(np.complex128)) + rt
    r_ex = (xt - alpha * rt) / (1 - alpha)
    ref = float(np.abs(r_ex).max())

    def stats(r):
        d = np.abs(r.astype(np.complex128) - r_ex) / ref
        return f'max {d.max():.3e}  rms {np.sqrt((d ** 2).mean()):.3e}'
    print(f'{name} {key}: one iteration, |r - r_float64| / max|r| (max |r| = {ref:.3f})')
    print(f'  numpy c64 (oracle, BLAS)   {stats(o["r"])}', flush=True)
    for v in [v for v in a.variants.split(',') if v]:
        eng, gemm = VARIANTS[v]
        T = VAMP(cfg, engine=eng, gemm=gemm).detect(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])
        torch.cuda.synchronize()
        print(f'  {v:25s}  {stats(c(T.r))}', flush=True)


if __name__ == '__main__':
    main()
