#!/usr/bin/env python3
"""Exploratory numerics probe (CPU, numpy; not on any product path): VAMP with GEMM1 reformulated
through the unitarity of the SVD factor (k == N: Vh V = I).

  q_{t+1} = Vh r~_{t+1} = ns (Vh x^_{t+1} - dxdr Vh r_t),   Vh r_t = w_t / (1 - alpha_t) + q_t

(r_t = V w_t / (1 - alpha_t) + r~_t, vamp.py:72-79), so GEMM1 only needs Vh x^ — available right
after the denoiser, before the batch-global scalars of vamp.py:85-94 are known.  This runs the
oracle's restatement both ways on the g4 golden inputs and checks both against the reference's
goldens with the GPU tests' bar (VER / SER within 1e-3, T by tests/test_gpu_vamp.py _check_T).

  python tools/unitary_probe.py [cfg2|cfg4] [every]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import golden_io as gio  # noqa: E402
from oracle import OracleConfig, loss_dict  # noqa: E402
from oracle import amp_oracle as O  # noqa: E402

C64, F32 = np.complex64, np.float32


def vamp_detect_u(U, s, Vh, y, SNR, cfg, unitary=True):
    """oracle.vamp_detect with GEMM1 = ns (Vh x^ - dxdr (w / (1 - alpha) + q)) when unitary."""
    U = np.asarray(U, C64); Vh = np.asarray(Vh, C64); y = np.asarray(y, C64)
    s = np.asarray(s, F32)
    B = y.shape[0]
    E = cfg.Na / cfg.Nr
    p = cfg.Na / cfg.Nt
    noise_var = E / SNR
    Uh = np.conj(U).T
    Vt = np.conj(Vh)
    s2 = (s * s).astype(F32)
    ytil = (y @ ((s[:, None] * Uh).astype(C64)).T).astype(C64)
    N = Vh.shape[1]
    r = np.zeros((B, N), C64)
    var = np.ones((B, N), F32)
    rt = np.full((B, N), F32(p), dtype=C64)
    s2t = p ** 2 * (1 - p) + (1 - p) ** 2 * p
    eta = s.shape[0] / N
    xm = None
    t = 0
    q_next = None
    for t in range(cfg.N_Layers):
        prev = var
        first = isinstance(s2t, float)
        vr = F32(noise_var / s2t) if first else F32(O._recip(s2t) * F32(noise_var))
        q = (rt @ Vh.T).astype(C64) if (q_next is None or not unitary) else q_next
        scale = O._recip(s2 + vr)
        xt = (scale * (ytil + vr * q)).astype(C64)
        varL = F32(F32(np.sum(scale, dtype=np.float64) / scale.size) * F32(noise_var))
        w = (xt - q).astype(C64)
        xt = (w @ Vt + rt).astype(C64)
        if first:
            xtv = F32(F32(eta) * varL + F32((1 - eta) * s2t))
            alpha = F32(xtv / F32(s2t))
            s2t32 = F32(s2t)
        else:
            xtv = F32(F32(eta) * varL + F32(F32(1 - eta) * s2t))
            alpha = F32(xtv / s2t)
            s2t32 = s2t
        alpha = O._clamp(alpha, O.VAR_RATIO_MIN, O.VAR_RATIO_MAX)
        inv1ma = O._recip(F32(1) - alpha)
        r = O._div_real(xt - alpha * rt, F32(1) - alpha)
        vhr = (w * inv1ma + q).astype(C64)                      # Vh r (Vh V = I)
        sigma2 = F32(F32(alpha / (F32(1) - alpha)) * s2t32)
        sigma2 = O._clamp(sigma2, O.VAR_MIN, O.VAR_MAX)
        xm, var = O.block_denoise(r, sigma2, cfg)
        P = (xm @ Vh.T).astype(C64)                              # Vh x^ (before the scalars)
        mean_var = F32(np.sum(var, dtype=np.float64) / var.size)
        dxdr = O._clamp(F32(mean_var / sigma2), O.VAR_RATIO_MIN, O.VAR_RATIO_MAX)
        ns = O._recip(F32(1) - dxdr)
        rt = ((xm - dxdr * r) * ns).astype(C64)
        q_next = ((P - dxdr * vhr) * ns).astype(C64)
        s2t = O._clamp(F32(F32(sigma2 * dxdr) * ns), O.VAR_MIN, O.VAR_MAX)
        if O.allclose_f32(var, prev):
            break
    return dict(r=r, xmmse=xm, var=var, T=t + 1)


def main():
    from test_gpu_vamp import _check_T, _config, _regen_inputs
    which = sys.argv[1] if len(sys.argv) > 1 else 'cfg2'
    every = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    curves = gio.g4_curves()
    bad = {False: 0, True: 0}
    n = 0
    for name in (f'{which}_vamp_16qam', f'{which}_vamp_qpsk'):
        ent = curves[name]
        keys = sorted(ent['points'], key=lambda k: (int(k.split('/')[0]), float(k.split('/')[1])))[::every]
        for key in keys:
            ref = ent['points'][key]
            seed, ebn0 = int(key.split('/')[0]), float(key.split('/')[1])
            cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'], device='cpu',
                          iterations=ent['iterations'])
            inp = _regen_inputs(cfg, seed, ebn0)
            c = lambda t: t.numpy()[..., 0] if t.dim() == 3 else t.numpy()  # noqa: E731
            ocfg = OracleConfig(ent['Nt'], ent['Na'], ent['Nr'], B=ent['B'], alphabet=ent['alphabet'],
                                iterations=ent['iterations'])
            line = f'{name:18s} {key:8s} ref T={int(ref["T"]):2d}/{int(ref.get("T_pert", ref["T"])):2d}'
            for uni in (False, True):
                out = vamp_detect_u(c(inp['U']), c(inp['s']), c(inp['Vh']), c(inp['y']), float(inp['SNR']), ocfg,
                                    unitary=uni)
                L = loss_dict(out['r'], out['xmmse'], c(inp['x']), inp['sym'], inp['idx'], out['T'], ocfg)
                ok = abs(float(L['ver']) - ref['ver']) <= 1e-3 and abs(float(L['ser']) - ref['ser']) <= 1e-3
                try:
                    _check_T(int(out['T']), int(ref['T']), ent['iterations'], ref['ver'], ref.get('T_pert'))
                except AssertionError:
                    ok = False
                bad[uni] += not ok
                line += (f'  {"unitary" if uni else "direct "} T={int(out["T"]):2d} dver={float(L["ver"]) - ref["ver"]:+.1e}'
                         f' dser={float(L["ser"]) - ref["ser"]:+.1e}{"" if ok else " FAIL"}')
            n += 1
            print(line, flush=True)
    print(f'{n} points: direct {bad[False]} fail, unitary {bad[True]} fail')


if __name__ == '__main__':
    torch.set_num_threads(8)
    main()
