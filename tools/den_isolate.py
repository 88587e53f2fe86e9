#!/usr/bin/env python3
"""Diagnostic (GPU): isolate the denoiser's share in VAMP's early-exit divergence.

Runs the numpy oracle's VAMP loop (oracle.vamp_detect: c64 GEMMs and float32 scalars on the host)
with its denoiser replaced by the GPU's amp_block_denoise (the library named by AMP_LIB_PATH, so
diagnostic builds with -DAMP_DEN_EXACT_EXP=1 / -DAMP_DEN_DIV=1 / -DAMP_DEN_Z64=1 can be compared),
at the golden points whose reference exit moved under perturbation, and prints T beside the
reference's and the oracle's own (float64 denoiser) T.  Also reports, at the first iteration, the
relative var error of the GPU denoiser against the float64 one on the same input.

  python tools/den_isolate.py [--points cfg4_vamp_qpsk:1/0,...] [--tag name]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]

import golden_io as gio  # noqa: E402
import oracle.amp_oracle as O  # noqa: E402


def gpu_denoiser(cfg_dev, stats, ref_den):
    import torch
    from vamp import block_denoise

    def den(r, tau, cfg):
        rd = torch.from_numpy(np.ascontiguousarray(r.astype(np.complex64))).to('cuda')
        xm, var = block_denoise(cfg_dev, rd, float(tau), mode=0)
        xm = xm.cpu().numpy()[..., 0]
        var = var.cpu().numpy()[..., 0]
        if 'first' not in stats:
            xr, vr = ref_den(r, tau, cfg)
            with np.errstate(invalid='ignore', divide='ignore'):
                rel = np.abs(var.astype(np.float64) - vr) / np.maximum(np.abs(vr), 1e-30)
            stats['first'] = (float(np.nanmax(rel)), float(np.nanmean(rel)),
                              float((var.astype(np.float64) - vr).sum() / max(abs(vr.sum()), 1e-30)))
        return xm, var
    return den


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', default='')
    ap.add_argument('--tag', default=os.path.basename(os.environ.get('AMP_LIB_PATH', 'default')))
    ap.add_argument('--oracle', action='store_true', help='also run the float64 oracle loop')
    a = ap.parse_args()
    from test_gpu_vamp import _config, _regen_inputs
    curves = gio.g4_curves()
    pts = []
    if a.points:
        pts = [tuple(p.split(':')) for p in a.points.split(',')]
    else:
        for n, ent in curves.items():
            if ent.get('algo') == 'vamp':
                pts += [(n, k) for k, rec in sorted(ent['points'].items()) if 'T_runs' in rec]
    for name, key in pts:
        ent = curves[name]
        ref = ent['points'][key]
        seed, ebn0 = int(key.split('/')[0]), float(key.split('/')[1])
        cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'], iterations=ent['iterations'],
                      device='cpu')
        inp = _regen_inputs(cfg, seed, ebn0)
        cfg_dev = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'],
                          iterations=ent['iterations'])
        ocfg = O.OracleConfig(ent['Nt'], ent['Na'], ent['Nr'], B=ent['B'], alphabet=ent['alphabet'],
                              iterations=ent['iterations'])
        np_ = lambda t: t.numpy()[..., 0] if t.dim() == 3 else t.numpy()   # noqa: E731
        args = (np_(inp['U']), np_(inp['s']), np_(inp['Vh']), np_(inp['y']), inp['SNR'], ocfg)
        line = f'{a.tag:24s} {name} {key}: ref T {int(ref["T"])} runs {sorted(int(t) for t in ref.get("T_runs", []))}'
        if a.oracle:
            line += f' | oracle64 {O.vamp_detect(*args)["T"]}'
        stats = {}
        saved = O.block_denoise
        O.block_denoise = gpu_denoiser(cfg_dev, stats, saved)
        try:
            T = O.vamp_detect(*args)['T']
        finally:
            O.block_denoise = saved
        mx, mean, bias = stats['first']
        line += f' | oracle+gpu-den {T}  (it0 var rel err max {mx:.2e} mean {mean:.2e} bias {bias:.2e})'
        print(line, flush=True)


if __name__ == '__main__':
    main()
