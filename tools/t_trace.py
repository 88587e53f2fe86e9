#!/usr/bin/env python3
"""Diagnostic (GPU): the early-exit trajectory of amp_vamp_run at one golden point — for every
iteration cap k = 1..max, the var output after k iterations, so that the host can form the
reference's exit test between consecutive iterations (vamp.py:185: allclose(var_k, var_{k-1}),
rtol 1e-5, atol 1e-8) and the batch mean var.  Prints per k: T reached, mean var, notclose count;
saves var_k for k in --save into gpurun_out/t_trace_<variant>.npz.

  python tools/t_trace.py [--point cfg4_vamp_qpsk:1/0] [--save 10,11,12]
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
from test_gpu_vamp import VARIANTS, _config, _regen_inputs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--point', default='cfg4_vamp_qpsk:1/0')
    ap.add_argument('--save', default='10,11,12')
    ap.add_argument('--variants', default='launches,persistent,persistent-f32,persistent-h2')
    a = ap.parse_args()
    from vamp import VAMP
    name, key = a.point.split(':')
    ent = gio.g4_curves()[name]
    seed, ebn0 = int(key.split('/')[0]), float(key.split('/')[1])
    save = {int(k) for k in a.save.split(',') if k}
    os.makedirs('gpurun_out', exist_ok=True)
    for variant in a.variants.split(','):
        eng, gemm = VARIANTS[variant]
        prev = None
        keep = {}
        for k in range(1, ent['iterations'] + 1):
            cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'], iterations=k)
            inp = _regen_inputs(cfg, seed, ebn0)
            det = VAMP(cfg, engine=eng, gemm=gemm)
            T = det.detect(inp['U'], inp['s'], inp['Vh'], inp['y'], inp['SNR'])
            torch.cuda.synchronize()
            var = T.buf.var.view(cfg.B, -1)[:, :cfg.Nt].float().cpu().numpy().copy()
            line = f'{variant:15s} k={k:2d} mean_var={np.float32(var.astype(np.float64).mean()):.7e}'
            if prev is not None:
                nc = int((~np.isclose(var, prev, rtol=1e-5, atol=1e-8)).sum())
                d = np.abs(var - prev)
                line += f' notclose={nc:8d} max|dvar|={d.max():.3e}'
            print(line, flush=True)
            if k in save:
                keep[f'var{k}'] = var
            prev = var
        np.savez_compressed(f'gpurun_out/t_trace_{variant}.npz', **keep)


if __name__ == '__main__':
    main()
