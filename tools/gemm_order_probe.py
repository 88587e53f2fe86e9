#!/usr/bin/env python3
"""Diagnostic (CPU): how the summation order / accuracy of VAMP's two per-iteration GEMMs
(vamp.py:67, 72) moves the reference's allclose early exit (vamp.py:185) at the golden points where
that exit is decided by rounding.  Runs the oracle restatement of the reference (float64 denoiser,
pinned to the reference by the g1-g4 goldens) with its c64 products computed as:

  blas      numpy / BLAS (the reference's CPU path; what the goldens were made with)
  exact     float64 products and sums, rounded to complex64 once (the most accurate)
  seq32     sequential float32 multiply-add over K in natural order (each step rounded: the
            accumulation pattern of an MFMA engine's f32 accumulator)
  seq32rN   the same in a seeded random K order (N = seed)
  blk32     eight interleaved float32 partial sums over K, added at the end (a BLAS-like kernel)
  grpG      per group of G K-terms one exact dot product added to the float32 accumulator (an MFMA
            engine's pattern: grp32 for the bf16x3 16x16x32 tiles, grp2 for the f32 32x32x2 ones)

  python tools/gemm_order_probe.py [--points cfg4_vamp_qpsk:1/0,...] [--variants blas,exact,seq32]
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

F32, F64 = np.float32, np.float64


def _seq32(order=None, nacc=1):
    """C = A @ B with float32 accumulation: for k in `order`, C_r += A_r B_r - A_i B_i and
    C_i += A_r B_i + A_i B_r, every product exact and every add rounded to float32 (an FMA per term);
    nacc interleaved partial sums (k mod nacc) added at the end."""
    def mm(a, b):
        a = np.asarray(a, np.complex64)
        b = np.asarray(b, np.complex64)
        K = a.shape[1]
        ks = np.arange(K) if order is None else order(K)
        ar, ai = a.real.astype(F64), a.imag.astype(F64)
        br, bi = b.real.astype(F64), b.imag.astype(F64)
        accs = [[np.zeros((a.shape[0], b.shape[1]), F32), np.zeros((a.shape[0], b.shape[1]), F32)] for _ in range(nacc)]
        for j, k in enumerate(ks):
            cr, ci = accs[j % nacc]
            x_r, x_i = ar[:, k:k + 1], ai[:, k:k + 1]
            y_r, y_i = br[k:k + 1, :], bi[k:k + 1, :]
            cr = (cr + x_r * y_r).astype(F32)
            cr = (cr - x_i * y_i).astype(F32)
            ci = (ci + x_r * y_i).astype(F32)
            ci = (ci + x_i * y_r).astype(F32)
            accs[j % nacc] = [cr, ci]
        cr, ci = accs[0]
        for c in accs[1:]:
            cr = (cr + c[0]).astype(F32)
            ci = (ci + c[1]).astype(F32)
        return (cr + 1j * ci).astype(np.complex64)
    return mm


def _grp32(kg=32):
    """An MFMA engine's accumulation: per K group of kg terms one exact dot product (float64),
    added to the float32 accumulator with one rounding (C_r += A_r.B_r, then C_r -= A_i.B_i; C_i
    likewise)."""
    def mm(a, b):
        a = np.asarray(a, np.complex64)
        b = np.asarray(b, np.complex64)
        K = a.shape[1]
        ar, ai = a.real.astype(F64), a.imag.astype(F64)
        br, bi = b.real.astype(F64), b.imag.astype(F64)
        cr = np.zeros((a.shape[0], b.shape[1]), F32)
        ci = np.zeros_like(cr)
        for k0 in range(0, K, kg):
            s = slice(k0, k0 + kg)
            cr = (cr + ar[:, s] @ br[s]).astype(F32)
            cr = (cr - ai[:, s] @ bi[s]).astype(F32)
            ci = (ci + ar[:, s] @ bi[s]).astype(F32)
            ci = (ci + ai[:, s] @ br[s]).astype(F32)
        return (cr + 1j * ci).astype(np.complex64)
    return mm


def variant_mm(v):
    if v == 'blas':
        return None
    if v == 'exact':
        return lambda a, b: (np.asarray(a, np.complex128) @ np.asarray(b, np.complex128)).astype(np.complex64)
    if v == 'seq32':
        return _seq32()
    if v.startswith('seq32r'):
        rs = int(v[6:] or 0)
        return _seq32(order=lambda K, rs=rs: np.random.default_rng(rs).permutation(K))
    if v.startswith('grp'):
        return _grp32(int(v[3:] or 32))
    if v == 'blk32':
        return _seq32(nacc=8)
    raise ValueError(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', default='cfg4_vamp_qpsk:0/0,cfg4_vamp_qpsk:1/0,cfg4_vamp_qpsk:2/0')
    ap.add_argument('--variants', default='blas,exact,blk32,seq32,seq32r1,seq32r2')
    a = ap.parse_args()
    from test_gpu_vamp import _config, _regen_inputs
    curves = gio.g4_curves()
    for p in a.points.split(','):
        name, key = p.split(':')
        ent = curves[name]
        ref = ent['points'][key]
        seed, ebn0 = int(key.split('/')[0]), float(key.split('/')[1])
        cfg = _config(ent['Nt'], ent['Na'], ent['Nr'], ent['B'], ent['alphabet'], iterations=ent['iterations'],
                      device='cpu')
        inp = _regen_inputs(cfg, seed, ebn0)
        ocfg = O.OracleConfig(ent['Nt'], ent['Na'], ent['Nr'], B=ent['B'], alphabet=ent['alphabet'],
                              iterations=ent['iterations'])
        np_ = lambda t: t.numpy()[..., 0] if t.dim() == 3 else t.numpy()   # noqa: E731
        args = (np_(inp['U']), np_(inp['s']), np_(inp['Vh']), np_(inp['y']), inp['SNR'], ocfg)
        out = {}
        for v in a.variants.split(','):
            # 'V+y': the variant for the y~ product too; 'y:V': for y~ only
            if v.startswith('y:'):
                mm, my = None, variant_mm(v[2:])
            elif v.endswith('+y'):
                mm = my = variant_mm(v[:-2])
            else:
                mm, my = variant_mm(v), None
            out[v] = O.vamp_detect(*args, mm=mm, mm_y=my)['T']
            print(f'  {name} {key} {v}: T {out[v]}', flush=True)
        print(f'{name} {key}: reference T {int(ref["T"])} runs {sorted(int(t) for t in ref.get("T_runs", []))} | '
              + ' '.join(f'{v}={t}' for v, t in out.items()), flush=True)


if __name__ == '__main__':
    main()
