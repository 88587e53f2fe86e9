#!/usr/bin/env python3
"""Diagnostic (CPU): which part of the float32 denoiser's arithmetic moves VAMP's allclose early
exit (vamp.py:185) away from the reference's at the reference-moved golden points.

Runs oracle.vamp_detect with the reference's float64 denoiser, with float32 models of a denoiser
('f32': the round-4 model, whose Z - Z_m is a float32 subtraction; 'gs...': the scalar gfx950 form
of amp_denoise.h operation for operation, exclusive sums included), and with hybrids that give one
part of a model more precision, and prints T per variant beside the reference's recorded T runs.
Outcome: the round-4 model's T = 20 came from its cancelling subtraction,
which the GPU code does not have; the faithful model and the GPU's own denoiser inside the oracle
loop (tools/den_isolate.py) give the reference's T.

  python tools/den_precision_probe.py [--points cfg4_vamp_qpsk:1/0.0,...]
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


def den_variant(kind):
    """A float32-model denoiser with the parts named in `kind` in float64:
    'exp'   eta = float32(exp(float64 argument)) (correctly rounded weights);
    'exp64' eta kept in float64;
    'sum'   every sum (Z, Z_m, sum a eta, sum |x-a|^2 eta) in float64;
    'x64'   x = sum a eta / Z kept in float64 for the variance;
    'gpu'   the argument formed as the GPU does: exp2((xi - smax) * log2e), float32 each step."""
    kinds = set(kind.split('+')) if kind else set()

    def den(r, tau, cfg):
        B = r.shape[0]
        sv = np.asarray(r, O.C64).reshape(B, cfg.L, cfg.M)
        it = F32(1) / F32(tau)
        ur = (sv.real.astype(F32) * it).astype(F32)
        ui = (sv.imag.astype(F32) * it).astype(F32)
        sym = cfg.symbols.astype(np.complex64)
        cre, cim = sym.real.astype(F32), sym.imag.astype(F32)
        with np.errstate(under='ignore', invalid='ignore', divide='ignore', over='ignore'):
            xi = (ur[..., None] * cre + ui[..., None] * cim).astype(F32)
            smax = xi.max(axis=(2, 3), keepdims=True)
            if 'gpu' in kinds:
                d = ((xi - smax).astype(F32) * F32(1.4426950408889634)).astype(F32)
                eta = np.exp2(d.astype(F64)).astype(F32)
            elif 'exp64' in kinds:
                eta = np.exp(xi.astype(F64) - smax.astype(F64))
            elif 'exp' in kinds:
                eta = np.exp(xi.astype(F64) - smax.astype(F64)).astype(F32)
            else:
                eta = np.exp((xi - smax).astype(F32)).astype(F32)
            allsum = 'sum' in kinds
            az = F64 if (allsum or 'sz' in kinds) else F32      # Z, Z_m, Z - Z_m, 1 / Z
            ax = F64 if (allsum or 'sx' in kinds) else F32      # sum a eta
            av = F64 if (allsum or 'sv' in kinds) else F32      # sum |x - a|^2 eta
            af = F64 if (allsum or 'fin' in kinds) else F32     # the final var formula
            zm = eta.astype(az).sum(axis=-1, dtype=az)
            z = zm.sum(axis=2, keepdims=True, dtype=az)
            iz = (az(1) / z).astype(az)
            if 'excl' in kinds:
                ze = (z - zm).astype(F64).astype(az) if az == F64 else \
                    (zm.astype(F64).sum(axis=2, keepdims=True) - zm.astype(F64)).astype(F32)
            else:
                ze = (z - zm).astype(az)
            xr = ((eta.astype(ax) * cre.astype(ax)).sum(axis=-1, dtype=ax) * iz).astype(ax)
            xim = ((eta.astype(ax) * cim.astype(ax)).sum(axis=-1, dtype=ax) * iz).astype(ax)
            if 'x64' not in kinds:
                xr, xim = xr.astype(F32), xim.astype(F32)
            dr, di = xr[..., None].astype(av) - cre.astype(av), xim[..., None].astype(av) - cim.astype(av)
            vs = ((dr * dr + di * di) * eta.astype(av)).sum(axis=-1, dtype=av)
            var = ((xr.astype(af) ** 2 + xim.astype(af) ** 2) * (ze.astype(af) * iz.astype(af))
                   + vs.astype(af) * iz.astype(af)).astype(F32)
        return (xr + 1j * xim).astype(O.C64).reshape(B, -1), var.reshape(B, -1)
    return den


def _fma32(a, b, c):
    """float32 fma (exact product, one rounding)."""
    return (a.astype(F64) * b.astype(F64) + c.astype(F64)).astype(F32)


def den_gpu_scalar(zsum='f32', vsum='f32'):
    """The scalar denoiser of amp_denoise.h (denoise_sections_g), operation for operation:
    fma logits, exp2((xi - smax) * log2e) on v_exp_f32 (modelled as correctly rounded), per
    position sums in k order with fma, the butterfly exclusive sum of Z over the section's lanes,
    v_rcp_f32 (modelled as correctly rounded), var = |x|^2 (ze iz) + vs iz.
    zsum='f64': Z and the exclusive sums carried in float64 (the candidate fix);
    vsum='f64': the variance sum and the final formula in float64."""
    def den(r, tau, cfg):
        B = r.shape[0]
        sv = np.asarray(r, O.C64).reshape(B, cfg.L, cfg.M)
        it = F32(1) / F32(tau)
        ur = (sv.real.astype(F32) * it).astype(F32)
        ui = (sv.imag.astype(F32) * it).astype(F32)
        sym = cfg.symbols.astype(np.complex64)
        cre, cim = sym.real.astype(F32), sym.imag.astype(F32)
        K, M = len(cre), cfg.M
        with np.errstate(under='ignore', invalid='ignore', divide='ignore', over='ignore'):
            xk = [_fma32(ur, np.full_like(ur, cre[k]), (ui * cim[k]).astype(F32)) for k in range(K)]
            lmax = xk[0]
            for k in range(1, K):
                lmax = np.maximum(lmax, xk[k])
            smax = lmax.max(axis=2, keepdims=True)
            zm = np.zeros_like(ur); a = np.zeros_like(ur); b = np.zeros_like(ur)
            es = []
            for k in range(K):
                d = ((xk[k] - smax).astype(F32) * F32(1.4426950408889634)).astype(F32)
                e = np.exp2(d.astype(F64)).astype(F32)
                es.append(e)
                zm = (zm + e).astype(F32)
                a = _fma32(np.full_like(e, cre[k]), e, a)
                b = _fma32(np.full_like(e, cim[k]), e, b)
            zt = zm.astype(F64 if zsum == 'f64' else F32)
            ze = np.zeros_like(zt)
            idx = np.arange(M)
            o = 1
            while o < M:
                p = zt[..., idx ^ o]
                ze = (ze + p).astype(zt.dtype)
                zt = (zt + p).astype(zt.dtype)
                o *= 2
            if zsum == 'f64':
                iz64 = 1.0 / zt
                iz = iz64.astype(F32)
                xr = (a.astype(F64) * iz64).astype(F32); xi = (b.astype(F64) * iz64).astype(F32)
            else:
                iz = (F32(1) / zt).astype(F32)
                xr = (a * iz).astype(F32); xi = (b * iz).astype(F32)
            if vsum == 'f64':
                vs = np.zeros(ur.shape, F64)
                for k in range(K):
                    dr = xr.astype(F64) - cre[k]; di = xi.astype(F64) - cim[k]
                    vs = vs + (dr * dr + di * di) * es[k]
            else:
                vs = np.zeros_like(ur)
                for k in range(K):
                    dr = (xr - cre[k]).astype(F32); di = (xi - cim[k]).astype(F32)
                    vs = _fma32(_fma32(dr, dr, (di * di).astype(F32)), es[k], vs)
            if zsum == 'f64' or vsum == 'f64':
                izd = 1.0 / zt.astype(F64)
                var = ((xr.astype(F64) ** 2 + xi.astype(F64) ** 2) * (ze.astype(F64) * izd)
                       + vs.astype(F64) * izd).astype(F32)
            else:
                x2 = (xr * xr + (xi * xi).astype(F32)).astype(F32)
                var = ((x2 * (ze * iz).astype(F32)).astype(F32) + (vs * iz).astype(F32)).astype(F32)
        return (xr + 1j * xi).astype(O.C64).reshape(B, -1), var.reshape(B, -1)
    return den


def run_point(name, key, variants):
    from test_gpu_vamp import _config, _regen_inputs
    ent = gio.g4_curves()[name]
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
    saved = O.block_denoise
    for v in variants:
        try:
            if v.startswith('gs'):      # gs, gs-z64, gs-v64, gs-z64-v64: den_gpu_scalar
                O.block_denoise = den_gpu_scalar('f64' if 'z64' in v else 'f32', 'f64' if 'v64' in v else 'f32')
            elif v != 'ref':
                O.block_denoise = den_variant('' if v == 'f32' else v)
            out[v] = O.vamp_detect(*args)['T']
        finally:
            O.block_denoise = saved
    print(f'{name} {key}: ref T {ref["T"]} runs {sorted(int(t) for t in ref.get("T_runs", []))} '
          f'den-runs {sorted(int(t) for t in ref.get("T_runs_den", []))} | ' +
          ' '.join(f'{v}={t}' for v, t in out.items()), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', default='')
    ap.add_argument('--variants', default='ref,f32,gpu,exp,exp64,sum,x64,exp+sum,exp+sum+x64,gpu+sum+x64')
    a = ap.parse_args()
    pts = []
    if a.points:
        for p in a.points.split(','):
            n, k = p.split(':')
            pts.append((n, k))
    else:
        for n, ent in gio.g4_curves().items():
            if ent.get('algo') == 'vamp':
                pts += [(n, k) for k, rec in sorted(ent['points'].items()) if 'T_runs' in rec]
    for n, k in pts:
        run_point(n, k, a.variants.split(','))


if __name__ == '__main__':
    main()
