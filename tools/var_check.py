"""Diagnostic companion of epochs_diag.py (DIAG_DUMP=1): recompute the persistent engine's
denoiser variance in float64 from the dumped r and 1/sigma2 (vamp.py:109-118) and report the
relative error of the kernel's float32 var per lane group of the wave (lanes 0-15, ..., 48-63;
cfg2: M = 16, one section per 16 lanes), to see whether one lane group is off.
  python tools/var_check.py DUMP.npy ALPHABET"""
import sys

import numpy as np


def main():
    d = np.load(sys.argv[1])            # [iters, nwg, 4, 16, 2N]
    alph = sys.argv[2]
    if alph == 'QPSK':
        a = np.array([1, 1j, -1, -1j])        # config.py QPSK table
    else:
        raise SystemExit('QPSK only')
    iters, nwg, _, R, twoN = d.shape
    N = twoN // 2
    M = 16
    rel = {g: [] for g in range(4)}
    for t in range(iters):
        for w in range(nwg):
            inv = np.float32(d[t, w, 3, 1, N])
            if not np.isfinite(inv) or inv == 0:
                continue
            r = d[t, w, 1, :, 0::2].astype(np.float32) + 1j * d[t, w, 1, :, 1::2].astype(np.float32)
            var = d[t, w, 3, :, :N].astype(np.float64)
            ur = (r.real * inv).astype(np.float32).astype(np.float64)
            ui = (r.imag * inv).astype(np.float32).astype(np.float64)
            xi = ur[..., None] * a.real + ui[..., None] * a.imag            # [16, N, K]
            xs = xi.reshape(R, N // M, M, -1)
            eta = np.exp(xs - xs.max(axis=(2, 3), keepdims=True))
            Z = eta.sum(axis=(2, 3), keepdims=True)
            xm = (eta * a).sum(axis=3) / Z[..., 0]
            P = eta.sum(axis=3) / Z[..., 0]
            v = np.abs(xm) ** 2 * (1 - P) + (np.abs(xm[..., None] - a) ** 2 * eta).sum(axis=3) / Z[..., 0]
            v = v.reshape(R, N)
            e = np.abs(var - v) / np.maximum(np.abs(v), 1e-30)
            for g in range(4):
                rel[g].append(e[:, g * M:(g + 1) * M].ravel())
    for g in range(4):
        x = np.concatenate(rel[g])
        print(f'lanes {16 * g:2d}-{16 * g + 15:2d}: n={x.size} rel err median {np.median(x):.2e} '
              f'p99.9 {np.quantile(x, 0.999):.2e} max {x.max():.2e} n>1e-3: {(x > 1e-3).sum()}')


if __name__ == '__main__' and len(sys.argv) <= 3:
    main()


def explain(path, alph='QPSK', limit=12):
    """For each var element with a relative error > 1e-3: the exclusive section sum ze the
    kernel's var implies (var = |x|^2 ze / Z + vs / Z, amp_denoise.h) against the true one and
    the four butterfly contributions (xor 1, xor 2, half-row mirror, row mirror), to see which
    step of group_sum_excl_c delivered a wrong value."""
    d = np.load(path)
    a = np.array([1, 1j, -1, -1j])
    iters, nwg, _, R, twoN = d.shape
    N, M = twoN // 2, 16
    shown = 0
    for t in range(iters):
        for w in range(nwg):
            inv = np.float32(d[t, w, 3, 1, N])
            if not np.isfinite(inv) or inv == 0:
                continue
            r = d[t, w, 1, :, 0::2].astype(np.float64) + 1j * d[t, w, 1, :, 1::2]
            var = d[t, w, 3, :, :N].astype(np.float64)
            for row in range(R):
                for s in range(N // M):
                    sec = r[row, s * M:(s + 1) * M]
                    ur = (sec.real * inv).astype(np.float32).astype(np.float64)
                    ui = (sec.imag * inv).astype(np.float32).astype(np.float64)
                    xi = ur[:, None] * a.real + ui[:, None] * a.imag
                    eta = np.exp(xi - xi.max())
                    zt = eta.sum(1)
                    Z = zt.sum()
                    xm = (eta * a).sum(1) / Z
                    vs = (np.abs(xm[:, None] - a) ** 2 * eta).sum(1)
                    ze = Z - zt
                    v = np.abs(xm) ** 2 * ze / Z + vs / Z
                    vg = var[row, s * M:(s + 1) * M]
                    bad = np.nonzero(np.abs(vg - v) > 1e-3 * np.abs(v))[0]
                    for m in bad:
                        zimp = (vg[m] * Z - vs[m]) / max(np.abs(xm[m]) ** 2, 1e-300)
                        idx = np.arange(M)
                        c1 = zt[m ^ 1]
                        c2 = zt[(idx ^ (m ^ 2)) < 2].sum() if False else zt[[m ^ 2, m ^ 3]].sum()
                        h = m & ~7
                        c4 = zt[[i for i in range(h, h + 8) if (i & 4) != (m & 4)]].sum()
                        c8 = zt[[i for i in range(M) if (i & 8) != (m & 8)]].sum()
                        zd, vd = d[t, w, 4, row, s * M + m], d[t, w, 4, row, N + s * M + m]
                        print(f'    dumped ze {zd:.6e} vs {vd:.6e}; f64 vs {vs[m]:.6e}')
                        print(f't{t} wg{w} row{row} sec{s} m{m}: var gpu {vg[m]:.6e} f64 {v[m]:.6e}; '
                              f'ze implied {zimp:.6e} true {ze[m]:.6e}; steps xor1 {c1:.3e} xor2 {c2:.3e} '
                              f'half {c4:.3e} row {c8:.3e}; zt[m] {zt[m]:.3e}')
                        shown += 1
                        if shown >= limit:
                            return


if __name__ == '__main__' and len(sys.argv) > 3 and sys.argv[3] == 'explain':
    explain(sys.argv[1], sys.argv[2])
