"""Diagnostic: side-by-side epochs vs sequential forwards, bit by bit, per epoch (cfg2 shape).
  python tools/epochs_diag.py ALPHABET EBN0 E [repeats]

Besides the r / xmmse words it compares the exchange records every workgroup published per
iteration (the 32-byte granule pairs of amp_persist.h part_publish, left in the workspace after the
launch): for every epoch the first iteration whose published partials differ from the sequential
forward's, and which workgroups differ there.  If the partials of iteration t-1 are identical
everywhere but a few workgroups publish different partials at t, those workgroups computed from
identical inputs differently (a local fault: LDS, scratch, a stale global read); if every
workgroup differs at t although the partials of t-1 were identical, the gathered scalars differed
(an exchange fault).  AMP_PERSIST_WG2=1 runs two workgroups per CU (8 cfg2 epochs per launch)."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import amp_native as nat  # noqa: E402
from test_gpu_epochs import _cfg, _epochs  # noqa: E402
from vamp import VAMP  # noqa: E402


def granules(ws: torch.Tensor, d, k, iters, epochs):
    off = (C.c_uint64 * 5)()
    nat.check(nat.lib().amp_vamp_debug_offsets(C.byref(d), k, iters, epochs, off), 'amp_vamp_debug_offsets')
    nwg = epochs * ((d.B + 15) // 16)
    n = iters * nwg * 32
    g = ws[int(off[0]):int(off[0]) + n].cpu().numpy().view(np.uint32).reshape(iters, nwg, 8)
    return g


def main():
    alph, ebn0, E = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
    rep = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    dev = torch.device('cuda:0')
    cfg = _cfg(64, 4, 128, 1024, alph)
    chan, SNR, eps = _epochs(cfg, E, ebn0, seed=3)
    mv = lambda t: t.to(dev).contiguous()  # noqa: E731
    U, s, Vh = (mv(t) for t in chan)
    det = VAMP(cfg)
    d = cfg.dims()
    k, iters, wpe = 64, cfg.N_Layers, cfg.B // 16
    print('max_epochs', det.max_epochs(k), 'WG2', os.environ.get('AMP_PERSIST_WG2'), flush=True)
    dump_on = os.environ.get('DIAG_DUMP', '0') == '1'
    twoN = 2 * cfg.Nt
    dump = torch.zeros(iters * E * wpe * 5 * 16 * twoN if dump_on else 1, dtype=torch.float32, device=dev)
    if dump_on:
        nat.lib().amp_vamp_debug_dump(C.c_void_p(dump.data_ptr()))

    def dumped(nwg):
        torch.cuda.synchronize()
        return dump[:iters * nwg * 5 * 16 * twoN].view(iters, nwg, 5, 16, twoN).cpu().numpy().copy()

    seq = []
    for x, sym, idx, y in eps:
        if dump_on:
            dump.zero_()
        L = det(U, s, Vh, mv(y), SNR, mv(x), sym, idx)
        T = int(L.loss['T'])
        g = granules(det._bufs.ws, d, k, iters, 1)
        seq.append((T, det.last.r.clone(), det.last.xmmse.clone(), g, dumped(wpe) if dump_on else None))
    for rr in range(rep):
        if dump_on:
            dump.zero_()
        Ls = det.forward_epochs(U, s, Vh, [mv(e[3]) for e in eps], SNR, [mv(e[0]) for e in eps],
                                [e[1] for e in eps], [e[2] for e in eps])
        r, xm, _ = det.last_epochs
        torch.cuda.synchronize()
        ws = nat.WORKSPACE.get(dev, 'vamp_epochs', 0)
        g = granules(ws, d, k, iters, E)
        dd = dumped(E * wpe) if dump_on else None
        if dump_on and os.environ.get('DIAG_SAVE'):
            np.save(f"{os.environ['DIAG_SAVE']}_rep{rr}.npy", dd)
            np.save(f"{os.environ['DIAG_SAVE']}_rep{rr}_small.npy", dd[:, :2])
        out, detail = [], []
        for e in range(E):
            T = int(Ls[e].loss['T'])
            dr = (r[e].view(torch.int32) != seq[e][1].view(torch.int32)).sum().item()
            dx = (xm[e].view(torch.int32) != seq[e][2].view(torch.int32)).sum().item()
            ge = g[:, e * wpe:(e + 1) * wpe, :]
            gs = seq[e][3]
            first = None
            for t in range(min(T, seq[e][0])):
                # payload words: sumvar lo/hi, notclose, maxabs, minsecmax (tags differ by generation)
                pe = ge[t][:, [0, 1, 2, 4, 5]]
                ps = gs[t][:, [0, 1, 2, 4, 5]]
                diff = np.nonzero((pe != ps).any(axis=1))[0]
                # tags must be the launch's (gen * (iters + 1) + t + 1): constant offset per launch
                if first is None and diff.size:
                    first = (t, diff.tolist()[:12], int(diff.size))
                    w = int(diff[0])
                    f64 = lambda q: q[:2].copy().view(np.float64)[0]  # noqa: E731
                    f32 = lambda q, i: q[i:i + 1].copy().view(np.float32)[0]  # noqa: E731
                    detail.append(f'      e{e} t{t} wg{w}: seq sumvar={f64(gs[t][w])!r} nc={gs[t][w][2]} '
                                  f'max={f32(gs[t][w], 4)!r} minsec={f32(gs[t][w], 5)!r} | '
                                  f'epochs sumvar={f64(ge[t][w])!r} nc={ge[t][w][2]} max={f32(ge[t][w], 4)!r} '
                                  f'minsec={f32(ge[t][w], 5)!r}')
            if dump_on:
                names = ('w', 'r', 'xmmse', 'var|wavesums', 'ze|vs')
                found = None
                for t in range(min(T, seq[e][0])):
                    for ph in range(5):
                        a = dd[t, e * wpe:(e + 1) * wpe, ph]
                        b = seq[e][4][t, :, ph]
                        neq = a.view(np.uint32) != b.view(np.uint32)
                        if neq.any():
                            wgs = np.nonzero(neq.any(axis=(1, 2)))[0]
                            w0 = int(wgs[0])
                            rows, cols = np.nonzero(neq[w0])
                            found = (t, names[ph], wgs.tolist()[:10], int(neq.sum()), w0, rows.tolist()[:8],
                                     cols.tolist()[:8], float(np.abs(a[w0] - b[w0]).max()))
                            break
                    if found:
                        break
                detail.append(f'      e{e} first state diff (t, phase, wgs, n, wg, rows, cols, maxabs): {found}')
            tags = ge[:T, :, 3] - np.arange(1, T + 1)[:, None]
            tag_ok = bool((tags == tags[0, 0]).all() and (ge[:T, :, 7] == ge[:T, :, 3]).all())
            out.append(f'e{e}:T{T}/{seq[e][0]} dr{dr} dx{dx} tags_ok={tag_ok} first_diff={first}')
        print(f'rep {rr}:', flush=True)
        for o in out:
            print('   ', o, flush=True)
        for o in detail:
            print(o, flush=True)


if __name__ == '__main__':
    main()
