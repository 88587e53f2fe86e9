"""Diagnostic: side-by-side epochs vs sequential forwards, bit by bit, per epoch (cfg2 shape).
  python tools/epochs_diag.py ALPHABET EBN0 E [repeats]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]
import torch  # noqa: E402
from test_gpu_epochs import _cfg, _epochs  # noqa: E402
from vamp import VAMP  # noqa: E402

alph, ebn0, E = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
rep = int(sys.argv[4]) if len(sys.argv) > 4 else 2
dev = torch.device('cuda:0')
cfg = _cfg(64, 4, 128, 1024, alph)
chan, SNR, eps = _epochs(cfg, E, ebn0, seed=3)
mv = lambda t: t.to(dev).contiguous()  # noqa: E731
U, s, Vh = (mv(t) for t in chan)
det = VAMP(cfg)
seq = []
for x, sym, idx, y in eps:
    L = det(U, s, Vh, mv(y), SNR, mv(x), sym, idx)
    seq.append((int(L.loss['T']), det.last.r.clone(), det.last.xmmse.clone()))
for k in range(rep):
    Ls = det.forward_epochs(U, s, Vh, [mv(e[3]) for e in eps], SNR, [mv(e[0]) for e in eps], [e[1] for e in eps],
                            [e[2] for e in eps])
    r, xm, _ = det.last_epochs
    out = []
    for e in range(E):
        dr = (r[e].view(torch.int32) != seq[e][1].view(torch.int32)).sum().item()
        dx = (xm[e].view(torch.int32) != seq[e][2].view(torch.int32)).sum().item()
        out.append(f'e{e}:T{int(Ls[e].loss["T"])}/{seq[e][0]} dr{dr} dx{dx}')
    print(f'rep {k}:', ' '.join(out), flush=True)
