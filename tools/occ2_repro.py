#!/usr/bin/env python3
"""Diagnostic (round 4): is the two-waves-per-SIMD corruption of the packed
denoiser tied to the VGPR spills of the OCC = 2 instantiation?  Runs 8 cfg2 epochs in one launch
(two workgroups per CU) `reps` times against 8 sequential forwards and counts the repetitions
whose r / xmmse / var words differ.  The library under test comes from AMP_LIB_PATH:
  lib/libampsparc.so                  production (scalar denoiser at OCC = 2)
  lib_diag/libampsparc_pk_du4.so      packed denoiser at OCC = 2, QPSK DU = 4 (20 VGPR spills)
  lib_diag/libampsparc_pk_du2.so      packed denoiser at OCC = 2, QPSK DU = 2 (no VGPR spill)

  AMP_LIB_PATH=... python tools/occ2_repro.py [reps]
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', 'tests'), os.path.join(HERE, '..'),
                os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]
import torch  # noqa: E402
from test_gpu_epochs import _cfg, _epochs, _run_both  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device('cuda', 0)
    print('lib', os.environ.get('AMP_LIB_PATH', 'default'))
    for alphabet, ebn0 in (('QPSK', 6.0), ('QPSK', 2.0), ('16QAM', 8.0)):
        cfg = _cfg(64, 4, 128, 1024, alphabet)
        chan, SNR, eps = _epochs(cfg, 8, ebn0, seed=3)
        det, seq, grp = _run_both(cfg, chan, SNR, eps, dev)
        mv = lambda t: t.to(dev).contiguous()  # noqa: E731
        U, s, Vh = (mv(t) for t in chan)
        bad = 0
        first = None
        for rep in range(reps):
            if rep:
                grp = det.forward_epochs(U, s, Vh, [mv(e[3]) for e in eps], SNR, [mv(e[0]) for e in eps],
                                         [e[1] for e in eps], [e[2] for e in eps])
            r, xm, var = det.last_epochs
            diff = []
            for e, (ls, st, r0, x0, v0) in enumerate(seq):
                nv = int((var[e].view(torch.int32) != v0.view(torch.int32)).sum())
                nr = int((r[e].view(torch.int32) != r0.view(torch.int32)).sum())
                if nv or nr or int(grp[e].loss['T']) != int(ls['T']):
                    diff.append((e, nr, nv))
            if diff:
                bad += 1
                first = first or (rep, diff[:3])
        print(f'{alphabet} {ebn0:4.1f} dB: {bad} of {reps} repetitions differ from the sequential forwards'
              + (f'; first {first}' if first else ''), flush=True)


if __name__ == '__main__':
    main()
