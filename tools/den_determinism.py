"""Diagnostic: run-to-run bit identity and float64 accuracy of the launch-engine block denoiser
(amp_block_denoise, vamp.py:96-119; many waves per SIMD) per 16-lane group, QPSK / 16-QAM.
  python tools/den_determinism.py ALPHABET [reps]
Draws r as a noisy section-sparse signal (one constellation point per section plus noise), runs
the denoiser `reps` times, counts words that differ from the first run, and reports the relative
error of var against a float64 recompute per lane group (position m within the 64-lane wave)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..'), os.path.join(HERE, '..', 'amp-sparc-spatialmodulation_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from config import Config  # noqa: E402
from vamp import block_denoise  # noqa: E402


def main():
    alph = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    Nt, Na, B = 256, 4, 8192          # M = 64: one section per wave
    if len(sys.argv) > 3:
        Nt, Na = int(sys.argv[3]), int(sys.argv[4])
    cfg = Config(Nt, Na, 2 * Nt, 1, 1, batch=B, generator_mode='sparc', iterations=20, alphabet=alph,
                 channel_profile='uniform', channel_truncation='tail', device='cuda')
    M = Nt // Na
    sym = np.asarray(cfg.symbols, dtype=np.complex128)
    rng = np.random.default_rng(0)
    x = np.zeros((B, Nt), np.complex64)
    pos = rng.integers(0, M, size=(B, Na))
    k = rng.integers(0, len(sym), size=(B, Na))
    for a in range(Na):
        x[np.arange(B), a * M + pos[:, a]] = sym[k[:, a]]
    r = (x + 0.25 * (rng.standard_normal((B, Nt)) + 1j * rng.standard_normal((B, Nt)))).astype(np.complex64)
    rt = torch.from_numpy(r).cuda().view(B, Nt, 1)
    tau = 0.05
    outs = []
    for _ in range(reps):
        xm, var = block_denoise(cfg, rt, tau, 0)
        torch.cuda.synchronize()
        outs.append((xm.cpu().numpy().copy(), var.cpu().numpy().copy()))
    nd = [int((o[1].view(np.uint32) != outs[0][1].view(np.uint32)).sum()) +
          int((o[0].view(np.uint64) != outs[0][0].view(np.uint64)).sum()) for o in outs[1:]]
    print(f'{alph} Nt={Nt} M={M}: words differing from run 0 in runs 1..{reps - 1}: {nd}')
    # float64 recompute (vamp.py:109-118 with the per-section shift)
    inv = np.float32(1.0) / np.float32(tau)
    ur = (r.real * inv).astype(np.float32).astype(np.float64)
    ui = (r.imag * inv).astype(np.float32).astype(np.float64)
    xi = (ur[..., None] * sym.real + ui[..., None] * sym.imag).reshape(B, Na, M, -1)
    eta = np.exp(xi - xi.max(axis=(2, 3), keepdims=True))
    Z = eta.sum(axis=(2, 3), keepdims=True)[..., 0]
    xr = (eta * sym).sum(3) / Z
    P = eta.sum(3) / Z
    v = (np.abs(xr) ** 2 * (1 - P) + (np.abs(xr[..., None] - sym) ** 2 * eta).sum(3) / Z).reshape(B, Nt)
    for i, (_, vg) in enumerate(outs[:3]):
        e = np.abs(vg.reshape(B, Nt) - v) / np.maximum(np.abs(v), 1e-30)
        lane = np.arange(Nt) % min(M, 64)
        line = []
        for g in range(0, min(M, 64), 16):
            sel = e[:, (lane >= g) & (lane < g + 16)]
            line.append(f'lanes {g}-{g + 15}: >1e-3 {(sel > 1e-3).sum()} max {sel.max():.1e}')
        print(f'  run {i}: ' + '; '.join(line))


if __name__ == '__main__':
    main()
