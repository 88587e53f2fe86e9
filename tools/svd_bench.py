#!/usr/bin/env python3
"""Throughput of the per-channel SVD of Model(rng='device') (vamp_model.py:57-58: one SVD per
new channel) on the GPU, cfg4 shape (A: 512 x 256 complex64), by method:
  svd1      torch.linalg.svd of one channel (the round-3 path)
  svdK      torch.linalg.svd of K channels stacked (one batched call)
  gramK     the Hermitian eigendecomposition of the K Gram matrices A^H A (torch.linalg.eigh,
            batched): Vh = eigenvectors^H, s = sqrt(eigenvalues) (descending), U = A V / s
Prints ms per channel and the reconstruction / orthogonality error of each.

  python tools/svd_bench.py [--n 512] [--N 256] [--K 1,8,32]
"""
import argparse
import json
import time

import torch


def gram_svd(A):
    """Batched SVD of tall complex A [..., n, N] (n >= N) through eigh of A^H A."""
    G = A.mH @ A
    w, V = torch.linalg.eigh(G)                      # ascending
    w = w.flip(-1).clamp_min(0)
    V = V.flip(-1)
    s = w.sqrt()
    U = (A @ V) / s.unsqueeze(-2).to(A.dtype)
    return U, s, V.mH


def errs(A, U, s, Vh):
    R = (U * s.unsqueeze(-2).to(U.dtype)) @ Vh
    rec = float(((R - A).abs().amax() / A.abs().amax()).item())
    I = torch.eye(Vh.shape[-2], dtype=Vh.dtype, device=Vh.device)
    orth = float((Vh @ Vh.mH - I).abs().amax().item())
    orthu = float((U.mH @ U - I).abs().amax().item())
    return rec, orth, orthu


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=512)
    ap.add_argument('--N', type=int, default=256)
    ap.add_argument('--K', default='1,8,32')
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(1)
    for K in [int(k) for k in a.K.split(',')]:
        A = (torch.randn(K, a.n, a.N, 2, device=dev, generator=g) / (2 * a.n) ** 0.5)
        A = torch.view_as_complex(A.contiguous())
        for name, fn in (('svd', lambda X: torch.linalg.svd(X, full_matrices=False)), ('gram', gram_svd)):
            fn(A)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                U, s, Vh = fn(A)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            rec, orth, orthu = errs(A, U, s, Vh)
            print(json.dumps({'method': f'{name}{K}', 'ms_per_call': round(ms, 3), 'ms_per_channel': round(ms / K, 3),
                              'max_rel_reconstruction_err': rec, 'max_VhVh^H-I': orth, 'max_U^HU-I': orthu}),
                  flush=True)


if __name__ == '__main__':
    main()
