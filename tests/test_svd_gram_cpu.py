"""svd_gram (model.py): the throughput-mode SVD of Model(rng='device') is a thin SVD of the
channel — reconstruction, orthonormal factors, descending singular values equal to LAPACK's —
for tall and wide shapes, and it falls back to torch.linalg.svd on an ill-conditioned matrix."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'amp-sparc-spatialmodulation_amd'))
from model import svd_gram  # noqa: E402


def _rand(n, N, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.complex(torch.randn(n, N, generator=g), torch.randn(n, N, generator=g)) / (2 * n) ** 0.5


@pytest.mark.parametrize('n,N', [(512, 256), (128, 64), (64, 128), (256, 256)])
def test_svd_gram_is_a_thin_svd(n, N):
    A = _rand(n, N, n + N)
    U, s, Vh = svd_gram(A)
    k = min(n, N)
    assert U.shape == (n, k) and s.shape == (k,) and Vh.shape == (k, N)
    R = (U * s.to(U.dtype)) @ Vh
    assert float((R - A).abs().max() / A.abs().max()) < 5e-5
    eye = torch.eye(k, dtype=A.dtype)
    assert float((U.mH @ U - eye).abs().max()) < 5e-5
    assert float((Vh @ Vh.mH - eye).abs().max()) < 5e-5
    assert bool((s[:-1] >= s[1:]).all())
    s_ref = torch.linalg.svdvals(A.to(torch.complex128)).to(torch.float32)
    np.testing.assert_allclose(s.numpy(), s_ref.numpy(), rtol=1e-4, atol=1e-6)


def test_svd_gram_falls_back_when_ill_conditioned():
    A = _rand(64, 32, 5)
    U, s, Vh = torch.linalg.svd(A, full_matrices=False)
    s = s.clone()
    s[-1] = s[0] * 1e-6                               # condition number 1e6
    B = (U * s.to(U.dtype)) @ Vh
    U2, s2, Vh2 = svd_gram(B)
    R = (U2 * s2.to(U2.dtype)) @ Vh2
    assert float((R - B).abs().max() / B.abs().max()) < 1e-5
    assert float(s2[-1] / s2[0]) < 1e-5
