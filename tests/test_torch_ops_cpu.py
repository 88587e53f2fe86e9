"""The TORCH_LIBRARY(amp) custom-op library (csrc/amp_torch_ops.cpp): it loads without a GPU,
registers every schema SURVEY.md §8(b) names, and has no CPU kernel (CPU tensors raise: the
product path has no CPU fallback).  The device results are checked in test_gpu_torch_ops.py."""
import numpy as np
import pytest
import torch

OPS = ('vamp_run', 'bamp_run', 'scamp_run', 'block_denoise', 'map_decide_count')


def test_ops_registered():
    import amp_native as nat
    ops = nat.torch_ops()
    for name in OPS:
        op = getattr(ops, name)
        assert op.default._schema.name == f'amp::{name}'


def test_cpu_tensors_raise():
    import amp_native as nat
    ops = nat.torch_ops()
    sym = torch.tensor(np.array([1, 1j, -1, -1j]))
    r = torch.zeros(2, 16, dtype=torch.complex64)
    with pytest.raises((NotImplementedError, RuntimeError)):
        ops.block_denoise(r, torch.tensor(0.5), 0, 16, 2, sym, [0, 1, 3, 2])
