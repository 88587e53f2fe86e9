"""g6 (BASELINE cfg5 shape, correlated channel): the build's input replica reproduces the
reference-side inputs bit for bit (SHA-256 of A and x) and y to float32 rounding."""
import hashlib

import numpy as np
import pytest

from cfg5_inputs import cfg5_inputs, g6_curves, g6_points


def _sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.numpy()).tobytes()).hexdigest()


@pytest.mark.parametrize('name,key', g6_points()[:2] + g6_points()[-2:])
def test_cfg5_inputs_replica(name, key):
    ent = g6_curves()[name]
    ref = ent['points'][key]
    seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
    inp = cfg5_inputs(ent, seed, EbN0)
    assert _sha(inp['A']) == ref['sha_A']
    assert _sha(inp['x']) == ref['sha_x']
    y2 = float(np.sum(np.abs(inp['y'].numpy().astype(np.complex128)) ** 2))
    assert abs(y2 - ref['y_abs2_sum']) <= 1e-5 * ref['y_abs2_sum']
