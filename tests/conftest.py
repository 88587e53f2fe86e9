"""Test configuration: the `gpu` marker and import paths.

The product package directory uses flat module names (config, channel, data, vamp,
bamp, scamp, loss) exactly like the reference, so the reference's drivers import it
unchanged; tests put it on sys.path the same way.
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'amp-sparc-spatialmodulation_amd')
GOLDEN = os.path.join(REPO, 'tests', 'golden')
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (ROCm device); run with -m gpu')


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope='session')
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no ROCm device')
    return torch.device('cuda:0')


@pytest.fixture(autouse=True)
def _no_silent_grid_rescue(request):
    """A persistent grid that times out is re-run on the launch engine in-process
    (vamp.LazyResult._check_grid) and would otherwise let a "persistent" parity test pass on the
    launch engine: every test except tests/test_gpu_rescue.py (which forces rescues on purpose)
    fails when a rescue happened during it."""
    def total():
        mod = sys.modules.get('vamp')
        return getattr(getattr(mod, 'LazyResult', None), 'rescues_total', 0) if mod else 0
    before = total()
    yield
    if os.path.basename(str(request.node.fspath)) == 'test_gpu_rescue.py':
        return
    n = total() - before
    if n:
        pytest.fail(f'{n} persistent grid rescue(s) during this test: the persistent engine lost its grid '
                    'and the launch engine produced the result')
