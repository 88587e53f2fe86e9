"""The drop-in claim: the reference's own drivers, launched through
tools/run_reference_driver.py, bind every detector-path name to THIS package, not to the
reference's files.  Reads the reference drivers as plain files in the build container (skipped
where /root/reference is absent, e.g. on the GPU box); nothing is executed on a device."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'amp-sparc-spatialmodulation_amd')
REF = os.environ.get('AMP_REFERENCE', '/root/reference')

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason='reference checkout not present')

# driver file -> the names it imports from the modules this package replaces
DRIVERS = {
    'vamp_model.py': ('Config', 'Data', 'Channel', 'Loss', 'VAMP'),
    'bamp_model.py': ('Config', 'Data', 'Channel', 'Loss', 'BAMP'),
    'scamp_model.py': ('Config', 'Data', 'Channel', 'Loss', 'SCAMP'),
}

PROBE = r'''
import json, sys, inspect
sys.dont_write_bytecode = True
sys.path.insert(0, {tools!r})
import run_reference_driver as rrd
mod = rrd.import_driver({driver!r})
out = {{}}
for name in {names!r}:
    obj = getattr(mod, name)
    out[name] = inspect.getsourcefile(obj)
out['Model'] = inspect.getsourcefile(mod.Model)
print(json.dumps(out))
'''


@pytest.mark.parametrize('driver', sorted(DRIVERS))
def test_reference_driver_binds_package(driver):
    path = os.path.join(REF, driver)
    if not os.path.exists(path):
        pytest.skip(f'{driver} not in the reference')
    pytest.importorskip('matplotlib')      # the drivers import the reference's plotter
    code = PROBE.format(tools=os.path.join(REPO, 'tools'), driver=path, names=DRIVERS[driver])
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1')
    # run from a scratch directory, the way the launcher is used (not from the reference's)
    out = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, env=env, cwd=REPO,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    import json
    files = json.loads(out.stdout.strip().splitlines()[-1])
    for name in DRIVERS[driver]:
        assert os.path.abspath(files[name]).startswith(PKG), (name, files[name])
    # the driver's own Model class stays the reference's (it is the code being dropped onto)
    assert os.path.abspath(files['Model']).startswith(os.path.abspath(REF)), files['Model']


def test_plain_python_would_load_the_reference():
    """Why the launcher exists: `python driver.py` puts the driver's directory first, ahead of
    PYTHONPATH, so a flat `import vamp` there resolves to the reference's file."""
    code = 'import sys; sys.dont_write_bytecode = True; import vamp; print(vamp.__file__)'
    env = dict(os.environ, PYTHONPATH=PKG, PYTHONDONTWRITEBYTECODE='1')
    out = subprocess.run([sys.executable, '-c',
                          f'import sys; sys.path.insert(0, {REF!r}); exec({code!r})'],
                         capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert os.path.abspath(out.stdout.strip()).startswith(os.path.abspath(REF))
