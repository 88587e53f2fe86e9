#!/usr/bin/env python3
"""Run a reference-style driver script against THIS build instead of the reference's modules.

    python tools/run_reference_driver.py /path/to/reference/vamp_model.py [args...]

``python vamp_model.py`` puts the script's own directory at ``sys.path[0]``, so its flat imports
(``from vamp import VAMP``, ``from loss import Loss`` ...) resolve to the reference's files
whatever PYTHONPATH says.  This launcher puts the package directory FIRST and the driver's
directory after it (for the modules the package does not replace, e.g. ``plotter``), then
runs the script as ``__main__`` with ``runpy`` — so every module the package provides
(config, channel, data, loss, vamp, bamp, scamp, shrink, model) comes from the gfx950 build.

``import_driver(path)`` does the same for a driver imported as a module (its ``__main__``
block does not run); tests use it to check what the driver's names resolve to.
"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'amp-sparc-spatialmodulation_amd')

# the modules of the package that shadow the reference's files of the same name
PROVIDED = ('config', 'channel', 'data', 'loss', 'vamp', 'bamp', 'scamp', 'shrink', 'model')


def _prepare_path(driver: str) -> None:
    ddir = os.path.dirname(os.path.abspath(driver))
    sys.path[:] = [p for p in sys.path if os.path.abspath(p or '.') not in (PKG, ddir)]
    sys.path.insert(0, PKG)
    sys.path.append(ddir)
    # a module of the same name imported earlier from elsewhere would win: drop it
    for name in PROVIDED:
        mod = sys.modules.get(name)
        if mod is not None and not os.path.abspath(getattr(mod, '__file__', '') or '').startswith(PKG):
            del sys.modules[name]


def import_driver(driver: str, name: str = 'reference_driver'):
    """Import a driver file as a module with the package's modules first on sys.path."""
    import importlib.util
    _prepare_path(driver)
    spec = importlib.util.spec_from_file_location(name, driver)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main(argv):
    if not argv:
        print(__doc__)
        return 2
    driver = argv[0]
    sys.dont_write_bytecode = True    # never write __pycache__ next to a read-only driver
    _prepare_path(driver)
    sys.argv = [driver] + list(argv[1:])
    runpy.run_path(driver, run_name='__main__')
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
