"""ORACLE — test infrastructure, not product code.

A CPU (numpy) restatement of the reference detector path of
AhmedKishki/AMP-SPARC-SpatialModulation, used ONLY as the checker:

* ``tests/`` compare the HIP path against it,
* ``__graft_entry__.smoke()`` checks one small GPU invocation against it,
* ``bench.py`` times it as the ``cpu_baseline`` leg (kind ``"port"``).

Nothing in the product package imports this module; the product fails
loudly when its HIP library is missing instead of falling back here.

Parity pinning: the restatement is checked against golden vectors produced by
running the reference itself in the build container
(``tests/golden/make_goldens.py``), see ``tests/test_oracle_goldens.py``.
"""
from .amp_oracle import *  # noqa: F401,F403
