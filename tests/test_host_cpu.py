"""CPU: host logic of the product (no GPU needed).

* the C-ABI library exports every entry point include/amp_sparc.h declares
  (loaded, no compute calls);
* Config mirrors the reference's constants (checked against the oracle's restatement);
* the host RNG replica (Channel.generate_as_sparc, Data.generate_message, Channel.awgn)
  reproduces the reference's streams bit-for-bit: SHA-256 of (A, x, labels) and the
  energy of y recorded by the reference in tests/golden/g4_curves.json.
"""
import hashlib
import os
import re

import numpy as np
import pytest
import torch

import golden_io as gio
from oracle import OracleConfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, 'include', 'amp_sparc.h')


def test_library_exports_every_declared_symbol():
    import amp_native as nat
    lib = nat.lib()
    decl = re.findall(r'^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(amp_[a-z_0-9]+)\s*\(', open(HEADER).read(), re.M)
    assert len(decl) >= 15
    for name in decl:
        assert hasattr(lib, name), name
        assert name in nat.SIGNATURES, f'{name} missing from the ctypes binding'
    assert b'gfx950' in lib.amp_build_info()


def test_struct_layouts_match_header():
    import ctypes as C
    import amp_native as nat
    assert nat.AMP_MAX_K == 64
    assert C.sizeof(nat.AmpConstellation) == 8 + 64 * 4 * 2 + 64 * 8 * 2 + 64 * 4
    assert C.sizeof(nat.AmpDims) == 40
    assert C.sizeof(nat.AmpStatus) == 32
    assert C.sizeof(nat.AmpCounts) == 13 * 8
    assert nat.AmpVampArgs.noise_var.offset == 48 and C.sizeof(nat.AmpVampArgs) == 112
    # amp_vamp_decide_args: x, sym, idx, (ibits_trunc, pad), counts, host_record
    assert nat.AmpVampDecideArgs.counts.offset == 32 and nat.AmpVampDecideArgs.host_record.offset == 40
    assert C.sizeof(nat.AmpVampDecideArgs) == 48
    # amp_status at byte 0 and amp_counts at byte 64 of a 256-byte result record (vamp.py LazyResult)
    assert C.sizeof(nat.AmpStatus) <= 64 and 64 + C.sizeof(nat.AmpCounts) <= 256


def test_workspace_sizes():
    import ctypes as C
    from config import Config
    import amp_native as nat
    cfg = Config(256, 8, 512, 1, 1, batch=4096, generator_mode='sparc', alphabet='16QAM',
                 channel_profile='uniform', channel_truncation='tail', device='cpu')
    d = cfg.dims()
    ws = nat.lib().amp_vamp_workspace_bytes(C.byref(d), 256, 20)
    assert 20e6 < ws < 80e6, ws
    assert nat.lib().amp_vamp_workspace_bytes(C.byref(d), 0, 20) == 0


@pytest.mark.parametrize('alph', ['OOK', 'BPSK', '4ASK', 'QPSK', '8PSK', '16PSK', '16QAM'])
@pytest.mark.parametrize('dims', [(64, 4, 128, 1, 1), (128, 16, 32, 25, 6), (16, 2, 32, 3, 2)])
def test_config_constants(alph, dims):
    from config import Config
    Nt, Na, Nr, Lin, Lh = dims
    c = Config(Nt, Na, Nr, Lin, Lh, batch=7, generator_mode='sparc', alphabet=alph,
               channel_profile='uniform', channel_truncation='tail', device='cpu')
    o = OracleConfig(Nt, Na, Nr, Lin=Lin, Lh=Lh, B=7, alphabet=alph)
    assert np.array_equal(c.symbols, o.symbols) and c.symbols.dtype == o.symbols.dtype
    assert c.gray == o.gray and c.K == o.K and c.symbol_bits == o.symbol_bits
    assert c.code_rate == o.code_rate and c.index_bits == o.index_bits
    assert c.shannon_limit_dB == o.shannon_limit_dB and c.Ns == o.Ns and c.Lout == o.Lout
    assert c.name == f'{alph},sparc/uniform,tail/Nt={Nt},Na={Na},Nr={Nr},Lh={Lh},Lin={Lin}'
    k = c.constellation()
    assert k.K == c.K and abs(k.re64[0] - np.real(c.symbols[0])) == 0


def test_config_assertions():
    from config import Config
    with pytest.raises(AssertionError):
        Config(64, 4, 128, 1, 1, alphabet='64QAM')
    with pytest.raises(AssertionError):
        Config(64, 5, 128, 1, 1, generator_mode='sparc')


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


CURVES = gio.g4_curves()
RNG_POINTS = [(name, key) for name, ent in sorted(CURVES.items()) for key in sorted(ent['points'])[:2]]


@pytest.mark.parametrize('name,key', RNG_POINTS)
def test_rng_replica_bit_exact(name, key):
    from config import Config
    from channel import Channel
    from data import Data
    ent = CURVES[name]
    ref = ent['points'][key]
    seed, EbN0 = int(key.split('/')[0]), float(key.split('/')[1])
    cfg = Config(ent['Nt'], ent['Na'], ent['Nr'], 1, 1, batch=ent['B'], generator_mode='sparc',
                 iterations=ent['iterations'], alphabet=ent['alphabet'], channel_profile='uniform',
                 channel_truncation='tail', device='cpu')
    np.random.seed(seed)
    torch.manual_seed(seed)
    ch, da = Channel(cfg), Data(cfg)
    W, A = ch.generate_as_sparc()
    if ent['algo'] == 'vamp':
        torch.linalg.svd(A, full_matrices=False)     # consumes no RNG; kept for call order
    x, sym, idx = da.generate_message()
    noise = ch.awgn(cfg.snr(EbN0))
    assert _sha(A.numpy()) == ref['sha_A']
    assert _sha(x.numpy()) == ref['sha_x']
    assert _sha(np.asarray(sym, np.int64)) == ref['sha_sym']
    y = A @ x + noise
    e = float(np.sum(np.abs(y.numpy().astype(np.complex128)) ** 2))
    assert abs(e - ref['y_abs2_sum']) <= 1e-6 * ref['y_abs2_sum']


def test_segmented_replica_matches_draw_loop():
    """Vectorised draws == the reference's per-section choice(M), choice(K) loop (data.py:82-87)."""
    from config import Config
    from data import Data
    for alph, Nt, Na in [('QPSK', 64, 4), ('OOK', 32, 4), ('8PSK', 24, 2)]:
        cfg = Config(Nt, Na, 2 * Nt, 2, 1, batch=5, generator_mode='sparc', alphabet=alph, device='cpu')
        np.random.seed(3)
        x, sym, idx = Data(cfg).generate_message()
        np.random.seed(3)
        M, K, S = Nt // Na, len(cfg.symbols), 5 * Na * 2
        xl = np.zeros((S, M), np.complex64)
        for s in range(S):
            p = np.random.choice(M)
            k = np.random.choice(K)
            xl[s, p] = cfg.symbols[k]
        assert np.array_equal(x.numpy().ravel(), xl.ravel())
        assert np.array_equal(idx, xl.ravel().nonzero()[0])


def test_detector_api_surface():
    """The reference's class surface (vamp.py / bamp.py / scamp.py: Tracker, Layer.forward(T),
    the detector's forward) and the lazy read-back every detector shares — checked on the CPU so
    a broken host mirror is caught before a GPU run."""
    import inspect
    import vamp
    import bamp
    import scamp
    for mod, det, layer in ((vamp, 'VAMP', 'VAMPLayer'), (bamp, 'BAMP', 'BAMPLayer'), (scamp, 'SCAMP', 'SCAMPLayer')):
        D, Ly, T = getattr(mod, det), getattr(mod, layer), getattr(mod, 'Tracker')
        for m in ('forward', 'detect', '_result_slot', '_arm'):
            assert callable(getattr(D, m, None)), (det, m)
        assert 'T' in inspect.signature(Ly.forward).parameters
        for m in ('prepare', 'finalize', 'status'):
            assert callable(getattr(T, m, None)), (det, m)
