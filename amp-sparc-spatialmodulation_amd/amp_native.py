"""ctypes binding of the gfx950 C-ABI library ``lib/libampsparc.so`` (include/amp_sparc.h).

The product path has no fallback: if the library is missing, or a tensor handed to it
is not a ROCm device tensor, the call raises.  ``build()`` compiles it in-tree with hipcc.
"""
from __future__ import annotations

import ctypes as C
import os
import warnings
import subprocess

import numpy as np
import torch   # noqa: F401  (loads torch's HIP runtime first: one runtime per process)

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
LIB_PATH = os.environ.get('AMP_LIB_PATH') or os.path.join(HERE, 'lib', 'libampsparc.so')   # AMP_LIB_PATH: A/B builds

AMP_MAX_K = 64      # include/amp_sparc.h (K in {1, 2, 4, 8, 16, 64})


class AmpConstellation(C.Structure):
    _fields_ = [('K', C.c_int32), ('symbol_bits', C.c_int32),
                ('re', C.c_float * AMP_MAX_K), ('im', C.c_float * AMP_MAX_K),
                ('re64', C.c_double * AMP_MAX_K), ('im64', C.c_double * AMP_MAX_K),
                ('gray', C.c_int32 * AMP_MAX_K)]


class AmpDims(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ('B', 'Nt', 'Na', 'Nr', 'Lin', 'Lout', 'N', 'n', 'L', 'M')]


class AmpStatus(C.Structure):
    _fields_ = [('T', C.c_int32), ('nan_state', C.c_int32), ('stopped', C.c_int32), ('gemm', C.c_int32),
                ('last_scalar', C.c_float * 4)]


class AmpCounts(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ('ier', 'ser', 'iber', 'sber', 'ver', 'verf', 'verm', 'verL', 'fer')] + \
               [(n, C.c_double) for n in ('mse', 'msef', 'msem', 'mseL')]


ENGINE_AUTO, ENGINE_LAUNCHES, ENGINE_PERSISTENT = 0, 1, 2   # amp_vamp_args.engine
GEMM_AUTO, GEMM_F32, GEMM_X3, GEMM_H2, GEMM_I8 = 0, 1, 2, 3, 4   # amp_vamp_args.gemm


class AmpVampArgs(C.Structure):
    _fields_ = [('U', C.c_void_p), ('s', C.c_void_p), ('Vh', C.c_void_p), ('y', C.c_void_p),
                ('k', C.c_int32), ('max_iter', C.c_int32), ('engine', C.c_int32), ('gemm', C.c_int32),
                ('noise_var', C.c_double), ('sparsity', C.c_double),
                ('r', C.c_void_p), ('xmmse', C.c_void_p), ('var', C.c_void_p), ('status', C.c_void_p),
                ('ws', C.c_void_p), ('ws_bytes', C.c_size_t)]


class AmpVamp2Args(C.Structure):
    _fields_ = [('U', C.c_void_p), ('s', C.c_void_p), ('Vh', C.c_void_p), ('y', C.c_void_p),
                ('k', C.c_int32), ('max_iter', C.c_int32), ('sigma2', C.c_double), ('damping', C.c_double),
                ('r', C.c_void_p), ('xmmse', C.c_void_p), ('var', C.c_void_p), ('status', C.c_void_p),
                ('ws', C.c_void_p), ('ws_bytes', C.c_size_t)]


class AmpVampDecideArgs(C.Structure):
    _fields_ = [('x', C.c_void_p), ('sym', C.c_void_p), ('idx', C.c_void_p), ('ibits_trunc', C.c_int32),
                ('pad', C.c_int32), ('counts', C.c_void_p), ('host_record', C.c_void_p)]


class AmpVampShard(C.Structure):
    _fields_ = [('xbuf', C.c_void_p), ('xbuf_bytes', C.c_size_t), ('B_global', C.c_int32), ('row_offset', C.c_int32),
                ('gen', C.c_uint32), ('pad', C.c_int32)]


class AmpBampArgs(C.Structure):
    _fields_ = [('H', C.c_void_p), ('y', C.c_void_p), ('max_iter', C.c_int32), ('denoiser', C.c_int32),
                ('noise_var', C.c_double), ('xmap', C.c_void_p), ('xmmse', C.c_void_p), ('var', C.c_void_p),
                ('status', C.c_void_p), ('ws', C.c_void_p), ('ws_bytes', C.c_size_t),
                ('P0', C.c_float), ('Ps', C.c_float), ('gemm', C.c_int32), ('pad', C.c_int32)]


class AmpScampArgs(C.Structure):
    _fields_ = [('W', C.c_void_p), ('A', C.c_void_p), ('y', C.c_void_p), ('max_iter', C.c_int32),
                ('engine', C.c_int32), ('gemm', C.c_int32), ('pad', C.c_int32), ('noise_var', C.c_double),
                ('xmap', C.c_void_p), ('xmmse', C.c_void_p),
                ('psi', C.c_void_p), ('status', C.c_void_p), ('ws', C.c_void_p), ('ws_bytes', C.c_size_t)]


# amp_allreduce_fn (include/amp_sparc.h): all-reduce `count` float64 words at a device pointer
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_void_p)
ALLREDUCE_SUM, ALLREDUCE_MAX = 0, 1

_P = C.c_void_p
_I = C.c_int32
_D = C.POINTER(AmpDims)
_K = C.POINTER(AmpConstellation)

# name -> (restype, argtypes); mirrors include/amp_sparc.h
SIGNATURES = {
    'amp_vamp_workspace_bytes': (C.c_size_t, [_D, _I, _I]),
    'amp_vamp_select_engine': (C.c_int, [_D, _I, _I]),
    'amp_vamp_select_gemm': (C.c_int, [_D, _I, _I]),
    'amp_vamp2_workspace_bytes': (C.c_size_t, [_D, _I]),
    'amp_vamp2_run': (C.c_int, [_D, _K, C.POINTER(AmpVamp2Args), _P]),
    'amp_vamp_persist_trace': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), _P, _P]),
    'amp_scamp_persist_trace': (C.c_int, [_D, _K, C.POINTER(AmpScampArgs), _P, _P]),
    'amp_vamp_run': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), _P]),
    'amp_vamp_prepare': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), _P]),
    'amp_vamp_iterate': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), _I, _P]),
    'amp_vamp_finalize': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), _P]),
    'amp_vamp_profile': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), C.POINTER(C.c_float), _P]),
    'amp_vamp_detect_count': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), C.POINTER(AmpVampDecideArgs), _P]),
    'amp_vamp_epochs_workspace_bytes': (C.c_size_t, [_D, _I, _I, _I]),
    'amp_vamp_debug_offsets': (C.c_int, [_D, _I, _I, _I, C.POINTER(C.c_uint64)]),
    'amp_vamp_debug_dump': (C.c_int, [_P]),
    'amp_vamp_max_epochs': (C.c_int, [_D, _I]),
    'amp_vamp_max_epochs_gemm': (C.c_int, [_D, _I, _I]),
    'amp_vamp_epochs_ch_eligible': (C.c_int, [_D, _I, _I]),
    'amp_debug_persist_timing': (C.c_int, [_I]),
    'amp_debug_persist_time': (C.c_int, [C.POINTER(C.c_int32), C.POINTER(C.c_float)]),
    'amp_set_allreduce_hook': (C.c_int, [_P, _P]),
    'amp_vamp_run_sharded': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), _I, _P]),
    'amp_bamp_run_sharded': (C.c_int, [_D, _K, C.POINTER(AmpBampArgs), _I, _P]),
    'amp_scamp_run_sharded': (C.c_int, [_D, _K, C.POINTER(AmpScampArgs), _I, _P]),
    'amp_map_decide_count_rows': (C.c_int, [_D, _K, _P, _P, _P, _P, _P, _I, C.c_int64, _P, _P, _P, C.c_size_t, _P]),
    'amp_vamp_detect_count_epochs': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), C.POINTER(AmpVampDecideArgs), _I,
                                               _P]),
    'amp_vamp_detect_count_epochs_ch': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), C.POINTER(AmpVampDecideArgs), _I,
                                                  C.c_int64, C.c_int64, C.c_int64, _P]),
    'amp_stream_create_cu_range': (C.c_int, [_I, _I, C.POINTER(C.c_void_p)]),
    'amp_stream_destroy': (C.c_int, [_P]),
    'amp_vamp_shard_xbuf_bytes': (C.c_size_t, [_I, _I]),
    'amp_vamp_shard_reset': (C.c_int, [_P, _P]),
    'amp_vamp_detect_count_shard': (C.c_int, [_D, _K, C.POINTER(AmpVampArgs), C.POINTER(AmpVampDecideArgs),
                                              C.POINTER(AmpVampShard), _P]),
    'amp_bamp_workspace_bytes': (C.c_size_t, [_D, _I]),
    'amp_bamp_run': (C.c_int, [_D, _K, C.POINTER(AmpBampArgs), _P]),
    'amp_bamp_prepare': (C.c_int, [_D, _K, C.POINTER(AmpBampArgs), _P]),
    'amp_bamp_iterate': (C.c_int, [_D, _K, C.POINTER(AmpBampArgs), _I, _P]),
    'amp_bamp_finalize': (C.c_int, [_D, _K, C.POINTER(AmpBampArgs), _P]),
    'amp_bamp_random_denoise': (C.c_int, [_K, C.c_int64, _P, _P, C.c_float, C.c_float, _P, _P, _P]),
    'amp_scamp_workspace_bytes': (C.c_size_t, [_D, _I]),
    'amp_scamp_select_engine': (C.c_int, [_D, _I]),
    'amp_scamp_run': (C.c_int, [_D, _K, C.POINTER(AmpScampArgs), _P]),
    'amp_scamp_detect_count': (C.c_int, [_D, _K, C.POINTER(AmpScampArgs), C.POINTER(AmpVampDecideArgs), _P]),
    'amp_scamp_prepare': (C.c_int, [_D, _K, C.POINTER(AmpScampArgs), _P]),
    'amp_scamp_iterate': (C.c_int, [_D, _K, C.POINTER(AmpScampArgs), _I, _P]),
    'amp_scamp_finalize': (C.c_int, [_D, _K, C.POINTER(AmpScampArgs), _P]),
    'amp_block_denoise': (C.c_int, [_D, _K, _P, _I, C.c_float, _P, _P, _P, _P, C.c_size_t, _P]),
    'amp_block_denoise_workspace_bytes': (C.c_size_t, [_D]),
    'amp_map_decide_count': (C.c_int, [_D, _K, _P, _P, _P, _P, _P, _I, _P, _P, _P, C.c_size_t, _P]),
    'amp_segmented_decide_count': (C.c_int, [_D, _K, _P, _P, _P, _P, _P, _I, _P, _P, _P, C.c_size_t, _P]),
    'amp_random_decide_count': (C.c_int, [_D, _K, _P, _P, _P, _P, _P, _I, _P, _P, _P, C.c_size_t, _P]),
    'amp_map_decide_workspace_bytes': (C.c_size_t, [_D]),
    'amp_shrink_bayes': (C.c_int, [_K, C.c_int64, _I, _P, C.c_float, _P, C.c_float, C.c_float, _P, _P]),
    'amp_shrink_ook': (C.c_int, [C.c_int64, _I, _P, C.c_float, _P, C.c_float, _P, _P, _P, C.c_size_t, _P]),
    'amp_shrink_ook_workspace_bytes': (C.c_size_t, [C.c_int64]),
    'amp_shrink_sw_ook': (C.c_int, [C.c_int64, _I, _I, _P, C.c_float, _P, _P, _P, _P]),
    'amp_gemm_nt_f32': (C.c_int, [_P, _I, _I, _I, _P, _I, _I, _P, _I, _I, _P]),
    'amp_build_cweight': (C.c_int, [_P, C.c_int64, C.c_int64, _I, _P, _I, _I, _P, _I, _I, _P]),
    'amp_last_error': (C.c_char_p, []),
    'amp_build_info': (C.c_char_p, []),
}

_lib = None
OPS_PATH = os.path.join(HERE, 'lib', 'libamp_torch_ops.so')
_ops_loaded = False


def torch_ops():
    """torch.ops.amp — the C ABI registered as PyTorch-ROCm custom ops (csrc/amp_torch_ops.cpp,
    TORCH_LIBRARY(amp)): vamp_run, bamp_run, scamp_run, block_denoise, map_decide_count.  Only
    a ROCm device kernel is registered: CPU tensors raise (no CPU fallback)."""
    global _ops_loaded
    if not _ops_loaded:
        if not os.path.exists(OPS_PATH):
            raise RuntimeError(f'{OPS_PATH} not found: run __graft_entry__.build()')
        lib()                          # libampsparc.so first (the op library links against it)
        torch.ops.load_library(OPS_PATH)
        _ops_loaded = True
    return torch.ops.amp


class AmpError(RuntimeError):
    """A non-zero status from the C ABI (bad argument, workspace, launch failure)."""


def build(verbose: bool = False) -> str:
    """Compile csrc/*.hip for gfx950 into lib/libampsparc.so (hipcc, in-tree)."""
    jobs = str(min(8, os.cpu_count() or 1))
    out = subprocess.run(['make', '-C', CSRC, '-j', jobs], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError('HIP build failed:\n' + out.stdout[-4000:] + out.stderr[-4000:])
    if verbose:
        print(out.stdout)
    return LIB_PATH


# Environment switches that only the diagnostic build reads (amp_host.h diag_env)
DIAG_SWITCHES = ('AMP_BAMP_KC', 'AMP_BAND_GEMM', 'AMP_BAMP_GEMM', 'AMP_BAMP_X3_ROWS', 'AMP_SCAMP_KC', 'AMP_SCAMP_GEMM',
                 'AMP_SCAMP_LAUNCH_GEMM', 'AMP_SCAMP_X3_WAVES', 'AMP_VAMP_GEMM', 'AMP_YTIL_IN_KERNEL', 'AMP_YTIL_X3',
                 'AMP_PERSIST_WG2', 'AMP_EPOCHS_TWO_PER_CU', 'AMP_VAMP_X3_WAVES', 'AMP_FIX_GRID', 'AMP_GRID_DENOISER', 'AMP_SECTION_BN',
                 'AMP_FOLD_LAUNCH', 'AMP_HOST_RECORD', 'AMP_SHARD_ANY_STREAM')


def lib():
    """The loaded library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'{LIB_PATH} not found: run __graft_entry__.build() (HIP extension missing; '
                               'there is no CPU fallback)')
        L = C.CDLL(LIB_PATH)
        stray = sorted(k for k in os.environ if k in DIAG_SWITCHES)
        if stray and not os.environ.get('AMP_LIB_PATH'):
            warnings.warn(f'{", ".join(stray)}: A/B switches of the diagnostic build, ignored by the shipped '
                          'library (make -C amp-sparc-spatialmodulation_amd/csrc DIAG=1, then '
                          'AMP_LIB_PATH=amp-sparc-spatialmodulation_amd/lib_diag/libampsparc_diag.so)',
                          RuntimeWarning, stacklevel=2)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name, None)
            if f is None:
                if os.environ.get('AMP_LIB_PATH'):   # an A/B build that predates this entry point
                    continue
                raise AttributeError(f'{LIB_PATH}: undefined symbol {name} (stale build: run __graft_entry__.build())')
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def unload():
    """Synchronise and dlclose the library while the HIP runtime (and any attached profiler) is
    still up: its code objects are then unregistered before interpreter teardown instead of
    from the loader's exit-time destructors, which ran after rocprofv3 had finalised and
    crashed it (observed on the box, r01)."""
    global _lib
    if _lib is None:
        return
    torch.cuda.synchronize()
    WORKSPACE.clear()
    import _ctypes
    _ctypes.dlclose(_lib._handle)
    _lib = None


def check(rc: int, what: str):
    if rc != 0:
        raise AmpError(f'{what} failed ({rc}): {lib().amp_last_error().decode()}')


def dptr(t: torch.Tensor, dtype=None, name: str = 'tensor') -> int:
    """Device pointer of a contiguous ROCm tensor (no copies, no CPU fallback)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f'{name}: expected a torch.Tensor, got {type(t).__name__}')
    if t.device.type != 'cuda':
        raise ValueError(f'{name}: the HIP path needs a ROCm device tensor (got {t.device}); '
                         'there is no CPU fallback')
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f'{name}: expected {dtype}, got {t.dtype}')
    if not t.is_contiguous():
        raise ValueError(f'{name}: must be contiguous')
    if t.is_conj() or t.is_neg():
        # a lazy conjugate / negation view: its memory does not hold its values
        raise ValueError(f'{name}: lazy conj/neg view; call .resolve_conj().resolve_neg() first')
    return t.data_ptr()


def fold_launch() -> bool:
    """A diagnostic library (AMP_LIB_PATH, `make DIAG=1`) with AMP_FOLD_LAUNCH=1 or AMP_HOST_RECORD=0
    (A/B runs): the persistent engines leave the counter fold to a launch of their own and the record
    is copied back as for the other engines.  The shipped library always folds in-kernel and writes
    the host record (amp_host.h fold_in_kernel)."""
    return bool(os.environ.get('AMP_LIB_PATH')) and (os.environ.get('AMP_FOLD_LAUNCH') == '1' or
                                                    os.environ.get('AMP_HOST_RECORD') == '0')


# amp_status.gemm (include/amp_sparc.h AMP_ARITH_*): the GEMM arithmetic a forward ran
ARITH_NAMES = {0: None, 1: 'f32', 2: 'bf16x3', 3: 'fp16x2', 4: 'int8x4'}


_CU_STREAMS = {}


def cu_range_stream(cu0: int, cu1: int, device=None):
    """A torch stream whose kernels run only on CUs [cu0, cu1) (amp_stream_create_cu_range), one per
    (range, device) for the life of the process: torch's caching allocator remembers the streams
    its blocks were used on and queries them when the blocks are freed (down to interpreter exit),
    so the HIP stream is never destroyed under it."""
    dev = torch.device('cuda', torch.cuda.current_device()) if device is None else torch.device(device)
    key = (int(cu0), int(cu1), dev.index)
    st = _CU_STREAMS.get(key)
    if st is None:
        h = C.c_void_p()
        with torch.cuda.device(dev):
            check(lib().amp_stream_create_cu_range(cu0, cu1, C.byref(h)), 'amp_stream_create_cu_range')
        st = _CU_STREAMS[key] = torch.cuda.ExternalStream(h.value, device=dev)
    return st


def stream_ptr(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def make_constellation(symbols: np.ndarray, gray, symbol_bits: int) -> AmpConstellation:
    sym = np.asarray(symbols).astype(np.complex128)
    c = AmpConstellation()
    c.K = len(sym)
    c.symbol_bits = int(symbol_bits)
    for i, a in enumerate(sym):
        c.re[i] = float(np.float32(a.real))
        c.im[i] = float(np.float32(a.imag))
        c.re64[i] = float(a.real)
        c.im64[i] = float(a.imag)
        c.gray[i] = int(gray[i])
    return c


class Workspace:
    """Cached device workspace per (device, purpose, size)."""

    def __init__(self):
        self._bufs = {}

    def get(self, device, key, nbytes: int) -> torch.Tensor:
        k = (str(device), key)
        b = self._bufs.get(k)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
            self._bufs[k] = b
        return b

    def clear(self):
        self._bufs.clear()


WORKSPACE = Workspace()
