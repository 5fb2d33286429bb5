"""ctypes binding of libsmmd_hip.so (the C ABI in include/smmd_hip.h).

The library is the only compute path for the hot ops: there is no CPU or
eager-PyTorch fallback.  Importing this module does not touch the GPU;
``lib()`` loads the shared object on first use and raises ``SmmdLibraryError``
when it is missing, so a box without the build fails loudly.

Device buffers are torch tensors (PyTorch is the allocator and the stream
owner); every call is issued on ``torch.cuda.current_stream()``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported before the .so: shares HIP runtime)

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.environ.get('SMMD_HIP_LIB', os.path.join(_PKG_ROOT, 'lib', 'libsmmd_hip.so'))
# an explicitly named library (A/B runs of another build) skips the stamp check
_CHECK_STAMP = 'SMMD_HIP_LIB' not in os.environ
CSRC = os.path.join(_PKG_ROOT, 'csrc')
HEADER = os.path.join(os.path.dirname(_PKG_ROOT), 'include', 'smmd_hip.h')

SMMD_MAX_TERMS = 8
SMMD_SN_MAX_LAYERS = 32
SN_P1_READY = 1            # smmd_sn_power_iter_ex flag
ADAM_SN_GDIRECT = 1        # smmd_adam_flat_sn2 flag
OPT_MAX_FUSED = 96         # tensors smmd_adam_flat_sn takes in one call
SN_MAX_FUSED = 16          # SN layers smmd_adam_flat_sn takes in one call
ABI_VERSION = 17

KIND_RBF, KIND_RQ, KIND_DISTANCE, KIND_DOT = 0, 1, 2, 3
SMMD_EUNSUPPORTED = 4       # smmd_status (include/smmd_hip.h)


class SmmdLibraryError(RuntimeError):
    """libsmmd_hip.so is missing or failed to load."""


class SmmdError(RuntimeError):
    """A libsmmd_hip.so entry point returned a non-OK smmd_status."""


class KernelDesc(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32),
                ('n_terms', ctypes.c_int32),
                ('param', ctypes.c_double * SMMD_MAX_TERMS),
                ('wt', ctypes.c_double * SMMD_MAX_TERMS),
                ('add_dot', ctypes.c_double),
                ('tanh_inputs', ctypes.c_int32),
                ('has_const_diag', ctypes.c_int32),
                ('const_diag', ctypes.c_double)]


class SnLayer(ctypes.Structure):
    _fields_ = [('W', ctypes.c_void_p),
                ('W_eff', ctypes.c_void_p),
                ('u', ctypes.c_void_p),
                ('v', ctypes.c_void_p),
                ('sigma', ctypes.c_void_p),
                ('s', ctypes.c_void_p),
                ('G', ctypes.c_void_p),
                ('gW', ctypes.c_void_p),
                ('gs', ctypes.c_void_p),
                ('N', ctypes.c_int32),
                ('K', ctypes.c_int32),
                ('fold', ctypes.c_int32)]


class PolySums(ctypes.Structure):
    """smmd_poly_sums: (rows, cols, diag, stats) of one smmd_poly_kernel_sums call."""
    _fields_ = [('rows', ctypes.c_void_p),
                ('cols', ctypes.c_void_p),
                ('diag', ctypes.c_void_p),
                ('stats', ctypes.c_void_p)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# name -> (restype, argtypes)
_SIGS = {
    'smmd_status_string': (ctypes.c_char_p, [_I]),
    'smmd_abi_version': (_I, []),
    'smmd_source_hash': (ctypes.c_char_p, []),
    'smmd_mmd2_workspace_bytes': (_SZ, [_I, _I, _I]),
    'smmd_mmd2_fwd': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _P, _I, _I, _I, _I, _I, _I, _I,
                           _P, _P, _P, _P, _P, _SZ, _P]),
    'smmd_mmd2_combine': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _I, _I, _P, _P]),
    'smmd_witness_fwd': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _P, _I, _P, _I, _I, _P, _P, _P]),
    'smmd_witness_bwd': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _P, _I, _P, _I, _I, _P, _P, _P,
                              _P, _P]),
    'smmd_kernel_matrix_fwd': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _P, _I, _I, _P, _P]),
    'smmd_kernel_matrix_bwd': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _P, _I, _I, _P, _P, _P,
                                    _P]),
    'smmd_scaled_loss_workspace_bytes': (_SZ, [_I, _I64]),
    'smmd_scaled_loss_fwd': (_I, [_P, _I, _I, _I, _I64, _P, _I, _P, _F, _I, _I, _P, _P, _P, _SZ,
                                  _P]),
    'smmd_scaled_loss_finalize': (_I, [_P, _F, _I, _I, _P]),
    'smmd_smmd_loss_fwd': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _P, _I, _I, _I, _P, _I, _I,
                                _I64, _P, _I, _F, _I, _I, _P, _P, _P, _P, _P, _P, _P, _SZ, _P,
                                _SZ, _P]),
    'smmd_smmd_loss_bwd': (_I, [_P, _I, _I, _I64, _P, _I, _P, _F, _I, _I, _P, _P, _P, _I, _P, _I,
                                _I, _P, _P, _P, _P, _P]),
    'smmd_scaled_loss_bwd': (_I, [_P, _I, _I, _I, _I64, _P, _I, _P, _F, _I, _I, _P, _P, _P, _P,
                                  _P]),
    'smmd_smmd_loss_fwd_gathered': (_I, [ctypes.POINTER(KernelDesc), _P, _I, _P, _I, _I, _I, _P,
                                         _I, _I, _F, _I, _I, _P, _P, _P, _P, _P, _P, _SZ, _P, _SZ,
                                         _P]),
    'smmd_smmd_loss_bwd_ex': (_I, [_P, _I, _I, _I, _I64, _P, _I, _P, _F, _I, _I, _P, _P, _P, _I,
                                   _P, _I, _I, _P, _P, _P, _P, _P]),
    'smmd_sn_workspace_bytes': (_SZ, [ctypes.POINTER(SnLayer), _I]),
    'smmd_sn_power_iter': (_I, [ctypes.POINTER(SnLayer), _I, _I, _F, _I, _P, _SZ, _P]),
    'smmd_sn_power_iter_ex': (_I, [ctypes.POINTER(SnLayer), _I, _I, _F, _I, _I, _P, _SZ, _P]),
    'smmd_sn_weight_bwd': (_I, [ctypes.POINTER(SnLayer), _I, _P, _SZ, _P]),
    'smmd_sn_grad_stats': (_I, [ctypes.POINTER(SnLayer), _I, _P, _SZ, _P]),
    'smmd_sn_clip_g': (_I, [ctypes.POINTER(SnLayer), _I, _F, _P, _SZ, _P]),
    'smmd_adam_flat_sn2': (_I, [_P, _P, _P, _P, ctypes.POINTER(ctypes.c_int64), _I, _F, _F, _F,
                                _F, _F, _F, _I64, _P, _P, _SZ, ctypes.POINTER(SnLayer),
                                ctypes.POINTER(ctypes.c_int32), _I, _P, _SZ, _I, _P]),
    'smmd_opt_workspace_bytes': (_SZ, [ctypes.POINTER(ctypes.c_int64), _I]),
    'smmd_clip_by_norm_flat': (_I, [_P, ctypes.POINTER(ctypes.c_int64), _I, _F, _P, _SZ, _P]),
    'smmd_adam_flat': (_I, [_P, _P, _P, _P, ctypes.POINTER(ctypes.c_int64), _I, _F, _F, _F, _F,
                            _F, _F, _I64, _P, _SZ, _P]),
    'smmd_adam_flat_sn': (_I, [_P, _P, _P, _P, ctypes.POINTER(ctypes.c_int64), _I, _F, _F, _F,
                               _F, _F, _F, _I64, _P, _SZ, ctypes.POINTER(SnLayer),
                               ctypes.POINTER(ctypes.c_int32), _I, _P, _SZ, _P]),
    'smmd_adam_flat_ex': (_I, [_P, _P, _P, _P, ctypes.POINTER(ctypes.c_int64), _I, _F, _F, _P,
                               _F, _F, _F, _P, _SZ, ctypes.POINTER(SnLayer),
                               ctypes.POINTER(ctypes.c_int32), _I, _P, _SZ, _P]),
    'smmd_poly_sums_workspace_bytes': (_SZ, [_I, _I, _I]),
    'smmd_poly_kernel_sums': (_I, [_P, _I, _P, _I, _I, ctypes.c_double, ctypes.c_double, _I, _P,
                                   _P, _P, _P, _P, _SZ, _P]),
    'smmd_poly_mmd2_var': (_I, [ctypes.POINTER(PolySums), ctypes.POINTER(PolySums),
                                ctypes.POINTER(PolySums), _I, ctypes.c_double, _I, _P, _P]),
    'smmd_fold_pool_weights': (_I, [ctypes.POINTER(_P), ctypes.POINTER(_P),
                                    ctypes.POINTER(ctypes.c_int64), _I, _I, _P]),
    'smmd_fold_up_weight': (_I, [_P, _P, _I, _I, _I, _P]),
    'smmd_conv1x1_supported': (_I, [_I, _I, _I, _I]),
    'smmd_conv1x1_workspace_bytes': (_SZ, [_I, _I, _I, _I]),
    'smmd_conv1x1': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_conv1x1_t': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_conv1x1_wgrad_supported': (_I, [_I, _I, _I, _I]),
    'smmd_conv1x1_wgrad_workspace_bytes': (_SZ, [_I, _I, _I, _I]),
    'smmd_conv1x1_wgrad': (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_conv1x1_wgrad_acc': (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_channel_sum_workspace_bytes': (_SZ, [_I, _I]),
    'smmd_channel_sum': (_I, [_P, _I, _I, _I, _P, _P, _SZ, _P]),
    'smmd_conv3x3_thin': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    'smmd_mask_pool2': (_I, [_P, _P, _P, _P, _I, _P, _F, _F, _I64, _I, _I, _P, _P, _P]),
    'smmd_mask_pool2_adj': (_I, [_P, _P, _P, _F, _F, _I64, _I, _I, _P, _P]),
    'smmd_up_add': (_I, [_P, _P, _P, _P, _I, _I64, _I, _I, _P, _P]),
    'smmd_bn_relu_workspace_bytes': (_SZ, [_I, _I]),
    'smmd_bn_relu_fwd': (_I, [_P, _I, _I, _I, _P, _P, _P, _P, _F, _F, _P, _P, _SZ, _P]),
    'smmd_bn_relu_fwd_save': (_I, [_P, _I, _I, _I, _P, _P, _P, _P, _F, _F, _P, _P, _P, _SZ, _P]),
    'smmd_bn_relu_bwd': (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'smmd_conv3x3_thin_wgrad_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_conv3x3_thin_wgrad': (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_conv3x3_thin_wgrad_acc': (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino3x3_supported': (_I, [_I, _I, _I, _I, _I]),
    'smmd_wino3x3_filter_bytes': (_SZ, [_I, _I]),
    'smmd_wino3x3_filter': (_I, [_P, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino3x3_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_wino3x3_conv': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino3x3_conv_relu': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino3x3_conv_mask': (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino3x3_conv2_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_wino3x3_conv2': (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2_supported': (_I, [_I, _I, _I, _I, _I]),
    'smmd_wino4x4s2t_supported': (_I, [_I, _I, _I, _I, _I]),
    'smmd_wino4x4s2_filter_bytes': (_SZ, [_I, _I]),
    'smmd_wino4x4s2_filter': (_I, [_P, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2t_filter': (_I, [_P, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_wino4x4s2t_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_wino4x4s2_conv': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2_conv_acc': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2_conv2_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_wino4x4s2_conv2': (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2t_conv': (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2t_conv_mask': (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_row_lrelu_sum': (_I, [_P, _P, _P, _P, _P, _I64, _I, _F, _P]),
    'smmd_row_lrelu_bcast': (_I, [_P, _P, _P, _P, _I64, _I, _F, _P]),
    'smmd_wino3x3_wgrad_supported': (_I, [_I, _I, _I, _I, _I]),
    'smmd_wino3x3_wgrad_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_wino3x3_wgrad': (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino3x3_wgrad_acc': (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino3x3_filter_sn': (_I, [_P, _P, _P, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2_filter_sn': (_I, [_P, _P, _P, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2t_filter_sn': (_I, [_P, _P, _P, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2_wgrad_supported': (_I, [_I, _I, _I, _I, _I]),
    'smmd_wino4x4s2_wgrad_workspace_bytes': (_SZ, [_I, _I, _I, _I, _I]),
    'smmd_wino4x4s2_wgrad': (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_wino4x4s2_wgrad_acc': (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _SZ, _P]),
    'smmd_poly_diff_ratio': (_I, [ctypes.POINTER(PolySums), ctypes.POINTER(PolySums),
                                  ctypes.POINTER(PolySums), ctypes.POINTER(PolySums), _I, _P,
                                  _P]),
}

EXPORTED_SYMBOLS = tuple(_SIGS)

_lock = threading.Lock()
_lib = None


def source_hash():
    """The stamp csrc/Makefile compiles into the library: the first 16 hex
    digits of SHA-256 over csrc/*.hip and csrc/*.hpp (names in byte order),
    then include/smmd_hip.h."""
    import hashlib
    names = sorted(f for f in os.listdir(CSRC) if f.endswith(('.hip', '.hpp')))
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, f) for f in names] + [HEADER]:
        with open(path, 'rb') as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def lib():
    """Load libsmmd_hip.so once (raises SmmdLibraryError if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise SmmdLibraryError(
                    'libsmmd_hip.so not found at %s -- build it with '
                    '`python -c "import __graft_entry__ as g; g.build()"` or '
                    '`make -C scaled-mmd-gan_amd/csrc`' % LIB_PATH)
            try:
                handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            except OSError as e:
                raise SmmdLibraryError('failed to load %s: %s' % (LIB_PATH, e)) from e
            for name, (res, args) in _SIGS.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            if handle.smmd_abi_version() != ABI_VERSION:
                raise SmmdLibraryError('ABI version mismatch')
            if _CHECK_STAMP and os.path.isdir(CSRC):
                built, now = handle.smmd_source_hash().decode(), source_hash()
                if built != now:
                    raise SmmdLibraryError(
                        '%s was built from other sources (stamp %s, sources %s): rebuild '
                        'with `make -C scaled-mmd-gan_amd/csrc`' % (LIB_PATH, built, now))
            _lib = handle
    return _lib


def check(status: int, what: str):
    if status != 0:
        msg = lib().smmd_status_string(status).decode()
        raise SmmdError('%s failed: %s' % (what, msg))


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_cuda(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise SmmdError('libsmmd_hip needs device tensors (got %s on %s): there is no CPU '
                            'path' % (tuple(t.shape), t.device))
        if t.dtype != torch.float32:
            raise SmmdError('libsmmd_hip computes in fp32 (got %s)' % t.dtype)


# ---------------------------------------------------------------------------
# optional per-entry-point timing with HIP events on the current stream
# (used by bench.py; a no-op unless enabled)
# ---------------------------------------------------------------------------
class _Timing:
    enabled = False
    records = {}
    nbytes = {}       # entry point -> algorithmic bytes summed over its timed calls
    nflops = {}       # entry point -> executed MFMA flops summed over its timed calls


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_NULL = _NullCtx()


class _EventCtx:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.s = torch.cuda.Event(enable_timing=True)
        self.e = torch.cuda.Event(enable_timing=True)
        self.s.record()
        return self

    def __exit__(self, *a):
        self.e.record()
        _Timing.records.setdefault(self.name, []).append((self.s, self.e))
        return False


def timed(name):
    """Context manager bracketing one library call with HIP events."""
    return _EventCtx(name) if _Timing.enabled else _NULL


def add_bytes(name, n):
    """Algorithmic HBM bytes of one call of an entry point whose size varies
    call to call (bench.py reports the mean per call)."""
    if _Timing.enabled:
        _Timing.nbytes[name] = _Timing.nbytes.get(name, 0) + int(n)


def add_flops(name, n):
    """Executed matrix-core flops of one call (the Winograd convolution's
    point products; bench.py reports the mean per call)."""
    if _Timing.enabled:
        _Timing.nflops[name] = _Timing.nflops.get(name, 0) + int(n)


def timing_flops():
    """{entry point: mean executed flops per timed call} (add_flops users)."""
    return {k: f / len(_Timing.records[k]) for k, f in _Timing.nflops.items()
            if _Timing.records.get(k)}


def timing_bytes():
    """{entry point: mean algorithmic bytes per timed call} (add_bytes users)."""
    return {k: b / len(_Timing.records[k]) for k, b in _Timing.nbytes.items()
            if _Timing.records.get(k)}


def enable_timing(on=True):
    _Timing.enabled = on


def timing_ms():
    """{entry point: (calls, mean ms)} over the recorded events (syncs)."""
    torch.cuda.synchronize()
    return {k: (len(v), sum(s.elapsed_time(e) for s, e in v) / len(v))
            for k, v in _Timing.records.items() if v}


def reset_timing():
    _Timing.records = {}
    _Timing.nbytes = {}
    _Timing.nflops = {}


# ---------------------------------------------------------------------------
# workspaces: zero-filled at allocation, owned per (device, stream, tag)
# ---------------------------------------------------------------------------
_ws_cache = {}
# Workspaces a HIP-graph capture was handed: a captured launch keeps their raw
# address for every replay, so one superseded by a larger request must stay
# allocated (freeing it returned it to its graph pool -- or, once the last
# tensor of an earlier capture's pool was gone, to the device -- and the next
# replay of the graph that recorded it wrote through a stale address)
_ws_captured = set()
_ws_retired = []


def workspace(tag: str, nbytes: int, device: torch.device):
    key = (device.index, torch.cuda.current_stream(device).cuda_stream, tag)
    buf = _ws_cache.get(key)
    capturing = torch.cuda.is_current_stream_capturing()
    if buf is None or buf.numel() < nbytes:
        if buf is not None and key in _ws_captured:
            _ws_retired.append(buf)
        _ws_captured.discard(key)
        buf = torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _ws_cache[key] = buf
    if capturing:
        _ws_captured.add(key)
    return buf


def clear_workspaces():
    """Drop the cached workspaces (none that a live step graph recorded: call
    it with no graphs alive)."""
    _ws_cache.clear()
    _ws_captured.clear()
    _ws_retired.clear()
