"""Convolution with an explicit second-order rule (PyTorch-ROCm / MIOpen).

The SMMD critic update differentiates THROUGH the critic's input gradient
(the scaling regulariser, gan/core/ops.py:228-233 + model.py:382-390), so
every critic convolution is differentiated twice.  PyTorch's generic
double-backward computes the weight term of that second pass as a FORWARD
convolution of batch/channel-transposed tensors whose "filter" is a whole
activation map (e.g. MIOpen problem ``-n 512 -c 64 -H 8 -W 8 -k 512 -y 8 -x 8``),
which MIOpen runs at 2-4 ms a call on MI355X.  Here the pass is spelled out
with the three standard primitives on the layer's own shapes:

  y = conv(x, w)            gx = Dx(gy, w)          gw = Dw(x, gy)
  second order, given ggx (and ggw):
    d/dgy = conv(ggx, w) + conv(x, ggw)
    d/dw  = Dw(ggx, gy)
    d/dx  = Dx(gy, ggw)

so it uses MIOpen's forward, backward-data and backward-weights kernels --
except for the thin 3x3 layers (a critic's 3-channel input conv, a
generator's 3-channel output layer), whose three primitives run on the
library's `smmd_conv3x3_thin*` kernels (csrc/smmd_thin.hip), the wide 3x3
stride-1 layers, whose forward and backward-data primitives run on the
library's fused Winograd F(2x2, 3x3) MFMA kernel (`smmd_wino3x3_*`,
csrc/smmd_wino.hip) and whose weight gradient runs on `smmd_wino3x3_wgrad`
(csrc/smmd_wino_wgrad.hip), and the 4x4 stride-2 layers (folded ConvMeanPool
/ UpsampleConv), whose forward and transposed convolutions run on the
polyphase Winograd kernels (`smmd_wino4x4s2*`, csrc/smmd_wino_s2.hip).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

_aten = torch.ops.aten

# >0 while an autograd.grad call that needs input gradients ONLY is running
# (the critic Jacobian of the scaling regulariser).  A custom Function cannot
# see which edges the engine needs, so without this every conv of that pass
# would also run a weight-gradient kernel whose result is discarded.
_input_only = [0]


class input_grad_only:
    def __enter__(self):
        _input_only[0] += 1

    def __exit__(self, *a):
        _input_only[0] -= 1


# storages whose gradient a backward pass does not need although they require
# grad: the critic step's real images (a leaf only for the Jacobian of the
# scaling regulariser; the parameter backward never reads their gradient)
_no_dx = set()


class no_input_grad:
    """Within the block, convolutions whose input IS `t` skip their input
    gradient (returned as None: the engine treats it as zero)."""

    def __init__(self, t):
        self.key = t.data_ptr()

    def __enter__(self):
        _no_dx.add(self.key)

    def __exit__(self, *a):
        _no_dx.discard(self.key)


# ---------------------------------------------------------------------------
# thin 3x3 convolutions on the library (SMMD_THIN_CONV=0: MIOpen for them too)
# ---------------------------------------------------------------------------
THIN = os.environ.get('SMMD_THIN_CONV', '1') != '0'
THIN_MAX_W = 64          # the library's cross-lane column tiling (smmd_thin.hip)


def thin_applicable(x, cin, cout, k, stride, padding):
    """True when conv(x, [cout, cin, k, k], stride, padding) -- and its input
    and weight gradients -- run on the library's thin kernels: an NCHW fp32
    device tensor, 3 x 3 at stride 1 with padding 1, one side <= 4 channels,
    width <= 64."""
    s = tuple(stride) if isinstance(stride, (list, tuple)) else (stride, stride)
    p = tuple(padding) if isinstance(padding, (list, tuple)) else (padding, padding)
    return (THIN and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and x.is_contiguous() and k == 3 and s == (1, 1) and p == (1, 1)
            and min(cin, cout) <= 4 and x.shape[1] == cin and x.shape[3] <= THIN_MAX_W)


def _thin_conv(x, w, b, mode):
    """smmd_conv3x3_thin: mode 0 conv(x, w) + b (w [co, ci, 3, 3]); mode 1 the
    input gradient of a conv with weight w [ci', co', 3, 3] at upstream x."""
    from . import _lib
    x = x.contiguous()
    w = w.contiguous()
    if b is not None:
        b = b.contiguous()
    _lib.require_cuda(x, w)
    N, ci, H, W = x.shape
    co = w.shape[0] if mode == 0 else w.shape[1]
    y = torch.empty((N, co, H, W), dtype=x.dtype, device=x.device)
    _lib.add_bytes('smmd_conv3x3_thin', (x.numel() + y.numel()) * 4)
    with _lib.timed('smmd_conv3x3_thin'):
        st = _lib.lib().smmd_conv3x3_thin(_lib.ptr(x), _lib.ptr(w),
                                          _lib.ptr(b) if b is not None else None, _lib.ptr(y),
                                          N, ci, co, H, W, int(mode),
                                          _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_conv3x3_thin')
    return y


def _gw_out(into, shape, like):
    """the weight gradient's output: a new tensor, or `into` (a contiguous
    earlier contribution the *_acc entry point adds to; convops._late_gw)."""
    if into is None:
        return torch.empty(shape, dtype=like.dtype, device=like.device), ''
    assert tuple(into.shape) == tuple(shape) and into.is_contiguous()
    return into, '_acc'


def _thin_wgrad(gy, x, into=None):
    """smmd_conv3x3_thin_wgrad: gw[o][i][t] = sum gy[n, o, p] x[n, i, p + d(t)]
    (into: added to it)."""
    from . import _lib
    gy = gy.contiguous()
    x = x.contiguous()
    _lib.require_cuda(gy, x)
    N, co, H, W = gy.shape
    ci = x.shape[1]
    L = _lib.lib()
    nbytes = L.smmd_conv3x3_thin_wgrad_workspace_bytes(N, ci, co, H, W)
    ws = _lib.workspace('thin_wgrad', nbytes, gy.device)
    gw, acc = _gw_out(into, (co, ci, 3, 3), gy)
    _lib.add_bytes('smmd_conv3x3_thin_wgrad', (gy.numel() + x.numel()) * 4)
    with _lib.timed('smmd_conv3x3_thin_wgrad'):
        st = getattr(L, 'smmd_conv3x3_thin_wgrad' + acc)(
            _lib.ptr(gy), _lib.ptr(x), _lib.ptr(gw), N, ci, co, H, W, _lib.ptr(ws), ws.numel(),
            _lib.stream_handle(gy.device))
    _lib.check(st, 'smmd_conv3x3_thin_wgrad')
    return gw


# ---------------------------------------------------------------------------
# wide 3x3 stride-1 convolutions on the library's Winograd kernel
# (SMMD_WINO=0: MIOpen for them)
# ---------------------------------------------------------------------------
WINO = os.environ.get('SMMD_WINO', '1') != '0'


def _under_2g(x, out_per_in_channel):
    """The Winograd kernels address their input and output by 32-bit byte
    offsets into a 0x7fffffff-byte buffer range (2^31 is the out-of-range
    sentinel): both under 2^29 floats = 2 GiB (out_per_in_channel: output
    elements per input element of one channel plane, e.g. cout for a same-size
    conv).  The library's *_supported checks hold the same bound."""
    plane = x.shape[0] * x.shape[2] * x.shape[3]
    return x.numel() < (1 << 29) and plane * out_per_in_channel < (1 << 29)


def wino_applicable(x, cin, cout, k, stride, padding):
    """True when conv(x, [cout, cin, 3, 3], stride 1, padding 1) runs on
    `smmd_wino3x3_conv`: an NCHW fp32 contiguous device tensor with even height
    and width, cin % 8 == 0 and cout % 64 == 0."""
    s = tuple(stride) if isinstance(stride, (list, tuple)) else (stride, stride)
    p = tuple(padding) if isinstance(padding, (list, tuple)) else (padding, padding)
    return (WINO and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and x.is_contiguous() and k == 3 and s == (1, 1) and p == (1, 1)
            and x.shape[1] == cin and cin % 8 == 0 and cout % 64 == 0
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 and x.shape[2] > 0
            and x.shape[3] > 0 and x.shape[0] > 0 and _under_2g(x, cout))


# transformed filters of the weights in use: a critic step convolves each
# weight several times (real and fake forward, the Jacobian's and the loss's
# input gradients, the double backward), and its transform costs 7-15 us.
# An entry is valid while its weight is the same live tensor at the same torch
# version and FlatAdam epoch (the fused optimizer writes parameters without
# bumping versions; the SN bank's W_eff is a new tensor every refresh).  The
# entry holds the weight only through a weak reference whose finalizer drops
# the entry when the weight is freed, so a superseded W_eff or folded filter
# takes its transform with it instead of pinning both until an eviction.  Not
# used during HIP-graph capture (a replay must re-transform what it convolves):
# there the capture's own cache below serves the step's repeated transforms.
# Shared by the 3x3 and the stride-2 kernels, capped at 1 GiB of transforms
# (a 512 -> 1024 stride-2 filter transforms to 75 MB), oldest first.
_WINO_CACHE = {}        # key -> (weakref to w, version, epoch, u)
_WINO_CACHE_MAX_BYTES = 1 << 30
_wino_cache_bytes = [0]


# A step-graph capture's own filter cache (StepGraphs._capture arms it): inside
# one captured step every weight keeps its values (the update comes last), so
# a weight convolved several times is transformed once and the later launches
# read the graph-pool buffer the first one wrote -- in every replay too.  It
# holds the weights strongly (no id reuse) and lives for one capture only: a
# buffer of another graph's pool must never be read.
_CAPTURE_CACHE = [None]


def arm_capture_cache(on):
    _CAPTURE_CACHE[0] = {} if on else None


def _filter_cache_get(key, w):
    """(cached transform or None, whether the result may be stored)."""
    if not torch.cuda.is_current_stream_capturing():
        return _cache_get(key, w), True
    cc = _CAPTURE_CACHE[0]
    if cc is None:
        return None, False
    e = cc.get(key)
    if e is not None and e[0] is w and e[1] == w._version:
        return e[2], True
    return None, True


def _filter_cache_put(key, w, u):
    if not torch.cuda.is_current_stream_capturing():
        _cache_put(key, w, u)
    elif _CAPTURE_CACHE[0] is not None:
        _CAPTURE_CACHE[0][key] = (w, w._version, u)


def _cache_get(key, w):
    e = _WINO_CACHE.get(key)
    if e is not None and e[0]() is w and e[1] == w._version and e[2] == _param_epoch(w):
        return e[3]
    return None


def _cache_drop(key, ref=None):
    """Remove `key` (only if it still holds `ref`, when given)."""
    e = _WINO_CACHE.get(key)
    if e is not None and (ref is None or e[0] is ref):
        del _WINO_CACHE[key]
        _wino_cache_bytes[0] -= e[3].numel() * e[3].element_size()


def _cache_put(key, w, u):
    import weakref
    _cache_drop(key)
    nb = u.numel() * u.element_size()
    while _WINO_CACHE and _wino_cache_bytes[0] + nb > _WINO_CACHE_MAX_BYTES:
        _cache_drop(next(iter(_WINO_CACHE)))
    ref = weakref.ref(w, lambda r, k=key: _cache_drop(k, r))
    _WINO_CACHE[key] = (ref, w._version, _param_epoch(w), u)
    _wino_cache_bytes[0] += nb


# Effective SN weights the refresh did not write (sn.SpectralNormBank.lazy):
# the Winograd filter transforms form them from the raw W and the device
# sigma and s (smmd_wino3x3_filter_sn, smmd_wino4x4s2(t)_filter_sn, bit-identical
# to transforming a written W_eff), and every other consumer materialises the
# values first (`materialize`).  id(tensor) -> [weakref, SN entry, fold, done,
# stamp].  The values are formed from the entry's CURRENT W, sigma and s, so a
# record is valid only while they are the ones of its refresh: `stamp` holds
# the entry's refresh generation and the weight's FlatAdam epoch and version,
# and a reader after a later refresh or update gets an error instead of the
# values of another W (model._detach_step_state drops lazy tensors at the end
# of every step, so the training loop never holds one that long).
_LAZY = {}


class StaleLazyWeight(RuntimeError):
    pass


def _lazy_stamp(entry):
    W = entry.weight
    return (getattr(entry, 'refresh_gen', 0), _param_epoch(W), W._version)


def register_lazy(w, entry, fold):
    import weakref
    key = id(w)
    ref = weakref.ref(w, lambda r, k=key: _LAZY.pop(k, None) if (
        _LAZY.get(k) is not None and _LAZY[k][0] is r) else None)
    _LAZY[key] = [ref, entry, bool(fold), False, _lazy_stamp(entry)]


def is_lazy(w):
    """True for an unwritten lazy W_eff, current or stale."""
    rec = _LAZY.get(id(w))
    return rec is not None and rec[0]() is w and not rec[3]


def _lazy(w):
    rec = _LAZY.get(id(w))
    if rec is None or rec[0]() is not w or rec[3]:
        return None
    if rec[4] != _lazy_stamp(rec[1]):
        raise StaleLazyWeight(
            'an unwritten spectrally normalised weight (W_eff) of an earlier refresh was '
            'read after its layer was refreshed or updated; its values can no longer be '
            'formed (materialize it before the update, or use the current W_eff)')
    return rec


def materialize(w):
    """Write the values of a lazily refreshed SN weight (W_eff = (W / sigma) s,
    or its ConvMeanPool fold) into ``w`` before a consumer reads them directly
    (MIOpen, the thin kernels, an unfold); a no-op for any other tensor."""
    rec = _lazy(w)
    if rec is None:
        return w
    e, fold = rec[1], rec[2]
    with torch.no_grad():
        W = e.weight
        s = e.scale
        weff = torch.div(W, e.sigma)
        if s is not None and s.numel() > 0:
            weff = weff.mul_(s)
        if fold:
            _fold_launch_into([weff.contiguous()], [w], adjoint=False)
        else:
            w.copy_(weff.view_as(w))
    rec[3] = True
    return w


def _param_epoch(w):
    from . import optim as _optim
    return _optim.param_epoch(w)


def _wino_filter(w, co, ci, mode):
    from . import _lib
    key = (id(w), 'w3', mode)
    u, store = _filter_cache_get(key, w)
    if u is not None:
        return u
    L = _lib.lib()
    u = torch.empty(L.smmd_wino3x3_filter_bytes(co, ci) // 4, dtype=w.dtype, device=w.device)
    lz = _lazy(w)
    with _lib.timed('smmd_wino3x3_filter'):
        if lz is not None:      # from the raw SN weight: W_eff was never written
            e = lz[1]
            sc = e.scale if e.scale is not None and e.scale.numel() > 0 else None
            st = L.smmd_wino3x3_filter_sn(_lib.ptr(e.weight), _lib.ptr(e.sigma), _lib.ptr(sc), co,
                                          ci, int(mode), _lib.ptr(u), u.numel() * 4,
                                          _lib.stream_handle(w.device))
        else:
            st = L.smmd_wino3x3_filter(_lib.ptr(w), co, ci, int(mode), _lib.ptr(u), u.numel() * 4,
                                       _lib.stream_handle(w.device))
    _lib.check(st, 'smmd_wino3x3_filter')
    if store:
        _filter_cache_put(key, w, u)
    return u


def clear_wino_cache():
    _WINO_CACHE.clear()
    _wino_cache_bytes[0] = 0


def _wino_conv(x, w, b, mode, relu=False, mask=None):
    """smmd_wino3x3_filter + smmd_wino3x3_conv: mode 0 conv(x, w) + b
    (w [co, ci, 3, 3]); mode 1 the input gradient of a conv with weight
    w [ci', co', 3, 3] at upstream x.  mask (y's shape): y = (mask <= 0 ? 0 :
    y), smmd_wino3x3_conv_mask."""
    from . import _lib
    x = x.contiguous()
    w = w.contiguous()
    if b is not None:
        b = b.contiguous()
    _lib.require_cuda(x, w, b)
    N, ci, H, W = x.shape
    co = w.shape[0] if mode == 0 else w.shape[1]
    L = _lib.lib()
    u = _wino_filter(w, co, ci, mode)
    y = torch.empty((N, co, H, W), dtype=x.dtype, device=x.device)
    nb = L.smmd_wino3x3_workspace_bytes(N, ci, co, H, W)
    ws = _lib.workspace('wino', nb, x.device) if nb else None
    _lib.add_bytes('smmd_wino3x3_conv', (x.numel() + y.numel()) * 4)
    # 16 transform-point products per 2 x 2 output tile and (ci, co) pair
    _lib.add_flops('smmd_wino3x3_conv', 2 * 16 * N * (H // 2) * (W // 2) * ci * co)
    with _lib.timed('smmd_wino3x3_conv'):
        if mask is not None:
            assert mask.shape == y.shape and mask.is_contiguous() and mask.dtype == y.dtype
            st = L.smmd_wino3x3_conv_mask(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(mask),
                                          _lib.ptr(y), N, ci, co, H, W, _lib.ptr(ws), nb,
                                          _lib.stream_handle(x.device))
        else:
            fn = L.smmd_wino3x3_conv_relu if relu else L.smmd_wino3x3_conv
            st = fn(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, ci, co, H, W,
                    _lib.ptr(ws), nb, _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_wino3x3_conv')
    return y


def _wino_conv2(x, w, x2, w2):
    """conv(x, w) + conv(x2, w2) (3x3 stride 1 SAME, same shapes) in ONE
    smmd_wino3x3_conv2 launch: the input-channel loop runs over both pairs."""
    from . import _lib
    x, x2 = x.contiguous(), x2.contiguous()
    w, w2 = w.contiguous(), w2.contiguous()
    _lib.require_cuda(x, w, x2, w2)
    N, ci, H, W = x.shape
    co = w.shape[0]
    L = _lib.lib()
    u = _wino_filter(w, co, ci, 0)
    u2 = _wino_filter(w2, co, ci, 0)
    y = torch.empty((N, co, H, W), dtype=x.dtype, device=x.device)
    nb = L.smmd_wino3x3_conv2_workspace_bytes(N, ci, co, H, W)
    ws = _lib.workspace('wino', nb, x.device) if nb else None
    _lib.add_bytes('smmd_wino3x3_conv', (2 * x.numel() + y.numel()) * 4)
    _lib.add_flops('smmd_wino3x3_conv', 2 * 2 * 16 * N * (H // 2) * (W // 2) * ci * co)
    with _lib.timed('smmd_wino3x3_conv'):
        st = L.smmd_wino3x3_conv2(_lib.ptr(x), _lib.ptr(u), _lib.ptr(x2), _lib.ptr(u2), None,
                                  _lib.ptr(y), N, ci, co, H, W, _lib.ptr(ws), nb,
                                  _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_wino3x3_conv2')
    return y


# the weight gradient of those layers (SMMD_WINO_WGRAD=0: MIOpen)
WINO_WGRAD = os.environ.get('SMMD_WINO_WGRAD', '1') != '0'


def _wino_wgrad(x, gy, into=None):
    """smmd_wino3x3_wgrad: gw [co, ci, 3, 3] of conv(x, W, stride 1, pad 1) at gy
    (into: added to it)."""
    from . import _lib
    x = x.contiguous()
    gy = gy.contiguous()
    _lib.require_cuda(x, gy)
    N, ci, H, W = x.shape
    co = gy.shape[1]
    L = _lib.lib()
    nb = L.smmd_wino3x3_wgrad_workspace_bytes(N, ci, co, H, W)
    ws = _lib.workspace('wino_wgrad', nb, x.device)
    gw, acc = _gw_out(into, (co, ci, 3, 3), x)
    _lib.add_bytes('smmd_wino3x3_wgrad', (x.numel() + gy.numel()) * 4)
    _lib.add_flops('smmd_wino3x3_wgrad', 2 * 16 * N * (H // 2) * (W // 2) * ci * co)
    with _lib.timed('smmd_wino3x3_wgrad'):
        st = getattr(L, 'smmd_wino3x3_wgrad' + acc)(
            _lib.ptr(x), _lib.ptr(gy), _lib.ptr(gw), N, ci, co, H, W, _lib.ptr(ws), nb,
            _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_wino3x3_wgrad')
    return gw


def _wgrad_ok(x, gy, w, stride, padding):
    return (WINO_WGRAD and _is_wino(x, w, stride, padding, 0) and gy.is_contiguous()
            and x.shape[1] % 64 == 0 and gy.shape[1] % 64 == 0 and x.shape[3] % 4 == 0)


def _is_wino(x, w, stride, padding, mode):
    """mode 0: conv(x, w); mode 1: its input gradient at upstream x (x has
    w.shape[0] channels, the result w.shape[1])."""
    if w.dim() != 4 or w.shape[2] != 3 or w.shape[3] != 3:
        return False
    ci, co = (w.shape[1], w.shape[0]) if mode == 0 else (w.shape[0], w.shape[1])
    return wino_applicable(x, ci, co, 3, stride, padding)


# ---------------------------------------------------------------------------
# 4x4 stride-2 pad-1 convolutions (the folded ConvMeanPool layers) and their
# transposed form (their input gradient; the generator's folded
# UpsampleConv) on the library's polyphase Winograd F(2x2, 2x2) kernels
# (smmd_wino4x4s2*, csrc/smmd_wino_s2.hip; SMMD_WINO_S2=0: MIOpen for them)
# ---------------------------------------------------------------------------
WINO_S2 = os.environ.get('SMMD_WINO_S2', '1') != '0'


def _s2_shape_ok(x, stride, padding):
    s = tuple(stride) if isinstance(stride, (list, tuple)) else (stride, stride)
    p = tuple(padding) if isinstance(padding, (list, tuple)) else (padding, padding)
    return (WINO_S2 and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and x.is_contiguous() and s == (2, 2) and p == (1, 1) and x.shape[0] > 0)


def _is_s2(x, w, stride, padding):
    """conv(x, w [co, ci, 4, 4], stride 2, padding 1) on smmd_wino4x4s2_conv:
    H, W % 4 == 0, ci % 2 == 0, co % 64 == 0."""
    return (w.dim() == 4 and w.shape[2] == 4 and w.shape[3] == 4 and _s2_shape_ok(x, stride, padding)
            and x.shape[1] == w.shape[1] and w.shape[1] % 2 == 0 and w.shape[0] % 64 == 0
            and x.shape[2] % 4 == 0 and x.shape[3] % 4 == 0 and _under_2g(x, w.shape[0] / 4))


def _is_s2t(g, w, stride, padding):
    """conv_transpose(g, w [k, c, 4, 4], stride 2, padding 1) on
    smmd_wino4x4s2t_conv: g [n, k, hg, wg] with hg, wg even, k % 8 == 0,
    c % 64 == 0."""
    return (w.dim() == 4 and w.shape[2] == 4 and w.shape[3] == 4 and _s2_shape_ok(g, stride, padding)
            and g.shape[1] == w.shape[0] and w.shape[0] % 8 == 0 and w.shape[1] % 64 == 0
            and g.shape[2] % 2 == 0 and g.shape[3] % 2 == 0 and _under_2g(g, w.shape[1] * 4))


def _s2_filter(w, transposed):
    from . import _lib
    key = (id(w), 's2', transposed)
    u, store = _filter_cache_get(key, w)
    if u is not None:
        return u
    L = _lib.lib()
    a, b = w.shape[0], w.shape[1]
    u = torch.empty(L.smmd_wino4x4s2_filter_bytes(a, b) // 4, dtype=w.dtype, device=w.device)
    lz = _lazy(w)
    with _lib.timed('smmd_wino4x4s2_filter'):
        if lz is not None:      # from the raw SN weight (and its fold): W' was never written
            e = lz[1]
            sc = e.scale if e.scale is not None and e.scale.numel() > 0 else None
            fn = L.smmd_wino4x4s2t_filter_sn if transposed else L.smmd_wino4x4s2_filter_sn
            st = fn(_lib.ptr(e.weight), _lib.ptr(e.sigma), _lib.ptr(sc), int(lz[2]), a, b,
                    _lib.ptr(u), u.numel() * 4, _lib.stream_handle(w.device))
        else:
            fn = L.smmd_wino4x4s2t_filter if transposed else L.smmd_wino4x4s2_filter
            st = fn(_lib.ptr(w), a, b, _lib.ptr(u), u.numel() * 4, _lib.stream_handle(w.device))
    _lib.check(st, 'smmd_wino4x4s2_filter')
    if store:
        _filter_cache_put(key, w, u)
    return u


def _s2_conv(x, w, b, into=None):
    """conv2d(x, w, b, stride 2, padding 1) on smmd_wino4x4s2_conv (into: added
    to it, smmd_wino4x4s2_conv_acc, and returned)."""
    from . import _lib
    x = x.contiguous()
    w = w.contiguous()
    if b is not None:
        b = b.contiguous()
    _lib.require_cuda(x, w, b)
    N, ci, H, W = x.shape
    co = w.shape[0]
    L = _lib.lib()
    u = _s2_filter(w, False)
    shape = (N, co, H // 2, W // 2)
    if into is not None:
        assert tuple(into.shape) == shape and into.is_contiguous() and into.dtype == x.dtype
    y = torch.empty(shape, dtype=x.dtype, device=x.device) if into is None else into
    nb = L.smmd_wino4x4s2_workspace_bytes(N, ci, co, H, W)
    ws = _lib.workspace('wino_s2', nb, x.device) if nb else None
    _lib.add_bytes('smmd_wino4x4s2_conv', (x.numel() + y.numel()) * 4)
    # 9 point products per 2 x 2 output tile and (phase channel, co) pair
    _lib.add_flops('smmd_wino4x4s2_conv', 2 * 9 * N * (H // 4) * (W // 4) * 4 * ci * co)
    fn = L.smmd_wino4x4s2_conv if into is None else L.smmd_wino4x4s2_conv_acc
    with _lib.timed('smmd_wino4x4s2_conv'):
        st = fn(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, ci, co, H, W, _lib.ptr(ws),
                nb, _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_wino4x4s2_conv')
    return y


def _s2_conv2(x, w, x2, w2):
    """conv(x, w) + conv(x2, w2) (4x4 stride 2 pad 1, same shapes) in ONE
    smmd_wino4x4s2_conv2 launch."""
    from . import _lib
    x, x2 = x.contiguous(), x2.contiguous()
    w, w2 = w.contiguous(), w2.contiguous()
    _lib.require_cuda(x, w, x2, w2)
    N, ci, H, W = x.shape
    co = w.shape[0]
    L = _lib.lib()
    u = _s2_filter(w, False)
    u2 = _s2_filter(w2, False)
    y = torch.empty((N, co, H // 2, W // 2), dtype=x.dtype, device=x.device)
    nb = L.smmd_wino4x4s2_conv2_workspace_bytes(N, ci, co, H, W)
    ws = _lib.workspace('wino_s2', nb, x.device) if nb else None
    _lib.add_bytes('smmd_wino4x4s2_conv', (2 * x.numel() + y.numel()) * 4)
    _lib.add_flops('smmd_wino4x4s2_conv', 2 * 2 * 9 * N * (H // 4) * (W // 4) * 4 * ci * co)
    with _lib.timed('smmd_wino4x4s2_conv'):
        st = L.smmd_wino4x4s2_conv2(_lib.ptr(x), _lib.ptr(u), _lib.ptr(x2), _lib.ptr(u2), None,
                                    _lib.ptr(y), N, ci, co, H, W, _lib.ptr(ws), nb,
                                    _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_wino4x4s2_conv2')
    return y


def _s2t_conv(g, w, b, mask=None):
    """conv_transpose2d(g, w [k, c, 4, 4], b, stride 2, padding 1) on
    smmd_wino4x4s2t_conv (the input gradient of conv(., w, stride 2)); with
    mask (the conv's input, a ReLU output) TF's ReLU gradient of it in the same
    launch (smmd_wino4x4s2t_conv_mask): threshold_backward(dx, mask, 0)."""
    from . import _lib
    g = g.contiguous()
    w = w.contiguous()
    if b is not None:
        b = b.contiguous()
    _lib.require_cuda(g, w, b)
    N, k, Hg, Wg = g.shape
    c = w.shape[1]
    L = _lib.lib()
    u = _s2_filter(w, True)
    y = torch.empty((N, c, 2 * Hg, 2 * Wg), dtype=g.dtype, device=g.device)
    nb = L.smmd_wino4x4s2t_workspace_bytes(N, k, c, Hg, Wg)
    ws = _lib.workspace('wino_s2t', nb, g.device) if nb else None
    _lib.add_bytes('smmd_wino4x4s2t_conv', (g.numel() + y.numel()) * 4)
    _lib.add_flops('smmd_wino4x4s2t_conv', 2 * 9 * N * (Hg // 2) * (Wg // 2) * 4 * k * c)
    if mask is not None:
        mask = mask.contiguous()
        assert mask.shape == y.shape and mask.dtype == y.dtype
        _lib.add_bytes('smmd_wino4x4s2t_conv', mask.numel() * 4)
    with _lib.timed('smmd_wino4x4s2t_conv'):
        if mask is None:
            st = L.smmd_wino4x4s2t_conv(_lib.ptr(g), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, k,
                                        c, Hg, Wg, _lib.ptr(ws), nb, _lib.stream_handle(g.device))
        else:
            st = L.smmd_wino4x4s2t_conv_mask(_lib.ptr(g), _lib.ptr(u), _lib.ptr(b),
                                             _lib.ptr(mask), _lib.ptr(y), N, k, c, Hg, Wg,
                                             _lib.ptr(ws), nb, _lib.stream_handle(g.device))
    _lib.check(st, 'smmd_wino4x4s2t_conv')
    return y


# the weight gradient of the stride-2 layers on the polyphase Winograd kernel
# (smmd_wino4x4s2_wgrad, csrc/smmd_wino_s2_wgrad.hip; SMMD_WINO_S2_WGRAD=0: MIOpen)
WINO_S2_WGRAD = os.environ.get('SMMD_WINO_S2_WGRAD', '1') != '0'


def _s2_wgrad_ok(x, gy, co):
    """gw [co, ci, 4, 4] of conv(x, ., stride 2, pad 1) at gy runs on
    smmd_wino4x4s2_wgrad: NCHW fp32 contiguous device tensors of the shapes
    the kernel tiles."""
    if not (WINO_S2_WGRAD and x.is_cuda and gy.is_cuda and x.dtype == torch.float32
            and gy.dtype == torch.float32 and x.dim() == 4 and gy.dim() == 4
            and x.is_contiguous() and gy.is_contiguous()):
        return False
    n, ci, h, w = x.shape
    if tuple(gy.shape) != (n, co, h // 2, w // 2):
        return False
    from . import _lib
    return bool(_lib.lib().smmd_wino4x4s2_wgrad_supported(n, ci, co, h, w))


def _s2_wgrad(x, gy, into=None):
    """smmd_wino4x4s2_wgrad: gw [co, ci, 4, 4] of conv(x, W', stride 2, pad 1)
    at gy [n, co, h/2, w/2] (into: added to it)."""
    from . import _lib
    _lib.require_cuda(x, gy)
    N, ci, H, W = x.shape
    co = gy.shape[1]
    L = _lib.lib()
    nb = L.smmd_wino4x4s2_wgrad_workspace_bytes(N, ci, co, H, W)
    ws = _lib.workspace('wino_s2_wgrad', nb, x.device)
    gw, acc = _gw_out(into, (co, ci, 4, 4), x)
    _lib.add_bytes('smmd_wino4x4s2_wgrad', (x.numel() + gy.numel()) * 4)
    # 9 point products per 2 x 2 output tile and (phase column, co) pair
    _lib.add_flops('smmd_wino4x4s2_wgrad', 2 * 9 * N * (H // 4) * (W // 4) * 4 * ci * co)
    with _lib.timed('smmd_wino4x4s2_wgrad'):
        st = getattr(L, 'smmd_wino4x4s2_wgrad' + acc)(
            _lib.ptr(x), _lib.ptr(gy), _lib.ptr(gw), N, ci, co, H, W, _lib.ptr(ws), nb,
            _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_wino4x4s2_wgrad')
    return gw


def _s2_weight_grad(gy, x, w, stride, padding, into=None):
    """gw of conv(x, w [co, ci, 4, 4], stride 2, pad 1) at gy: the library's
    polyphase kernel where it tiles the shapes, MIOpen otherwise (into: added
    to it; the returned tensor is then `into`)."""
    if _s2_wgrad_ok(x, gy, w.shape[0]):
        return _s2_wgrad(x.contiguous(), gy.contiguous(), into)
    return _aten.convolution_backward(gy, x, w, None, stride, padding, [1, 1], False,
                                      [0, 0], 1, [False, True, False])[1]


class _ConvT2dS2(torch.autograd.Function):
    """conv_transpose2d(x, w [cin, cout, 4, 4], b, stride 2, padding 1): the
    generator's folded UpsampleConv.  Backward: grad_x = conv(g, w, stride 2)
    on the forward Winograd kernel, grad_w on the stride-2 weight-gradient
    kernel (x and g in swapped roles), grad_b the channel sum (the generator
    step differentiates it once)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return _s2t_conv(x, w, b)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = _s2_conv(gy, w, None) if _is_s2(gy, w, 2, 1) else F.conv2d(gy, w, None, 2, 1)
        if ctx.needs_input_grad[1]:
            # conv_transpose(x, w) = Dx of conv(., w): its weight gradient is
            # the stride-2 conv's weight gradient at input gy, upstream x
            if _s2_wgrad_ok(gy, x.contiguous(), w.shape[0]):
                gw = _s2_wgrad(gy, x.contiguous())
            else:
                _, gw, _ = _aten.convolution_backward(gy, x, w, None, [2, 2], [1, 1], [1, 1], True,
                                                      [0, 0], 1, [False, True, False])
        if ctx.has_b and ctx.needs_input_grad[2]:
            gb = bias_grad(gy)
        return gx, gw, gb


def conv_transpose_s2(x, w, b=None):
    """F.conv_transpose2d(x, w, b, stride=2, padding=1) with the Winograd
    kernels on device tensors they tile, PyTorch otherwise."""
    if _is_s2t(x, w, 2, 1):
        return _ConvT2dS2.apply(x, w, b)
    return F.conv_transpose2d(x, w, b, stride=2, padding=1)


# SMMD_CONV1X1=0: the 1x1 shortcut convolutions on MIOpen
CONV1X1 = os.environ.get('SMMD_CONV1X1', '1') != '0'


def _is_c1(x, w, stride, padding):
    """A 1x1 stride-1 unpadded conv on an NCHW fp32 contiguous device tensor
    (the residual shortcuts, block.py:28-40): `smmd_conv1x1*`."""
    return (CONV1X1 and w.dim() == 4 and tuple(w.shape[2:]) == (1, 1)
            and list(stride) == [1, 1] and list(padding) == [0, 0] and x.is_cuda
            and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 4
            and x.is_contiguous() and x.shape[1] == w.shape[1] and x.data_ptr() % 16 == 0)


def _c1_gemm(a, x, b, m, ta=False):
    """y [N, m, H, W] = a [m, r] . x [N, r, H, W] (+ b) on smmd_conv1x1 (ta: a
    given as its transpose [r, m], smmd_conv1x1_t), or None when the library
    does not tile the shape."""
    from . import _lib
    N, r, H, W = x.shape
    P = H * W
    L = _lib.lib()
    if not L.smmd_conv1x1_supported(N, r, m, P) or a.data_ptr() % 16:
        return None
    y = torch.empty((N, m, H, W), dtype=x.dtype, device=x.device)
    if b is not None:
        b = b.contiguous()
    nb = L.smmd_conv1x1_workspace_bytes(N, r, m, P)
    ws = _lib.workspace('conv1x1', nb, x.device) if nb else None
    _lib.add_bytes('smmd_conv1x1', (x.numel() + y.numel() + a.numel()) * 4)
    _lib.add_flops('smmd_conv1x1', 2 * N * P * r * m)
    fn = L.smmd_conv1x1_t if ta else L.smmd_conv1x1
    with _lib.timed('smmd_conv1x1'):
        st = fn(_lib.ptr(a), _lib.ptr(x), _lib.ptr(b), _lib.ptr(y), N, r, m, P, _lib.ptr(ws), nb,
                _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_conv1x1')
    return y


def _c1_fwd(x, w, b):
    w = materialize(w)
    return _c1_gemm(w.reshape(w.shape[0], w.shape[1]).contiguous(), x, b, w.shape[0])


def _c1_wt(w):
    """W^T [cin, cout] of a 1x1 weight, cached like the filter transforms (a
    critic step takes several input gradients of each shortcut)."""
    key = (id(w), 'c1t')
    u, store = _filter_cache_get(key, w)
    if u is not None:
        return u
    u = materialize(w).reshape(w.shape[0], w.shape[1]).t().contiguous()
    if store:
        _filter_cache_put(key, w, u)
    return u


# SMMD_C1_DX_T=0: the input gradient from a W^T copy (_c1_wt) instead of W
C1_DX_T = os.environ.get('SMMD_C1_DX_T', '1') != '0'


def _c1_dx(gy, w):
    if C1_DX_T:
        wm = materialize(w).reshape(w.shape[0], w.shape[1])
        if wm.is_contiguous():
            return _c1_gemm(wm, gy, None, w.shape[1], ta=True)
    return _c1_gemm(_c1_wt(w), gy, None, w.shape[1])


def _c1_wgrad(gy, x, into=None):
    from . import _lib
    N, C, H, W = x.shape
    K = gy.shape[1]
    P = H * W
    L = _lib.lib()
    if (not L.smmd_conv1x1_wgrad_supported(N, C, K, P) or gy.data_ptr() % 16
            or not gy.is_contiguous()):
        return None
    gw, acc = _gw_out(into, (K, C, 1, 1), x)
    nb = L.smmd_conv1x1_wgrad_workspace_bytes(N, C, K, P)
    ws = _lib.workspace('conv1x1_wgrad', nb, x.device) if nb else None
    _lib.add_bytes('smmd_conv1x1_wgrad', (x.numel() + gy.numel() + gw.numel()) * 4)
    _lib.add_flops('smmd_conv1x1_wgrad', 2 * N * P * C * K)
    with _lib.timed('smmd_conv1x1_wgrad'):
        st = getattr(L, 'smmd_conv1x1_wgrad' + acc)(
            _lib.ptr(gy), _lib.ptr(x), _lib.ptr(gw), N, C, K, P, _lib.ptr(ws), nb,
            _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_conv1x1_wgrad')
    return gw


def _is_thin(x, w, stride, padding):
    return thin_applicable(x, w.shape[1], w.shape[0], w.shape[2], stride, padding) \
        and w.shape[2] == w.shape[3]


def _fwd(x, w, b, stride, padding, ymask=None, into=None):
    """conv(x, w) + b: the library's kernels or MIOpen.  ymask (the output's
    shape): the result masked as threshold_backward(y, ymask, 0), in the 3x3
    Winograd kernel's epilogue where it runs there.  into (not with ymask):
    the result added to it (into + y, in the stride-2 kernel's epilogue where
    it runs there) and returned."""
    if into is not None:
        if _is_s2(x, w, stride, padding) and into.is_contiguous():
            return _s2_conv(x, w, b, into)
        return into.add_(_fwd(x, w, b, stride, padding))
    if ymask is not None:
        if (_is_wino(x, w, stride, padding, 0) and ymask.is_contiguous()
                and os.environ.get('SMMD_WINO8', '1') != '0'):
            return _wino_conv(x, w, b, 0, mask=ymask)
        return _aten.threshold_backward(_fwd(x, w, b, stride, padding), ymask, 0.0)
    if _is_thin(x, w, stride, padding):
        return _thin_conv(x, materialize(w), b, 0)
    if _is_wino(x, w, stride, padding, 0):
        return _wino_conv(x, w, b, 0)
    if _is_s2(x, w, stride, padding):
        return _s2_conv(x, w, b)
    if _is_c1(x, w, stride, padding):
        y = _c1_fwd(x, w, b)
        if y is not None:
            return y
    return F.conv2d(x, materialize(w), b, stride, padding)


# conv(x, w) + conv(x2, w2) as one pair launch (SMMD_CONV_PAIR=0: two
# launches and an add)
CONV_PAIR = os.environ.get('SMMD_CONV_PAIR', '1') != '0'


def _fwd2(x, w, x2, w2, stride, padding):
    """conv(x, w) + conv(x2, w2) on one library launch when both convs take
    the same Winograd path; None otherwise."""
    if not (CONV_PAIR and x.shape == x2.shape and w.shape == w2.shape):
        return None
    if _is_wino(x, w, stride, padding, 0) and _is_wino(x2, w2, stride, padding, 0):
        return _wino_conv2(x, w, x2, w2)
    if _is_s2(x, w, stride, padding) and _is_s2(x2, w2, stride, padding):
        return _s2_conv2(x, w, x2, w2)
    return None


def _bwd(gy, x, w, stride, padding, mask, xmask=None, gw_into=None):
    """(Dx, Dw) of conv(x, w) at upstream gy via the native backward kernels.
    xmask (the input x, a ReLU output whose producer skips its mask): Dx
    returned as threshold_backward(Dx, x, 0), inside the stride-2 transposed
    conv's launch where it runs there.  gw_into: Dw is added into it (the
    library's *_wgrad_acc kernels, or an add after the others) and returned."""
    gx, gw, fused = _bwd_core(gy, x, w, stride, padding, mask, xmask, gw_into)
    if xmask is not None and gx is not None and not fused:
        gx = _aten.threshold_backward(gx, xmask, 0.0)
    if gw_into is not None and gw is not None and gw is not gw_into:
        gw_into.add_(gw)
        gw = gw_into
    return gx, gw


def _bwd_core(gy, x, w, stride, padding, mask, xmask, into=None):
    """_bwd's kernels: (Dx, Dw, Dx already masked by xmask)."""
    if mask[0] and not (_is_wino(gy, w, stride, padding, 1) or _is_s2t(gy, w, stride, padding)):
        materialize(w)          # a direct reader of w's values below
    if _is_thin(x, w, stride, padding):
        gx = _thin_conv(gy, w, None, 1) if mask[0] else None
        gw = _thin_wgrad(gy, x, into) if mask[1] else None
        return gx, gw, False
    if _is_c1(x, w, stride, padding) and _is_c1(gy, w.transpose(0, 1), stride, padding):
        gx = _c1_dx(gy, w) if mask[0] else None
        gw = _c1_wgrad(gy, x, into) if mask[1] else None
        # an output the library did not tile comes from aten ALONE: a gw the
        # *_wgrad_acc kernel already added into `into` must not be formed twice
        need_x, need_w = mask[0] and gx is None, mask[1] and gw is None
        if need_x or need_w:
            ax, aw, _ = _aten.convolution_backward(gy, x, materialize(w), None, stride, padding,
                                                   [1, 1], False, [0, 0], 1,
                                                   [need_x, need_w, False])
            gx = ax if need_x else gx
            gw = aw if need_w else gw
        return gx, gw, False
    if mask[1] and _wgrad_ok(x, gy, w, stride, padding):
        gw = _wino_wgrad(x, gy, into)
        gx = None
        if mask[0]:
            gx = (_wino_conv(gy, w, None, 1) if _is_wino(gy, w, stride, padding, 1) else
                  _aten.convolution_backward(gy, x, w, None, stride, padding, [1, 1], False,
                                             [0, 0], 1, [True, False, False])[0])
        return gx, gw, False
    if mask[0] and _is_wino(gy, w, stride, padding, 1):
        gx = _wino_conv(gy, w, None, 1)
        gw = None
        if mask[1]:
            _, gw, _ = _aten.convolution_backward(gy, x, w, None, stride, padding, [1, 1], False,
                                                  [0, 0], 1, [False, True, False])
        return gx, gw, False
    s2 = (w.dim() == 4 and tuple(w.shape[2:]) == (4, 4) and _s2_shape_ok(x, stride, padding)
          and tuple(x.shape[2:]) == (2 * gy.shape[2], 2 * gy.shape[3]))
    if s2 and (mask[1] or _is_s2t(gy, w, stride, padding)):
        gx = gw = None
        fused = False
        if mask[0]:
            if _is_s2t(gy, w, stride, padding):
                fused = xmask is not None and xmask.shape == x.shape
                gx = _s2t_conv(gy, w, None, mask=xmask if fused else None)
            else:
                gx = _aten.convolution_backward(gy, x, w, None, stride, padding, [1, 1], False,
                                                [0, 0], 1, [True, False, False])[0]
        if mask[1]:
            gw = _s2_weight_grad(gy, x, w, stride, padding, into)
        return gx, gw, fused
    gx, gw, _ = _aten.convolution_backward(gy, x, w, None, stride, padding, [1, 1], False,
                                           [0, 0], 1, [mask[0], mask[1], False])
    return gx, gw, False


class _ConvBackward(torch.autograd.Function):
    """(gx, gw) = backward of conv(x, w); differentiable once more.  mask_in:
    gx = threshold_backward(Dx, x, 0) (x a ReLU output whose producer skips
    its mask, _Conv2d's mask_in), and so is the gradient this node returns
    for x.  gy_mask (gy is that masked gx of a mask_in node, _Conv2dReLU with
    consumer_masks): the gradient this node returns for gy is masked by it --
    in the 3x3 Winograd epilogue (smmd_wino3x3_conv_mask) -- and the mask_in
    node, whose only upstream that is, skips its own mask of it
    (_ggx_masked; the select is idempotent, so the result is bit-identical)."""

    @staticmethod
    def forward(ctx, x, w, gy, stride, padding, want_w, mask_in=False, gy_mask=None):
        ctx.save_for_backward(x, w, gy, gy_mask)
        ctx.cfg = (stride, padding, mask_in)
        ctx._smmd_mask_in = bool(mask_in)
        # an output nobody differentiates (the placeholder gw of the input-only
        # Jacobian pass, or gx/gw unused by the loss) arrives as None instead
        # of a materialised zero tensor: otherwise every critic conv of the
        # double backward ran conv(x, 0) and Dx(gy, 0) on it
        ctx.set_materialize_grads(False)
        gx, gw = _bwd(gy, x, w, stride, padding, (True, want_w), x if mask_in else None)
        # gw None (the input-only pass): a non-tensor output, discarded by the
        # caller -- no placeholder tensor, so no fill kernel per call
        return gx, gw

    @staticmethod
    def backward(ctx, ggx, ggw):
        x, w, gy, gy_mask = ctx.saved_tensors
        stride, padding, mask_in = ctx.cfg
        need_x, need_w, need_gy = ctx.needs_input_grad[:3]
        g_x = g_w = g_gy = into = None
        if ggx is not None:
            ggx = ggx.contiguous(memory_format=_fmt(x))
            # gx = m * Dx(gy): its adjoint masks ggx first (unless the node
            # that produced ggx masked it already, _Conv2dReLU's gy_mask)
            if mask_in and not getattr(ctx, '_smmd_ggx_masked', False):
                ggx = (_ReluMask.apply(ggx, x) if torch.is_grad_enabled()
                       else _aten.threshold_backward(ggx, x, 0.0))
        fused_mask = gy_mask is not None and not torch.is_grad_enabled()
        # another node's gradient for the same gy input (a critic block's
        # main path and shortcut both read _ReluPool's gu): this one is
        # computed into it and none returned -- the sum autograd would form
        shared = _shared_gy_key(ctx) if (need_gy and ggx is not None and ggw is None
                                         and gy_mask is None) else None
        gy_into = _late['gy'].get(shared) if shared is not None else None
        # the upstream's gradient conv(ggx, w) + conv(x, ggw): one pair launch
        # when both take the same Winograd path, else two convs and their sum
        pair = None
        if need_gy and ggx is not None and ggw is not None:
            pair = _fwd2(ggx, w, x, ggw, stride, padding)
        if ggx is not None:
            if need_gy and pair is None:
                g_gy = _fwd(ggx, w, None, stride, padding,
                            gy_mask if fused_mask and ggw is None else None,
                            gy_into[1] if gy_into is not None else None)
            if need_w:
                into = _late_target(w)
                _, g_w = _bwd(gy, ggx, w, stride, padding, (False, True), None, into)
        if ggw is not None:
            if need_gy and pair is None:
                t = _fwd(x, ggw, None, stride, padding)
                g_gy = t if g_gy is None else g_gy + t
            if need_x:
                g_x, _ = _bwd(gy, x, ggw, stride, padding, (True, False),
                              x if mask_in else None)
        if pair is not None:
            g_gy = pair
        if gy_mask is not None and g_gy is not None and not (fused_mask and ggx is not None
                                                             and ggw is None):
            g_gy = (_ReluMask.apply(g_gy.contiguous(), gy_mask) if torch.is_grad_enabled()
                    else _aten.threshold_backward(g_gy, gy_mask, 0.0))
        if shared is not None and g_gy is not None:
            if gy_into is not None:     # added into the earlier contribution
                g_gy = None
                _late['gy_acc'] += 1
            elif g_gy.is_contiguous():
                _late['gy'][shared] = (ctx.next_functions[2][0], g_gy)
        return g_x, _late_gw(w, g_w, into), g_gy, None, None, None, None, None


# Late sums of weight gradients (SMMD_WGRAD_LATE_SUM=0: off).  A critic
# weight (an SN bank output, marked by SpectralNormBank.refresh) is convolved
# by the real and the fake forward and by the double backward, and autograd
# adds those contributions as they arrive -- one latency-bound add kernel per
# weight and extra contribution, ~26 per critic step.  While armed (around the
# critic step's backward, MMD_GAN.d_step) the first contribution of such a
# weight goes to autograd as usual and the later ones are queued; the SN
# node's backward (their only consumer, which autograd runs after every
# contribution exists) first adds the queue in arrival order with one
# multi-tensor add per round: the same sums in the same order, bit-identical.
WGRAD_LATE_SUM = os.environ.get('SMMD_WGRAD_LATE_SUM', '1') != '0'
WGRAD_ACC = os.environ.get('SMMD_WGRAD_ACC', '1') != '0'    # later ones into the first
# the same for two double-backward nodes' gradients of one gy input
# (_ConvBackward, _shared_gy_key; SMMD_GY_ACC=0: autograd adds them).
# Single-consumer rule (both sums): every gradient reaching such an edge must
# come from a node that takes part in the sum.  A native autograd gradient to
# the same edge makes autograd's input buffer a new tensor (first + other), and
# later in-place adds into `first` would be lost; for the SN weights
# check_late_delivery enforces it at the SN node.  The gy sums are armed only
# for _ReluPool's gu, whose consumers are the block's two convolutions.
GY_ACC = os.environ.get('SMMD_GY_ACC', '1') != '0'
_late = {'armed': False, 'first': {}, 'queue': [], 'queued': 0, 'gy': {}, 'gy_acc': 0}
# (queued, gy_acc: running counts)


def arm_late_wgrad_sums(on):
    """Start (True) or end (False) a backward whose SN-weight gradients are
    summed late (flush_late_wgrad_sums); ending drops any state."""
    _late['armed'] = bool(on) and WGRAD_LATE_SUM
    _late['first'].clear()
    _late['queue'].clear()
    _late['gy'].clear()


# Late sums of bias gradients (SMMD_BIAS_LATE_SUM=0: off): a critic conv bias
# gets one gradient per pass (real, fake), and autograd adds them -- one
# latency-bound add launch per bias, and a copy where one channel sum feeds
# two biases (_ReluPool's bx and by).  While armed (MMD_GAN.d_step, one
# process, gathered gradients, .grad None at the start) every contribution is
# queued instead and flush_late_bias_sums forms .grad after the backward:
# first + second by one out-of-place multi-tensor add (+ later ones in
# place), the sums autograd forms in arrival order, bit for bit.
BIAS_LATE_SUM = os.environ.get('SMMD_BIAS_LATE_SUM', '1') != '0'
_lateb = {'armed': False, 'queue': [], 'queued': 0, 'closed': set()}


def arm_late_bias_sums(on):
    _lateb['armed'] = bool(on) and BIAS_LATE_SUM
    _lateb['queue'].clear()
    _lateb['closed'].clear()


def late_bias_armed():
    return _lateb['armed']


def _late_bias(p, g):
    """g for autograd, or None: queued for p.grad."""
    if (g is None or p is None or not _lateb['armed'] or not p.is_leaf
            or torch.is_grad_enabled()):
        return g
    if id(p) in _lateb['closed']:
        # its gradient was already handed to its all-reduce bucket
        raise RuntimeError('late bias sum: a gradient contribution of a bias (%s) arrived after '
                           'its SN layer group flushed it (SMMD_BIAS_LATE_SUM=0 avoids the '
                           'late sums)' % (tuple(p.shape),))
    _lateb['queue'].append((p, g))
    _lateb['queued'] += 1
    return None


def flush_late_bias_sums(params=None):
    """p.grad = the sum of p's queued contributions in arrival order (round 1:
    one out-of-place _foreach_add of the first two of every parameter; round
    r > 1: one in-place _foreach_add_ of the r-th); a single contribution is
    taken as it is, cloned when another parameter holds the same tensor.  A
    parameter whose .grad already exists (the data-parallel step's views into
    the flat gradient, zeroed before the backward) gets the sum added into it,
    all of them by one more multi-tensor add: 0 + sum, the same values.
    ``params``: only these parameters (a data-parallel SN group's biases,
    whose buckets are then notified; a later contribution to one of them is
    an error), else every queued one.  Returns the parameters it set."""
    q = _lateb['queue']
    if params is not None:
        ids = {id(p) for p in params}
        _lateb['closed'].update(ids)
        take = [(p, g) for p, g in q if id(p) in ids]
        q[:] = [(p, g) for p, g in q if id(p) not in ids]
    else:
        take = list(q)
        q.clear()
    if not take:
        return []
    per = {}
    for p, g in take:
        per.setdefault(id(p), (p, []))[1].append(g)
    into_p, into_t = [], []

    def assign(p, t):
        if p.grad is None:
            p.grad = t
        else:                       # (an existing .grad: the flat view, or autograd's own)
            into_p.append(p.grad)
            into_t.append(t)
    with torch.no_grad():
        pairs = [(p, gs) for p, gs in per.values() if len(gs) >= 2]
        if pairs:
            sums = torch._foreach_add([gs[0] for _, gs in pairs], [gs[1] for _, gs in pairs])
            r = 2
            while True:
                more = [(k, gs[r]) for k, (_, gs) in enumerate(pairs) if len(gs) > r]
                if not more:
                    break
                torch._foreach_add_([sums[k] for k, _ in more], [g for _, g in more])
                r += 1
            for (p, _), t in zip(pairs, sums):
                assign(p, t)
        held = {}
        for p, gs in per.values():
            if len(gs) == 1:
                held[id(gs[0])] = held.get(id(gs[0]), 0) + 1
        for p, gs in per.values():
            if len(gs) == 1:
                assign(p, gs[0].clone() if (held[id(gs[0])] > 1 and p.grad is None) else gs[0])
        if into_p:
            torch._foreach_add_(into_p, into_t)
    return [p for p, _ in per.values()]


def _shared_gy_key(ctx):
    """The autograd edge of a _ConvBackward node's gy input -- (producer node,
    output index): two nodes with the same edge have their gradients for gy
    summed by autograd into one input of that producer, which runs after both
    -- or None outside an armed backward.  The producer node is kept alive by
    the entry (_late['gy'], cleared by arm_late_wgrad_sums), so its id is not
    reused while the key stands."""
    if not (GY_ACC and _late['armed']) or torch.is_grad_enabled():
        return None
    fn, nr = ctx.next_functions[2]
    return None if fn is None else (id(fn), nr)


def _late_target(w):
    """w's first gradient contribution of the armed backward (a later one is
    computed straight into it by the library's *_wgrad_acc kernels), or None."""
    if not (WGRAD_ACC and _late['armed'] and getattr(w, '_smmd_late_sum', False)):
        return None
    f = _late['first'].get(id(w))
    return f[1] if f is not None and f[0] is w else None


def _late_gw(w, gw, into=None):
    """gw for autograd, or None: added into w's first contribution already
    (into, _late_target), or queued onto it."""
    if gw is not None and into is not None and gw is into:
        _late['queued'] += 1
        return None
    if gw is None or not _late['armed'] or not getattr(w, '_smmd_late_sum', False):
        return gw
    f = _late['first'].get(id(w))
    if f is None or f[0] is not w:
        _late['first'][id(w)] = (w, gw)
        return gw
    _late['queue'].append((f[1], gw))
    _late['queued'] += 1
    return None


def check_late_delivery(out_ids, grads):
    """The late sums' invariant, checked at the SN node: the gradient autograd
    delivers for a marked SN output must BE its first recorded contribution
    (the tensor later terms were queued onto or computed into).  Another
    consumer sending a native autograd gradient to the same edge would make
    autograd's input buffer a new tensor (first + other), and every term
    added into `first` after that would be lost silently -- so raise instead.
    out_ids: id() of the node's outputs, in the order of grads."""
    if not _late['armed']:
        return
    for oid, g in zip(out_ids, grads):
        f = _late['first'].get(oid)
        if f is None or id(f[0]) != oid:
            continue
        if g is None or g.data_ptr() != f[1].data_ptr():
            raise RuntimeError(
                'late weight-gradient sum: the SN output %s received a gradient other than '
                'its recorded first contribution (a consumer outside convops._Conv2d / '
                '_LinOut / _Outer sent it a native gradient); run with '
                'SMMD_WGRAD_LATE_SUM=0' % (tuple(f[0].shape),))


def flush_late_wgrad_sums():
    """Add the queued contributions into their first ones, in arrival order:
    round r adds each weight's r-th queued term (one _foreach_add_ per round,
    no tensor twice in one launch)."""
    q = _late['queue']
    if not q:
        return
    rounds = []
    seen = {}
    for acc, g in q:
        r = seen.get(id(acc), 0)
        seen[id(acc)] = r + 1
        if r == len(rounds):
            rounds.append(([], []))
        rounds[r][0].append(acc)
        rounds[r][1].append(g)
    with torch.no_grad():
        for accs, gs in rounds:
            torch._foreach_add_(accs, gs)
    q.clear()


def _fmt(t):
    if t.dim() == 4 and not t.is_contiguous() and t.is_contiguous(
            memory_format=torch.channels_last):
        return torch.channels_last
    return torch.contiguous_format


class _Conv2d(torch.autograd.Function):
    """conv(x, w) + b.  mask_in (x a ReLU output whose producer,
    _Conv2dReLU with consumer_masks, skips its mask): the input gradient is
    returned already masked by x > 0 -- inside the stride-2 transposed conv's
    launch (smmd_wino4x4s2t_conv_mask) instead of a threshold_backward pass."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, mask_in=False):
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, padding, b is not None, mask_in)
        ctx.bias_ref = b                    # the parameter (_late_bias)
        return _fwd(x, w, b, stride, padding)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        stride, padding, has_b, mask_in = ctx.cfg
        gy = gy.contiguous(memory_format=_fmt(x))
        want_w = ctx.needs_input_grad[1] and _input_only[0] == 0
        want_x = ctx.needs_input_grad[0] and not (_no_dx and x.data_ptr() in _no_dx)
        into = None
        if torch.is_grad_enabled():          # create_graph: keep it differentiable
            gx, gw = _ConvBackward.apply(x, w, gy, stride, padding, want_w, mask_in)
            if not want_w:
                gw = None
        elif want_x or want_w:
            into = _late_target(w) if want_w else None
            gx, gw = _bwd(gy, x, w, stride, padding, (want_x, want_w), x if mask_in else None,
                          into)
        else:
            gx = gw = None
        gb = (bias_grad(gy) if (has_b and ctx.needs_input_grad[2] and _input_only[0] == 0)
              else None)
        return gx, _late_gw(w, gw, into), _late_bias(ctx.bias_ref, gb), None, None, None


def bias_grad(gy):
    """sum of gy over (N, H, W): the conv bias gradient (TF BiasAddGrad,
    snops.py:89-90).  An NCHW device tensor outside a create_graph pass runs
    `smmd_channel_sum` (csrc/smmd_bias.hip, fixed-order two-stage sum); a
    gradient that must itself be differentiable (create_graph, e.g. the
    witness penalty), channels_last or host tensors use torch's reduction."""
    if (not gy.is_cuda or torch.is_grad_enabled() or gy.dim() != 4
            or not gy.is_contiguous()):
        return gy.sum(dim=(0, 2, 3))
    from . import _lib
    _lib.require_cuda(gy)
    N, C, H, W = gy.shape
    L = _lib.lib()
    nbytes = L.smmd_channel_sum_workspace_bytes(N, C)
    ws = _lib.workspace('channel_sum', nbytes, gy.device)
    out = torch.empty(C, dtype=gy.dtype, device=gy.device)
    _lib.add_bytes('smmd_channel_sum', (gy.numel() + C) * 4)
    with _lib.timed('smmd_channel_sum'):
        st = L.smmd_channel_sum(_lib.ptr(gy), N, C, H * W, _lib.ptr(out), _lib.ptr(ws),
                                ws.numel(), _lib.stream_handle(gy.device))
    _lib.check(st, 'smmd_channel_sum')
    return out


class _ReluMask(torch.autograd.Function):
    """g -> g * (r > 0) (threshold_backward(g, r, 0), TF's relu gradient) as
    the differentiable node of a create_graph backward.  Its own gradient is
    the same mask for g and None for r: the mask's derivative is zero, and
    autograd's ThresholdBackwardBackward0 materialised it as a zero tensor
    (a fill of the activation's size) that the engine then added to r's other
    gradient (a full-size add) -- per critic layer of every critic step."""

    @staticmethod
    def forward(ctx, g, r):
        ctx.save_for_backward(r)
        return _aten.threshold_backward(g, r, 0.0)

    @staticmethod
    def backward(ctx, gg):
        r, = ctx.saved_tensors
        if gg is None or not ctx.needs_input_grad[0]:
            return None, None
        gg = gg.contiguous()
        return ((_ReluMask.apply(gg, r) if torch.is_grad_enabled()
                 else _aten.threshold_backward(gg, r, 0.0)), None)


class _Conv2dReLU(torch.autograd.Function):
    """relu(conv(x, w) + b) with the ReLU in the Winograd kernel's epilogue (the
    critic's first conv of each down block, block.py:44-46, norm off): no
    pre-activation is written.  Backward: the mask (r > 0) of the output, as
    TF's relu gradient, then the conv's backward (differentiable: the double
    backward of the scaling regulariser)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, padding, consumer_masks=False):
        r = _wino_conv(x, w, b, 0, relu=True)
        ctx.save_for_backward(x, w, r)
        ctx.cfg = (stride, padding, b is not None, consumer_masks)
        ctx.bias_ref = b
        return r

    @staticmethod
    def backward(ctx, gr):
        x, w, r = ctx.saved_tensors
        stride, padding, has_b, consumer_masks = ctx.cfg
        if consumer_masks:
            # r's only consumer is a conv with mask_in (ResidualBlock.down_parts):
            # every gradient that reaches r -- its input gradient, and in the
            # double backward _ConvBackward's for its saved x -- is masked already
            gy = gr.contiguous()
        elif torch.is_grad_enabled():
            gy = _ReluMask.apply(gr.contiguous(), r)
        else:
            gy = _aten.threshold_backward(gr.contiguous(), r, 0.0)
        want_w = ctx.needs_input_grad[1] and _input_only[0] == 0
        want_x = ctx.needs_input_grad[0] and not (_no_dx and x.data_ptr() in _no_dx)
        want_b = has_b and ctx.needs_input_grad[2] and _input_only[0] == 0
        into = None
        if torch.is_grad_enabled():
            # (a differentiable bias gradient is a second consumer of gr: then
            # the mask_in node keeps its own mask)
            gx, gw = _ConvBackward.apply(
                x, w, gy, stride, padding, want_w, False,
                r if consumer_masks and not want_b and _ggx_masked(gr) else None)
            if not want_w:
                gw = None
        elif want_x or want_w:
            into = _late_target(w) if want_w else None
            gx, gw = _bwd(gy, x, w, stride, padding, (want_x, want_w), None, into)
        else:
            gx = gw = None
        gb = bias_grad(gy) if want_b else None
        return gx, _late_gw(w, gw, into), _late_bias(ctx.bias_ref, gb), None, None, None


# the double backward's gradient of a consumer-masked conv-ReLU's upstream
# masked where it is produced (SMMD_GGX_MASK_FUSE=0: by the consumer)
GGX_MASK_FUSE = os.environ.get('SMMD_GGX_MASK_FUSE', '1') != '0'


def _ggx_masked(gr):
    """gr (a consumer-masked ReLU output's gradient) is exactly the input
    gradient of one mask_in _ConvBackward node: mark that node so that it
    skips its mask of the gradient it receives for gr -- which then comes
    only from the node built on gr here, masking it (_ConvBackward gy_mask)."""
    fn = gr.grad_fn
    if not (GGX_MASK_FUSE and fn is not None and gr.output_nr == 0
            and getattr(fn, '_smmd_mask_in', False)):
        return False
    fn._smmd_ggx_masked = True
    return True


def conv2d_relu(x, w, b=None, stride=1, padding=0, consumer_masks=False):
    """relu(conv2d(x, w, b)): one Winograd launch on the 3x3 layers it tiles
    (SMMD_CONV_RELU=0: a separate ReLU), the two ops otherwise.
    consumer_masks: the output's only consumer is a conv2d(..., mask_in=True),
    which returns its input gradient masked, so this ReLU's backward skips
    the mask (the separate-ReLU form keeps it: masking twice is exact)."""
    s = (stride, stride) if isinstance(stride, int) else tuple(stride)
    p = (padding, padding) if isinstance(padding, int) else tuple(padding)
    if CONV_RELU and _is_wino(x, w, list(s), list(p), 0):
        return _Conv2dReLU.apply(x, w, b, list(s), list(p), bool(consumer_masks and RELU_MASK_FUSE))
    return F.relu(conv2d(x, w, b, stride, padding))


CONV_RELU = os.environ.get('SMMD_CONV_RELU', '1') != '0'


# SMMD_RELU_MASK_FUSE=0: the critic's conv-ReLU keeps its own mask pass
# (threshold_backward) instead of its consumer's masked input gradient
RELU_MASK_FUSE = os.environ.get('SMMD_RELU_MASK_FUSE', '1') != '0'


def conv2d(x, w, b=None, stride=1, padding=0, mask_in=False):
    """F.conv2d with the MIOpen-friendly second-order rule above.  mask_in: x
    is a ReLU output; the input gradient comes back masked by x > 0 (see
    conv2d_relu's consumer_masks)."""
    s = (stride, stride) if isinstance(stride, int) else tuple(stride)
    p = (padding, padding) if isinstance(padding, int) else tuple(padding)
    return _Conv2d.apply(x, w, b, list(s), list(p), bool(mask_in and RELU_MASK_FUSE))


class _Up2Quarter(torch.autograd.Function):
    """g -> nearest-upsample(g / 4): the adjoint of the 2x2 mean pool."""

    @staticmethod
    def forward(ctx, g):
        return F.interpolate(g * 0.25, scale_factor=2, mode='nearest')

    @staticmethod
    def backward(ctx, gg):
        return _MeanPool2.apply(gg)


class _MeanPool2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return F.avg_pool2d(x, 2)

    @staticmethod
    def backward(ctx, g):
        return _Up2Quarter.apply(g.contiguous())


def _fold_launch(srcs, adjoint):
    """smmd_fold_pool_weights over a list of layers, ONE launch on the current
    stream (device tensors only)."""
    from . import _lib
    import ctypes
    _lib.require_cuda(*srcs)
    srcs = [materialize(t).contiguous() for t in srcs]
    dsts = [torch.empty(t.shape[:2] + ((3, 3) if adjoint else (4, 4)), dtype=t.dtype,
                        device=t.device) for t in srcs]
    n = len(srcs)
    P = ctypes.c_void_p * n
    nf = (ctypes.c_int64 * n)(*[t.numel() // (16 if adjoint else 9) for t in srcs])
    with _lib.timed('smmd_fold_pool_weights'):
        st = _lib.lib().smmd_fold_pool_weights(P(*[t.data_ptr() for t in srcs]),
                                               P(*[t.data_ptr() for t in dsts]), nf, n,
                                               int(adjoint), _lib.stream_handle(srcs[0].device))
    _lib.check(st, 'smmd_fold_pool_weights')
    return tuple(dsts)


def _fold_launch_into(srcs, dsts, adjoint):
    """smmd_fold_pool_weights from ``srcs`` into the existing contiguous
    ``dsts`` (e.g. gradient views of a flat buffer), ONE launch."""
    from . import _lib
    import ctypes
    n = len(srcs)
    P = ctypes.c_void_p * n
    nf = (ctypes.c_int64 * n)(*[t.numel() // (16 if adjoint else 9) for t in srcs])
    with _lib.timed('smmd_fold_pool_weights'):
        st = _lib.lib().smmd_fold_pool_weights(P(*[t.data_ptr() for t in srcs]),
                                               P(*[t.data_ptr() for t in dsts]), nf, n,
                                               int(adjoint), _lib.stream_handle(srcs[0].device))
    _lib.check(st, 'smmd_fold_pool_weights')


def _fold_torch(w):
    return F.avg_pool2d(F.pad(w, (1, 1, 1, 1)), 2, stride=1)


def _fold_adj_torch(g):
    return F.avg_pool2d(g, 2, stride=1)


class _FoldPool(torch.autograd.Function):
    """W_l [cout, cin, 3, 3] -> W'_l [cout, cin, 4, 4] for every listed layer."""

    @staticmethod
    def forward(ctx, *ws):
        if ws[0].is_cuda:
            return _fold_launch(ws, 0)
        return tuple(_fold_torch(w) for w in ws)

    @staticmethod
    def backward(ctx, *gs):
        return _FoldPoolAdj.apply(*gs)


class _FoldPoolAdj(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *gs):
        # 1/4 sum_{a,b} g[u+a, v+b] = the 2x2 stride-1 mean of the 4x4 gradient
        if gs[0].is_cuda:
            return _fold_launch(gs, 1)
        return tuple(_fold_adj_torch(g) for g in gs)

    @staticmethod
    def backward(ctx, *ggs):
        return _FoldPool.apply(*ggs)


def fold_pool_weights(ws):
    """fold_pool_weight over a list of layers: one HIP launch forward, one for
    the adjoint in the backward."""
    out = _FoldPool.apply(*ws)
    return list(out) if isinstance(out, tuple) else [out]


def fold_pool_weight(w):
    """W [cout, cin, 3, 3] -> W' [cout, cin, 4, 4] with
    meanpool2(conv(x, W, stride 1, pad 1)) == conv(x, W', stride 2, pad 1):
    W'[s, t] = 1/4 sum_{a, b in {0, 1}} W[s - a, t - b], i.e. a 2x2 stride-1
    mean over W zero-padded by one (ConvMeanPool, gan/core/resnet/block.py:63-66,
    as one strided conv).  Device tensors run the HIP fold
    (`smmd_fold_pool_weights`, csrc/smmd_fold.hip) and its adjoint, each the
    other's backward, so the op is differentiable to any order; host tensors
    (CPU module tests, the oracle's mirror) use the same sums in torch."""
    return fold_pool_weights([w])[0]


def unfold_pool_weight(w4):
    """Inverse of fold_pool_weight on its image: W [cout, cin, 3, 3] from
    W' = fold(W) by back-substitution, W[s, t] = 4 W'[s, t] - W[s-1, t] -
    W[s, t-1] - W[s-1, t-1] (differentiable torch ops; the fallback for a
    ConvMeanPool whose bank wrote only the folded filter but whose input has
    odd spatial size)."""
    rows = []
    for s_ in range(3):
        row = []
        for t_ in range(3):
            v = 4.0 * w4[:, :, s_, t_]
            if s_ > 0:
                v = v - rows[s_ - 1][t_]
            if t_ > 0:
                v = v - row[t_ - 1]
            if s_ > 0 and t_ > 0:
                v = v - rows[s_ - 1][t_ - 1]
            row.append(v)
        rows.append(row)
    return torch.stack([torch.stack(r, -1) for r in rows], -2)


def fold_up_weight(w):
    """W [cout, cin, 3, 3] -> K [cin, cout, 4, 4] with
    conv(upsample_nearest2(x), W, stride 1, pad 1) == conv_transpose(x, K, stride 2, pad 1):
    per axis the two output phases see taps (W0, W1 + W2) and (W0 + W1, W2) of
    x, i.e. K = flip([W0, W0 + W1, W1 + W2, W2]) = flip(4 fold_pool_weight(W))
    (UpsampleConv, gan/core/resnet/block.py:53-60, without the 4x larger
    upsampled input; linear, so differentiable to any order).  Device tensors
    run `smmd_fold_up_weight` (one launch each way, K contiguous; the torch
    form was pad, avg_pool2d, scale, flip and a transposing copy, and its
    backward's avg_pool2d_backward alone took 127 us on the 1024 -> 512
    layer); host tensors the torch ops."""
    if w.is_cuda and w.dim() == 4 and tuple(w.shape[2:]) == (3, 3) and w.dtype == torch.float32:
        return _FoldUp.apply(w)
    return torch.flip(_fold_torch(w) * 4.0, (2, 3)).transpose(0, 1)


def _fold_up_launch(src, adjoint):
    from . import _lib
    src = src.contiguous()
    if adjoint:                       # gK [cin, cout, 4, 4] -> gW [cout, cin, 3, 3]
        cin, cout = src.shape[0], src.shape[1]
        dst = torch.empty(cout, cin, 3, 3, device=src.device, dtype=src.dtype)
    else:                             # W [cout, cin, 3, 3] -> K [cin, cout, 4, 4]
        cout, cin = src.shape[0], src.shape[1]
        dst = torch.empty(cin, cout, 4, 4, device=src.device, dtype=src.dtype)
    _lib.add_bytes('smmd_fold_up_weight', 25 * cout * cin * 4)
    with _lib.timed('smmd_fold_up_weight'):
        st = _lib.lib().smmd_fold_up_weight(_lib.ptr(src), _lib.ptr(dst), cout, cin,
                                            int(adjoint), _lib.stream_handle(src.device))
    _lib.check(st, 'smmd_fold_up_weight')
    return dst


class _FoldUp(torch.autograd.Function):
    """fold_up_weight on the library; its backward is the adjoint launch,
    whose backward is this forward again (the map is linear)."""

    @staticmethod
    def forward(ctx, w):
        return _fold_up_launch(materialize(w), False)

    @staticmethod
    def backward(ctx, gk):
        return _FoldUpAdj.apply(gk)


class _FoldUpAdj(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gk):
        return _fold_up_launch(gk, True)

    @staticmethod
    def backward(ctx, ggw):
        return _FoldUp.apply(ggw)


def mean_pool2(x):
    """2x2 mean pool, the reference's add_n of the four strided slices / 4
    (gan/core/resnet/block.py:65, :71), as a linear op whose backward is one
    nearest-upsample of g/4 (and whose double backward is the pool again),
    instead of four strided-slice backwards (zero fill + copy each)."""
    if x.shape[2] % 2 or x.shape[3] % 2:
        return (x[:, :, ::2, ::2] + x[:, :, 1::2, ::2] + x[:, :, ::2, 1::2]
                + x[:, :, 1::2, 1::2]) / 4.
    return _MeanPool2.apply(x)


# ---------------------------------------------------------------------------
# a critic down block's input: the main path's ReLU and the shortcut's mean
# pool in one read, their gradients in one write (csrc/smmd_relupool.hip;
# SMMD_RELU_POOL=0: relu + mean_pool2 as separate torch ops).  The input may
# arrive as the previous block's two paths (their add fused) or as the first
# conv's pre-activation (its leaky ReLU fused: relu(lrelu(h)) = relu(h)).
# ---------------------------------------------------------------------------
RELU_POOL = os.environ.get('SMMD_RELU_POOL', '1') != '0'


def relu_pool_applicable(x, y=None):
    """An NCHW fp32 device tensor with even height and width % 4 == 0 (and y,
    if given, of the same shape and layout)."""
    ok = (RELU_POOL and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
          and x.is_contiguous() and x.shape[2] % 2 == 0 and x.shape[3] % 4 == 0)
    if ok and y is not None:
        ok = y.shape == x.shape and y.dtype == x.dtype and y.is_contiguous() and y.is_cuda
    return ok


def _mask_pool(x, y, m, slope_m, slope_p, masked=True, pooled=True, bx=None, by=None):
    """smmd_mask_pool2: with u = (x + bx) (+ (y + by)), (u s_m(m), pool(u s_p(m)));
    m None: the mask source is u; either output may be skipped."""
    from . import _lib
    x = x.contiguous()
    y = y.contiguous() if y is not None else None
    m = m.contiguous() if m is not None else None
    _lib.require_cuda(*[t for t in (x, y, m, bx, by) if t is not None])
    N, C, H, W = x.shape
    out_m = torch.empty_like(x) if masked else None
    out_p = torch.empty((N, C, H // 2, W // 2), dtype=x.dtype, device=x.device) if pooled else None
    nb = x.numel() * (1 + (y is not None) + (m is not None) + masked) + \
        (out_p.numel() if pooled else 0)
    _lib.add_bytes('smmd_mask_pool2', nb * 4)
    with _lib.timed('smmd_mask_pool2'):
        st = _lib.lib().smmd_mask_pool2(_lib.ptr(x), _lib.ptr(y), _lib.ptr(bx), _lib.ptr(by), C,
                                        _lib.ptr(m), float(slope_m), float(slope_p), N * C, H, W,
                                        _lib.ptr(out_m), _lib.ptr(out_p),
                                        _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_mask_pool2')
    return out_m, out_p


def _mask_pool_adj(a, b, m, slope_m, slope_p):
    """smmd_mask_pool2_adj: a s_m(m) + s_p(m) nearest_up(b / 4) (a or b None: absent)."""
    from . import _lib
    m = m.contiguous()
    a = a.contiguous() if a is not None else None
    b = b.contiguous() if b is not None else None
    _lib.require_cuda(m, *[t for t in (a, b) if t is not None])
    N, C, H, W = m.shape
    out = torch.empty_like(m)
    nb = out.numel() * (2 + (a is not None)) + (b.numel() if b is not None else 0)
    _lib.add_bytes('smmd_mask_pool2_adj', nb * 4)
    with _lib.timed('smmd_mask_pool2_adj'):
        st = _lib.lib().smmd_mask_pool2_adj(_lib.ptr(a), _lib.ptr(b), _lib.ptr(m), float(slope_m),
                                            float(slope_p), N * C, H, W, _lib.ptr(out),
                                            _lib.stream_handle(m.device))
    _lib.check(st, 'smmd_mask_pool2_adj')
    return out


class _MaskPool(torch.autograd.Function):
    """(x; m) -> (x s_m(m), pool(x s_p(m))): linear in x, the mask m constant."""

    @staticmethod
    def forward(ctx, x, m, slope_m, slope_p):
        ctx.save_for_backward(m)
        ctx.slopes = (slope_m, slope_p)
        ctx.set_materialize_grads(False)
        return _mask_pool(x, None, m, slope_m, slope_p)

    @staticmethod
    def backward(ctx, ga, gb):
        if ga is None and gb is None:
            return None, None, None, None
        m, = ctx.saved_tensors
        return _MaskPoolAdj.apply(ga, gb, m, *ctx.slopes), None, None, None


class _MaskPoolAdj(torch.autograd.Function):
    """(a, b; m) -> a s_m(m) + s_p(m) up(b) / 4: the adjoint of _MaskPool, and
    its backward (and the other way round), so every order of differentiation
    stays on the two kernels."""

    @staticmethod
    def forward(ctx, a, b, m, slope_m, slope_p):
        ctx.save_for_backward(m)
        ctx.slopes = (slope_m, slope_p)
        return _mask_pool_adj(a, b, m, slope_m, slope_p)

    @staticmethod
    def backward(ctx, g):
        m, = ctx.saved_tensors
        need_a, need_b = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if not (need_a or need_b):
            return None, None, None, None, None
        ga, gb = _MaskPool.apply(g, m, *ctx.slopes)
        return (ga if need_a else None), (gb if need_b else None), None, None, None


class _ReluPool(torch.autograd.Function):
    """(x, y, bx, by) -> (relu(u), pool(u s_p(u))), u = (x + bx) + (y + by) (y,
    bx, by may be None): the ReLU output is the backward's mask (its sign is
    u's); the gradient of u goes to x and y, its channel sum to bx and by."""

    @staticmethod
    def forward(ctx, x, y, bx, by, slope_p):
        r, p = _mask_pool(x, y, None, 0.0, slope_p, bx=bx, by=by)
        ctx.save_for_backward(r)
        ctx.slope_p = slope_p
        ctx.has = (y is not None, bx is not None, by is not None)
        ctx.bias_refs = (bx, by)
        ctx.set_materialize_grads(False)
        return r, p

    @staticmethod
    def backward(ctx, gr, gp):
        if gr is None and gp is None:
            return None, None, None, None, None
        r, = ctx.saved_tensors
        gu = _MaskPoolAdj.apply(gr, gp, r, 0.0, ctx.slope_p)
        has_y, has_bx, has_by = ctx.has
        gb = None
        if (has_bx and ctx.needs_input_grad[2]) or (has_by and ctx.needs_input_grad[3]):
            if _input_only[0] == 0:         # not the Jacobian's input-only pass
                gb = bias_grad(gu)
        bx, by = ctx.bias_refs
        return (gu, (gu if has_y else None), _late_bias(bx, gb if has_bx else None),
                _late_bias(by, gb if has_by else None), None)


def relu_pool(x, y=None, slope_p=1.0, bx=None, by=None):
    """A critic down block's two input ops (block.py:44, :69-71) on u = (x +
    bx) + (y + by) (y None: u = x + bx; bx, by: the previous block's conv
    biases, None when already applied): (relu(u), mean_pool2(u)) with slope_p
    1, or with slope_p 0.2 (relu(lrelu(u)), mean_pool2(lrelu(u))) -- u the
    first conv's output, architecture.py:393.  One HIP pass each way on
    device tensors, the torch composition otherwise."""
    if relu_pool_applicable(x, y):
        return _ReluPool.apply(x, y, bx, by, float(slope_p))
    u = x if bx is None else x + bx.view(1, -1, 1, 1)
    if y is not None:
        u = u + (y if by is None else y + by.view(1, -1, 1, 1))
    if slope_p != 1.0:
        u = F.leaky_relu(u, slope_p)
    return F.relu(u), mean_pool2(u)


# ---------------------------------------------------------------------------
# a generator up block's output: up(s + bs) + (h + bh) in one pass
# (csrc/smmd_relupool.hip smmd_up_add; SMMD_UP_ADD=0: the torch ops)
# ---------------------------------------------------------------------------
UP_ADD = os.environ.get('SMMD_UP_ADD', '1') != '0'


def up_add_applicable(s, h):
    """s [N, C, H/2, W/2] and h [N, C, H, W]: NCHW fp32 device tensors, H even,
    W % 4 == 0."""
    return (UP_ADD and h.is_cuda and s.is_cuda and h.dtype == torch.float32
            and s.dtype == torch.float32 and h.dim() == 4 and h.is_contiguous()
            and s.is_contiguous() and h.shape[2] % 2 == 0 and h.shape[3] % 4 == 0
            and tuple(s.shape) == (h.shape[0], h.shape[1], h.shape[2] // 2, h.shape[3] // 2))


class _UpAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s, bs, h, bh):
        from . import _lib
        _lib.require_cuda(s, h)
        N, C, H, W = h.shape
        out = torch.empty_like(h)
        _lib.add_bytes('smmd_up_add', (2 * h.numel() + s.numel()) * 4)
        with _lib.timed('smmd_up_add'):
            st = _lib.lib().smmd_up_add(_lib.ptr(s), _lib.ptr(bs), _lib.ptr(h), _lib.ptr(bh), C,
                                        N * C, H, W, _lib.ptr(out),
                                        _lib.stream_handle(h.device))
        _lib.check(st, 'smmd_up_add')
        ctx.has = (bs is not None, bh is not None)
        return out

    @staticmethod
    def backward(ctx, g):
        # the nearest upsample's adjoint is the 2x2 window sum: avg_pool2d's
        # ((g00 + g01) + g10) + g11 with divisor 1 -- the sum / 4 * 4 of the
        # unfused form (exact: a power-of-two scale), one kernel instead of two
        g = g.contiguous()
        gs = (F.avg_pool2d(g, 2, divisor_override=1) if ctx.needs_input_grad[0] or ctx.has[0]
              else None)
        gbs = bias_grad(gs) if ctx.has[0] and ctx.needs_input_grad[1] else None
        gbh = bias_grad(g) if ctx.has[1] and ctx.needs_input_grad[3] else None
        return gs, gbs, g, gbh


def up_add(s, bs, h, bh):
    """up(s + bs) + (h + bh) (block.py:50 of an up block, biases per channel,
    either may be None): one HIP pass on device tensors, torch ops otherwise."""
    if up_add_applicable(s, h):
        return _UpAdd.apply(s, bs, h, bh)
    if bs is not None:
        s = s + bs.view(1, -1, 1, 1)
    if bh is not None:
        h = h + bh.view(1, -1, 1, 1)
    return F.interpolate(s, scale_factor=2, mode='nearest') + h


# ---------------------------------------------------------------------------
# the critic's tail: lrelu(u + v).sum(dim=(2, 3)) (architecture.py:430-433, the
# last block's two paths, the final lrelu and tf.reduce_sum) in one launch,
# its backward in one, its double backward in one (csrc/smmd_relupool.hip;
# SMMD_TAIL=0: the torch ops -- an add, the lrelu and the sum forward, the
# expand + leaky_relu_backward and, in the double backward, a zero fill and
# an add of it for the mask input)
TAIL = os.environ.get('SMMD_TAIL', '1') != '0'


def _tail_ok(u, v):
    return (TAIL and u.is_cuda and u.dtype == torch.float32 and u.dim() == 4
            and u.is_contiguous() and (u.shape[2] * u.shape[3]) % 4 == 0
            and u.data_ptr() % 16 == 0
            and (v is None or (v.shape == u.shape and v.dtype == u.dtype and v.is_contiguous()
                               and v.data_ptr() % 16 == 0)))


def _row_sum(a, b, mu, mv, slope):
    from . import _lib
    N, C, H, W = a.shape
    y = torch.empty((N, C), dtype=a.dtype, device=a.device)
    _lib.add_bytes('smmd_row_lrelu_sum', a.numel() * 4 * (1 + (b is not None) + (mu is not None)
                                                          + (mv is not None)))
    with _lib.timed('smmd_row_lrelu_sum'):
        st = _lib.lib().smmd_row_lrelu_sum(_lib.ptr(a), _lib.ptr(b), _lib.ptr(mu), _lib.ptr(mv),
                                           _lib.ptr(y), N * C, H * W, float(slope),
                                           _lib.stream_handle(a.device))
    _lib.check(st, 'smmd_row_lrelu_sum')
    return y


class _TailBcast(torch.autograd.Function):
    """g [N, C] -> g * s(u + v) [N, C, H, W]: the tail's backward; its own
    adjoint is the masked row sum (the mask inputs get no gradient)."""

    @staticmethod
    def forward(ctx, g, u, v, slope):
        from . import _lib
        g = g.contiguous()
        N, C, H, W = u.shape
        out = torch.empty_like(u)
        _lib.add_bytes('smmd_row_lrelu_bcast', u.numel() * 4 * (2 + (v is not None)))
        with _lib.timed('smmd_row_lrelu_bcast'):
            st = _lib.lib().smmd_row_lrelu_bcast(_lib.ptr(g), _lib.ptr(u), _lib.ptr(v),
                                                 _lib.ptr(out), N * C, H * W, float(slope),
                                                 _lib.stream_handle(u.device))
        _lib.check(st, 'smmd_row_lrelu_bcast')
        ctx.save_for_backward(u, v)
        ctx.slope = slope
        return out

    @staticmethod
    def backward(ctx, gg):
        u, v = ctx.saved_tensors
        if gg is None or not ctx.needs_input_grad[0]:
            return None, None, None, None
        return _row_sum(gg.contiguous(), None, u, v, ctx.slope), None, None, None


class _TailSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, v, slope):
        ctx.save_for_backward(u, v)
        ctx.slope = slope
        return _row_sum(u, v, None, None, slope)

    @staticmethod
    def backward(ctx, g):
        u, v = ctx.saved_tensors
        if g is None:
            return None, None, None
        gh = (_TailBcast.apply(g, u, v, ctx.slope) if torch.is_grad_enabled()
              else _TailBcast.forward(_NoCtx(), g, u, v, ctx.slope))
        return gh, (gh if v is not None else None), None


class _NoCtx:
    """a stand-in ctx for calling a Function's forward directly (no graph)."""

    def save_for_backward(self, *a):
        pass


def lrelu_rowsum(u, v=None, slope=0.2):
    """leaky_relu(u + v, slope).sum(dim=(2, 3)) (v None: u alone)."""
    if _tail_ok(u, v):
        return _TailSum.apply(u, v, slope)
    h = u if v is None else u + v
    return F.leaky_relu(h, slope).sum(dim=(2, 3))
