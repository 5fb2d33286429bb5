"""SN-aware layers (gan/core/snops.py, gan/core/resnet/ops/conv2d.py) on
PyTorch-ROCm.

The conv / matmul math runs on MIOpen / hipBLASLt; the spectral
normalisation is NOT done per layer: each SN layer registers with its
network's :class:`~gan.core.sn.SpectralNormBank`, which writes ``w_eff``
(= s * W / sigma, snops.py:82-84) for every layer in one HIP launch set
before the critic runs.  TF 'SAME' padding is reproduced exactly
(asymmetric padding where TF pads more on the bottom/right).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .convops import conv2d, conv2d_relu, thin_applicable


def same_pad(n_in, k, s):
    """TF 'SAME': total = max((ceil(n/s) - 1) s + k - n, 0), before = total // 2."""
    n_out = -(-n_in // s)
    total = max((n_out - 1) * s + k - n_in, 0)
    return total // 2, total - total // 2


def _trunc_normal_(t, std):
    nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2 * std, b=2 * std)


def _glorot_uniform_(t, fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    nn.init.uniform_(t, -lim, lim)


class _SNMixin:
    """with_sn: forward uses self.w_eff (set by the bank); with_learnable_sn_scale
    makes ``sn_scale`` trainable (snops.py:82).  A ConvMeanPool conv
    (``sn_fold``) may instead receive its pool-folded 4 x 4 filter straight
    from the bank (``w_fold``); ``effective_weight`` then unfolds it, for the
    rare call that needs the 3 x 3 filter (odd spatial sizes)."""

    sn_fold = False

    def _init_sn(self, with_sn, with_learnable_sn_scale, scale):
        self.with_sn = with_sn
        if with_sn:
            self.sn_scale = nn.Parameter(torch.full((1,), float(scale)),
                                         requires_grad=with_learnable_sn_scale)
        self.w_eff = None
        self.w_fold = None

    def effective_weight(self):
        if not self.with_sn:
            return self.weight
        if self.w_eff is None:
            if getattr(self, 'w_fold', None) is not None:
                from .convops import materialize, unfold_pool_weight
                self.w_eff = unfold_pool_weight(materialize(self.w_fold))
                return self.w_eff
            raise RuntimeError('SN layer used before its SpectralNormBank.refresh()')
        return self.w_eff


class Conv2d(nn.Module, _SNMixin):
    """snops.conv2d / resnet Conv2D: NCHW conv with TF SAME padding.
    init: 'truncated_normal' (snops.py:77-78) or 'glorot_uniform'
    (resnet/ops/conv2d.py:26-27)."""

    def __init__(self, cin, cout, k=5, stride=2, bias=True, with_sn=False,
                 with_learnable_sn_scale=False, scale=1.0, init='truncated_normal', stddev=0.02):
        super().__init__()
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        if init == 'glorot_uniform':
            _glorot_uniform_(self.weight, k * k * cin, k * k * cout)
        else:
            _trunc_normal_(self.weight, stddev)
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None
        self._init_sn(with_sn, with_learnable_sn_scale, scale)

    def forward(self, x, with_bias=True, relu=False, consumer_masks=False, mask_in=False):
        """with_bias False: the convolution alone (a consumer adds self.bias);
        relu: relu(conv + bias) (convops.conv2d_relu), consumer_masks: its
        only consumer is a conv with mask_in (x a ReLU output: the input
        gradient comes back masked, convops.conv2d)."""
        w = self.effective_weight()
        b = self.bias if with_bias else None
        ph = same_pad(x.shape[2], self.k, self.stride)
        pw = same_pad(x.shape[3], self.k, self.stride)
        if relu:
            if ph[0] == ph[1] and pw[0] == pw[1]:
                return conv2d_relu(x, w, b, self.stride, (ph[0], pw[0]), consumer_masks)
            return F.relu(self.forward(x, with_bias, mask_in=mask_in))
        if ph[0] == ph[1] and pw[0] == pw[1]:
            return conv2d(x, w, b, self.stride, (ph[0], pw[0]), mask_in=mask_in)
        x = F.pad(x, (pw[0], pw[1], ph[0], ph[1]))
        return conv2d(x, w, b, self.stride, 0, mask_in=mask_in)


class Deconv2d(nn.Module, _SNMixin):
    """snops.deconv2d: tf.nn.conv2d_transpose with SAME padding, output = in * s.
    Weight kept as torch stores it, [cin, cout, k, k]; its SN rows are the
    input channels, matching the reference reshape [kh*kw*cout, cin]
    (snops.py:114-117)."""

    def __init__(self, cin, cout, k=5, stride=2, bias=True, with_sn=False,
                 with_learnable_sn_scale=False, scale=1.0, stddev=0.02):
        super().__init__()
        self.cin, self.cout, self.k, self.stride = cin, cout, k, stride
        self.weight = nn.Parameter(torch.empty(cin, cout, k, k))
        nn.init.normal_(self.weight, 0.0, stddev)
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None
        self._init_sn(with_sn, with_learnable_sn_scale, scale)

    def forward(self, x):
        w = self.effective_weight()
        h, wd = x.shape[2] * self.stride, x.shape[3] * self.stride
        before, _ = same_pad(h, self.k, self.stride)
        if self.stride == 1 and before == 1 and thin_applicable(x, self.cin, self.cout, self.k,
                                                                1, 1):
            # a stride-1 SAME transposed conv is the conv with the flipped,
            # transposed filter: the generator's dim -> 3 output layer then runs
            # on the library's thin kernels (csrc/smmd_thin.hip)
            return conv2d(x, w.flip(2, 3).transpose(0, 1), self.bias, 1, 1)
        y = F.conv_transpose2d(x, w, self.bias, self.stride, before)
        if y.shape[2] != h or y.shape[3] != wd:
            y = y[:, :, :h, :wd]
        return y


class Linear(nn.Module, _SNMixin):
    """snops.linear: weight [out, in] (reference Matrix [in, out]),
    random-normal init (snops.py:175-176)."""

    def __init__(self, cin, cout, bias=True, with_sn=False, with_learnable_sn_scale=False,
                 scale=1.0, stddev=0.01, bias_start=0.0):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cout, cin))
        nn.init.normal_(self.weight, 0.0, stddev)
        self.bias = nn.Parameter(torch.full((cout,), float(bias_start))) if bias else None
        self._init_sn(with_sn, with_learnable_sn_scale, scale)

    def forward(self, x):
        w = self.effective_weight()
        if LINEAR_MV and w.shape[0] == 1 and x.dim() == 2 and x.is_cuda:
            # one output feature (the critic's output layer at dof_dim 1): a
            # matrix-vector product; hipBLASLt ran this [B, F] x [F, 1] GEMM on
            # one workgroup, 32 us per call
            if LINEAR_NODE:
                return _LinOut.apply(x, w, self.bias).unsqueeze(1)
            y = (torch.mv(x, w.view(-1)) if self.bias is None
                 else torch.addmv(self.bias, x, w.view(-1)))
            return y.unsqueeze(1)
        return F.linear(x, w, self.bias)


def batch_norm(c):
    """tf.layers.batch_normalization(momentum=.9, eps=1e-5, training=True)
    (snops.py:31-40, resnet/ops/batchnorm.py:10-18)."""
    return nn.BatchNorm2d(c, eps=1e-5, momentum=0.1)


# SMMD_LINEAR_MV=0: a single-output linear layer through F.linear (hipBLASLt)
LINEAR_MV = os.environ.get('SMMD_LINEAR_MV', '1') != '0'
# SMMD_LINEAR_NODE=0: that layer's backward by torch's AddmvBackward0
LINEAR_NODE = os.environ.get('SMMD_LINEAR_NODE', '1') != '0'


class _LinOut(torch.autograd.Function):
    """y [B] = x [B, F] . w [1, F] + b (snops.py:46-66 linear at one output,
    the critic's last layer): torch.mv / addmv forward.  Backward: dx = dy w
    (an outer product, _Outer under create_graph), dw = x^T dy, db = sum dy,
    the ops AddmvBackward0 runs; the weight gradient skipped in an input-only
    pass (convops.input_grad_only), and dw / db handed to convops' late sums
    (an SN weight's contributions summed at its SN node, a bias's after the
    backward) instead of autograd's adds."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.bias_ref = b
        v = w.view(-1)
        return torch.mv(x, v) if b is None else torch.addmv(b, x, v)

    @staticmethod
    def backward(ctx, gy):
        from . import convops
        x, w = ctx.saved_tensors
        full = convops._input_only[0] == 0
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = (_Outer.apply(gy, w) if torch.is_grad_enabled()
                  else torch.outer(gy, w.view(-1)))
        if ctx.needs_input_grad[1] and full:
            gw = convops._late_gw(w, torch.mv(x.t(), gy).view(1, -1))
        if ctx.bias_ref is not None and ctx.needs_input_grad[2] and full:
            gb = convops._late_bias(ctx.bias_ref, gy.sum(0, keepdim=True))
        return gx, gw, gb


class _Outer(torch.autograd.Function):
    """dx = g w of _LinOut under create_graph (the scaling regulariser's
    Jacobian pass): its own backward as two matrix-vector products (gemv)
    instead of MulBackward0's broadcast multiplies and sums."""

    @staticmethod
    def forward(ctx, g, w):
        ctx.save_for_backward(g, w)
        return torch.outer(g, w.view(-1))

    @staticmethod
    def backward(ctx, gg):
        from . import convops
        g, w = ctx.saved_tensors
        g_g = torch.mv(gg, w.view(-1)) if ctx.needs_input_grad[0] else None
        g_w = None
        if ctx.needs_input_grad[1]:
            g_w = convops._late_gw(w, torch.mv(gg.t(), g).view(1, -1))
        return g_g, g_w


# SMMD_BN_RELU=0: torch's BatchNorm2d + relu for the generator outside autograd
BN_RELU = os.environ.get('SMMD_BN_RELU', '1') != '0'


# SMMD_BN_RELU_GRAD=0: with a gradient (the generator step) torch's / MIOpen's
# batch norm + relu instead of the library's forward and backward
BN_RELU_GRAD = os.environ.get('SMMD_BN_RELU_GRAD', '1') != '0'


def _bn_relu_fwd(bn, x, save):
    from . import _lib
    N, C, H, W = x.shape
    L = _lib.lib()
    ws = _lib.workspace('bn_relu', L.smmd_bn_relu_workspace_bytes(N, C), x.device)
    y = torch.empty_like(x)
    _lib.add_bytes('smmd_bn_relu_fwd', 3 * x.numel() * 4)
    with _lib.timed('smmd_bn_relu_fwd'):
        st = L.smmd_bn_relu_fwd_save(_lib.ptr(x), N, C, H * W, _lib.ptr(bn.weight),
                                     _lib.ptr(bn.bias), _lib.ptr(bn.running_mean),
                                     _lib.ptr(bn.running_var), float(bn.momentum), float(bn.eps),
                                     _lib.ptr(y), _lib.ptr(save), _lib.ptr(ws), ws.numel(),
                                     _lib.stream_handle(x.device))
    _lib.check(st, 'smmd_bn_relu_fwd')
    _count_batch(bn)
    return y


def _count_batch(bn):
    """nn.BatchNorm2d's num_batches_tracked += 1, counted on the host and added
    to the device buffer when a state_dict is taken: with momentum set it is
    bookkeeping only (TF's batch norm has none), and a device add per call was
    one kernel launch per layer per step (9 x ~4 us per generator forward).
    A load_state_dict drops the pending count with the value it replaces.
    While a step graph is captured (StepGraphs) the host code runs once, at
    capture: there the device add is captured instead, so every replay counts."""
    if bn.num_batches_tracked.is_cuda and torch.cuda.is_current_stream_capturing():
        with torch.no_grad():
            bn.num_batches_tracked.add_(1)
        return
    if getattr(bn, '_smmd_batches', None) is None:
        bn._smmd_batches = 0
        bn.register_state_dict_pre_hook(_flush_batches)
        bn._register_load_state_dict_pre_hook(_drop_batches, with_module=True)
    bn._smmd_batches += 1


def _flush_batches(module, prefix, keep_vars):
    if module._smmd_batches:
        with torch.no_grad():
            module.num_batches_tracked.add_(module._smmd_batches)
        module._smmd_batches = 0


def _drop_batches(module, state_dict, prefix, *args):
    module._smmd_batches = 0


class _BNReLU(torch.autograd.Function):
    """relu(batch_norm(x)) in training mode with the library's two-pass
    forward (statistics; normalise + ReLU + moving averages) and backward
    (smmd_bn_relu_bwd: the channel sums of gz and gz xhat; then dx, dgamma,
    dbeta).  A second-order backward (a critic with batch norm inside the
    scaling regulariser's double backward) is formed from torch ops on the
    saved statistics, so it stays differentiable."""

    @staticmethod
    def forward(ctx, x, gamma, beta, bn):
        C = x.shape[1]
        save = torch.empty(4 * C, device=x.device, dtype=torch.float32)
        y = _bn_relu_fwd(bn, x, save)
        ctx.save_for_backward(x, gamma, beta, save)
        ctx.eps = float(bn.eps)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, gamma, beta, save = ctx.saved_tensors
        N, C, H, W = x.shape
        if torch.is_grad_enabled():             # create_graph: differentiable torch ops
            # the batch statistics recomputed from x, so the second order keeps
            # their dependence on x
            mean = x.mean((0, 2, 3), keepdim=True)
            inv = torch.rsqrt(x.var((0, 2, 3), unbiased=False, keepdim=True) + ctx.eps)
            xh = (x - mean) * inv
            z = xh * gamma.view(1, C, 1, 1) + beta.view(1, C, 1, 1)
            gz = gy * (z > 0).to(gy.dtype)
            gb = gz.sum((0, 2, 3))
            gg = (gz * xh).sum((0, 2, 3))
            M = float(N * H * W)
            gx = (gamma.view(1, C, 1, 1) * inv) * (gz - gb.view(1, C, 1, 1) / M
                                                   - xh * gg.view(1, C, 1, 1) / M)
            return gx, gg, gb, None
        from . import _lib
        gy = gy.contiguous()
        L = _lib.lib()
        ws = _lib.workspace('bn_relu', L.smmd_bn_relu_workspace_bytes(N, C), x.device)
        gx = torch.empty_like(x)
        gg = torch.empty(C, device=x.device, dtype=torch.float32)
        gb = torch.empty(C, device=x.device, dtype=torch.float32)
        _lib.add_bytes('smmd_bn_relu_bwd', 5 * x.numel() * 4)
        with _lib.timed('smmd_bn_relu_bwd'):
            st = L.smmd_bn_relu_bwd(_lib.ptr(x), _lib.ptr(gy), N, C, H * W, _lib.ptr(beta),
                                    _lib.ptr(save), _lib.ptr(gx), _lib.ptr(gg), _lib.ptr(gb),
                                    _lib.ptr(ws), ws.numel(), _lib.stream_handle(x.device))
        _lib.check(st, 'smmd_bn_relu_bwd')
        return gx, gg, gb, None


def _bn_relu_ok(bn, x):
    return (isinstance(bn, nn.BatchNorm2d) and bn.training and bn.track_running_stats
            and bn.affine and bn.momentum is not None and x.is_cuda
            and x.dtype == torch.float32 and x.dim() == 4 and x.is_contiguous()
            and (x.shape[2] * x.shape[3]) % 4 == 0 and x.data_ptr() % 16 == 0)


def bn_relu(bn, x):
    """relu(bn(x)) (resnet/block.py:42-47 Normalize then tf.nn.relu) for a
    training-mode nn.BatchNorm2d on an NCHW device tensor, on the library:
    without a gradient (the generator's forward in every critic step) the
    two-pass smmd_bn_relu_fwd (batch statistics, moving averages, normalise +
    ReLU in one write); with one (the generator step) the same forward and
    smmd_bn_relu_bwd (_BNReLU).  Otherwise the torch modules."""
    if BN_RELU and _bn_relu_ok(bn, x):
        if not torch.is_grad_enabled():
            return _bn_relu_fwd(bn, x, None)
        if BN_RELU_GRAD:
            return _BNReLU.apply(x, bn.weight, bn.bias, bn)
    return F.relu(bn(x))


def lrelu(x, leak=0.2):
    """max(x, leak * x)  (snops.py:165-166)."""
    return F.leaky_relu(x, leak)


def sn_modules(module):
    return [m for m in module.modules() if isinstance(m, _SNMixin) and m.with_sn]
