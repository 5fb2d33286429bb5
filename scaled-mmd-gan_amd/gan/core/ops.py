"""Hot-path helpers of gan/core/ops.py and the scaled-loss op.

* ``safer_norm`` / ``sq_sum`` / ``dot``: small reductions (gan/core/ops.py:
  203-225) used by the gradient penalty; plain tensor reductions.
* ``jacobian_columns`` + ``scaled_loss``: ``squared_norm_jacobian``
  (ops.py:228-233) fused with ``add_scaling`` (gan/core/model.py:366-403) and
  ``apply_scaling`` (gan/core/smmd.py:21-23, :40-42) in libsmmd_hip: one
  HBM pass over the input-gradient, one single-block finalize, and a one-pass
  backward that feeds PyTorch's double-backward through the critic.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib
from .collectives import all_reduce_
from .convops import input_grad_only
from .mmd import _eps


def safer_norm(tensor, axis=None, keep_dims=False, epsilon=_eps):
    """sqrt(sum(t^2, axis) + eps)  (gan/core/ops.py:203-206)."""
    sq = tensor * tensor
    if axis is None:
        s = sq.sum()
    else:
        s = sq.sum(dim=axis, keepdim=keep_dims)
    return torch.sqrt(s + epsilon)


def sq_sum(t, name=None):
    """sum(t ** 2)  (gan/core/ops.py:209-213)."""
    return (t * t).sum()


def dot(x, y, name=None):
    """<x, y> of two vectors  (gan/core/ops.py:216-225)."""
    if x.dim() != 1 or y.dim() != 1:
        raise ValueError('dot expects rank-1 tensors')
    return (x * y).sum()


_SEEDS = {}


def grad_seed(y, i=None):
    """The gradient d(sum y[:, i]) / dy (i None: d(sum y) / dy) as a constant
    tensor, kept per shape outside a graph capture: seeding autograd with it
    gives the same gradient as differentiating the select and the sum -- the
    same ones in the same places -- without their zero, copy and fill
    kernels.  (Autograd never adds into a seed it does not own alone.)"""
    key = (tuple(y.shape), y.dtype, y.device, i)
    t = _SEEDS.get(key)
    if t is None:
        if i is None:
            t = torch.ones(y.shape, dtype=y.dtype, device=y.device)
        else:
            t = torch.zeros(y.shape, dtype=y.dtype, device=y.device)
            t[:, i] = 1
        if y.is_cuda and torch.cuda.is_current_stream_capturing():
            return t
        _SEEDS[key] = t
    return t


def jacobian_columns(y, x, create_graph=True):
    """Stack of d(sum_b y[b, i]) / dx for every critic output column i
    (gan/core/ops.py:230-231): returns [d, *x.shape].  The critic has no
    cross-sample coupling in the configs (no BN in D), so
    row b of column i is d y[b, i] / d x[b].  Each column's pass is seeded
    with grad_seed(y, i), the gradient of y[:, i].sum() w.r.t. y."""
    d = y.shape[1]
    cols = []
    for i in range(d):
        with input_grad_only():       # no weight-gradient kernels in this pass
            g, = torch.autograd.grad(y, x, grad_outputs=grad_seed(y, i),
                                     create_graph=create_graph, retain_graph=True)
        cols.append(g)
    return torch.stack(cols, 0) if d > 1 else cols[0].unsqueeze(0)


class _ScaledLoss(torch.autograd.Function):
    """g_loss = base * f(scale), scale = 1 / (sc * Q + 1),
    Q = mean_b sum_c ||jac[c, b]||^2 (+ mean(feat^2) for 'value_and_grad'),
    f = id (SMMD) or sqrt (SWGAN)."""

    @staticmethod
    def forward(ctx, base, jac, feat, sc, variant, sqrt_scale, b_total, group, pre):
        _lib.require_cuda(base, jac, feat)
        jac = jac.contiguous()
        n_cols, b = jac.shape[0], jac.shape[1]
        per = jac[0, 0].numel()
        dev = jac.device
        L = _lib.lib()
        base = base.reshape(1).contiguous()
        feat_c = feat.contiguous() if feat is not None else None
        dof = feat_c.shape[1] if feat_c is not None else 0
        s = _lib.stream_handle(dev)
        per_sample = torch.empty(b, device=dev, dtype=torch.float32)
        if pre is not None:
            # global J / nD already known (gathered with the step's features):
            # only the single-thread finalize runs
            out = torch.zeros(8, device=dev, dtype=torch.float32)
            out[3:5] = pre
            out[5:6] = base.detach()
            _lib.check(L.smmd_scaled_loss_finalize(_lib.ptr(out), float(sc), variant,
                                                   sqrt_scale, s), 'smmd_scaled_loss_finalize')
            group = None
        else:
            out = torch.empty(8, device=dev, dtype=torch.float32)
            nbytes = L.smmd_scaled_loss_workspace_bytes(n_cols * b, per)
            ws = _lib.workspace('scaled_loss', nbytes, dev)
            args = (_lib.ptr(jac), n_cols, b, b_total, per, _lib.ptr(feat_c), dof,
                    _lib.ptr(base), float(sc), variant, sqrt_scale, _lib.ptr(out),
                    _lib.ptr(per_sample), _lib.ptr(ws), ws.numel(), s)
            with _lib.timed('smmd_scaled_loss_fwd'):
                st = L.smmd_scaled_loss_fwd(*args)
            _lib.check(st, 'smmd_scaled_loss_fwd')
        if group is not None:
            # J and nD are partial means over the global batch: sum them
            all_reduce_(out[3:5], group)
            _lib.check(L.smmd_scaled_loss_finalize(_lib.ptr(out), float(sc), variant,
                                                   sqrt_scale, s), 'smmd_scaled_loss_finalize')
        ctx.save_for_backward(jac, feat_c, out)
        ctx.cfg = (n_cols, b, b_total, per, dof, float(sc), variant, sqrt_scale)
        ctx.mark_non_differentiable(out, per_sample)
        return out[0].view(()), out, per_sample

    @staticmethod
    def backward(ctx, g_gloss, g_out, g_ps):
        jac, feat, out = ctx.saved_tensors
        n_cols, b, b_total, per, dof, sc, variant, sqrt_scale = ctx.cfg
        dev = jac.device
        go = g_gloss.reshape(1).contiguous().to(torch.float32)
        d_base = torch.empty(1, device=dev, dtype=torch.float32)
        gjac = torch.empty_like(jac)
        gfeat = torch.empty_like(feat) if (feat is not None and variant == 1) else None
        args = (_lib.ptr(jac), n_cols, b, b_total, per, _lib.ptr(feat), dof, _lib.ptr(out), sc,
                variant, sqrt_scale, _lib.ptr(go), _lib.ptr(d_base), _lib.ptr(gjac),
                _lib.ptr(gfeat), _lib.stream_handle(dev))
        with _lib.timed('smmd_scaled_loss_bwd'):
            st = _lib.lib().smmd_scaled_loss_bwd(*args)
        _lib.check(st, 'smmd_scaled_loss_bwd')
        if feat is not None and gfeat is None:
            gfeat = torch.zeros_like(feat)
        return d_base.view(()), gjac, gfeat, None, None, None, None, None, None


def _b_total(jac, process_group):
    from .collectives import is_dp
    group = process_group if is_dp(process_group) else None
    return group, jac.shape[1] * (dist.get_world_size(group) if group is not None else 1)


def scaling_partials(jac, feat=None, variant='grad', process_group=None):
    """This rank's share of (J, nD) over the global batch -- sum over its rows
    divided by the global batch size -- as a detached [2] tensor: the partials
    a collectives.StepExchange gathers with the critic features so the scale
    needs no all-reduce of its own (``scaled_loss(..., pre=sum of them)``)."""
    v = {'grad': 0, 'value_and_grad': 1}[variant]
    _, b_total = _b_total(jac, process_group)
    jac = jac.detach().contiguous()
    n_cols, b, per = jac.shape[0], jac.shape[1], jac[0, 0].numel()
    feat_c = feat.detach().contiguous() if (feat is not None and v == 1) else None
    dof = feat_c.shape[1] if feat_c is not None else 0
    dev = jac.device
    L = _lib.lib()
    out = torch.empty(8, device=dev, dtype=torch.float32)
    ws = _lib.workspace('scaled_loss', L.smmd_scaled_loss_workspace_bytes(n_cols * b, per), dev)
    with _lib.timed('smmd_scaled_loss_fwd'):
        st = L.smmd_scaled_loss_fwd(_lib.ptr(jac), n_cols, b, b_total, per, _lib.ptr(feat_c), dof,
                                    None, 0.0, v, 0, _lib.ptr(out), None, _lib.ptr(ws),
                                    ws.numel(), _lib.stream_handle(dev))
    _lib.check(st, 'smmd_scaled_loss_fwd')
    return out[3:5]


def scaled_loss(base, jac, feat=None, sc=10.0, variant='grad', sqrt_scale=False,
                process_group=None, pre=None):
    """Apply the scaling regulariser to ``base`` (mmd2 for SMMD, the critic
    mean difference for SWGAN).  ``jac`` = jacobian_columns(d_images, images).

    Returns (g_loss, aux) with aux a detached 8-vector
    [g_loss, d_loss, scale, J, norm_discriminator, base, 0, 0] and, in the
    all-gather mode, J / nD over the global batch: all-reduced here, or
    ``pre`` = their global values already gathered (collectives.StepExchange)."""
    v = {'grad': 0, 'value_and_grad': 1}[variant]
    if v == 1 and feat is None:
        raise ValueError("scaling_variant 'value_and_grad' needs the critic output")
    group, b_total = _b_total(jac, process_group)
    g, out, _ = _ScaledLoss.apply(base, jac, feat if v == 1 else None, sc, v,
                                  1 if sqrt_scale else 0, b_total, group, pre)
    return g, out


class _ScaleFactor(torch.autograd.Function):
    """scale = 1 / (sc * Q + 1) alone (model.py:387-390), for an overridden
    apply_scaling: the same HIP pass as _ScaledLoss without a base loss.  The
    backward reuses smmd_scaled_loss_bwd with base := 1 and f = id, whose
    dL/dQ = go * base * (-sc scale^2) is then exactly d scale / dQ * go."""

    @staticmethod
    def forward(ctx, jac, feat, sc, variant, b_total, group, pre):
        _lib.require_cuda(jac, feat)
        jac = jac.contiguous()
        n_cols, b = jac.shape[0], jac.shape[1]
        per = jac[0, 0].numel()
        dev = jac.device
        L = _lib.lib()
        feat_c = feat.contiguous() if feat is not None else None
        dof = feat_c.shape[1] if feat_c is not None else 0
        s = _lib.stream_handle(dev)
        if pre is not None:
            out = torch.zeros(8, device=dev, dtype=torch.float32)
            out[3:5] = pre
            _lib.check(L.smmd_scaled_loss_finalize(_lib.ptr(out), float(sc), variant, 0, s),
                       'smmd_scaled_loss_finalize')
            group = None
        else:
            out = torch.empty(8, device=dev, dtype=torch.float32)
            per_sample = torch.empty(b, device=dev, dtype=torch.float32)
            ws = _lib.workspace('scaled_loss',
                                L.smmd_scaled_loss_workspace_bytes(n_cols * b, per), dev)
            with _lib.timed('smmd_scaled_loss_fwd'):
                st = L.smmd_scaled_loss_fwd(_lib.ptr(jac), n_cols, b, b_total, per,
                                            _lib.ptr(feat_c), dof, None, float(sc), variant, 0,
                                            _lib.ptr(out), _lib.ptr(per_sample), _lib.ptr(ws),
                                            ws.numel(), s)
            _lib.check(st, 'smmd_scaled_loss_fwd')
        if group is not None:
            all_reduce_(out[3:5], group)
            _lib.check(L.smmd_scaled_loss_finalize(_lib.ptr(out), float(sc), variant, 0, s),
                       'smmd_scaled_loss_finalize')
        ctx.save_for_backward(jac, feat_c, out)
        ctx.cfg = (n_cols, b, b_total, per, dof, float(sc), variant)
        ctx.mark_non_differentiable(out)
        return out[2].clone().view(()), out

    @staticmethod
    def backward(ctx, g_scale, g_out):
        jac, feat, out = ctx.saved_tensors
        n_cols, b, b_total, per, dof, sc, variant = ctx.cfg
        unit = out.clone()
        unit[5] = 1.0                      # base := 1, so dL/dQ = g_scale d scale / dQ
        go = g_scale.reshape(1).contiguous().to(torch.float32)
        gjac = torch.empty_like(jac)
        gfeat = torch.empty_like(feat) if (feat is not None and variant == 1) else None
        with _lib.timed('smmd_scaled_loss_bwd'):
            st = _lib.lib().smmd_scaled_loss_bwd(
                _lib.ptr(jac), n_cols, b, b_total, per, _lib.ptr(feat), dof, _lib.ptr(unit), sc,
                variant, 0, _lib.ptr(go), None, _lib.ptr(gjac), _lib.ptr(gfeat),
                _lib.stream_handle(jac.device))
        _lib.check(st, 'smmd_scaled_loss_bwd')
        if feat is not None and gfeat is None:
            gfeat = torch.zeros_like(feat)
        return gjac, gfeat, None, None, None, None, None


def scaling_factor(jac, feat=None, sc=10.0, variant='grad', process_group=None, pre=None):
    """scale of MMD_GAN.add_scaling (model.py:382-390) as a differentiable
    0-dim tensor, for an ``apply_scaling(scale)`` override.  Returns (scale,
    aux) with aux as in ``scaled_loss`` (g_loss, d_loss and base unset)."""
    v = {'grad': 0, 'value_and_grad': 1}[variant]
    if v == 1 and feat is None:
        raise ValueError("scaling_variant 'value_and_grad' needs the critic output")
    group, b_total = _b_total(jac, process_group)
    scale, out = _ScaleFactor.apply(jac, feat if v == 1 else None, sc, v, b_total, group, pre)
    return scale, out


class _SqNormJac(torch.autograd.Function):
    @staticmethod
    def forward(ctx, jac):
        _lib.require_cuda(jac)
        jac = jac.contiguous()
        n_cols, b = jac.shape[0], jac.shape[1]
        per = jac[0, 0].numel()
        dev = jac.device
        L = _lib.lib()
        out = torch.empty(8, device=dev, dtype=torch.float32)
        per_sample = torch.empty(b, device=dev, dtype=torch.float32)
        ws = _lib.workspace('scaled_loss', L.smmd_scaled_loss_workspace_bytes(n_cols * b, per),
                            dev)
        _lib.check(L.smmd_scaled_loss_fwd(_lib.ptr(jac), n_cols, b, b, per, None, 0, None, 0.0,
                                          0, 0, _lib.ptr(out), _lib.ptr(per_sample), _lib.ptr(ws),
                                          ws.numel(), _lib.stream_handle(dev)),
                   'smmd_scaled_loss_fwd')
        ctx.save_for_backward(jac)
        return per_sample

    @staticmethod
    def backward(ctx, g):
        jac, = ctx.saved_tensors
        return 2.0 * jac * g.view(1, -1, *([1] * (jac.dim() - 2)))


def squared_norm_jacobian(y, x):
    """sum_i ||d y[:, i] / d x||^2 per sample  (gan/core/ops.py:228-233)."""
    return _SqNormJac.apply(jacobian_columns(y, x))
