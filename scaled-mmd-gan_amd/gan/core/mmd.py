"""MMD kernels and the MMD^2 estimator on the MI355X hot path.

Drop-in for the reference's ``gan/core/mmd.py`` (names, signatures, default
parameters and the ``(K_XX, K_XY, K_YY, const_diagonal)`` contract of
``_<kind>_kernel``), re-implemented on ``libsmmd_hip.so``:

* ``mmd2(_rbf_kernel(X, Y))`` -- the loss of ``SMMD.set_loss``
  (gan/core/smmd.py:11-15) -- runs as ONE fused HIP launch that never
  materialises the N x N matrices and produces d mmd2 / dX, dY in the same
  sweep (``smmd_mmd2_fwd``).
* The kernel functions return a lazy :class:`KernelMatrices`; its elements are
  materialised (by ``smmd_kernel_matrix_fwd``) only when a caller indexes or
  unpacks it, exactly like the reference tuple.
* ``K_XY_only=True`` returns the materialised K_XY (gan/core/mmd.py:72-73).

All arithmetic is fp32 on the GPU.  There is no CPU path: tensors must live on
a ROCm device and the library must be built (see ``_lib``).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from .collectives import all_reduce_, gather_rows, is_dp
from . import _lib

_eps = 1.0e-5   # gan/core/mmd.py:6


def mysqrt(x):
    """sqrt(max(x + eps, 0))  (gan/core/mmd.py:12)."""
    return torch.sqrt(torch.clamp(x + _eps, min=0.0))


# ---------------------------------------------------------------------------
# kernel specification
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class KernelSpec:
    """One member of the kernel family (gan/core/mmd.py:18-188).

    const_diag is None where the reference returns ``False`` (the estimator
    then subtracts the trace, mmd.py:212-213)."""
    name: str
    kind: int
    params: tuple = ()
    wts: tuple = ()
    add_dot: float = 0.0
    tanh: bool = False
    const_diag: float | None = None
    _desc: object = field(default=None, compare=False, repr=False)

    def desc(self):
        d = _lib.KernelDesc()
        d.kind = self.kind
        d.n_terms = len(self.params)
        for i, (p, w) in enumerate(zip(self.params, self.wts)):
            d.param[i] = float(p)
            d.wt[i] = float(w)
        d.add_dot = float(self.add_dot)
        d.tanh_inputs = 1 if self.tanh else 0
        d.has_const_diag = 0 if self.const_diag is None else 1
        d.const_diag = 0.0 if self.const_diag is None else float(self.const_diag)
        return d


_RQ_DOT = {'mix_rq': 0.0, 'mix_rq_dot': .1, 'mix_rq_1dot': 1., 'mix_rq_10dot': 10.,
           'mix_rq_01dot': .1, 'mix_rq_001dot': .01, 'tanh_mix_rq': 0.0}

KERNEL_NAMES = ('rbf', 'mix_rbf', 'mix_rq', 'mix_rq_dot', 'mix_rq_1dot', 'mix_rq_10dot',
                'mix_rq_01dot', 'mix_rq_001dot', 'tanh_mix_rq', 'distance', 'tanh_distance',
                'dot')


def get_kernel_spec(name: str, **kw) -> KernelSpec:
    """``config.kernel`` string -> KernelSpec with the reference defaults."""
    if name == 'rbf':                                           # mmd.py:55
        sigma, wt = kw.get('sigma', 1.), kw.get('wt', 1.)
        return KernelSpec('rbf', _lib.KIND_RBF, (sigma,), (wt,), const_diag=float(wt))
    if name == 'mix_rbf':                                       # mmd.py:85-87
        sigmas = tuple(kw.get('sigmas', (2.0, 5.0, 10.0, 20.0, 40.0, 80.0)))
        wts = tuple(kw.get('wts') or [1] * len(sigmas))
        return KernelSpec('mix_rbf', _lib.KIND_RBF, sigmas, wts, const_diag=float(sum(wts)))
    if name in _RQ_DOT:                                         # mmd.py:119-188
        alphas = tuple(kw.get('alphas', (.1, 1., 10.)))
        wts = tuple(kw.get('wts') or [1.] * len(alphas))
        add_dot = float(kw.get('add_dot', _RQ_DOT[name]))
        # quirk kept: const diagonal = sum(wts) even when add_dot > 0 (mmd.py:182-188)
        return KernelSpec(name, _lib.KIND_RQ, alphas, wts, add_dot=add_dot,
                          tanh=(name == 'tanh_mix_rq'), const_diag=float(sum(wts)))
    if name in ('distance', 'tanh_distance'):                   # mmd.py:18-41
        return KernelSpec(name, _lib.KIND_DISTANCE, tanh=(name == 'tanh_distance'))
    if name == 'dot':                                           # mmd.py:44-52
        return KernelSpec('dot', _lib.KIND_DOT)
    raise ValueError('unknown kernel %r (known: %s)' % (name, ', '.join(KERNEL_NAMES)))


def _as_spec(kernel, **kw) -> KernelSpec:
    if isinstance(kernel, KernelSpec):
        return kernel
    return get_kernel_spec(kernel, **kw)


def _features(t):
    if t.dim() == 1:
        t = t.unsqueeze(1)
    if t.dim() != 2:
        raise ValueError('critic features must be [batch, dof] (got %s)' % (tuple(t.shape),))
    _lib.require_cuda(t)
    return t.contiguous()


# ---------------------------------------------------------------------------
# fused MMD^2 (forward + unit gradient in one launch)
# ---------------------------------------------------------------------------
# In the all-gather mode a global batch of at most this many rows per side is
# evaluated whole on every rank (one more launch-bound sweep, no all-reduce of
# partial sums); larger ones are row-sharded, each rank its own rows against
# all columns, with the 8 partial sums all-reduced.
FULL_ROWS = int(os.environ.get('SMMD_GLOBAL_FULL_ROWS', '4096'))


class _MMD2Fused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, Y, spec, biased, group, exchange):
        X = _features(X)
        Y = _features(Y)
        if X.shape[1] != Y.shape[1]:
            raise ValueError('X and Y feature dims differ: %d vs %d' % (X.shape[1], Y.shape[1]))
        dev = X.device
        L = _lib.lib()
        need_grad = ctx.needs_input_grad[0] or ctx.needs_input_grad[1]
        d = X.shape[1]
        ml, nl = X.shape[0], Y.shape[0]
        shard = False
        if is_dp(group):
            world, rank = dist.get_world_size(group), dist.get_rank(group)
            if exchange is not None and exchange.group is group and not exchange.used:
                Xa, Ya = exchange.gather(X, Y)     # the step's one packed all-gather
            else:
                # ONE all-gather of the packed local rows [X; Y] (latency-bound:
                # 2 x 256 B per rank at batch 64), then each side's rows in rank order
                Za = gather_rows(torch.cat([X, Y], 0), group).view(world, ml + nl, d)
                Xa = Za[:, :ml].reshape(world * ml, d)
                Ya = Za[:, ml:].reshape(world * nl, d)
            shard = max(Xa.shape[0], Ya.shape[0]) > FULL_ROWS
            own = (rank * ml, (rank + 1) * ml, rank * nl, (rank + 1) * nl)
        else:
            group = None
            Xa, Ya = X, Y
        m, n = Xa.shape[0], Ya.shape[0]
        rows = own if shard else (0, m, 0, n)
        sums = torch.empty(8, device=dev, dtype=torch.float32)
        out = torch.empty(1, device=dev, dtype=torch.float32)
        gx = gy = None
        if need_grad:
            gx = torch.empty((rows[1] - rows[0], d), device=dev, dtype=torch.float32)
            gy = torch.empty((rows[3] - rows[2], d), device=dev, dtype=torch.float32)
        nbytes = L.smmd_mmd2_workspace_bytes(m, n, d)
        ws = _lib.workspace('mmd2', nbytes, dev)
        desc = spec.desc()
        args = (desc, _lib.ptr(Xa), m, _lib.ptr(Ya), n, d, 1 if biased else 0, *rows,
                _lib.ptr(sums), _lib.ptr(out), _lib.ptr(gx), _lib.ptr(gy), _lib.ptr(ws),
                ws.numel(), _lib.stream_handle(dev))
        with _lib.timed('smmd_mmd2_fwd'):
            st = L.smmd_mmd2_fwd(*args)
        _lib.check(st, 'smmd_mmd2_fwd')
        if group is not None and shard:
            all_reduce_(sums, group)
            _lib.check(L.smmd_mmd2_combine(desc, _lib.ptr(sums), m, n, 1 if biased else 0,
                                           _lib.ptr(out), _lib.stream_handle(dev)),
                       'smmd_mmd2_combine')
        elif group is not None and need_grad:
            # the whole batch was evaluated: this rank's rows of the gradient
            gx = gx[own[0]:own[1]]
            gy = gy[own[2]:own[3]]
        ctx.save_for_backward(gx, gy)
        ctx.mark_non_differentiable(sums)
        return out.view(()), sums

    @staticmethod
    def backward(ctx, g_mmd2, g_sums):
        gx, gy = ctx.saved_tensors
        dX = dY = None
        if gx is not None:
            dX = gx * g_mmd2
            dY = gy * g_mmd2
        return dX, dY, None, None, None, None


def mmd2_fused(X, Y, kernel='rbf', biased=False, process_group=None, return_sums=False,
               exchange=None, **kw):
    """mmd.mmd2(mmd._<kernel>_kernel(X, Y), biased) as one HIP launch.

    ``process_group`` (a torch.distributed group with >1 ranks) selects the
    all-gather mode: every rank contributes its local rows of X and Y, sees
    the full (world * batch) pairwise kernel, and gets the same estimator
    and the gradient of its own rows.  Messages: one all-gather of the packed
    rows (carried by ``exchange``, a collectives.StepExchange, when given),
    plus one all-reduce of 8 floats only when the global batch exceeds
    FULL_ROWS per side and the sweep is row-sharded."""
    spec = _as_spec(kernel, **kw)
    val, sums = _MMD2Fused.apply(X, Y, spec, bool(biased), process_group, exchange)
    return (val, sums) if return_sums else val


# ---------------------------------------------------------------------------
# the SMMD loss in one launch: mmd2 and the scaled loss of one process (or a
# tower), when the Jacobian of the scaling regulariser is already known as
# mmd2 runs (model.set_tower_loss computes it ahead, ``pending_scale``)
# ---------------------------------------------------------------------------
TILE_MAX_ROWS = (16384 // 4 - 64) * 64      # csrc/smmd_kern.hpp TILE_MAX_RT * 64


def _env_first(name):
    """The first character of an environment flag, as the library reads it
    (csrc/smmd_mmd.hip: `e && e[0] == '1'`), or '' when unset."""
    return (os.environ.get(name) or '')[:1]


def fused_loss_path(m, n, d):
    """smmd_smmd_loss_fwd applies: smmd_mmd2_fwd's 2-D tiled path
    (csrc/smmd_mmd.hip use_tile, its flags parsed the same way) and
    SMMD_FUSED_LOSS not 0.  Should the library still answer
    SMMD_EUNSUPPORTED, _mmd2_scaled falls back to the two separate calls."""
    if _env_first('SMMD_FUSED_LOSS') == '0':
        return False
    if d > 8 or _env_first('SMMD_MMD_GRAM') == '1' or _env_first('SMMD_MMD_TILE') == '0':
        return False
    return m + n <= TILE_MAX_ROWS


class _FusedUnsupported(Exception):
    """smmd_smmd_loss_fwd returned SMMD_EUNSUPPORTED (the caller falls back)."""


class _SMMDLoss(torch.autograd.Function):
    """(mmd2, g_loss = mmd2 * scale) of one launch (smmd_smmd_loss_fwd) and
    their joint backward (smmd_smmd_loss_bwd)."""

    @staticmethod
    def forward(ctx, X, Y, jac, feat, spec, biased, sc, variant):
        X = _features(X)
        Y = _features(Y)
        _lib.require_cuda(jac, feat)
        jac = jac.contiguous()
        feat_c = feat.contiguous() if feat is not None else None
        dev = X.device
        L = _lib.lib()
        m, n, d = X.shape[0], Y.shape[0], X.shape[1]
        n_cols, b = jac.shape[0], jac.shape[1]
        per = jac[0, 0].numel()
        dof = feat_c.shape[1] if feat_c is not None else 0
        sums = torch.empty(8, device=dev, dtype=torch.float32)
        mm = torch.empty(1, device=dev, dtype=torch.float32)
        gx = torch.empty((m, d), device=dev, dtype=torch.float32)
        gy = torch.empty((n, d), device=dev, dtype=torch.float32)
        out = torch.empty(8, device=dev, dtype=torch.float32)
        per_sample = torch.empty(b, device=dev, dtype=torch.float32)
        ws = _lib.workspace('mmd2', L.smmd_mmd2_workspace_bytes(m, n, d), dev)
        lws = _lib.workspace('scaled_loss', L.smmd_scaled_loss_workspace_bytes(n_cols * b, per),
                             dev)
        _lib.add_bytes('smmd_smmd_loss_fwd', jac.numel() * 4 + 4 * (m + n) * d * 4)
        with _lib.timed('smmd_smmd_loss_fwd'):
            st = L.smmd_smmd_loss_fwd(
                spec.desc(), _lib.ptr(X), m, _lib.ptr(Y), n, d, 1 if biased else 0,
                _lib.ptr(jac), n_cols, b, per, _lib.ptr(feat_c), dof, float(sc), variant, 0,
                _lib.ptr(sums), _lib.ptr(mm), _lib.ptr(gx), _lib.ptr(gy), _lib.ptr(out),
                _lib.ptr(per_sample), _lib.ptr(ws), ws.numel(), _lib.ptr(lws), lws.numel(),
                _lib.stream_handle(dev))
        if st == _lib.SMMD_EUNSUPPORTED:
            raise _FusedUnsupported()
        _lib.check(st, 'smmd_smmd_loss_fwd')
        ctx.save_for_backward(gx, gy, jac, feat_c, out)
        ctx.cfg = (n_cols, b, per, dof, float(sc), variant, m, n, d)
        ctx.mark_non_differentiable(sums, out)
        # the unused outputs' gradients arrive as None, not as zero fills
        ctx.set_materialize_grads(False)
        return mm.view(()), out[0].view(()), sums, out

    @staticmethod
    def backward(ctx, g_mmd, g_loss, g_sums, g_out):
        gx, gy, jac, feat, out = ctx.saved_tensors
        n_cols, b, per, dof, sc, variant, m, n, d = ctx.cfg
        dev = gx.device
        go = (g_loss.reshape(1).contiguous().to(torch.float32) if g_loss is not None
              else torch.zeros(1, device=dev, dtype=torch.float32))
        gm = g_mmd.reshape(1).contiguous().to(torch.float32) if g_mmd is not None else None
        dX, dY = torch.empty_like(gx), torch.empty_like(gy)
        gjac = torch.empty_like(jac) if ctx.needs_input_grad[2] else None
        gfeat = (torch.empty_like(feat) if (feat is not None and variant == 1
                                            and ctx.needs_input_grad[3]) else None)
        # the Jacobian read and its gradient written (critic steps), the
        # features' unit gradients read and dX, dY written
        _lib.add_bytes('smmd_smmd_loss_bwd', (2 * jac.numel() * 4 if gjac is not None else 0)
                       + 2 * (m + n) * d * 4)
        with _lib.timed('smmd_smmd_loss_bwd'):
            st = _lib.lib().smmd_smmd_loss_bwd(
                _lib.ptr(jac), n_cols, b, per, _lib.ptr(feat), dof, _lib.ptr(out), sc, variant, 0,
                _lib.ptr(go), _lib.ptr(gm), _lib.ptr(gx), m, _lib.ptr(gy), n, d, _lib.ptr(gjac),
                _lib.ptr(gfeat), _lib.ptr(dX), _lib.ptr(dY), _lib.stream_handle(dev))
        _lib.check(st, 'smmd_smmd_loss_bwd')
        if feat is not None and gfeat is None and ctx.needs_input_grad[3]:
            gfeat = torch.zeros_like(feat)
        return dX, dY, gjac, gfeat, None, None, None, None


class _SMMDLossGathered(torch.autograd.Function):
    """The all-gather mode's SMMD loss: the step exchange's one packed
    all-gather, then ONE launch (smmd_smmd_loss_fwd_gathered) for the MMD^2
    sweep over the gathered global rows and the scaled loss, whose J / nD the
    kernel sums in rank order from the gathered per-rank partials; its
    backward is one smmd_smmd_loss_bwd_ex launch over this rank's rows and
    Jacobian (normaliser: the global batch).  Replaces, in that mode,
    smmd_mmd2_fwd + the torch sum of the partials + smmd_scaled_loss_finalize
    forward and the two separate backward passes."""

    @staticmethod
    def forward(ctx, X, Y, jac, feat, spec, biased, sc, variant, ex):
        X = _features(X)
        Y = _features(Y)
        _lib.require_cuda(jac, feat)
        jac = jac.contiguous()
        feat_c = feat.contiguous() if feat is not None else None
        dev = X.device
        L = _lib.lib()
        ml, nl, d = X.shape[0], Y.shape[0], X.shape[1]
        allp, Xa, Ya = ex.gather_packed(X, Y)
        allp = allp.contiguous()
        world, rank = ex.world, ex.rank
        m, n = Xa.shape[0], Ya.shape[0]
        n_cols, b = jac.shape[0], jac.shape[1]
        per = jac[0, 0].numel()
        dof = feat_c.shape[1] if feat_c is not None else 0
        sums = torch.empty(8, device=dev, dtype=torch.float32)
        mm = torch.empty(1, device=dev, dtype=torch.float32)
        gx = torch.empty((m, d), device=dev, dtype=torch.float32)
        gy = torch.empty((n, d), device=dev, dtype=torch.float32)
        out = torch.empty(8, device=dev, dtype=torch.float32)
        ws = _lib.workspace('mmd2', L.smmd_mmd2_workspace_bytes(m, n, d), dev)
        lws = _lib.workspace('scaled_loss', L.smmd_scaled_loss_workspace_bytes(1, 1), dev)
        stats = allp[:, (ml + nl) * d:]
        with _lib.timed('smmd_smmd_loss_fwd'):
            st = L.smmd_smmd_loss_fwd_gathered(
                spec.desc(), _lib.ptr(Xa), m, _lib.ptr(Ya), n, d, 1 if biased else 0,
                _lib.ptr(stats), world, allp.shape[1], float(sc), variant, 0, _lib.ptr(sums),
                _lib.ptr(mm), _lib.ptr(gx), _lib.ptr(gy), _lib.ptr(out), _lib.ptr(ws), ws.numel(),
                _lib.ptr(lws), lws.numel(), _lib.stream_handle(dev))
        _lib.check(st, 'smmd_smmd_loss_fwd_gathered')   # the Python gate mirrors use_tile
        ex.stats_total = out[3:5]
        gx_own = gx[rank * ml:(rank + 1) * ml]
        gy_own = gy[rank * nl:(rank + 1) * nl]
        ctx.save_for_backward(gx_own, gy_own, jac, feat_c, out)
        ctx.cfg = (n_cols, b, world * b, per, dof, float(sc), variant, ml, nl, d)
        ctx.mark_non_differentiable(sums, out)
        ctx.set_materialize_grads(False)
        return mm.view(()), out[0].view(()), sums, out

    @staticmethod
    def backward(ctx, g_mmd, g_loss, g_sums, g_out):
        gx, gy, jac, feat, out = ctx.saved_tensors
        n_cols, b, b_total, per, dof, sc, variant, m, n, d = ctx.cfg
        dev = gx.device
        go = (g_loss.reshape(1).contiguous().to(torch.float32) if g_loss is not None
              else torch.zeros(1, device=dev, dtype=torch.float32))
        gm = g_mmd.reshape(1).contiguous().to(torch.float32) if g_mmd is not None else None
        dX, dY = torch.empty_like(gx), torch.empty_like(gy)
        gjac = torch.empty_like(jac) if ctx.needs_input_grad[2] else None
        gfeat = (torch.empty_like(feat) if (feat is not None and variant == 1
                                            and ctx.needs_input_grad[3]) else None)
        with _lib.timed('smmd_smmd_loss_bwd'):
            st = _lib.lib().smmd_smmd_loss_bwd_ex(
                _lib.ptr(jac), n_cols, b, b_total, per, _lib.ptr(feat), dof, _lib.ptr(out), sc,
                variant, 0, _lib.ptr(go), _lib.ptr(gm), _lib.ptr(gx), m, _lib.ptr(gy), n, d,
                _lib.ptr(gjac), _lib.ptr(gfeat), _lib.ptr(dX), _lib.ptr(dY),
                _lib.stream_handle(dev))
        _lib.check(st, 'smmd_smmd_loss_bwd_ex')
        if feat is not None and gfeat is None and ctx.needs_input_grad[3]:
            gfeat = torch.zeros_like(feat)
        return dX, dY, gjac, gfeat, None, None, None, None, None


# SMMD_GLOBAL_FUSED_LOSS=0: the all-gather mode's loss as separate launches
GLOBAL_FUSED_LOSS = os.environ.get('SMMD_GLOBAL_FUSED_LOSS', '1') != '0'


def _mmd2_scaled_gathered(K, biased, ex):
    """mmd2 of K fused with the scaled loss in the all-gather mode (the step
    exchange carries the Jacobian partials), or None when it does not apply:
    a row-sharded global batch (> FULL_ROWS per side), a path the fused
    launch does not take, an overridden apply_scaling."""
    X, Y = K.X, K.Y
    group = current_loss_group()
    if not (GLOBAL_FUSED_LOSS and ex is not None and ex.fuse and not ex.used
            and ex.result is None and ex.jac is not None and ex.stats is not None
            and is_dp(group) and ex.group is group):
        return None
    if X.dim() == 1 or Y.dim() == 1 or X.shape[1] != Y.shape[1]:
        return None
    m, n, d = ex.world * X.shape[0], ex.world * Y.shape[0], X.shape[1]
    if max(m, n) > FULL_ROWS or not fused_loss_path(m, n, d):
        return None
    feat = ex.feat if ex.variant == 1 else None
    if ex.variant == 1 and feat is None:
        return None
    val, g, _, out = _SMMDLossGathered.apply(X, Y, ex.jac, feat, K.spec, bool(biased), ex.sc,
                                             ex.variant, ex)
    ex.result = (val, g, out)
    return val


class ScalePending:
    """The scaling regulariser's inputs known before ``set_loss`` runs (the
    Jacobian columns of the real batch, the critic output for nD): the first
    mmd2 of a KernelMatrices inside ``pending_scale(p)`` then runs fused with
    the scaled loss, leaving (mmd2, g_loss, aux) in ``p.result`` for
    ``add_scaling`` to pick up."""

    def __init__(self, jac, feat, sc, variant, fuse=True):
        self.jac, self.feat, self.sc = jac, feat, sc
        self.variant = {'grad': 0, 'value_and_grad': 1}[variant]
        self.fuse = fuse          # False: only the Jacobian is provided ahead
        self.result = None


class pending_scale:
    def __init__(self, pending):
        self.pending = pending

    def __enter__(self):
        self.prev = getattr(_scope, 'pending', None)
        _scope.pending = self.pending
        return self

    def __exit__(self, *a):
        _scope.pending = self.prev
        return False


def current_pending():
    return getattr(_scope, 'pending', None)


def _mmd2_scaled(K, biased, p):
    """mmd2 of K fused with the pending scaled loss, or None when it does not apply."""
    X, Y = K.X, K.Y
    if X.dim() == 1 or Y.dim() == 1 or X.shape[1] != Y.shape[1]:
        return None
    if not fused_loss_path(X.shape[0], Y.shape[0], X.shape[1]):
        return None
    feat = p.feat if p.variant == 1 else None
    if p.variant == 1 and feat is None:
        return None
    try:
        val, g, _, out = _SMMDLoss.apply(X, Y, p.jac, feat, K.spec, bool(biased), p.sc,
                                         p.variant)
    except _FusedUnsupported:      # the header's contract: make the two separate calls
        return None
    p.result = (val, g, out)
    return val


# ---------------------------------------------------------------------------
# materialised kernel matrices (tuple API)
# ---------------------------------------------------------------------------
class _KernelMatrix(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, B, spec):
        A = _features(A)
        B = _features(B)
        L = _lib.lib()
        out = torch.empty((A.shape[0], B.shape[0]), device=A.device, dtype=torch.float32)
        _lib.check(L.smmd_kernel_matrix_fwd(spec.desc(), _lib.ptr(A), A.shape[0], _lib.ptr(B),
                                            B.shape[0], A.shape[1], _lib.ptr(out),
                                            _lib.stream_handle(A.device)),
                   'smmd_kernel_matrix_fwd')
        ctx.save_for_backward(A, B)
        ctx.spec = spec
        return out

    @staticmethod
    def backward(ctx, G):
        A, B = ctx.saved_tensors
        G = G.contiguous()
        gA = torch.empty_like(A) if ctx.needs_input_grad[0] else None
        gB = torch.empty_like(B) if ctx.needs_input_grad[1] else None
        _lib.check(_lib.lib().smmd_kernel_matrix_bwd(
            ctx.spec.desc(), _lib.ptr(A), A.shape[0], _lib.ptr(B), B.shape[0], A.shape[1],
            _lib.ptr(G), _lib.ptr(gA), _lib.ptr(gB), _lib.stream_handle(A.device)),
            'smmd_kernel_matrix_bwd')
        return gA, gB, None


def kernel_matrix(A, B, kernel='rbf', **kw):
    """K(A, B) [na, nb] materialised (differentiable)."""
    return _KernelMatrix.apply(A, B, _as_spec(kernel, **kw))


class KernelMatrices:
    """The value of ``mmd._<kind>_kernel(X, Y)``: behaves as the reference
    tuple ``(K_XX, K_XY, K_YY, const_diagonal)`` (mmd.py:82, :116, :188, :37,
    :52), materialising on first element access, while ``mmd2`` consumes it
    without materialising anything."""

    def __init__(self, spec: KernelSpec, X, Y):
        self.spec, self.X, self.Y = spec, X, Y
        self._mats = None

    def _materialise(self):
        if self._mats is None:
            X, Y = self.X, self.Y
            self._mats = (kernel_matrix(X, X, self.spec), kernel_matrix(X, Y, self.spec),
                          kernel_matrix(Y, Y, self.spec),
                          False if self.spec.const_diag is None else self.spec.const_diag)
        return self._mats

    def __len__(self):
        return 4

    def __iter__(self):
        return iter(self._materialise())

    def __getitem__(self, i):
        return self._materialise()[i]


def _make(name, X, Y, K_XY_only, **kw):
    spec = get_kernel_spec(name, **kw)
    if K_XY_only:
        return kernel_matrix(X, Y, spec)
    return KernelMatrices(spec, X, Y)


def _distance_kernel(X, Y, K_XY_only=False):
    return _make('distance', X, Y, K_XY_only)


def _tanh_distance_kernel(X, Y, K_XY_only=False):
    return _make('tanh_distance', X, Y, K_XY_only)


def _dot_kernel(X, Y, K_XY_only=False):
    return _make('dot', X, Y, K_XY_only)


def _rbf_kernel(X, Y, sigma=1., wt=1., K_XY_only=False):
    return _make('rbf', X, Y, K_XY_only, sigma=sigma, wt=wt)


def _mix_rbf_kernel(X, Y, sigmas=(2.0, 5.0, 10.0, 20.0, 40.0, 80.0), wts=None, K_XY_only=False):
    return _make('mix_rbf', X, Y, K_XY_only, sigmas=sigmas, wts=wts)


def _mix_rq_kernel(X, Y, alphas=(.1, 1., 10.), wts=None, K_XY_only=False, add_dot=.0):
    return _make('mix_rq', X, Y, K_XY_only, alphas=alphas, wts=wts, add_dot=add_dot)


def _mix_rq_dot_kernel(X, Y, alphas=(.1, 1., 10.), wts=None, K_XY_only=False):
    return _make('mix_rq_dot', X, Y, K_XY_only, alphas=alphas, wts=wts)


def _mix_rq_1dot_kernel(X, Y, alphas=(.1, 1., 10.), wts=None, K_XY_only=False):
    return _make('mix_rq_1dot', X, Y, K_XY_only, alphas=alphas, wts=wts)


def _mix_rq_10dot_kernel(X, Y, alphas=(.1, 1., 10.), wts=None, K_XY_only=False):
    return _make('mix_rq_10dot', X, Y, K_XY_only, alphas=alphas, wts=wts)


def _mix_rq_01dot_kernel(X, Y, alphas=(.1, 1., 10.), wts=None, K_XY_only=False):
    return _make('mix_rq_01dot', X, Y, K_XY_only, alphas=alphas, wts=wts)


def _mix_rq_001dot_kernel(X, Y, alphas=(.1, 1., 10.), wts=None, K_XY_only=False):
    return _make('mix_rq_001dot', X, Y, K_XY_only, alphas=alphas, wts=wts)


def _tanh_mix_rq_kernel(X, Y, K_XY_only=False):
    return _make('tanh_mix_rq', X, Y, K_XY_only)


def get_kernel(name):
    """getattr(mmd, '_%s_kernel' % name) as the reference does (smmd.py:11)."""
    fn = globals().get('_%s_kernel' % name)
    if fn is None:
        raise ValueError('unknown kernel %r' % name)
    return fn


for _name in KERNEL_NAMES:              # lets spec_of map a kernel callable back
    globals()['_%s_kernel' % _name].kernel_name = _name


def spec_of(kernel):
    """KernelSpec of one of this module's ``_<kind>_kernel`` callables (with
    their default parameters), or None for any other callable."""
    name = getattr(kernel, 'kernel_name', None)
    return get_kernel_spec(name) if name is not None else None


# ---------------------------------------------------------------------------
# the batch a loss spans: in the all-gather data-parallel mode, mmd2 of a
# kernel value evaluated inside ``loss_group(group)`` is the estimator of the
# GLOBAL batch (every rank's rows), as model.set_tower_loss arranges around
# set_loss -- so a subclass's ``mmd.mmd2(kernel(G, images))`` needs no change
# ---------------------------------------------------------------------------
_scope = threading.local()


class loss_group:
    """``with loss_group(group, exchange):`` -- mmd2 inside spans ``group``'s
    global batch; ``exchange`` (collectives.StepExchange) carries its
    all-gather together with the step's other small messages."""

    def __init__(self, group, exchange=None):
        self.group = group if is_dp(group) else None
        self.exchange = exchange if self.group is not None else None

    def __enter__(self):
        self.prev = (getattr(_scope, 'group', None), getattr(_scope, 'exchange', None))
        _scope.group, _scope.exchange = self.group, self.exchange
        return self

    def __exit__(self, *a):
        _scope.group, _scope.exchange = self.prev
        return False


def current_loss_group():
    return getattr(_scope, 'group', None)


def current_exchange():
    return getattr(_scope, 'exchange', None)


# ---------------------------------------------------------------------------
# estimator
# ---------------------------------------------------------------------------
def mmd2(K, biased=False):
    """gan/core/mmd.py:194-196.  A KernelMatrices argument takes the fused
    path; an explicit 4-tuple of matrices is reduced as given."""
    if isinstance(K, KernelMatrices):
        p = current_pending()
        if p is not None and p.fuse and p.result is None and current_loss_group() is None:
            val = _mmd2_scaled(K, biased, p)
            if val is not None:
                return val
        val = _mmd2_scaled_gathered(K, biased, current_exchange())
        if val is not None:
            return val
        return mmd2_fused(K.X, K.Y, K.spec, biased, process_group=current_loss_group(),
                          exchange=current_exchange())
    K_XX, K_XY, K_YY, const_diagonal = K
    return _mmd2(K_XX, K_XY, K_YY, const_diagonal, biased)


def _mmd2(K_XX, K_XY, K_YY, const_diagonal=False, biased=False):
    """gan/core/mmd.py:199-220 on explicit matrices."""
    m = float(K_XX.shape[0])
    n = float(K_YY.shape[0])
    if biased:
        return (K_XX.sum() / (m * m) + K_YY.sum() / (n * n) - 2 * K_XY.sum() / (m * n))
    if const_diagonal is not False:
        trace_X = m * float(const_diagonal)
        trace_Y = n * float(const_diagonal)
    else:
        trace_X = torch.diagonal(K_XX).sum()
        trace_Y = torch.diagonal(K_YY).sum()
    return ((K_XX.sum() - trace_X) / (m * (m - 1)) + (K_YY.sum() - trace_Y) / (n * (n - 1))
            - 2 * K_XY.sum() / (m * n))


# ---------------------------------------------------------------------------
# witness function of the gradient penalty (gan/core/model.py:336-339)
# ---------------------------------------------------------------------------
class _WitnessGrad(torch.autograd.Function):
    """dH = d(sum_i witness_i)/dH with a HIP second-order backward."""

    @staticmethod
    def forward(ctx, H, R, F, spec):
        H, R, F = _features(H), _features(R), _features(F)
        dH = torch.empty_like(H)
        w = torch.empty(H.shape[0], device=H.device, dtype=torch.float32)
        _lib.check(_lib.lib().smmd_witness_fwd(
            spec.desc(), _lib.ptr(H), H.shape[0], _lib.ptr(R), R.shape[0], _lib.ptr(F),
            F.shape[0], H.shape[1], _lib.ptr(w), _lib.ptr(dH), _lib.stream_handle(H.device)),
            'smmd_witness_fwd')
        ctx.save_for_backward(H, R, F)
        ctx.spec = spec
        ctx.mark_non_differentiable(w)
        return dH, w

    @staticmethod
    def backward(ctx, gdH, gw):
        H, R, F = ctx.saved_tensors
        gdH = gdH.contiguous()
        gH, gR, gF = torch.empty_like(H), torch.empty_like(R), torch.empty_like(F)
        _lib.check(_lib.lib().smmd_witness_bwd(
            ctx.spec.desc(), _lib.ptr(H), H.shape[0], _lib.ptr(R), R.shape[0], _lib.ptr(F),
            F.shape[0], H.shape[1], _lib.ptr(gdH), _lib.ptr(gH), _lib.ptr(gR), _lib.ptr(gF),
            _lib.stream_handle(H.device)), 'smmd_witness_bwd')
        return gH, gR, gF, None


def witness_and_grad(H, R, F, kernel='rbf', **kw):
    """(d sum_i w_i / dH, w) with w_i = mean_j K(H_i,R_j) - mean_j K(H_i,F_j)."""
    dH, w = _WitnessGrad.apply(H, R, F, _as_spec(kernel, **kw))
    return dH, w


# ---------------------------------------------------------------------------
# Polynomial-kernel MMD statistics: the KID scorer and the 3-sample test of
# the learning-rate scheduler (gan/core/mmd.py:296-539 numpy/TF versions,
# gan/compute_scores.py:232-335).  K = (gamma <a, b> + coef0)^degree is
# evaluated tile by tile on the f32 matrix cores (smmd_poly_kernel_sums) and
# never materialised; the estimators run in double on the device.
# ---------------------------------------------------------------------------
class PolySums:
    """Row sums, column sums, diagonal and {sum K, sum K^2, sum diag,
    sum diag^2} of one polynomial kernel matrix (device float64 tensors)."""

    __slots__ = ('rows', 'cols', 'diag', 'stats', 'shape')

    def __init__(self, rows, cols, diag, stats, shape):
        self.rows, self.cols, self.diag, self.stats, self.shape = rows, cols, diag, stats, shape

    def c_struct(self):
        return _lib.PolySums(self.rows.data_ptr(), self.cols.data_ptr(), self.diag.data_ptr(),
                             self.stats.data_ptr())


def _codes(x, device=None):
    if not torch.is_tensor(x):
        x = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
    dev = device or (x.device if x.is_cuda else torch.device('cuda', torch.cuda.current_device()))
    return x.to(device=dev, dtype=torch.float32).contiguous()


def polynomial_kernel_sums(A, B, degree=3, gamma=None, coef0=1):
    """Sums of K = (gamma A B^T + coef0)^degree (sklearn polynomial_kernel;
    gamma None -> 1 / dim) without forming K."""
    A = _codes(A)
    B = _codes(B, A.device)
    _lib.require_cuda(A, B)
    na, dim = A.shape
    nb = B.shape[0]
    if B.shape[1] != dim:
        raise ValueError('feature widths differ: %d vs %d' % (dim, B.shape[1]))
    g = 1.0 / dim if gamma is None else float(gamma)
    dev = A.device
    rows = torch.empty(na, device=dev, dtype=torch.float64)
    cols = torch.empty(nb, device=dev, dtype=torch.float64)
    diag = torch.zeros(min(na, nb), device=dev, dtype=torch.float64)
    stats = torch.empty(4, device=dev, dtype=torch.float64)
    L = _lib.lib()
    nbytes = L.smmd_poly_sums_workspace_bytes(na, nb, dim)
    ws = _lib.workspace('poly', nbytes, dev)
    with _lib.timed('smmd_poly_kernel_sums'):
        _lib.check(L.smmd_poly_kernel_sums(_lib.ptr(A), na, _lib.ptr(B), nb, dim, g, float(coef0),
                                           int(degree), _lib.ptr(rows), _lib.ptr(cols),
                                           _lib.ptr(diag), _lib.ptr(stats), _lib.ptr(ws),
                                           ws.numel(), _lib.stream_handle(dev)),
                   'smmd_poly_kernel_sums')
    return PolySums(rows, cols, diag, stats, (na, nb))


_ESTIMATORS = {'unbiased': 0, 'biased': 1, 'u-statistic': 2}


def poly_mmd2_and_variance(xx, yy, xy, var_at_m=None, mmd_est='unbiased'):
    """mmd2 and var_est of gan/compute_scores.py:246-335 from three PolySums
    records (device double tensor [2])."""
    m = xx.shape[0]
    if not (xx.shape == yy.shape == xy.shape == (m, m)):
        raise ValueError('KID statistics need equal sample sizes')
    out = torch.empty(2, device=xx.rows.device, dtype=torch.float64)
    _lib.check(_lib.lib().smmd_poly_mmd2_var(
        xx.c_struct(), yy.c_struct(), xy.c_struct(), m,
        float(var_at_m) if var_at_m is not None else -1.0, _ESTIMATORS[mmd_est],
        _lib.ptr(out), _lib.stream_handle(xx.rows.device)), 'smmd_poly_mmd2_var')
    return out


class YRelatedSums(tuple):
    """(K_XY sums, K_YY sums) of gan/core/mmd.py:436 -- the record the
    3-sample scheduler keeps for an earlier sample Z."""


def np_diff_polynomial_mmd2_and_ratio_with_saving(X, Y, saved_sums_for_Z):
    """gan/core/mmd.py:429-441: K = (<.,.>/dim + 1)^3.  Returns the Y-related
    sums when saved_sums_for_Z is None, else (mmd2(X,Y) - mmd2(X,Z), the test
    statistic, Y-related sums)."""
    X = _codes(X)
    Y = _codes(Y, X.device)
    xy = polynomial_kernel_sums(X, Y)
    yy = polynomial_kernel_sums(Y, Y)
    mine = YRelatedSums((xy, yy))
    if saved_sums_for_Z is None:
        return mine
    xz, zz = saved_sums_for_Z
    m = yy.shape[0]
    out = torch.empty(2, device=X.device, dtype=torch.float64)
    _lib.check(_lib.lib().smmd_poly_diff_ratio(yy.c_struct(), xy.c_struct(), zz.c_struct(),
                                               xz.c_struct(), m, _lib.ptr(out),
                                               _lib.stream_handle(X.device)),
               'smmd_poly_diff_ratio')
    diff, ratio = out.tolist()
    return diff, ratio, mine
