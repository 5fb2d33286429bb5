"""Spectral normalisation on the MI355X hot path.

Drop-in for gan/core/sn.py (``spectral_normed_weight``, ``NO_OPS``) plus the
batched form the networks use: :class:`SpectralNormBank` runs the power
iteration, sigma and ``W_eff = s * W / sigma`` for EVERY SN layer of a network
in one set of HIP launches (``smmd_sn_power_iter``) and the matching backward
in another (``smmd_sn_weight_bwd``).

Layout note: weights are kept as PyTorch stores them, flattened to
[N = out channels, K].  The reference reshapes its [kh, kw, Cin, Cout] weight
to [kh*kw*Cin, Cout] (sn.py:18-19); that is the transpose of ours up to a
permutation of K, which leaves sigma and u unchanged (v is permuted).
"""
from __future__ import annotations

import os
import warnings

import torch

from . import _lib

NO_OPS = 'NO_OPS'         # gan/core/sn.py:9
SN_EPS = 1e-12            # gan/core/sn.py:12
# SMMD_SN_FOLD=0: ConvMeanPool SN layers get W_eff and a separate fold launch
SN_FOLD = os.environ.get('SMMD_SN_FOLD', '1') != '0'


def _folds(e, W):
    """This call writes the layer's pool-folded filter (smmd_sn_layer.fold)."""
    return (e.fold and W.dim() == 4 and tuple(W.shape[2:]) == (3, 3) and W.is_contiguous()
            and W.data_ptr() % 16 == 0)


def truncated_normal_(t, std=1.0):
    """tf.truncated_normal_initializer: normal re-drawn outside 2 std."""
    with torch.no_grad():
        torch.nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2 * std, b=2 * std)
    return t


def _launch_refresh(bank, update_u, flags, Ws, ss):
    """The refresh launch set (smmd_sn_power_iter_ex): every layer's W_eff or
    pool-folded W'.  Returns (outs, folds)."""
    n = len(bank.entries)
    outs = []
    arr = (_lib.SnLayer * n)()
    # lazy in a captured step too: the filter transforms that stand in for
    # P3's writes are captured kernels reading W, sigma and s at replay time
    lazy = bank.lazy if (bank.lazy and os.environ.get('SMMD_SN_LAZY_GRAPH', '1') != '0') else ()
    for i, (e, W, s) in enumerate(zip(bank.entries, Ws, ss)):
        # each output channel's K values must be contiguous: true for the
        # default and the channels_last layouts (SN is invariant to the
        # order of K, see the module docstring)
        if _memfmt(W) is None:
            raise ValueError('SN weight %d is neither contiguous nor channels_last' % i)
        fold = _folds(e, W)
        W_eff = (torch.empty(W.shape[0], W.shape[1], 4, 4, device=W.device,
                             dtype=torch.float32) if fold else torch.empty_like(W))
        outs.append(W_eff)
        L = arr[i]
        L.fold = 1 if fold else 0
        L.W = W.data_ptr()
        # every refresh rewrites the entry's sigma (and u): a lazy W_eff of an
        # earlier refresh can no longer be formed (convops._lazy raises)
        e.refresh_gen = getattr(e, 'refresh_gen', 0) + 1
        if i in lazy and bool(fold) == bool(e.fold) and W.is_contiguous():
            # consumed only through the Winograd filter transforms, which form
            # it from W, sigma and s (convops.register_lazy): P3 skips it.
            # Only an OIHW-contiguous W: the _filter_sn kernels read it as
            # OIHW, and a channels_last W_eff placeholder copied by a
            # .contiguous() would escape the registry unwritten
            from .convops import register_lazy
            register_lazy(W_eff, e, fold)
            L.W_eff = None
        else:
            L.W_eff = W_eff.data_ptr()
        L.u = e.u.data_ptr()
        L.v = e.v.data_ptr()
        L.sigma = e.sigma.data_ptr()
        L.s = s.data_ptr() if s is not None and s.numel() > 0 else None
        L.N, L.K = e.N, e.K
    dev = Ws[0].device
    lib = _lib.lib()
    args = (arr, n, bank.num_iters, SN_EPS, 1 if update_u else 0, flags, _lib.ptr(bank.ws),
            bank.ws.numel(), _lib.stream_handle(dev))
    with _lib.timed('smmd_sn_power_iter'):
        st = lib.smmd_sn_power_iter_ex(*args)
    _lib.check(st, 'smmd_sn_power_iter_ex')
    return outs, [bool(a.fold) for a in arr]


def _gdirect_scales_ok(bank, ss, needs):
    """G-direct writes dL/ds straight into each learnable scale's gradient,
    which must therefore exist (a view of the optimizer's flat buffer, zeroed
    before the step: the kernel OVERWRITES it, it does not accumulate).  A
    scale that needs a gradient but has no `.grad` takes the dense backward."""
    for e, s, need in zip(bank.entries, ss, needs):
        if need and s is not None and s.numel() > 0 and e.scale.grad is None:
            return False
    return True


class _SNBatch(torch.autograd.Function):
    @staticmethod
    def forward(ctx, bank, update_u, flags, *tensors):
        n = len(bank.entries)
        Ws, ss = tensors[:n], tensors[n:]
        outs, folds = _launch_refresh(bank, update_u, flags, Ws, ss)
        ctx.bank = bank
        ctx.folds = folds
        ctx.save_for_backward(*Ws, *ss)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        from . import convops
        convops.flush_late_wgrad_sums()     # the conv nodes' queued G contributions
        convops.check_late_delivery(getattr(ctx, '_smmd_out_ids', ()), grads)
        bank = ctx.bank
        n = len(bank.entries)
        saved = ctx.saved_tensors
        Ws, ss = saved[:n], saved[n:]
        if bank._gd_armed and _gdirect_scales_ok(bank, ss, ctx.needs_input_grad[3 + n:]):
            return _SNBatch._backward_gdirect(ctx, bank, Ws, ss, grads)
        arr = (_lib.SnLayer * n)()
        gWs, gss, keep = [], [], []
        for i, (e, W, s, G) in enumerate(zip(bank.entries, Ws, ss, grads)):
            fold = ctx.folds[i]
            if G is None:
                G = (torch.zeros(W.shape[0], W.shape[1], 4, 4, device=W.device,
                                 dtype=torch.float32) if fold else torch.zeros_like(W))
            G = G.contiguous() if fold else G.contiguous(memory_format=_memfmt(W))
            keep.append(G)
            gW = torch.empty_like(W)
            gs = torch.empty(1, device=W.device, dtype=torch.float32)
            gWs.append(gW)
            gss.append(gs if (s is not None and s.numel() > 0) else None)
            L = arr[i]
            L.W = W.data_ptr()
            L.u = e.u.data_ptr()
            L.v = e.v.data_ptr()
            L.sigma = e.sigma.data_ptr()
            L.s = s.data_ptr() if s is not None and s.numel() > 0 else None
            L.G = G.data_ptr()
            L.gW = gW.data_ptr()
            L.gs = gs.data_ptr()
            L.N, L.K = e.N, e.K
            L.fold = 1 if fold else 0
        args = (arr, n, _lib.ptr(bank.ws), bank.ws.numel(), _lib.stream_handle(Ws[0].device))
        with _lib.timed('smmd_sn_weight_bwd'):
            st = _lib.lib().smmd_sn_weight_bwd(*args)
        _lib.check(st, 'smmd_sn_weight_bwd')
        gs_out = []
        for s, gs in zip(ss, gss):
            if gs is None:
                gs_out.append(None)
            else:
                gs_out.append(gs.view_as(s))
        return (None, None, None, *gWs, *gs_out)


    @staticmethod
    def _backward_gdirect(ctx, bank, Ws, ss, grads):
        """The G-direct backward (one process, the critic's update next):
        dL/dW is not formed.  smmd_sn_grad_stats reduces what the fused
        update needs from G and writes dL/ds straight into the scale's
        gradient (a view of the optimizer's flat buffer); G is kept on the
        bank for FlatAdam.step (smmd_adam_flat_sn2, SMMD_ADAM_SN_GDIRECT).
        No gradient is returned for W or s, so autograd runs no accumulation
        for them."""
        n = len(bank.entries)
        arr = (_lib.SnLayer * n)()
        keep = []
        for i, (e, W, s, G) in enumerate(zip(bank.entries, Ws, ss, grads)):
            fold = ctx.folds[i]
            if G is None:
                G = (torch.zeros(W.shape[0], W.shape[1], 4, 4, device=W.device,
                                 dtype=torch.float32) if fold else torch.zeros_like(W))
            G = G.contiguous() if fold else G.contiguous(memory_format=_memfmt(W))
            keep.append(G)
            L = arr[i]
            L.W = W.data_ptr()
            L.u = e.u.data_ptr()
            L.v = e.v.data_ptr()
            L.sigma = e.sigma.data_ptr()
            has_s = s is not None and s.numel() > 0
            L.s = s.data_ptr() if has_s else None
            sg = e.scale.grad if has_s else None
            L.gs = sg.data_ptr() if sg is not None else None
            L.G = G.data_ptr()
            L.N, L.K = e.N, e.K
            L.fold = 1 if fold else 0
        args = (arr, n, _lib.ptr(bank.ws), bank.ws.numel(), _lib.stream_handle(Ws[0].device))
        with _lib.timed('smmd_sn_grad_stats'):
            st = _lib.lib().smmd_sn_grad_stats(*args)
        _lib.check(st, 'smmd_sn_grad_stats')
        bank._gd_pending = (keep, [bool(f) for f in ctx.folds])
        return (None, None, None) + (None,) * (2 * n)


class _SNGroup(torch.autograd.Function):
    """One gradient bucket's SN layers as their own autograd node (data
    parallel runs, ``SpectralNormBank.set_groups``): the refresh ran once for
    all layers (the outputs are the bank's), but each group's backward fires
    as soon as ITS layers' W_eff gradients are complete, so its bucket's
    all-reduce is issued while the rest of the backward runs."""

    @staticmethod
    def forward(ctx, bank, members, *tensors):
        k = len(members)
        ctx.bank, ctx.members = bank, members
        ctx.save_for_backward(*tensors)
        return tuple(bank._fresh[i] for i in members) if k > 1 else bank._fresh[members[0]]

    @staticmethod
    def backward(ctx, *grads):
        from . import convops
        convops.flush_late_wgrad_sums()     # the conv nodes' queued G contributions
        convops.check_late_delivery(getattr(ctx, '_smmd_out_ids', ()), grads)
        bank, members = ctx.bank, ctx.members
        k = len(members)
        saved = ctx.saved_tensors
        res = bank._group_backward(members, saved[:k], saved[k:], grads)
        return (None, None) + res


def _memfmt(W):
    if W.is_contiguous():
        return torch.contiguous_format
    if W.dim() == 4 and W.is_contiguous(memory_format=torch.channels_last):
        return torch.channels_last
    return None


class SNEntry:
    """State of one SN layer: u [N] (truncated normal, sn.py:20-21), v [K],
    sigma [1]; the weight and scale parameters live in the layer module."""

    def __init__(self, module, weight_name='weight', scale_name='sn_scale'):
        self.module = module
        self.weight_name = weight_name
        self.scale_name = scale_name
        W = getattr(module, weight_name)
        self.N = W.shape[0]
        self.K = W[0].numel()
        dev = W.device
        self.u = truncated_normal_(torch.empty(self.N, device=dev, dtype=torch.float32))
        self.v = torch.zeros(self.K, device=dev, dtype=torch.float32)
        self.sigma = torch.ones(1, device=dev, dtype=torch.float32)
        # a ConvMeanPool conv: the bank writes its pool-folded filter
        self.fold = SN_FOLD and bool(getattr(module, 'sn_fold', False))

    @property
    def weight(self):
        return getattr(self.module, self.weight_name)

    @property
    def scale(self):
        return getattr(self.module, self.scale_name, None)

    def to(self, device):
        self.u = self.u.to(device)
        self.v = self.v.to(device)
        self.sigma = self.sigma.to(device)


class SpectralNormBank:
    """All SN layers of one network, normalised together once per step.

    ``refresh(update_u)`` computes W_eff for every layer (one HIP launch set)
    and stores it on each module as ``module.w_eff``; it is reused by every
    critic call of the step (real, fake, GP), which also removes the
    reference's u read/assign race."""

    def __init__(self, modules, num_iters=1):
        self._init_state([SNEntry(m) for m in modules], num_iters)

    def _init_state(self, entries, num_iters):
        self.entries = entries
        self.num_iters = num_iters
        self.ws = None
        self._p1_token = None
        # G-direct (one process): while armed, the SN backward leaves
        # (G tensors, folds) in _gd_pending for the optimizer's fused update
        self._gd_armed = False
        self._gd_pending = None
        # data parallel: the layers split into autograd groups (one per
        # gradient bucket, set_groups) and, while armed, their dL/dW and dL/ds
        # written straight into the optimizer's flat gradient (_direct)
        self.groups = None
        self._direct = None
        self._direct_armed = False
        # data parallel G-direct (either mode): while armed, a group's backward
        # writes G (the adjoint fold of G' for ConvMeanPool layers) into the
        # SN weights' .grad views instead of dL/dW, the buckets sum G over the
        # ranks, and dp_gdirect_finish runs the stats on the sum
        self._dpgd_armed = False
        # layers whose W_eff the refresh does not write (set_lazy)
        self.lazy = set()
        self._fresh = None
        self._folds = None
        self._alloc_ws()

    def _state_token(self):
        # storage and version of every W and u: an in-place write through
        # torch (copy_, load_state_dict, broadcast into the parameter) bumps a
        # version; the fused optimizer's own write does not
        return tuple((e.weight.data_ptr(), e.weight._version, e.u.data_ptr(), e.u._version)
                     for e in self.entries)

    def mark_p1_ready(self):
        """Called by FlatAdam right after smmd_adam_flat_sn wrote the first
        pass of the next power iteration into ``ws``."""
        self._p1_token = self._state_token()

    def invalidate(self):
        self._p1_token = None

    def _alloc_ws(self):
        if not self.entries:
            return
        arr = (_lib.SnLayer * len(self.entries))()
        for i, e in enumerate(self.entries):
            arr[i].N, arr[i].K = e.N, e.K
        nbytes = _lib.lib().smmd_sn_workspace_bytes(arr, len(self.entries))
        dev = self.entries[0].weight.device
        self.ws = torch.zeros(nbytes, dtype=torch.uint8, device=dev)

    def to(self, device):
        for e in self.entries:
            e.to(device)
        self._p1_token = None
        self._alloc_ws()

    def refresh(self, update_u=True):
        if not self.entries:
            return []
        Ws = [e.weight for e in self.entries]
        ss = [e.scale if e.scale is not None else torch.empty(0, device=Ws[0].device)
              for e in self.entries]
        _lib.require_cuda(*Ws)
        ready = self._p1_token is not None and self._p1_token == self._state_token()
        self._p1_token = None
        flags = _lib.SN_P1_READY if ready else 0
        if (self.groups is not None and torch.is_grad_enabled()
                and any(t.requires_grad for t in list(Ws) + list(ss))):
            with torch.no_grad():
                fresh, self._folds = _launch_refresh(self, bool(update_u), flags, Ws, ss)
            self._fresh = fresh
            outs = [None] * len(Ws)
            for members in self.groups:
                m = tuple(members)
                r = _SNGroup.apply(self, m, *[Ws[i] for i in m], *[ss[i] for i in m])
                r = r if isinstance(r, tuple) else (r,)
                if r[0].grad_fn is not None:     # the node's ctx (check_late_delivery)
                    r[0].grad_fn._smmd_out_ids = tuple(id(t) for t in r)
                for i, t in zip(m, r):
                    outs[i] = t
            self._fresh = None
        else:
            outs = _SNBatch.apply(self, bool(update_u), flags, *Ws, *ss)
            if outs and outs[0].grad_fn is not None:     # the node's ctx
                outs[0].grad_fn._smmd_out_ids = tuple(id(t) for t in outs)
        for e, w in zip(self.entries, outs):
            w._smmd_late_sum = True              # convops._late_gw: summed at the SN node
            if w.shape != e.weight.shape:        # the pool-folded 4 x 4 filter
                e.module.w_eff, e.module.w_fold = None, w
            else:
                e.module.w_eff, e.module.w_fold = w, None
        return list(outs)

    def set_groups(self, groups, direct=None):
        """Split the bank's autograd node into ``groups`` (lists of layer
        indices, in the order their gradients should be ready: the gradient
        buckets' order).  ``direct(members)``: called after a group's backward
        wrote its gradients into the parameters' .grad views (the armed
        direct mode), e.g. to issue the bucket's all-reduce."""
        groups = [list(g) for g in groups if len(g)] if groups else None
        if groups:
            covered = {i for g in groups for i in g}
            rest = [i for i in range(len(self.entries)) if i not in covered]
            if rest:
                groups.append(rest)
        self.groups = groups
        self._direct = direct

    def arm_direct(self, on=True):
        """Arm the direct-write group backward for the next backward pass."""
        self._direct_armed = bool(on) and self._direct is not None

    def set_lazy(self, indices):
        """Layers (bank indices) whose W_eff / W' the refresh leaves unwritten:
        their consumers are the Winograd convolutions, whose filter transforms
        read W, sigma and s directly (smmd_wino3x3_filter_sn,
        smmd_wino4x4s2(t)_filter_sn); any other reader materialises it
        (convops.materialize).  SMMD_SN_LAZY=0: none."""
        self.lazy = set(indices) if os.environ.get('SMMD_SN_LAZY', '1') != '0' else set()

    def arm_dp_gdirect(self, on=True, clip=0.0):
        """See below; clip > 0 (tower mode): each rank's dL/dW and dL/ds are
        clipped (model.py:449-455) before the sum, by scaling its G by the
        clip factor of the analytic norm (smmd_sn_grad_stats on the rank's G,
        then smmd_sn_clip_g)."""
        self._dpgd_clip = float(clip)
        self._arm_dp_gdirect(on)

    def _arm_dp_gdirect(self, on=True):
        """Arm the data-parallel G-direct backward (with arm_direct) for the
        next backward pass.  dL/dW = (s/sigma) G - (s <G, W> / sigma^2) u' v^T is
        linear in G given the replicated W, u', v, sigma and s, so the sum over
        ranks of dL/dW is that of the summed G: the buckets all-reduce G and
        the fused update forms dL/dW once (smmd_adam_flat_sn2)."""
        self._dpgd_armed = bool(on) and self._direct is not None

    def _layers(self, Gs, gss, folds):
        """The full SnLayer array (the workspace is carved by all layers) with
        G / gs only where given (None: the layer is skipped)."""
        n = len(self.entries)
        arr = (_lib.SnLayer * n)()
        for i, e in enumerate(self.entries):
            L = arr[i]
            L.W = e.weight.data_ptr()
            L.u = e.u.data_ptr()
            L.v = e.v.data_ptr()
            L.sigma = e.sigma.data_ptr()
            s = e.scale
            L.s = s.data_ptr() if s is not None and s.numel() > 0 else None
            L.G = Gs[i].data_ptr() if Gs[i] is not None else None
            L.gs = gss[i].data_ptr() if gss[i] is not None else None
            L.N, L.K = e.N, e.K
            L.fold = 1 if folds[i] else 0
        return arr

    def _scale_grad(self, e):
        s = e.scale
        return s.grad if (s is not None and s.numel() > 0 and s.requires_grad) else None

    def _group_write_g(self, members, Ws, ss, grads):
        """The data-parallel G-direct group backward: G into each SN weight's
        .grad view (fold layers: the adjoint fold of G', one launch for the
        group), the scale's .grad left zero (dp_gdirect_finish writes dL/ds
        from the summed G)."""
        folds_src, folds_dst = [], []
        for j, i in enumerate(members):
            e, W, G = self.entries[i], Ws[j], grads[j]
            gW = e.weight.grad
            if G is None:
                gW.zero_()
                continue
            if self._folds[i]:
                folds_src.append(G.contiguous())
                folds_dst.append(gW)
            else:
                gW.copy_(G.reshape(gW.shape))
        if folds_src:
            from .convops import _fold_launch_into
            _fold_launch_into(folds_src, folds_dst, adjoint=True)
        clip = getattr(self, '_dpgd_clip', 0.0)
        if clip > 0:
            # tower mode: this rank's clip_by_norm of dL/dW (and of dL/ds)
            # before the sum, through the analytic norm of its own G
            n = len(self.entries)
            Gs = [self.entries[i].weight.grad if i in members else None for i in range(n)]
            gss = [self._scale_grad(self.entries[i]) if i in members else None
                   for i in range(n)]
            arr = self._layers(Gs, gss, [False] * n)
            stream = _lib.stream_handle(Ws[0].device)
            with _lib.timed('smmd_sn_grad_stats'):
                st = _lib.lib().smmd_sn_grad_stats(arr, n, _lib.ptr(self.ws), self.ws.numel(),
                                                   stream)
            _lib.check(st, 'smmd_sn_grad_stats')
            st = _lib.lib().smmd_sn_clip_g(arr, n, float(clip), _lib.ptr(self.ws),
                                           self.ws.numel(), stream)
            _lib.check(st, 'smmd_sn_clip_g')
        self._direct(members)
        return (None,) * (2 * len(members))

    def dp_gdirect_finish(self, write_gs=True):
        """After the buckets' all-reduce: the stats of the summed G (in the SN
        weights' .grad views), then G pending for the fused update, which
        forms dL/dW (global mode: clips it with the analytic norm) and applies
        Adam.  write_gs: dL/ds from the summed G (global mode); tower mode
        keeps the all-reduced sum of the ranks' clipped dL/ds."""
        n = len(self.entries)
        Gs = [e.weight.grad for e in self.entries]
        gss = [self._scale_grad(e) if write_gs else None for e in self.entries]
        folds = [False] * n
        arr = self._layers(Gs, gss, folds)
        with _lib.timed('smmd_sn_grad_stats'):
            st = _lib.lib().smmd_sn_grad_stats(arr, n, _lib.ptr(self.ws), self.ws.numel(),
                                               _lib.stream_handle(Gs[0].device))
        _lib.check(st, 'smmd_sn_grad_stats')
        self._gd_pending = (Gs, folds)

    def _group_backward(self, members, Ws, ss, grads):
        """smmd_sn_weight_bwd for the group's layers (the full layer array with
        the others' G NULL: the workspace is carved by the whole array)."""
        if self._direct_armed and self._dpgd_armed:
            return self._group_write_g(members, Ws, ss, grads)
        n = len(self.entries)
        arr = (_lib.SnLayer * n)()
        direct = self._direct_armed
        outs_W, outs_s, keep = [], [], []
        for i, e in enumerate(self.entries):
            L = arr[i]
            L.N, L.K = e.N, e.K
            L.W = e.weight.data_ptr()
            L.u = e.u.data_ptr()
            L.v = e.v.data_ptr()
            L.sigma = e.sigma.data_ptr()
            L.fold = 1 if self._folds[i] else 0
        for j, i in enumerate(members):
            e, W, s, G = self.entries[i], Ws[j], ss[j], grads[j]
            fold = self._folds[i]
            if G is None:
                G = (torch.zeros(W.shape[0], W.shape[1], 4, 4, device=W.device,
                                 dtype=torch.float32) if fold else torch.zeros_like(W))
            G = G.contiguous() if fold else G.contiguous(memory_format=_memfmt(W))
            keep.append(G)
            has_s = s is not None and s.numel() > 0
            if direct:
                gW, gs = e.weight.grad, (e.scale.grad if has_s else None)
            else:
                gW = torch.empty_like(W)
                gs = torch.empty(1, device=W.device, dtype=torch.float32) if has_s else None
            outs_W.append(None if direct else gW)
            outs_s.append(None if (direct or gs is None) else gs.view_as(s))
            L = arr[i]
            L.W = W.data_ptr()
            L.s = s.data_ptr() if has_s else None
            L.G = G.data_ptr()
            L.gW = gW.data_ptr()
            L.gs = gs.data_ptr() if gs is not None else None
        args = (arr, n, _lib.ptr(self.ws), self.ws.numel(), _lib.stream_handle(Ws[0].device))
        with _lib.timed('smmd_sn_weight_bwd'):
            st = _lib.lib().smmd_sn_weight_bwd(*args)
        _lib.check(st, 'smmd_sn_weight_bwd')
        if direct:
            self._direct(members)
        return tuple(outs_W) + tuple(outs_s)

    def arm_gdirect(self, on=True):
        """Arm (or disarm) the G-direct backward for the next backward pass.
        Its dL/ds is WRITTEN (not accumulated) into each learnable scale's
        `.grad`, so the caller zeroes the gradients before the backward (the
        critic step does, right before it) and a scale without `.grad` makes
        that backward take the dense path (`_gdirect_scales_ok`)."""
        self._gd_armed = bool(on)
        if on:
            self._gd_pending = None

    def sigmas(self):
        return torch.cat([e.sigma for e in self.entries])

    def state_dict(self):
        return {'u': [e.u.clone() for e in self.entries]}

    def load_state_dict(self, sd):
        self._p1_token = None
        for e, u in zip(self.entries, sd['u']):
            e.u.copy_(u)


def spectral_normed_weight(W, u=None, num_iters=1, update_collection=None, with_sigma=False,
                           stop_grad=True):
    """gan/core/sn.py:16-59 for one weight in the REFERENCE layout
    (last dim = out).  ``u`` [1, N] is updated in place when
    ``update_collection is None`` (sn.py:39-46); any other value leaves it
    (NO_OPS semantics: the reference only queues the assign)."""
    if not stop_grad:
        raise NotImplementedError('stop_grad=False is not supported (the reference default '
                                  'and every caller use stop_grad=True, sn.py:16, :32-34)')
    N = W.shape[-1]
    if u is None:
        warnings.warn('spectral_normed_weight: no u given; a fresh truncated-normal u is used '
                      '(pass u to keep the power-iteration state)')
        u = truncated_normal_(torch.empty(1, N, device=W.device, dtype=torch.float32))
    Wt = W.reshape(-1, N).t().contiguous()          # [N, K]
    holder = torch.nn.Module()
    holder.weight = Wt
    bank = SpectralNormBank.__new__(SpectralNormBank)
    e = SNEntry.__new__(SNEntry)
    e.module, e.weight_name, e.scale_name = holder, 'weight', 'sn_scale'
    e.N, e.K, e.fold = N, Wt.shape[1], False
    e.u = u.reshape(N).detach().clone().contiguous()
    e.v = torch.zeros(e.K, device=W.device, dtype=torch.float32)
    e.sigma = torch.ones(1, device=W.device, dtype=torch.float32)
    bank._init_state([e], num_iters)
    W_eff_t, = _SNBatch.apply(bank, True, 0, Wt, torch.empty(0, device=W.device))
    if update_collection is None:
        with torch.no_grad():
            u.copy_(e.u.view_as(u))
    W_bar = W_eff_t.t().reshape(W.shape)
    if with_sigma:
        return W_bar, e.sigma[0]
    return W_bar
