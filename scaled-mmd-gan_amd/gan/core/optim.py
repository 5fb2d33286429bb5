"""Flat-buffer TF-semantics Adam with per-tensor clip_by_norm (libsmmd_hip).

Replaces the per-variable ``tf.clip_by_norm(g, 1.)`` of MMD_GAN.compute_grads
(gan/core/model.py:444-456) and ``tf.train.AdamOptimizer`` (model.py:405-412,
:458-468).  Every parameter of a network is re-pointed into ONE contiguous
fp32 buffer, and so is its gradient, so

* the data-parallel gradient exchange is a single RCCL all_reduce over
  ``flat_grad`` (one bucket of ~40 MB for the SNResNet critic), and
* clip + Adam for all tensors is one ``smmd_adam_flat`` launch set.

With a spectral-norm bank attached (``attach_sn``) the step is
``smmd_adam_flat_sn``: the SN weights are updated tile by tile together with
the first pass of the bank's next power iteration, which the next
``refresh`` then skips (one read of every SN weight less per step).
"""
from __future__ import annotations

import ctypes
import math
import struct
import os

import torch

from . import _lib


# Step count per parameter storage, bumped by every FlatAdam step: the update
# writes the parameters through the library, which does not advance torch's
# version counters, so caches of tensors derived from parameters
# (architecture.prefolded, _Up) key on param_epoch(w) as well.
_EPOCH = {}


def param_epoch(t):
    """FlatAdam steps applied so far to the storage `t` lives in (0 if none)."""
    return _EPOCH.get(t.untyped_storage().data_ptr(), 0)


def _f32(x):
    """x rounded to float32 (as a ctypes c_float argument is), as a Python float."""
    return struct.unpack('f', struct.pack('f', float(x)))[0]


class FlatAdam:
    def __init__(self, params, lr, beta1=0.5, beta2=0.9, eps=1e-8, clip_norm=1.0, name='opt'):
        self.name = name
        self.params = [p for p in params]
        if not self.params:
            raise ValueError('no parameters')
        dev = self.params[0].device
        _lib.require_cuda(*self.params)
        self.lr, self.beta1, self.beta2, self.eps = lr, beta1, beta2, eps
        self.clip_norm = clip_norm if clip_norm else 0.0
        sizes = [p.numel() for p in self.params]
        offs = [0]
        for s in sizes:     # tensor i owns [offs[i], offs[i+1]): size padded to 4 floats
            offs.append(offs[-1] + (s + 3) // 4 * 4)
        self.numel = offs[-1]
        self.param_numel = sum(sizes)
        self.offsets = (ctypes.c_int64 * len(offs))(*offs)
        self.flat_param = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        self.flat_grad = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        self.m = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        self.v = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        with torch.no_grad():
            for p, o, s in zip(self.params, offs, sizes):
                # keep each parameter's memory format (e.g. channels_last convs)
                view = self._view(self.flat_param, p, o)
                view.copy_(p)
                p.data = view
                p.grad = self._view(self.flat_grad, p, o)
        self.step_count = 0
        self._sn = None
        # gather mode (set per step by MMD_GAN in one process): zero_grad
        # drops the .grad views (an SN bank's weights and scales excepted),
        # autograd's accumulation nodes then keep each parameter's gradient
        # tensor as it is produced (no add kernel into a zeroed view per
        # parameter), and step() copies them into flat_grad with one
        # multi-tensor copy
        self.gather = False
        # graph mode (model.StepGraphs): the update reads its bias-corrected
        # step size from this device scalar, written before every replay
        self.graph_mode = False
        self.lr_t_dev = torch.zeros(1, device=dev, dtype=torch.float32)
        nbytes = _lib.lib().smmd_opt_workspace_bytes(self.offsets, len(self.params))
        self.ws = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=dev)

    @staticmethod
    def _view(flat, p, o):
        if p.is_contiguous():
            return flat[o:o + p.numel()].view_as(p)
        return torch.as_strided(flat, p.shape, p.stride(), o)

    def _gathering(self):
        return self.gather and not self.graph_mode

    def zero_grad(self, set_to_none=False):
        if self._gathering() and self._sn is None:
            for p in self.params:
                p.grad = None
            return
        self.flat_grad.zero_()
        if self._sn is not None:
            self._sn[0]._gd_pending = None
        # re-attach views in case autograd replaced a .grad tensor
        for i, p in enumerate(self.params):
            o, n = self.offsets[i], p.numel()
            if n and (p.grad is None or p.grad.data_ptr() != self.flat_grad[o:o + n].data_ptr()):
                p.grad = self._view(self.flat_grad, p, o)
        if self._gathering():
            # an SN bank's weights and scales keep their views (the G-direct
            # backward writes dL/ds into them, and no AccumulateGrad touches
            # the weights); the others gather (flat_grad already zero)
            keep = {id(t) for e in self._sn[0].entries for t in (e.weight, e.scale)
                    if t is not None}
            for p in self.params:
                if id(p) not in keep:
                    p.grad = None

    def _gather_grads(self, lo=0, hi=None):
        """Gather mode: every parameter's gradient (of tensors lo .. hi - 1:
        one all-reduce bucket, collectives.GradBuckets) into flat_grad (one
        _foreach_copy_; parameters without one get zeros) and the .grad views
        re-attached."""
        dst, src, empty = [], [], []
        hi = len(self.params) if hi is None else hi
        for i in range(lo, hi):
            p = self.params[i]
            if not p.numel():
                continue
            view = self._view(self.flat_grad, p, self.offsets[i])
            g = p.grad
            if g is None:
                empty.append(view)
            elif g.data_ptr() != view.data_ptr():
                dst.append(view)
                src.append(g)
            p.grad = view
        with torch.no_grad():
            if dst:
                torch._foreach_copy_(dst, src)
            if empty and self._sn is None:   # (with a bank zero_grad zeroed them)
                torch._foreach_zero_(empty)

    def _check_grads(self):
        if self._gathering():
            self._gather_grads()
        for i, p in enumerate(self.params):
            o, n = self.offsets[i], p.numel()
            if n and (p.grad is None or p.grad.data_ptr() != self.flat_grad[o:o + n].data_ptr()):
                raise RuntimeError('a parameter gradient was re-allocated outside flat_grad; '
                                   'call zero_grad() before backward()')

    def clip_(self, clip_norm=None):
        """Per-tensor clip_by_norm in place (the per-tower clip)."""
        c = self.clip_norm if clip_norm is None else clip_norm
        _lib.check(_lib.lib().smmd_clip_by_norm_flat(
            _lib.ptr(self.flat_grad), self.offsets, len(self.params), float(c),
            _lib.ptr(self.ws), self.ws.numel(), _lib.stream_handle(self.flat_grad.device)),
            'smmd_clip_by_norm_flat')

    def clip_range_(self, lo, hi, clip_norm=None):
        """clip_by_norm of tensors [lo, hi) in place (one gradient bucket)."""
        c = self.clip_norm if clip_norm is None else clip_norm
        sub = ctypes.cast(ctypes.byref(self.offsets, 8 * lo), ctypes.POINTER(ctypes.c_int64))
        _lib.check(_lib.lib().smmd_clip_by_norm_flat(
            _lib.ptr(self.flat_grad), sub, hi - lo, float(c), _lib.ptr(self.ws), self.ws.numel(),
            _lib.stream_handle(self.flat_grad.device)), 'smmd_clip_by_norm_flat')

    def attach_sn(self, bank):
        """Fuse the first power-iteration pass of ``bank`` (a
        SpectralNormBank whose weights are parameters of this optimizer) into
        ``step``.  Returns False, leaving the plain update, when the fused
        call does not apply (env SMMD_SN_FUSE_P1=0, no SN layers, too many
        tensors, a weight outside this optimizer)."""
        self._sn = None
        if os.environ.get('SMMD_SN_FUSE_P1', '1') == '0' or bank is None or not bank.entries:
            return False
        if len(self.params) > _lib.OPT_MAX_FUSED or len(bank.entries) > _lib.SN_MAX_FUSED:
            return False
        index = {id(p): i for i, p in enumerate(self.params)}
        idx = [index.get(id(e.weight)) for e in bank.entries]
        if any(i is None for i in idx):
            return False
        self._sn = (bank, (ctypes.c_int32 * len(idx))(*idx))
        return True

    def _sn_layers(self):
        bank, idx = self._sn
        base = self.flat_param.data_ptr()
        arr = (_lib.SnLayer * len(bank.entries))()
        pend = bank._gd_pending
        for k, e in enumerate(bank.entries):
            W = e.weight
            if W.data_ptr() != base + 4 * self.offsets[idx[k]]:
                return None         # re-pointed since attach_sn: plain update
            arr[k].W = W.data_ptr()
            arr[k].u = e.u.data_ptr()
            arr[k].N, arr[k].K = e.N, e.K
            if pend is not None:    # the G-direct update: G of the backward
                arr[k].G = pend[0][k].data_ptr()
                arr[k].fold = 1 if pend[1][k] else 0
                arr[k].v = e.v.data_ptr()
        return arr

    def dense_grad(self):
        """The flat gradient with every SN weight's dL/dW formed (a copy): under
        the G-direct update those ranges of ``flat_grad`` are never written
        (smmd_sn_weight_bwd from the kept G, for inspection and tests)."""
        if self._gathering():
            self._gather_grads()
        g = self.flat_grad.clone()
        if self._sn is None or self._sn[0]._gd_pending is None:
            return g
        bank, idx = self._sn
        G, folds = bank._gd_pending
        n = len(bank.entries)
        arr = (_lib.SnLayer * n)()
        gs = torch.empty(n, device=g.device, dtype=torch.float32)
        for k, e in enumerate(bank.entries):
            L = arr[k]
            L.W = e.weight.data_ptr()
            L.u = e.u.data_ptr()
            L.v = e.v.data_ptr()
            L.sigma = e.sigma.data_ptr()
            s = e.scale
            L.s = s.data_ptr() if s is not None and s.numel() > 0 else None
            L.G = G[k].data_ptr()
            L.gW = g.data_ptr() + 4 * self.offsets[idx[k]]
            L.gs = gs[k:k + 1].data_ptr()
            L.N, L.K = e.N, e.K
            L.fold = 1 if folds[k] else 0
        _lib.check(_lib.lib().smmd_sn_weight_bwd(arr, n, _lib.ptr(bank.ws), bank.ws.numel(),
                                                  _lib.stream_handle(g.device)),
                   'smmd_sn_weight_bwd')
        return g

    def lr_t(self, step=None, lr=None):
        """tf.train.AdamOptimizer's lr_t = lr sqrt(1 - b2^t) / (1 - b1^t) in
        double, as smmd_adam_flat computes it (model.py:405-412)."""
        t = self.step_count if step is None else step
        lr = self.lr if lr is None else lr
        # lr and the betas as the float32 values the library receives (its
        # adam_lr_t widens those to double): a graph replay's device lr_t is
        # then the eager update's bit for bit
        lr, b1, b2 = _f32(lr), _f32(self.beta1), _f32(self.beta2)
        return lr * math.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)

    def advance(self):
        """Host bookkeeping of one update (step count, parameter epoch); a
        graph replay of the update calls it instead of ``step``."""
        self.step_count += 1
        key = self.flat_param.untyped_storage().data_ptr()
        _EPOCH[key] = _EPOCH.get(key, 0) + 1

    def step(self, grad_scale=1.0, clip=True, lr=None):
        self._check_grads()
        self.advance()
        if self.graph_mode:
            self._step_dev(grad_scale, clip)
            return
        c = float(self.clip_norm) if clip else 0.0
        args = (_lib.ptr(self.flat_param), _lib.ptr(self.flat_grad), _lib.ptr(self.m),
                _lib.ptr(self.v), self.offsets, len(self.params), float(grad_scale), c,
                float(self.lr if lr is None else lr), float(self.beta1), float(self.beta2),
                float(self.eps), self.step_count, _lib.ptr(self.ws), self.ws.numel())
        stream = _lib.stream_handle(self.flat_grad.device)
        layers = self._sn_layers() if self._sn is not None else None
        if layers is not None:
            bank, idx = self._sn
            gd = bank._gd_pending is not None
            with _lib.timed('smmd_adam_flat_sn[%s]' % self.name):
                st = _lib.lib().smmd_adam_flat_sn2(
                    *args[:13], None, *args[13:], layers, idx, len(bank.entries),
                    _lib.ptr(bank.ws), bank.ws.numel(), _lib.ADAM_SN_GDIRECT if gd else 0, stream)
            _lib.check(st, 'smmd_adam_flat_sn2')
            bank._gd_pending = None
            bank.mark_p1_ready()
            return
        with _lib.timed('smmd_adam_flat[%s]' % self.name):
            st = _lib.lib().smmd_adam_flat(*args, stream)
        _lib.check(st, 'smmd_adam_flat')

    def _step_dev(self, grad_scale, clip):
        """The update with lr_t from ``lr_t_dev`` (smmd_adam_flat_ex): what a
        captured step graph replays.  Outside a capture the scalar is written
        here; during one the replaying code writes it before each replay."""
        if not torch.cuda.is_current_stream_capturing():
            self.lr_t_dev.fill_(self.lr_t())
        c = float(self.clip_norm) if clip else 0.0
        stream = _lib.stream_handle(self.flat_grad.device)
        layers = self._sn_layers() if self._sn is not None else None
        if layers is not None:
            bank, idx = self._sn
            gd = bank._gd_pending is not None
            st = _lib.lib().smmd_adam_flat_sn2(
                _lib.ptr(self.flat_param), _lib.ptr(self.flat_grad), _lib.ptr(self.m),
                _lib.ptr(self.v), self.offsets, len(self.params), float(grad_scale), c, 0.0,
                float(self.beta1), float(self.beta2), float(self.eps), 0,
                _lib.ptr(self.lr_t_dev), _lib.ptr(self.ws), self.ws.numel(), layers, idx,
                len(bank.entries), _lib.ptr(bank.ws), bank.ws.numel(),
                _lib.ADAM_SN_GDIRECT if gd else 0, stream)
            _lib.check(st, 'smmd_adam_flat_sn2')
            bank._gd_pending = None
            bank.mark_p1_ready()
            return
        st = _lib.lib().smmd_adam_flat_ex(
            _lib.ptr(self.flat_param), _lib.ptr(self.flat_grad), _lib.ptr(self.m),
            _lib.ptr(self.v), self.offsets, len(self.params), float(grad_scale), c,
            _lib.ptr(self.lr_t_dev), float(self.beta1), float(self.beta2), float(self.eps),
            _lib.ptr(self.ws), self.ws.numel(), None, None, 0, None, 0, stream)
        _lib.check(st, 'smmd_adam_flat_ex')

    def state_dict(self):
        return {'m': self.m.clone(), 'v': self.v.clone(), 'step': self.step_count,
                'lr': self.lr}

    def load_state_dict(self, sd):
        self.m.copy_(sd['m'])
        self.v.copy_(sd['v'])
        self.step_count = int(sd['step'])
        self.lr = float(sd['lr'])
