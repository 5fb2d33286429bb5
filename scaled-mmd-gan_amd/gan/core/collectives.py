"""The collectives of the data-parallel path, one place.

On MI355X the group is RCCL (backend "nccl") over xGMI and every call works
on device tensors in place.  A gloo group (the CPU rehearsal of the N > 1
path, or several ranks sharing one GPU in tests) has no device all-gather,
so device tensors are staged through host copies there; the values are the
same either way.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def force_dp():
    """SMMD_DP_FORCE=1: a world-size-1 group takes the data-parallel path
    (packed all-gather, bucketed in-backward all-reduce, parameter broadcast)
    instead of the one-process shortcuts, so the RCCL device branches below
    run on a one-GPU box (tests/test_gpu_dist.py::test_rccl_world1_*)."""
    import os
    return os.environ.get('SMMD_DP_FORCE', '0') != '0'


def is_dp(group):
    """True when ``group`` takes the data-parallel path: more than one rank,
    or any initialised group under SMMD_DP_FORCE=1."""
    if group is None:
        return False
    return dist.get_world_size(group) > 1 or force_dp()


def _host_staged(t, group):
    return t.is_cuda and dist.get_backend(group) == 'gloo'


def gather_rows(t, group):
    """all_gather_into_tensor of ``t`` [r, ...] -> [world * r, ...], rank order."""
    world = dist.get_world_size(group)
    shape = (world * t.shape[0],) + tuple(t.shape[1:])
    if _host_staged(t, group):
        out = torch.empty(shape, dtype=t.dtype)
        dist.all_gather_into_tensor(out, t.cpu(), group=group)
        return out.to(t.device)
    out = torch.empty(shape, dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def all_reduce_(t, group):
    """In-place SUM over the group."""
    if _host_staged(t, group):
        h = t.detach().cpu()
        dist.all_reduce(h, group=group)
        with torch.no_grad():
            t.copy_(h)
        return t
    dist.all_reduce(t, group=group)
    return t


def broadcast_(t, src, group):
    """In-place broadcast of ``t`` from global rank ``src``."""
    if _host_staged(t, group):
        h = t.detach().cpu()
        dist.broadcast(h, src, group=group)
        with torch.no_grad():
            t.copy_(h)
        return t
    dist.broadcast(t, src, group=group)
    return t


def all_reduce_async(t, group):
    """SUM in place, returning the pending work (None when it completed
    synchronously: the host-staged gloo path)."""
    if _host_staged(t, group):
        all_reduce_(t, group)
        return None
    return dist.all_reduce(t, group=group, async_op=True)


# ---------------------------------------------------------------------------
# one latency-bound collective per loss evaluation (the all-gather mode)
# ---------------------------------------------------------------------------
class StepExchange:
    """The small messages of one loss evaluation in the all-gather ('global')
    mode packed into ONE ``all_gather_into_tensor``: each rank's critic
    feature rows [X; Y] (d floats per row) and, when the scaling regulariser
    is on, its partial statistics (J and nD summed over its rows, already
    divided by the global batch).  Afterwards every rank holds the global
    batch -- mmd2 then runs over all rows, needing no all-reduce of partial
    sums -- and the global J / nD as the fixed rank-order sum of the gathered
    partials (the same bits on every rank).  Without an exchange (a custom
    set_loss, the gaussian-noise variant) the ops fall back to their own
    all-reduces."""

    def __init__(self, group):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.jac = None           # the Jacobian columns computed ahead of set_loss
        self.feat = None
        self.stats = None         # local partials [2] (J, nD), set ahead of gather
        self.stats_total = None   # global [2] after gather
        self.used = False
        # the fused loss of this mode (mmd._mmd2_scaled_gathered): set by
        # MMD_GAN._prepare_exchange when apply_scaling is SMMD's own
        self.fuse = False
        self.sc = None
        self.variant = 0
        self.result = None        # (mmd2, g_loss, out) of the fused launch

    def gather_packed(self, X, Y):
        """The all-gather alone: (allp [world, (ml + nl) d (+ 2)], X_all,
        Y_all), allp's tail columns being every rank's stats (the fused loss
        sums them in its own launch, mmd._SMMDLossGathered)."""
        if self.used:
            raise RuntimeError('StepExchange.gather runs once per loss evaluation')
        self.used = True
        ml, nl, d = X.shape[0], Y.shape[0], X.shape[1]
        parts = [X.reshape(-1), Y.reshape(-1)]
        if self.stats is not None:
            parts.append(self.stats.reshape(-1).to(X.dtype))
        packed = torch.cat(parts).view(1, -1)
        allp = gather_rows(packed, self.group).view(self.world, -1)
        Xa = allp[:, :ml * d].reshape(self.world * ml, d)
        Ya = allp[:, ml * d:(ml + nl) * d].reshape(self.world * nl, d)
        return allp, Xa, Ya

    def gather(self, X, Y):
        """[X; Y; stats] of every rank -> (X_all, Y_all) in rank order."""
        ml, nl, d = X.shape[0], Y.shape[0], X.shape[1]
        allp, Xa, Ya = self.gather_packed(X, Y)
        if self.stats is not None:
            tot = allp[0, (ml + nl) * d:].clone()
            for r in range(1, self.world):      # fixed rank order
                tot += allp[r, (ml + nl) * d:]
            self.stats_total = tot
        return Xa, Ya


# ---------------------------------------------------------------------------
# bucketed gradient all-reduce, issued from autograd hooks during backward
# ---------------------------------------------------------------------------
def _bucket_bytes():
    import os
    return int(float(os.environ.get('SMMD_BUCKET_MB', '16')) * (1 << 20))


class GradBuckets:
    """All-reduce (SUM) of a FlatAdam's flat gradient in contiguous buckets of
    about ``bucket_bytes``, formed from the last tensor backwards (the order
    the backward produces them).  Buckets are issued, async, from the
    post-accumulate-grad hooks as they complete, strictly in bucket order (a
    bucket that completes early waits for its predecessors), so every rank
    issues the same collectives in the same order whatever order its
    backward ran in; they overlap the rest of the backward.  ``finish``
    issues what no hook did (tensors without a gradient this step contribute
    their zeros) and waits for all.  ``clip_norm`` > 0 clips every tensor of
    a bucket before its all-reduce (the reference's per-tower clip_by_norm,
    model.py:449-455)."""

    def __init__(self, opt, group, bucket_bytes=None, clip_norm=0.0):
        self.opt, self.group = opt, group
        self.clip_norm = float(clip_norm)
        cap = _bucket_bytes() if bucket_bytes is None else int(bucket_bytes)
        # every rank must issue the same all-reduces: rank 0's bucket size wins
        # (an SMMD_BUCKET_MB that differs between ranks would otherwise hang)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            c = torch.tensor([cap], dtype=torch.int64, device=opt.flat_grad.device)
            src = dist.get_global_rank(group, 0) if group is not None else 0
            cap = int(broadcast_(c, src, group).item())
        self.bucket_bytes = cap
        offs = [int(o) for o in opt.offsets]
        n = len(opt.params)
        self.buckets = []
        hi = n
        while hi > 0:
            lo = hi - 1
            while lo > 0 and (offs[hi] - offs[lo - 1]) * 4 <= cap:
                lo -= 1
            self.buckets.append((lo, hi))
            hi = lo
        self.bucket_of = [0] * n
        for b, (lo, hi) in enumerate(self.buckets):
            for i in range(lo, hi):
                self.bucket_of[i] = b
        self._offs = offs
        self.armed = False
        self.left, self.works, self.next = [], [], 0
        self.counted = set()
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook(i))
                       for i, p in enumerate(opt.params)]
        self.launch_log = []      # bucket ids in issue order of the last step (tests)
        # tensors the bucket clip leaves alone (their owner clipped them: the
        # SN weights and scales under the tower-mode G-direct backward)
        self.clip_exclude = frozenset()
        # tensors whose arrival only notify() reports (see notify)
        self.notify_only = frozenset()

    def arm(self):
        """Call before the backward whose gradients this step exchanges."""
        self.armed = True
        self.left = [hi - lo for lo, hi in self.buckets]
        self.counted = set()
        self.next = 0
        self.works = []
        self.launch_log = []

    def _hook(self, i):
        def fn(_p):
            if i not in self.notify_only:
                self._arrive(i)
        return fn

    def _arrive(self, i):
        if self.armed:
            b = self.bucket_of[i]
            if i in self.counted:
                # counted once per step: a tensor written by an SN group node
                # (notify) still has its AccumulateGrad node run -- with no
                # gradient, the group returns None -- and this hook fires again;
                # counting both issued a bucket before its last tensor arrived
                return
            self.counted.add(i)
            self.left[b] -= 1
            while self.next < len(self.buckets) and self.left[self.next] <= 0:
                self._launch(self.next)

    def notify(self, i):
        """Tensor i's gradient is in place without autograd's accumulation
        (the SN group backward writes it directly): count it as a hook would.
        Tensors in ``notify_only`` (the late-summed biases of a data-parallel
        critic step, MMD_GAN.d_step) are counted by this call alone: their
        AccumulateGrad node runs, with no gradient, before the group writes them."""
        self._arrive(i)

    def _launch(self, b):
        lo, hi = self.buckets[b]
        self.next = b + 1
        self.launch_log.append(b)
        if getattr(self.opt, '_gathering', lambda: False)():
            # gather mode (AccumulateGrad kept each gradient as its own tensor,
            # no add into a zeroed view): the bucket's gradients copied into
            # its flat range by one multi-tensor copy, then reduced
            self.opt._gather_grads(lo, hi)
        if self.clip_norm > 0:
            i = lo
            while i < hi:                 # runs of tensors not excluded
                if i in self.clip_exclude:
                    i += 1
                    continue
                j = i
                while j < hi and j not in self.clip_exclude:
                    j += 1
                self.opt.clip_range_(i, j, self.clip_norm)
                i = j
        w = all_reduce_async(self.opt.flat_grad[self._offs[lo]:self._offs[hi]], self.group)
        if w is not None:
            self.works.append(w)

    def finish(self):
        """Issue what the hooks did not, then wait for every bucket."""
        if not self.armed:          # no backward was armed: exchange everything now
            self.arm()
        while self.next < len(self.buckets):
            self._launch(self.next)
        for w in self.works:
            w.wait()
        self.works = []
        self.armed = False

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
