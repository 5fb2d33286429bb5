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
