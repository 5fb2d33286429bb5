"""Scaled MMD (gan/core/smmd.py): SMMD and SWGAN on the HIP hot path."""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import mmd, ops
from .collectives import all_reduce_
from .model import MMD_GAN


class SMMD(MMD_GAN):
    """set_loss = mmd2(kernel(G, images)) scaled by 1/(sc*E||grad D||^2 + 1)
    (smmd.py:10-23, model.py:366-403).  The reference never adds the witness
    GP here."""

    def uses_scaling(self):
        return bool(self.config.with_scaling)

    def _critic_losses(self, images, fake, need_critic_grad):
        gp, self.gp = self.gp, 0.0        # SMMD.set_loss never calls add_gradient_penalty
        try:
            return super()._critic_losses(images, fake, need_critic_grad)
        finally:
            self.gp = gp


class SWGAN(MMD_GAN):
    """d_loss = mean(D(G)) - mean(D(images)), g_loss = -d_loss, scaled by
    sqrt(scale) (smmd.py:26-42); forces dof_dim = 1 (:28)."""

    def __init__(self, config, **kw):
        config.dof_dim = 1
        super().__init__(config, **kw)
        self.optim_name = 'swgan_loss'

    def uses_scaling(self):
        return bool(self.config.with_scaling)

    def base_loss(self, d_G, d_images):
        base = d_images.mean() - d_G.mean()          # g_loss = -(mean G - mean images)
        if self.dp_mode == 'global' and self.world > 1:
            base = base.clone()
            all_reduce_(base, self.group)
            base = base / self.world
        return base

    def apply_scaling(self, base, jac, d_images):
        return ops.scaled_loss(base, jac, d_images, sc=self.sc,
                               variant=self.config.scaling_variant, sqrt_scale=True,
                               process_group=self._dist_group() if self.dp_mode == 'global'
                               else None)

    def _critic_losses(self, images, fake, need_critic_grad):
        gp, self.gp = self.gp, 0.0
        try:
            return super()._critic_losses(images, fake, need_critic_grad)
        finally:
            self.gp = gp


def get_model(name):
    """Model dispatch of gan/main.py:139-152 (gan / wgan_gp / cramer are outside
    this build)."""
    if name == 'mmd':
        return MMD_GAN
    if name == 'smmd':
        return SMMD
    if name == 'swgan':
        return SWGAN
    if name in ('gan', 'wgan_gp', 'cramer'):
        raise NotImplementedError('model %r is outside this build (SURVEY.md section 2)' % name)
    raise ValueError('unknown model {}'.format(name))


__all__ = ['SMMD', 'SWGAN', 'get_model', 'mmd', 'torch']
