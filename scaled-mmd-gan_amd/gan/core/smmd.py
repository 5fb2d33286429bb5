"""Scaled MMD (gan/core/smmd.py): SMMD and SWGAN on the HIP hot path.

Same hooks as the reference: ``set_loss(G, images)`` builds the base loss and
calls ``add_scaling()``, which computes the scale and hands it to
``apply_scaling(scale)``.  A subclass overriding ``apply_scaling`` (as SWGAN
does in the reference) receives the scale tensor (0-dim, differentiable); the
classes' own ``apply_scaling`` runs fused with the scale in one HIP launch
(ops.scaled_loss) -- same value, fewer launches.
"""
from __future__ import annotations

import torch

from . import mmd
from .collectives import all_reduce_
from .model import MMD_GAN


class SMMD(MMD_GAN):
    """smmd.py:6-23: g_loss = mmd2(kernel(G, images)) * scale,
    scale = 1/(sc*E||grad D||^2 + 1) (model.py:366-403).  The reference never
    adds the witness GP here."""

    def set_loss(self, G, images):
        kernel = mmd.get_kernel(self.config.kernel)                # smmd.py:11
        self.g_loss = mmd.mmd2(kernel(G, images))
        self.d_loss = -self.g_loss
        self.optim_name = 'kernel_loss'
        self.add_scaling()

    def apply_scaling(self, scale):
        """smmd.py:21-23."""
        self.g_loss = self.g_loss * scale
        self.d_loss = -self.g_loss

    def _fused_scaling(self):
        return 'mul' if type(self).apply_scaling is SMMD.apply_scaling else None


class SWGAN(MMD_GAN):
    """smmd.py:26-42: d_loss = mean(D(G)) - mean(D(images)), g_loss = -d_loss,
    scaled by sqrt(scale); forces dof_dim = 1 (:28)."""

    def __init__(self, config, **kw):
        config.dof_dim = 1
        super().__init__(config, **kw)
        self.optim_name = 'swgan_loss'

    def _mean(self, t):
        """tf.reduce_mean over the loss's batch: the global batch in the
        all-gather mode (each rank's mean all-reduced / world)."""
        m = t.mean()
        grp = self._loss_group()
        if grp is not None:
            m = m.clone()
            all_reduce_(m, grp)
            m = m / self.world
        return m

    def set_loss(self, G, images):
        self.d_loss = self._mean(G) - self._mean(images)
        self.g_loss = -self.d_loss
        self.optim_name = 'swgan_loss'
        self.add_scaling()

    def apply_scaling(self, scale):
        """smmd.py:40-42."""
        self.g_loss = self.g_loss * torch.sqrt(scale)
        self.d_loss = -self.g_loss

    def _fused_scaling(self):
        return 'sqrt' if type(self).apply_scaling is SWGAN.apply_scaling else None


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
