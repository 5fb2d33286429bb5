"""MMD-GAN trainer (gan/core/model.py, MMD_GAN) on PyTorch-ROCm + libsmmd_hip.

One process per GPU.  A training step (one optimizer update, model.py:507-546):

  D step:  SN bank refresh (all critic layers, 1 HIP launch set)
           -> G(z) (no grad) -> critic(real), critic(fake)
           -> fused MMD^2 (1 HIP launch, gradient in the same sweep)
           -> jac = d critic(real) / d real   (PyTorch, create_graph)
           -> scaled loss (HIP) -> backward (PyTorch double backward + HIP ops)
           -> [RCCL all_reduce of the flat gradient in ~16 MB buckets, each
               issued from autograd hooks as its tensors' gradients land]
           -> clip_by_norm + TF-Adam over all critic tensors (1 HIP launch set)
  G step:  same forward with G in the graph; the scale is a constant for G
           (it depends on the critic only), so no double backward.

Data-parallel modes:
  'tower'  -- the reference's towers (model.py:187-266): local MMD^2 and scale
              per rank, per-rank clip_by_norm (inside each gradient bucket),
              bucketed all_reduce(SUM)/world, Adam.
  'global' -- the north-star mode: ONE all-gather per loss evaluation carries
              every rank's critic features and its J / nD partials
              (collectives.StepExchange), so each rank evaluates the full
              (world*batch) pairwise kernel and the global scale with no
              further small collective; parameter gradients bucketed
              all_reduce(SUM); clip; Adam.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist

from . import collectives, convops, mmd, ops
from .architecture import get_networks
from .collectives import GradBuckets, StepExchange
from .optim import FlatAdam
from .sn import SpectralNormBank
from .snops import sn_modules

GRAD_GATHER = os.environ.get('SMMD_GRAD_GATHER', '1') != '0'


class Timer:
    """gan/utils/timer.py: '[%8d][%s] msg' every `limit` steps and the first 10."""

    def __init__(self, start_time=None, limit=100):
        self.start_time = time.time() if start_time is None else start_time
        self.limit = limit

    def __call__(self, step, mess='', prints=True):
        if prints and (step % self.limit != 0) and (step > 10):
            return None
        t = int(time.time() - self.start_time)
        m, s = t // 60, t % 60
        h, m = m // 60, m % 60
        hms = '%2dh%02dm%02ds' % (h, m, s) if h else ('%5dm%02ds' % (m, s) if m else '%8ds' % s)
        msg = '[%8d][%s] %s' % (step, hms, mess)
        if prints:
            print(msg)
            return None
        return msg


def _winograd_fed(bank):
    """Indices of the SN layers whose convolutions run on the library's
    Winograd kernels in both directions (forward and input gradient) at any
    even input size: 3x3 stride-1 convs with 64-multiple channel counts, and
    4x4 stride-2 convs (the ConvMeanPool folds) whose transposed form tiles
    (smmd_wino3x3_*, smmd_wino4x4s2(t)_*).  Their W_eff is never read
    directly, so the refresh need not write it (SpectralNormBank.set_lazy)."""
    from . import snops
    out = []
    for i, e in enumerate(bank.entries):
        m = e.module
        if not isinstance(m, snops.Conv2d) or m.weight.dim() != 4:
            continue
        co, ci = m.weight.shape[0], m.weight.shape[1]
        if ci % 64 or co % 64:
            continue
        if e.fold and tuple(m.weight.shape[2:]) == (3, 3):
            out.append(i)
        elif (tuple(m.weight.shape[2:]) == (3, 3) and getattr(m, 'stride', 1) == 1
              and convops.WINO):
            out.append(i)
    return out


class MMD_GAN:
    """Base model: loss = mmd2 of the configured kernel (model.py:313-325),
    optional witness gradient penalty (:327-350) and L2 critic penalty
    (:352-364)."""

    def __init__(self, config, device=None, process_group=None, dp_mode='tower',
                 batch_size=None, output_size=None, c_dim=3, channels_last=False,
                 schedule='lean'):
        c = config
        # 'lean': a step computes only the gradient set it applies.
        # 'reference': every step also computes the other set and discards it,
        # as each sess.run of the reference does (model.py:514)
        if schedule not in ('lean', 'reference'):
            raise ValueError('schedule must be lean or reference')
        self.schedule = schedule
        if getattr(c, 'learning_rate_D', -1) < 0:               # model.py:18-19
            c.learning_rate_D = c.learning_rate
        if getattr(c, 'real_batch_size', -1) == -1:             # model.py:42-43
            c.real_batch_size = c.batch_size
        self.config = c
        self.device = device or torch.device('cuda', torch.cuda.current_device())
        self.group = process_group
        grouped = process_group is not None or (dist.is_available() and dist.is_initialized())
        self.world = dist.get_world_size(process_group) if grouped else 1
        self._dp_forced = bool(grouped and collectives.force_dp())
        if dp_mode not in ('tower', 'global'):
            raise ValueError(dp_mode)
        self.dp_mode = dp_mode
        self.batch_size = batch_size or c.batch_size
        self.real_batch_size = c.real_batch_size
        self.output_size = output_size or c.output_size
        self.c_dim = c_dim
        self.z_dim = c.z_dim
        self.timer = Timer()
        G_cls, D_cls = get_networks(c.architecture)
        dbn = bool(c.batch_norm) and (c.gradient_penalty <= 0)   # model.py:270
        self.generator = G_cls(c.gf_dim, c_dim, self.output_size, c.batch_norm,
                               z_dim=c.z_dim).to(self.device)
        self.discriminator = D_cls(c.df_dim, c.dof_dim, dbn, with_sn=c.with_sn,
                                   with_learnable_sn_scale=c.with_learnable_sn_scale,
                                   input_size=self.output_size).to(self.device)
        self.memory_format = torch.channels_last if channels_last else torch.contiguous_format
        if channels_last:               # NHWC activations and conv weights (MIOpen NHWC solvers)
            self.generator.to(memory_format=torch.channels_last)
            self.discriminator.to(memory_format=torch.channels_last)
        self.sn_D = SpectralNormBank(sn_modules(self.discriminator))
        self.sn_D.set_lazy(_winograd_fed(self.sn_D))
        self.sn_G = SpectralNormBank(sn_modules(self.generator))
        self.spec = mmd.get_kernel_spec(c.kernel) if c.kernel else None
        self.g_vars = [p for p in self.generator.parameters() if p.requires_grad]
        self.d_vars = [p for p in self.discriminator.parameters() if p.requires_grad]
        clip = 1.0 if c.clip_grad else 0.0
        self.g_optim = FlatAdam(self.g_vars, c.learning_rate, c.beta1, c.beta2, clip_norm=clip,
                                name='G')
        self.d_optim = FlatAdam(self.d_vars, c.learning_rate_D, c.beta1, c.beta2, clip_norm=clip,
                                name='D')
        # each optimizer step also writes the first power-iteration pass of
        # the next refresh of its network's SN bank
        self.d_optim.attach_sn(self.sn_D)
        self.g_optim.attach_sn(self.sn_G)
        self.lr = float(c.learning_rate)
        self.sc = float(c.scaling_coeff) if c.with_scaling else None
        self.gp = float(c.gradient_penalty)
        self.step = 0
        self.d_counter = 0
        self.g_counter = 0
        self.optim_name = 'kernel_loss'
        self.last = {}
        self._ex = None
        self._buckets = {}
        if self.dp:
            self._broadcast_params()
            for opt in (self.d_optim, self.g_optim):
                self._bucket_for(opt)
            self._group_sn(self.sn_D, self.d_optim)

    # ------------------------------------------------------------------
    @property
    def dp(self):
        """The data-parallel path: several ranks, or (SMMD_DP_FORCE=1) the one
        rank of an initialised group, which then runs the collectives on one
        GPU (collectives.force_dp)."""
        return self.world > 1 or getattr(self, '_dp_forced', False)

    def _dist_group(self):
        return self.group if self.dp else None

    def _broadcast_params(self):
        for opt in (self.g_optim, self.d_optim):
            dist.broadcast(opt.flat_param, 0, group=self.group)
        for bank in (self.sn_D, self.sn_G):
            for e in bank.entries:
                dist.broadcast(e.u, 0, group=self.group)

    def set_counters(self, step):
        """model.py:470-478."""
        c = self.config
        if self.g_counter == 0:
            d_steps = c.dsteps
            if (step % 500 == 0) or (step < 20):
                d_steps = c.start_dsteps
            self.d_counter = (self.d_counter + 1) % (d_steps + 1)
        if self.d_counter == 0:
            self.g_counter = (self.g_counter + 1) % c.gsteps

    def sample_z(self, n):
        return torch.empty(n, self.z_dim, device=self.device).uniform_(-1.0, 1.0)  # model.py:271

    # ------------------------------------------------------------------
    # the reference's loss hooks (model.py:268-403; SMMD / SWGAN override
    # set_loss and apply_scaling, smmd.py:10-42).  They work on the same
    # attributes the reference uses: self.images / self.G (critic inputs),
    # self.d_images / self.d_G (critic outputs, 'hF'), self.d_images_layers /
    # self.d_G_layers, and set self.g_loss / self.d_loss / self.optim_name.
    # ------------------------------------------------------------------
    def _loss_group(self):
        """The group the loss spans: all ranks in the all-gather mode."""
        return self._dist_group() if self.dp_mode == 'global' else None

    def set_tower_loss(self, images, fake, need_critic_grad):
        """The loss half of model.py:268-311: the critic on the real and the
        generated batch, then ``set_loss(self.d_G, self.d_images)``.
        ``need_critic_grad``: build the graph for d_loss w.r.t. the critic
        (the Jacobian's double backward, the penalties).  Returns
        (g_loss, d_loss, aux)."""
        D = self.discriminator
        c = self.config
        if images.dim() == 4:
            images = images.contiguous(memory_format=self.memory_format)
        if getattr(c, 'with_scaling', False) and not getattr(c, 'use_gaussian_noise', False):
            images = images.detach().requires_grad_(True)    # x_hat_data of add_scaling
        self.images = self._last_images = images
        self.G = fake
        self._need_critic_grad = need_critic_grad
        self.aux = None
        if getattr(c, "L2_discriminator_penalty", 0) > 0:
            self.d_images_layers = D(images, return_layers=True)
            self.d_G_layers = D(fake, return_layers=True)
            self.d_images = self.d_images_layers['hF']
            self.d_G = self.d_G_layers['hF']
        else:
            self.d_images_layers = self.d_G_layers = None
            self.d_images = D(images)
            self.d_G = D(fake)
        # mmd.mmd2 inside set_loss spans the global batch in the all-gather
        # mode, and one all-gather carries the features and the scale's partials
        grp = self._loss_group()
        self._ex = ex = self._prepare_exchange(grp) if grp is not None else None
        pend = self._prepare_scale() if grp is None else None
        try:
            with mmd.loss_group(grp, self._ex), mmd.pending_scale(pend):
                self.set_loss(self.d_G, self.d_images)
        finally:
            self._ex = None
        # the loss ran as ONE launch (smmd_smmd_loss_fwd / _fwd_gathered)
        self.fused_loss = ((pend is not None and pend.result is not None)
                           or (ex is not None and ex.result is not None))
        return self.g_loss, self.d_loss, self.aux

    def _scaling_ahead(self):
        c = self.config
        return (getattr(c, 'with_scaling', False) and not getattr(c, 'use_gaussian_noise', False)
                and c.scaling_variant in ('grad', 'value_and_grad'))

    def _prepare_scale(self):
        """One process (or a tower): the Jacobian of the scaling regulariser
        computed BEFORE set_loss, so the loss's mmd2 runs in one launch with
        the scaled loss (mmd.ScalePending, csrc smmd_smmd_loss_fwd) when
        apply_scaling is SMMD's own; add_scaling uses the same Jacobian
        otherwise."""
        if not self._scaling_ahead():
            return None
        need = self._need_critic_grad
        jac = ops.jacobian_columns(self.d_images, self.images, create_graph=need)
        feat = self.d_images
        if not need:
            jac, feat = jac.detach(), feat.detach()
        return mmd.ScalePending(jac, feat, self.sc, self.config.scaling_variant,
                                fuse=self._fused_scaling() == 'mul')

    def _prepare_exchange(self, grp):
        """The all-gather mode's StepExchange: with the scaling regulariser on
        the real batch (the configs' case) the Jacobian and this rank's J / nD
        partials are computed BEFORE set_loss, so they ride in mmd2's feature
        all-gather and add_scaling needs no collective."""
        ex = StepExchange(grp)
        c = self.config
        if (getattr(c, 'with_scaling', False) and not getattr(c, 'use_gaussian_noise', False)
                and c.scaling_variant in ('grad', 'value_and_grad')):
            need = self._need_critic_grad
            jac = ops.jacobian_columns(self.d_images, self.images, create_graph=need)
            ex.jac = jac if need else jac.detach()
            ex.feat = self.d_images if need else self.d_images.detach()
            ex.stats = ops.scaling_partials(ex.jac, ex.feat, c.scaling_variant, grp)
            # SMMD's own apply_scaling: set_loss's mmd2 and the scaled loss run
            # as ONE launch after the gather (mmd._SMMDLossGathered)
            ex.fuse = self._fused_scaling() == 'mul'
            ex.sc = self.sc
            ex.variant = {'grad': 0, 'value_and_grad': 1}[c.scaling_variant]
        return ex

    def set_loss(self, G, images):
        """model.py:313-325: mmd2 of the configured kernel, then the witness
        gradient penalty and the L2 critic penalty."""
        kernel = mmd.get_kernel(self.config.kernel)
        self.g_loss = mmd.mmd2(kernel(G, images))
        self.d_loss = -self.g_loss
        self.optim_name = 'kernel_loss'
        self.add_gradient_penalty(kernel, G, images)
        self.add_l2_penalty()

    def add_gradient_penalty(self, kernel, fake, real):
        """Witness GP (model.py:327-350): x_hat = (1-a) real + a fake images;
        witness_i = mean_j K(D(x_hat)_i, real_j) - mean_j K(D(x_hat)_i, fake_j)
        on the critic features; penalty = mean((||d sum(witness)/d x_hat||_C -
        1)^2), the norm over the CHANNEL axis only (model.py:341).  For the
        library's kernels the witness gradient at the critic output is the HIP
        witness op (with its own second-order backward); any other kernel
        callable runs through its K_XY_only matrices."""
        if self.config.gradient_penalty <= 0 or not self._need_critic_grad:
            return
        bs = min(self.batch_size, self.real_batch_size)
        real, fake = real[:bs], fake[:bs]
        alpha = torch.rand(bs, 1, 1, 1, device=self.device)
        x_hat_data = ((1.0 - alpha) * self.images[:bs].detach()
                      + alpha * self.G[:bs].detach()).requires_grad_(True)
        x_hat = self.discriminator(x_hat_data)                    # NO_OPS (model.py:335)
        spec = mmd.spec_of(kernel)
        if spec is not None:
            dH, _ = mmd.witness_and_grad(x_hat, real, fake, spec)
            g, = torch.autograd.grad(x_hat, x_hat_data, grad_outputs=dH, create_graph=True)
        else:
            witness = (kernel(x_hat, real, K_XY_only=True).mean(1)
                       - kernel(x_hat, fake, K_XY_only=True).mean(1))
            g, = torch.autograd.grad(witness.sum(), x_hat_data, create_graph=True)
        penalty = torch.mean((ops.safer_norm(g, axis=1) - 1.0) ** 2)
        self.d_loss = self.d_loss + penalty * self.gp
        self.optim_name += '_(gp %.1f)' % self.config.gradient_penalty

    def add_l2_penalty(self):
        """model.py:352-364: L2 * mean over the batch of the per-sample mean
        square of every critic layer output (real and generated calls)."""
        coeff = self.config.L2_discriminator_penalty
        if coeff <= 0 or not self._need_critic_grad:
            return
        penalty = 0.0
        for layers in (self.d_G_layers, self.d_images_layers):
            for layer in layers.values():
                penalty = penalty + (layer * layer).reshape(layer.shape[0], -1).mean(1)
        self.d_L2_penalty = coeff * torch.mean(penalty)
        self.d_loss = self.d_loss + self.d_L2_penalty
        self.optim_name += ' (L2 dp %.6f)' % coeff
        self.optim_name = self.optim_name.replace(') (', ', ')

    def add_scaling(self):
        """model.py:366-403: scale = 1 / (sc E||d D(x)/dx||^2 + 1) ('grad') or
        1 / (sc (E||dD/dx||^2 + E D(x)^2) + 1) ('value_and_grad'), x the real
        batch or, with use_gaussian_noise, N(0, 10^2) noise of its shape through
        one more critic call; then ``self.apply_scaling(scale)``.

        The Jacobian is PyTorch autograd (create_graph in a critic update); J,
        the scale and its backward are one HIP pass each over the Jacobian.
        When apply_scaling is the class's own (not overridden), scale and
        product run fused in the same launch (ops.scaled_loss)."""
        c = self.config
        if not c.with_scaling:          # the reference builds scale for summaries only
            return
        if c.scaling_variant not in ('grad', 'value_and_grad'):
            raise ValueError('scaling_variant must be grad or value_and_grad (model.py:387-390)')
        need = self._need_critic_grad
        ex, pre = getattr(self, '_ex', None), None
        pend = mmd.current_pending()
        fused = self._fused_scaling()
        if (pend is not None and pend.result is not None and fused == 'mul'
                and self.g_loss is pend.result[0]):
            # set_loss's mmd2 ran fused with this very scaling (one launch)
            _, self.g_loss, self.aux = pend.result
            self.d_loss = -self.g_loss
            return
        if (ex is not None and ex.result is not None and fused == 'mul'
                and self.g_loss is ex.result[0]):
            # the all-gather mode: set_loss's mmd2 ran fused with this scaling
            _, self.g_loss, self.aux = ex.result
            self.d_loss = -self.g_loss
            return
        if ex is not None and ex.jac is not None:
            jac, feat = ex.jac, ex.feat            # computed ahead (_prepare_exchange)
            pre = ex.stats_total                    # None if no mmd2 gathered them
        elif pend is not None:
            jac, feat = pend.jac, pend.feat        # computed ahead (_prepare_scale)
        else:
            if getattr(c, "use_gaussian_noise", False):
                x_hat_data = (torch.randn(self.images.shape, device=self.device) * 10.0) \
                    .contiguous(memory_format=self.memory_format).requires_grad_(True)
                x_hat = self.discriminator(x_hat_data)            # NO_OPS (model.py:370)
            else:
                x_hat_data, x_hat = self.images, self.d_images
            jac = ops.jacobian_columns(x_hat, x_hat_data, create_graph=need)
            if not need:
                jac = jac.detach()
            feat = x_hat if need else x_hat.detach()
        if fused is not None:
            self.g_loss, self.aux = ops.scaled_loss(
                self.g_loss, jac, feat, sc=self.sc, variant=c.scaling_variant,
                sqrt_scale=(fused == 'sqrt'), process_group=self._loss_group(), pre=pre)
            self.d_loss = -self.g_loss
        else:
            scale, self.aux = ops.scaling_factor(jac, feat, sc=self.sc,
                                                 variant=c.scaling_variant,
                                                 process_group=self._loss_group(), pre=pre)
            self.apply_scaling(scale)

    def _fused_scaling(self):
        """'mul' / 'sqrt' when apply_scaling is SMMD's / SWGAN's own (the
        scale and the product then run in one HIP launch), else None."""
        return None

    def apply_scaling(self, scale):
        raise NotImplementedError('apply_scaling is defined by SMMD / SWGAN (smmd.py:21-23, '
                                  ':40-42)')

    # kept for callers of the round-1 API
    def _critic_losses(self, images, fake, need_critic_grad):
        return self.set_tower_loss(images, fake, need_critic_grad)

    # ------------------------------------------------------------------
    def _bucket_for(self, opt):
        """The GradBuckets of ``opt`` (created on first use): tower mode clips
        each tensor inside its bucket before the all-reduce (model.py:449,
        :455), global mode sums raw gradients and clips after."""
        bk = getattr(self, '_buckets', None)
        if bk is None:
            bk = self._buckets = {}
        if id(opt) not in bk:
            clip = opt.clip_norm if self.dp_mode == 'tower' else 0.0
            bk[id(opt)] = GradBuckets(opt, self.group, clip_norm=clip)
        return bk[id(opt)]

    def _group_sn(self, bank, opt):
        """Data parallel: one SN autograd node per gradient bucket of ``opt``
        (sn._SNGroup), whose backward writes dL/dW and dL/ds straight into the
        flat gradient and counts them for their buckets, so a bucket's
        all-reduce is issued as soon as its layers' gradients exist instead of
        after the single SN backward at the end (and autograd adds nothing).
        SMMD_SN_DIRECT=0 keeps the single node."""
        import os
        if not bank.entries or os.environ.get('SMMD_SN_DIRECT', '1') == '0':
            return
        bk = self._bucket_for(opt)
        index = {id(p): i for i, p in enumerate(opt.params)}
        if any(id(e.weight) not in index for e in bank.entries):
            return
        groups = [[j for j, e in enumerate(bank.entries) if lo <= index[id(e.weight)] < hi]
                  for lo, hi in bk.buckets]

        def direct(members, _bk=bk, _bank=bank, _index=index):
            # the group's layers' biases: their queued contributions (late bias
            # sums; every one is in by now -- a layer's bias gradients come
            # from its own conv nodes or the downstream block input node, both
            # ahead of its SN node) added into their flat-gradient views, and
            # counted for their buckets like the weights
            biases = [b for b in (getattr(_bank.entries[j].module, 'bias', None)
                                  for j in members)
                      if isinstance(b, torch.Tensor) and b.requires_grad and id(b) in _index]
            if biases and convops.late_bias_armed():
                convops.flush_late_bias_sums(biases)
                for b in biases:
                    _bk.notify(_index[id(b)])
            for j in members:
                e = _bank.entries[j]
                for p in (e.weight, e.scale):
                    if p is not None and p.requires_grad and id(p) in _index:
                        _bk.notify(_index[id(p)])
        bank.set_groups(groups, direct)

    def _arm(self, opt):
        if self.dp:
            self._bucket_for(opt).arm()

    def _exchange(self, opt):
        if not self.dp:
            opt.step()
            return
        # buckets not already issued from the backward's hooks go now; wait all
        self._bucket_for(opt).finish()
        if getattr(self, '_dpgd', False) and opt is self.d_optim:
            # the buckets summed G: its stats (global: and dL/ds), then the
            # fused update
            self.sn_D.dp_gdirect_finish(write_gs=self.dp_mode == 'global')
        if self.dp_mode == 'tower':
            # per-tower clip done per bucket; the tower mean (model.py:257-258)
            opt.step(grad_scale=1.0 / self.world, clip=False)
        else:
            opt.step()

    def d_step(self, images):
        self.sn_D.refresh(update_u=True)
        if self.sn_G.entries:
            self.sn_G.refresh(update_u=True)
        ref = self.schedule == 'reference'
        with torch.set_grad_enabled(ref):
            fake = self.generator(self.sample_z(self.batch_size))
        for p in self.d_vars:
            p.requires_grad_(True)
        self.d_optim.gather = GRAD_GATHER and not self.dp
        self.d_optim.zero_grad()
        g_loss, d_loss, aux = self.set_tower_loss(images, fake, need_critic_grad=True)
        self._arm(self.d_optim)
        if ref:       # the generator's gradient set, computed and discarded
            torch.autograd.grad(g_loss, self.g_vars, retain_graph=True)
        gd = self._gdirect()
        dpgd = gd and self.dp
        self.sn_D.arm_gdirect(gd and not dpgd)
        self.sn_D.arm_direct(self.dp)        # the grouped SN nodes' direct writes
        tower_clip = self.d_optim.clip_norm if (dpgd and self.dp_mode == 'tower') else 0.0
        self.sn_D.arm_dp_gdirect(dpgd, clip=tower_clip)
        if self.dp:
            bk = self._bucket_for(self.d_optim)
            bk.clip_exclude = self._sn_tensor_ids() if tower_clip > 0 else frozenset()
        self._dpgd = dpgd
        convops.arm_late_wgrad_sums(True)
        # the bias gradients' later contributions added after the backward
        # (one process, gathered gradients: no hook reads .grad during it)
        # (data parallel: flushed per SN group into the flat-gradient views,
        # the buckets notified there -- MMD_GAN._group_sn)
        late_dp = self.dp and self.sn_D.groups is not None and self.sn_D._direct is not None
        convops.arm_late_bias_sums(self.d_optim.gather or late_dp)
        if self.dp:
            bk.notify_only = self._sn_bias_ids() if (late_dp and convops.late_bias_armed()) \
                else frozenset()
        try:
            if ref:
                d_loss.backward(inputs=self.d_vars)
            else:
                # the real images are a leaf only for the Jacobian: the critic's
                # first conv skips the input gradient nobody reads
                with convops.no_input_grad(self._last_images):
                    d_loss.backward(ops.grad_seed(d_loss))
            convops.flush_late_bias_sums()
        finally:
            convops.arm_late_wgrad_sums(False)
            convops.arm_late_bias_sums(False)
            self.sn_D.arm_gdirect(False)
            self.sn_D.arm_direct(False)
            self.sn_D.arm_dp_gdirect(False)
        self._exchange(self.d_optim)
        self._dpgd = False
        return self._detach_step_state()

    def _sn_bias_ids(self):
        """Flat-buffer tensor indices of the critic's SN layers' biases (the
        late-summed biases a data-parallel SN group flushes and notifies)."""
        index = {id(p): i for i, p in enumerate(self.d_optim.params)}
        return frozenset(index[id(b)] for b in (getattr(e.module, 'bias', None)
                                                for e in self.sn_D.entries)
                         if isinstance(b, torch.Tensor) and b.requires_grad and id(b) in index)

    def _sn_tensor_ids(self):
        """Flat-buffer tensor indices of the critic's SN weights and scales."""
        index = {id(p): i for i, p in enumerate(self.d_optim.params)}
        out = set()
        for e in self.sn_D.entries:
            for p in (e.weight, e.scale):
                if p is not None and id(p) in index:
                    out.add(index[id(p)])
        return frozenset(out)

    def _gdirect(self):
        """The critic's SN weight gradients go straight from G into the
        fused update (smmd_adam_flat_sn2 forms dL/dW from G): an SN-fused
        optimizer, SMMD_SN_GDIRECT not 0; one process (sn._SNBatch.
        _backward_gdirect), or several ranks (either mode) with the grouped SN
        nodes (the buckets all-reduce G itself: sn.arm_dp_gdirect; in tower
        mode each rank's G is first scaled by its own clip factor).
        SMMD_SN_DP_GDIRECT=0 keeps the dense dL/dW exchange for several ranks."""
        import os
        if not (self.d_optim._sn is not None and bool(self.sn_D.entries)
                and os.environ.get('SMMD_SN_GDIRECT', '1') != '0'):
            return False
        if not self.dp:
            return True
        return (self.sn_D.groups is not None and self.sn_D._direct is not None
                and os.environ.get('SMMD_SN_DP_GDIRECT', '1') != '0')

    def _detach_step_state(self):
        """After a step's backward: keep the reference attributes (self.g_loss,
        self.d_images, ...) as values, so no tensor keeps the step's autograd
        graph -- its activations, and the parameters' gradient-accumulation
        nodes bound to this step's stream -- alive into the next step (a
        captured step graph must create its own).  Returns (g_loss, d_loss,
        aux) detached."""
        for name in ('g_loss', 'd_loss', 'd_images', 'd_G', 'G', 'images', '_last_images'):
            v = getattr(self, name, None)
            if torch.is_tensor(v):
                setattr(self, name, v.detach())
        for name in ('d_images_layers', 'd_G_layers'):
            v = getattr(self, name, None)
            if v:
                setattr(self, name, {k: t.detach() for k, t in v.items()})
        aux = self.aux.detach() if torch.is_tensor(self.aux) else self.aux
        self.aux = aux
        # the SN layers' effective weights are outputs of the step's SN node
        # (whose backward holds the weights' accumulation nodes): keep values
        # (an unwritten lazy one is dropped: after the update its W, sigma and
        # s no longer define it; every step refreshes before using the critic)
        for bank in (self.sn_D, self.sn_G):
            for e in bank.entries:
                mod = e.module
                for name in ('w_eff', 'w_fold'):
                    t = getattr(mod, name, None)
                    if torch.is_tensor(t):
                        setattr(mod, name, None if convops.is_lazy(t) else t.detach())
        for net in (self.discriminator, self.generator):
            if getattr(net, '_fold_cache', None) is not None:
                net._fold_cache = None
        return self.g_loss, self.d_loss, aux

    def g_step(self, images):
        # critic weights are constants of the generator update: freeze them
        # BEFORE the SN refresh so W_eff does not require grad (otherwise the
        # backward runs every critic conv's weight-gradient kernel and the SN
        # weight backward, and discards them)
        ref = self.schedule == 'reference'
        if not ref:
            for p in self.d_vars:
                p.requires_grad_(False)
        try:
            self.sn_D.refresh(update_u=True)
            if self.sn_G.entries:
                self.sn_G.refresh(update_u=True)
            # one process: the generator's gradients gathered into the flat
            # buffer by one copy at the update (optim.FlatAdam.gather,
            # SMMD_GRAD_GATHER=0: accumulated into it parameter by parameter)
            # (data parallel: each bucket gathers its range before its
            # all-reduce, collectives.GradBuckets._launch)
            self.g_optim.gather = GRAD_GATHER
            self.g_optim.zero_grad()
            fake = self.generator(self.sample_z(self.batch_size))
            g_loss, d_loss, aux = self.set_tower_loss(images, fake, need_critic_grad=ref)
            if ref:   # the critic's gradient set, computed and discarded
                torch.autograd.grad(d_loss, self.d_vars, retain_graph=True)
            self._arm(self.g_optim)
            g_loss.backward(inputs=self.g_vars)
            self._exchange(self.g_optim)
        finally:
            for p in self.d_vars:
                p.requires_grad_(True)
        return self._detach_step_state()

    def train_step(self, images):
        """model.py:507-546 (lean: only the gradient set being applied)."""
        step = self.step
        self.set_counters(step)
        graphs = getattr(self, '_graphs', None)
        if self.d_counter == 0:
            g_loss, d_loss, aux = (graphs.run(False, images) if graphs is not None
                                   else self.g_step(images))
            self.step += 1                                   # global_step (model.py:460-463)
        else:
            g_loss, d_loss, aux = (graphs.run(True, images) if graphs is not None
                                   else self.d_step(images))
        self.last = {'g_loss': g_loss.detach(), 'd_loss': d_loss.detach(), 'aux': aux}
        return g_loss, d_loss, step

    def enable_graphs(self, on=True):
        """Run ``train_step`` as HIP-graph replays of the captured critic and
        generator steps (StepGraphs).  One GPU, lean schedule only."""
        if not on:
            if getattr(self, '_graphs', None) is not None:
                self._graphs.close()
            self._graphs = None
            return
        if self.dp:
            raise NotImplementedError('step graphs are single-GPU (the collectives run eagerly)')
        if self.schedule != 'lean':
            raise NotImplementedError("step graphs capture the lean schedule")
        self._graphs = StepGraphs(self)

    def check_finite(self):
        """NaN asserts of model.py:537-538 (forces a host sync)."""
        g = float(self.last['g_loss'])
        d = float(self.last['d_loss'])
        assert not np.isnan(g), 'NaN g_loss'
        assert not np.isnan(d), 'NaN d_loss'
        return g, d

    @torch.no_grad()
    def get_samples(self, n):
        """n generator samples [n, c, h, w] on the device, batch by batch
        (model.py:663-694, the NO_OPS sampler graph; BN in training mode as
        the reference's)."""
        out, have = [], 0
        while have < n:
            out.append(self.generator(self.sample_z(self.batch_size)))
            have += out[-1].shape[0]
        return torch.cat(out)[:n]

    def set_lr_sc(self, lr, sc):
        """Set the learning rate (both optimizers, model.py:410-411) and the
        scaling coefficient, e.g. after another rank's decay_ops."""
        c = self.config
        self.lr = lr
        self.g_optim.lr = lr
        self.d_optim.lr = lr * c.learning_rate_D / c.learning_rate
        if self.sc is not None and sc is not None:
            self.sc = sc

    def decay_ops(self):
        """lr *= decay_rate (min 1e-6) and sc *= sc_decay_rate (model.py:162, :173, :493-496)."""
        c = self.config
        self.lr = max(self.lr * c.decay_rate, 1e-6)
        self.g_optim.lr = self.lr
        self.d_optim.lr = self.lr * c.learning_rate_D / c.learning_rate
        if self.sc is not None:
            self.sc *= c.sc_decay_rate

    # checkpoint: torch state (the TF Saver format is out of scope)
    def save_checkpoint(self, checkpoint_dir, step=None):
        """model.py:585-593: 'MMDGAN.model-<step>' (every 2000 steps) or
        'best.model' (step None, the scorer's best KID); the 'checkpoint' file
        names the latest save, as TF's checkpoint state does."""
        import os
        os.makedirs(checkpoint_dir, exist_ok=True)
        name = 'best.model' if step is None else 'MMDGAN.model-%d' % step
        path = os.path.join(checkpoint_dir, name + '.pt')
        torch.save(self.state_dict(), path + '.tmp')
        os.replace(path + '.tmp', path)                      # never a torn checkpoint
        with open(os.path.join(checkpoint_dir, 'checkpoint.tmp'), 'w') as f:
            f.write(name + '\n')
        os.replace(os.path.join(checkpoint_dir, 'checkpoint.tmp'),
                   os.path.join(checkpoint_dir, 'checkpoint'))
        return path

    def load_checkpoint(self, checkpoint_dir, ckpt_name=''):
        """model.py:595-606: ``ckpt_name`` or the latest save; False if none."""
        import os
        if not ckpt_name:
            state = os.path.join(checkpoint_dir, 'checkpoint')
            if not os.path.exists(state):
                return False
            with open(state) as f:
                ckpt_name = f.read().strip()
        path = os.path.join(checkpoint_dir, ckpt_name)
        if not path.endswith('.pt'):
            path += '.pt'
        if not os.path.exists(path):
            return False
        self.load_state_dict(torch.load(path, map_location=self.device, weights_only=True))
        return True

    def state_dict(self):
        return {'G': self.generator.state_dict(), 'D': self.discriminator.state_dict(),
                'sn_D': self.sn_D.state_dict(), 'sn_G': self.sn_G.state_dict(),
                'g_optim': self.g_optim.state_dict(), 'd_optim': self.d_optim.state_dict(),
                'step': self.step, 'lr': self.lr, 'sc': self.sc,
                'counters': (self.d_counter, self.g_counter)}

    def load_state_dict(self, sd):
        self.generator.load_state_dict(sd['G'])
        self.discriminator.load_state_dict(sd['D'])
        self.sn_D.load_state_dict(sd['sn_D'])
        self.sn_G.load_state_dict(sd['sn_G'])
        self.g_optim.load_state_dict(sd['g_optim'])
        self.d_optim.load_state_dict(sd['d_optim'])
        self.step, self.lr, self.sc = sd['step'], sd['lr'], sd['sc']
        self.d_counter, self.g_counter = sd['counters']
        self.g_optim.lr = self.lr
        self.d_optim.lr = self.lr * self.config.learning_rate_D / self.config.learning_rate


class StepGraphs:
    """The lean training step as HIP-graph replays (one GPU).

    A step's ~800 kernel launches (MIOpen convolutions, PyTorch elementwise
    ops, the autograd double backward and the libsmmd_hip calls) are
    recorded once per step kind and replayed, which removes the host's
    per-launch cost and the idle gaps between the step's phases.  The kinds
    are the critic step (with or without the SN bank's first power-iteration
    pass already written by the previous critic update) and the generator
    step.  Everything a replay must change is read from device memory: the
    images (copied into a static buffer), z (the graph-safe RNG), the Adam
    step size (``FlatAdam.lr_t_dev``, written before every replay); the
    host-side folded-filter caches across steps are off while graphs are in
    use (within one captured step a weight's Winograd filter is transformed
    once, convops.arm_capture_cache), and the
    host bookkeeping of a step (optimizer step counts, the SN bank's
    first-pass token) is replayed by ``run``.  A new scaling coefficient is
    recaptured automatically; anything else that changes a launch argument
    (a checkpoint load re-pointing tensors, another batch shape) needs
    ``invalidate``."""

    def __init__(self, model):
        from . import architecture
        self.m = model
        self.graphs, self.outs = {}, {}
        self.pool = None
        self.images = None
        self.key = None
        architecture.CACHE_FOLDS = False
        for opt in (model.d_optim, model.g_optim):
            opt.graph_mode = True

    def close(self):
        from . import architecture
        architecture.CACHE_FOLDS = True
        for opt in (self.m.d_optim, self.m.g_optim):
            opt.graph_mode = False
        self.graphs, self.outs, self.pool = {}, {}, None

    def invalidate(self):
        self.graphs, self.outs = {}, {}

    @staticmethod
    def _ready(bank):
        return bool(bank.entries) and bank._p1_token is not None and \
            bank._p1_token == bank._state_token()

    def _kind(self, critic):
        m = self.m
        return (critic, self._ready(m.sn_D), self._ready(m.sn_G))

    def _bookkeeping(self, critic):
        """The host effects of one step that a replay does not re-run."""
        m = self.m
        opt = m.d_optim if critic else m.g_optim
        opt.advance()
        for bank in (m.sn_D, m.sn_G):
            bank._p1_token = None                 # each refresh consumes it
        if opt._sn is not None:
            opt._sn[0].mark_p1_ready()            # the fused update wrote P1

    def _capture(self, kind, critic):
        m = self.m
        tokens = (m.sn_D._p1_token, m.sn_G._p1_token)
        counts = (m.d_optim.step_count, m.g_optim.step_count)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        convops.arm_capture_cache(True)       # the step's repeated filter transforms
        try:
            with torch.cuda.graph(g, pool=self.pool):
                out = m.d_step(self.images) if critic else m.g_step(self.images)
        finally:
            convops.arm_capture_cache(False)
        self.pool = g.pool()
        # the capture ran the host side of one step without executing it
        m.sn_D._p1_token, m.sn_G._p1_token = tokens
        m.d_optim.step_count, m.g_optim.step_count = counts
        self.graphs[kind], self.outs[kind] = g, out

    def run(self, critic, images):
        m = self.m
        key = m.sc
        if key != self.key:                       # sc is baked into the graphs (lr is not)
            self.invalidate()
            self.key = key
        if self.images is None or self.images.shape != images.shape:
            self.images = torch.empty_like(images)
            self.invalidate()
        self.images.copy_(images)
        kind = self._kind(critic)
        if kind not in self.graphs:
            self._capture(kind, critic)
        opt = m.d_optim if critic else m.g_optim
        opt.lr_t_dev.fill_(opt.lr_t(opt.step_count + 1))
        self.graphs[kind].replay()
        self._bookkeeping(critic)
        # the capture's static outputs are overwritten by the next replay of
        # this kind: hand out copies (train_step's values, model.last)
        return tuple(t.clone() if torch.is_tensor(t) else t for t in self.outs[kind])
