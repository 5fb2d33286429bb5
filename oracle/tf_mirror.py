"""Op-by-op CPU mirror of the reference TF-1.x training step -- TEST / BASELINE
INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests).

TensorFlow 1.6 cannot run in this pipeline (BASELINE.md
section 2), so the CPU baseline is this restatement in torch-CPU fp32, which
materialises everything the TF graph materialises:

* the networks of oracle/ref_nets.py: the reference's TF layers (SAME convs,
  conv2d_transpose, add_n mean pools, concat + depth_to_space upsampling,
  training-mode batch norm) on weights in the reference's own variable layout
  and names -- written from gan/core/architecture.py and gan/core/resnet/,
  not from the product's modules, whose parameters are only copied in
* per SN layer: W_r reshape in the reference layout, 2 GEMVs, 2 l2-norms,
  sigma, W_bar = W_r / sigma, s * W_bar   (gan/core/sn.py:16-59, snops.py:81-84)
* K_XX, K_XY, K_YY via 3 matmuls + diag + clamp + exp, then 3 full sums
  (gan/core/mmd.py:55-82, :199-220)
* tf.gradients of every critic output w.r.t. the input, sum of squares, mean,
  scale (gan/core/ops.py:228-233, gan/core/model.py:382-390, smmd.py:21-23)
* per-variable tf.clip_by_norm and the TF Adam update (model.py:444-468)
"""
from __future__ import annotations

import math

import torch

from . import ref_nets as R
from . import smmd_oracle as O


def _l2n(v, eps=O.SN_EPS):
    return v / (torch.sqrt(torch.sum(v * v)) + eps)


def sn_weight_tf(W_ref, u, s):
    """spectral_normed_weight (sn.py:16-59) on a weight in the reference
    layout ([kh, kw, in, out] or [in, out]) and snops' ``s * W_bar``.
    Returns (s W_bar in the same layout, the new u)."""
    Wr = W_ref.reshape(-1, W_ref.shape[-1])
    with torch.no_grad():                       # stop_gradient on u', v' (sn.py:35-37)
        v = _l2n(u @ Wr.t())
        u_new = _l2n(v @ Wr)
    sigma = (v @ Wr @ u_new.t())[0, 0]
    W_bar = (Wr / sigma).reshape(W_ref.shape)
    if s is not None:
        W_bar = s * W_bar
    return W_bar, u_new


def rbf_mmd2_tf(X, Y, sigma=1.0, wt=1.0):
    XX, XY, YY = X @ X.t(), X @ Y.t(), Y @ Y.t()
    sx, sy = torch.diagonal(XX), torch.diagonal(YY)
    gamma = 1.0 / (2 * sigma ** 2)
    KXY = wt * torch.exp(-gamma * torch.clamp(-2 * XY + sx[:, None] + sy[None, :], min=0.0))
    KXX = wt * torch.exp(-gamma * torch.clamp(-2 * XX + sx[:, None] + sx[None, :], min=0.0))
    KYY = wt * torch.exp(-gamma * torch.clamp(-2 * YY + sy[:, None] + sy[None, :], min=0.0))
    m, n = float(X.shape[0]), float(Y.shape[0])
    return ((KXX.sum() - m * wt) / (m * (m - 1)) + (KYY.sum() - n * wt) / (n * (n - 1))
            - 2 * KXY.sum() / (m * n))


def squared_norm_jacobian(y, x):
    """ops.py:228-233: sum_i |d y[:, i] / d x|^2 per sample."""
    tot = 0.
    for i in range(y.shape[1]):
        g, = torch.autograd.grad(y[:, i].sum(), x, create_graph=True)
        tot = tot + torch.sum(g * g, dim=tuple(range(1, g.dim())))
    return tot


def arch_key(architecture):
    if 'g-resnet5' in architecture:          # architecture.py:451
        return 'g-resnet5'
    if architecture in ('snresnet', 'sngan'):
        return architecture
    raise ValueError('the TF mirror covers the BASELINE architectures (sngan, snresnet, '
                     'g-resnet5), not %r' % architecture)


def tf_adam_(params, grads, ms, vs, t, lr, b1, b2, eps=1e-8, clip=1.0):
    """Per-variable tf.clip_by_norm(g, 1.) (model.py:449, :455) then
    tf.train.AdamOptimizer's update (model.py:410-411, :458-468)."""
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    with torch.no_grad():
        for p, gr, m, v in zip(params, grads, ms, vs):
            if clip:
                inv = torch.rsqrt(torch.sum(gr * gr))
                gr = gr * torch.clamp(inv * clip, max=1.0)     # t c / max(|t|, c)
            m += (gr - m) * (1 - b1)
            v += (gr * gr - v) * (1 - b2)
            p -= lr_t * m / (torch.sqrt(v) + eps)


class TFMirrorStep:
    """One critic (D) update of SMMD exactly as the TF graph computes it, on
    oracle.ref_nets networks initialised from the product's G and D.

    ``cfg``: the gan.main flags (architecture, gf_dim, df_dim, dof_dim,
    output_size, c_dim, z_dim, batch_norm, gradient_penalty,
    with_sn, with_learnable_sn_scale, learning_rate, beta1, beta2,
    scaling_coeff)."""

    def __init__(self, cfg, G, D, sc=None):
        self.arch = arch_key(cfg.architecture)
        self.size, self.gdim = int(cfg.output_size), int(cfg.gf_dim)
        self.c_dim = int(getattr(cfg, 'c_dim', 3) or 3)
        self.z_dim = int(cfg.z_dim)
        d_bn = bool(cfg.batch_norm) and cfg.gradient_penalty <= 0        # model.py:270
        self.d_vars, self.g_vars, self.P, self.prod = R.bind(
            self.arch, G, D, self.gdim, int(cfg.df_dim), int(cfg.dof_dim), self.size,
            bool(cfg.with_sn), bool(cfg.with_learnable_sn_scale), bool(cfg.batch_norm),
            d_bn=d_bn and self.arch == 'g-resnet5', c_dim=self.c_dim, z_dim=self.z_dim)
        self.lr, self.b1, self.b2 = cfg.learning_rate, cfg.beta1, cfg.beta2
        self.sc = cfg.scaling_coeff if sc is None else sc
        self.sn_names = [v.name.rsplit('/', 1)[0] for v in self.d_vars if v.sn]
        # u: tf.truncated_normal_initializer() [1, out] (sn.py:20-21); tests
        # overwrite them with the product's
        self.us = {}
        for n in self.sn_names:
            W = self.P[n + '/w'] if (n + '/w') in self.P else self.P[n + '/Matrix']
            self.us[n] = torch.nn.init.trunc_normal_(torch.empty(1, W.shape[-1]), a=-2., b=2.)
        self.d_names = [v.name for v in self.d_vars if v.trainable]
        self.g_names = [v.name for v in self.g_vars if v.trainable]
        self.params = [self.P[n] for n in self.d_names]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    # -- graph pieces ---------------------------------------------------
    def sn_weights(self):
        """The critic's variables with every SN weight replaced by s W / sigma;
        advances u (update_collection=None on the real-image call)."""
        Q = dict(self.P)
        for n in self.sn_names:
            key = n + '/w' if (n + '/w') in self.P else n + '/Matrix'
            Q[key], self.us[n] = sn_weight_tf(self.P[key], self.us[n], self.P.get(n + '/s'))
        return Q

    def critic(self, Q, x, return_layers=False):
        return R.critic_forward(self.arch, Q, x, return_layers)

    def generator(self, z):
        return R.generator_forward(self.arch, self.P, z, self.gdim, self.c_dim, self.size)

    def to_product(self, name, t):
        """A reference-layout tensor (weight or its gradient) in the product's
        layout, for comparisons."""
        kind = next(v.kind for v in self.d_vars + self.g_vars if v.name == name)
        if kind in R.TO_REF:
            perm = R.TO_REF[kind]
            inv = [0] * len(perm)
            for i, p in enumerate(perm):
                inv[p] = i
            t = t.permute(*inv)
        return t.reshape(self.prod[name].shape)

    def losses(self, images, z):
        Q = self.sn_weights()
        fake = self.generator(z)
        x = images.detach().requires_grad_(True)
        d_images = self.critic(Q, x)
        d_G = self.critic(Q, fake)
        mmd2 = rbf_mmd2_tf(d_G, d_images)
        J = torch.mean(squared_norm_jacobian(d_images, x))
        g_loss = mmd2 * (1.0 / (self.sc * J + 1.0))
        return g_loss, -g_loss

    def grads(self, images, z=None):
        """(d_loss, {name: dL/dvar} in the reference layout, before clipping)
        of one critic update; advances u."""
        if z is None:
            z = torch.empty(images.shape[0], self.z_dim).uniform_(-1, 1)
        Q = self.sn_weights()
        with torch.no_grad():
            fake = self.generator(z)
        x = images.detach().requires_grad_(True)
        d_images = self.critic(Q, x)
        d_G = self.critic(Q, fake)
        mmd2 = rbf_mmd2_tf(d_G, d_images)
        J = torch.mean(squared_norm_jacobian(d_images, x))
        d_loss = -(mmd2 * (1.0 / (self.sc * J + 1.0)))
        gr = torch.autograd.grad(d_loss, self.params)
        return d_loss.detach(), dict(zip(self.d_names, gr))

    def step(self, images, z=None):
        d_loss, grads = self.grads(images, z)
        self.t += 1
        tf_adam_(self.params, [grads[n] for n in self.d_names], self.m, self.v, self.t,
                 self.lr, self.b1, self.b2)
        return float(d_loss)


class TFMirrorTrainer:
    """The reference's training loop on the CPU mirror: set_counters' 5 D + 1 G
    schedule (model.py:470-478) and, as every ``sess.run`` of train_step does
    (model.py:514, :522-533), BOTH gradient sets computed each step with one
    of them applied.  The CPU baseline of bench.py."""

    def __init__(self, cfg, G, D):
        self.critic = TFMirrorStep(cfg, G, D)
        c = self.critic
        self.g_params = [c.P[n] for n in c.g_names]
        self.gm = [torch.zeros_like(p) for p in self.g_params]
        self.gv = [torch.zeros_like(p) for p in self.g_params]
        self.gt = 0
        self.dsteps, self.start_dsteps, self.gsteps = cfg.dsteps, cfg.start_dsteps, cfg.gsteps
        self.step_no, self.d_counter, self.g_counter = 0, 0, 0

    def set_counters(self):
        if self.g_counter == 0:
            d = self.start_dsteps if (self.step_no % 500 == 0 or self.step_no < 20) \
                else self.dsteps
            self.d_counter = (self.d_counter + 1) % (d + 1)
        if self.d_counter == 0:
            self.g_counter = (self.g_counter + 1) % self.gsteps

    def train_step(self, images):
        """One sess.run: returns 'D' or 'G' (the update applied)."""
        c = self.critic
        self.set_counters()
        z = torch.empty(images.shape[0], c.z_dim).uniform_(-1, 1)
        g_loss, d_loss = c.losses(images, z)
        d_grads = torch.autograd.grad(d_loss, c.params, retain_graph=True)
        g_grads = torch.autograd.grad(g_loss, self.g_params)
        if self.d_counter == 0:
            self.gt += 1
            self.step_no += 1
            tf_adam_(self.g_params, g_grads, self.gm, self.gv, self.gt, c.lr, c.b1, c.b2)
            return 'G'
        c.t += 1
        tf_adam_(c.params, d_grads, c.m, c.v, c.t, c.lr, c.b1, c.b2)
        return 'D'
