"""Op-by-op CPU mirror of the reference TF-1.x training step -- TEST / BASELINE
INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests).

TensorFlow 1.6 cannot run in this pipeline (BASELINE.md
section 2), so the CPU baseline is this restatement in torch-CPU fp32, which
materialises everything the TF graph materialises:

* per SN layer: W_r reshape in the reference layout, 2 GEMVs, 2 l2-norms,
  sigma, W_bar = W_r / sigma, s * W_bar   (gan/core/sn.py:16-59, snops.py:84)
* K_XX, K_XY, K_YY via 3 matmuls + diag + clamp + exp, then 3 full sums
  (gan/core/mmd.py:55-82, :199-220)
* tf.gradients of the critic w.r.t. its input, sum of squares, mean, scale
  (gan/core/ops.py:228-233, gan/core/model.py:382-390, smmd.py:21-23)
* per-variable tf.clip_by_norm and the TF Adam update (model.py:444-468)

The convolution stack is the product's PyTorch module graph
(gan.core.architecture) with its convolutions and mean pools swapped back to
stock F.conv2d / F.avg_pool2d while the mirror runs (plain autograd, as the
TF graph is; ConvMeanPool and UpsampleConv in their literal conv -> pool and
upsample -> conv orders, not the product's folded stride-2 convs), and its SN weights produced here instead of by the HIP bank.
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.nn.functional as F

from . import smmd_oracle as O


def _l2n(v, eps=O.SN_EPS):
    return v / (torch.sqrt(torch.sum(v * v)) + eps)


def sn_weight_tf(W_torch, u, s, ref_layout_perm):
    """W_torch: module weight; ref_layout_perm maps it to the TF layout
    [kh, kw, Cin, Cout] (or [in, out] for linear).  Returns the effective
    weight in torch layout and the new u (sn.py:24-46)."""
    W_ref = W_torch.permute(*ref_layout_perm)
    Wr = W_ref.reshape(-1, W_ref.shape[-1])
    with torch.no_grad():
        v = _l2n(u @ Wr.t())
        u_new = _l2n(v @ Wr)
    sigma = (v @ Wr @ u_new.t())[0, 0]
    W_bar = (Wr / sigma).reshape(W_ref.shape)
    if s is not None:
        W_bar = s * W_bar
    inv = [0] * len(ref_layout_perm)
    for i, p in enumerate(ref_layout_perm):
        inv[p] = i
    return W_bar.permute(*inv), u_new


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


@contextlib.contextmanager
def stock_torch_ops():
    """Run the product modules with stock PyTorch conv / pool autograd."""
    from gan.core import architecture, snops
    saved = (snops.conv2d, architecture.mean_pool2, architecture.FOLD_POOL,
             architecture.FOLD_UP)
    snops.conv2d = lambda x, w, b=None, stride=1, padding=0: F.conv2d(x, w, b, stride, padding)
    architecture.mean_pool2 = lambda x: F.avg_pool2d(x, 2)
    architecture.FOLD_POOL = False       # the reference's literal conv -> mean-pool order
    architecture.FOLD_UP = False         # and upsample -> conv order
    try:
        yield
    finally:
        (snops.conv2d, architecture.mean_pool2, architecture.FOLD_POOL,
         architecture.FOLD_UP) = saved


class TFMirrorStep:
    """One critic (D) update of SMMD exactly as the TF graph computes it."""

    def __init__(self, G, D, sn_layers, lr=2e-4, beta1=0.5, beta2=0.9, sc=10.0, z_dim=128):
        self.G, self.D, self.sn_layers = G, D, sn_layers
        self.lr, self.b1, self.b2, self.sc, self.z_dim = lr, beta1, beta2, sc, z_dim
        self.us = [torch.randn(1, m.weight.shape[0]) for m in sn_layers]
        self.params = [p for p in D.parameters() if p.requires_grad]
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.t = 0

    def _sn(self):
        for i, m in enumerate(self.sn_layers):
            if m.weight.dim() == 4:
                perm = (2, 3, 1, 0)          # [Cout, Cin, kh, kw] -> [kh, kw, Cin, Cout]
            else:
                perm = (1, 0)                # [out, in] -> [in, out]
            s = m.sn_scale if hasattr(m, 'sn_scale') else None
            m.w_eff, self.us[i] = sn_weight_tf(m.weight, self.us[i], s, perm)

    def grads(self, images, z=None):
        """(d_loss, [dL/dp for p in D params] before clipping) of one critic
        update; advances u (update_collection=None on the real-image call)."""
        with stock_torch_ops():
            return self._grads(images, z)

    def _grads(self, images, z=None):
        self._sn()
        if z is None:
            z = torch.empty(images.shape[0], self.z_dim).uniform_(-1, 1)
        with torch.no_grad():
            fake = self.G(z)
        x = images.detach().requires_grad_(True)
        d_images = self.D(x)
        d_G = self.D(fake)
        mmd2 = rbf_mmd2_tf(d_G, d_images)
        g, = torch.autograd.grad(d_images[:, 0].sum(), x, create_graph=True)
        J = torch.sum(g * g, dim=(1, 2, 3)).mean()
        scale = 1.0 / (self.sc * J + 1.0)
        d_loss = -(mmd2 * scale)
        grads = torch.autograd.grad(d_loss, self.params)
        return d_loss.detach(), grads

    def step(self, images, z=None):
        d_loss, grads = self.grads(images, z)
        self.t += 1
        tf_adam_(self.params, grads, self.m, self.v, self.t, self.lr, self.b1, self.b2)
        return float(d_loss.detach())


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


class TFMirrorTrainer:
    """The reference's training loop on the CPU mirror: set_counters' 5 D + 1 G
    schedule (model.py:470-478) and, as every ``sess.run`` of train_step does
    (model.py:514, :522-533), BOTH gradient sets computed each step with one
    of them applied.  The CPU baseline of bench.py."""

    def __init__(self, G, D, sn_layers, lr=2e-4, beta1=0.5, beta2=0.9, sc=10.0, z_dim=128,
                 dsteps=5, start_dsteps=10, gsteps=1):
        self.critic = TFMirrorStep(G, D, sn_layers, lr, beta1, beta2, sc, z_dim)
        self.g_params = [p for p in G.parameters() if p.requires_grad]
        self.gm = [torch.zeros_like(p) for p in self.g_params]
        self.gv = [torch.zeros_like(p) for p in self.g_params]
        self.gt = 0
        self.dsteps, self.start_dsteps, self.gsteps = dsteps, start_dsteps, gsteps
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
        with stock_torch_ops():
            c = self.critic
            self.set_counters()
            c._sn()
            z = torch.empty(images.shape[0], c.z_dim).uniform_(-1, 1)
            fake = c.G(z)
            x = images.detach().requires_grad_(True)
            d_images = c.D(x)
            d_G = c.D(fake)
            mmd2 = rbf_mmd2_tf(d_G, d_images)
            g, = torch.autograd.grad(d_images[:, 0].sum(), x, create_graph=True)
            J = torch.sum(g * g, dim=(1, 2, 3)).mean()
            g_loss = mmd2 * (1.0 / (c.sc * J + 1.0))
            d_loss = -g_loss
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
