"""Generators / critics of the BASELINE configs (gan/core/architecture.py),
on PyTorch-ROCm, NCHW fp32.

Built: sngan (SNGANGenerator + SNGANDiscriminator, cifar10_smmd.yml),
snresnet (SNResNetGenerator + SNResNetDiscriminator, imagenet_smmd.yml),
g-resnet5 (ResNetGenerator + DCGAN5Discriminator, celebA_smmd.yml), plus the
plain dcgan / dcgan5 / sngan-dcgan5 / resnet5 variants.  The conditional
(label) networks are out of scope.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import convops
from . import optim as _optim
from .convops import (conv2d, conv_transpose_s2, fold_pool_weight, fold_pool_weights,
                      fold_up_weight, mean_pool2)
from .snops import Conv2d, Deconv2d, Linear, batch_norm, bn_relu, lrelu


def conv_sizes(size, layers, stride=2):
    """gan/utils/misc.py:228-232."""
    s = [int(size)]
    for _ in range(layers):
        s.append(int(-(-s[-1] // stride)))
    return tuple(s)


class _Identity(nn.Module):
    def forward(self, x):
        return x


def _bn_or_id(use, c):
    return batch_norm(c) if use else _Identity()


# ---------------------------------------------------------------------------
# ResNet blocks (gan/core/resnet/block.py:9-86)
# ---------------------------------------------------------------------------
# SMMD_FOLD_POOL=0 restores the literal conv -> mean-pool order (A/B, tests)
FOLD_POOL = os.environ.get('SMMD_FOLD_POOL', '1') != '0'
# SMMD_FOLD_UP=0 restores the literal upsample -> conv order of UpsampleConv
FOLD_UP = os.environ.get('SMMD_FOLD_UP', '1') != '0'
# SMMD_DEFER_BIAS=0: each critic block's two conv biases added by the convs
# themselves instead of inside the next block's fused input pass (A/B)
DEFER_BIAS = os.environ.get('SMMD_DEFER_BIAS', '1') != '0'
# Host-side caches of folded filters (the generator's across critic steps,
# the critic's across its real / fake calls).  A captured step graph
# (model.StepGraphs) must recompute them on every replay: it turns this off.
CACHE_FOLDS = True


class _Up(nn.Module):
    """UpsampleConv (block.py:53-60): concat x4 + depth_to_space(2) = nearest x2."""

    def __init__(self, cin, cout, k, bias, **sn):
        super().__init__()
        self.conv = Conv2d(cin, cout, k, 1, bias=bias, init='glorot_uniform', **sn)
        self._kcache = None

    def _folded(self, w):
        """fold_up_weight(w), contiguous.  Under no_grad (the generator's
        forward in every critic step) it is reused while w is the same
        unmodified tensor and no FlatAdam step ran: the generator's weights
        change once per 5 + 1 steps.  With grad enabled it is rebuilt every
        call: a cached K would carry an autograd graph that a non-retaining
        backward frees."""
        if torch.is_grad_enabled() or not CACHE_FOLDS:
            self._kcache = None
            return fold_up_weight(w).contiguous()
        key = (_optim.param_epoch(w), w._version)
        c = self._kcache
        if c is not None and c[0] == key and c[1] is w:
            return c[2]
        K = fold_up_weight(w).contiguous()
        self._kcache = (key, w, K)
        return K

    def forward(self, x):
        c = self.conv
        if FOLD_UP and c.stride == 1:
            if c.k == 1:     # a 1x1 conv commutes with the nearest upsample: 4x fewer flops
                return F.interpolate(c(x), scale_factor=2, mode='nearest')
            if c.k == 3:     # one 4x4 stride-2 transposed conv on the folded weight
                return conv_transpose_s2(x, self._folded(c.effective_weight()), c.bias)
        return c(F.interpolate(x, scale_factor=2, mode='nearest'))




class _ConvMeanPool(nn.Module):
    """block.py:63-66."""

    def __init__(self, cin, cout, k, bias, **sn):
        super().__init__()
        self.conv = Conv2d(cin, cout, k, 1, bias=bias, init='glorot_uniform', **sn)
        # the SN bank may write this conv's pool-folded filter directly
        self.conv.sn_fold = self.foldable()

    _w4 = None      # set by prefolded(): this call's folded weight

    def foldable(self):
        return FOLD_POOL and self.conv.k == 3 and self.conv.stride == 1

    def bias_deferrable(self, x):
        """The bias is a plain per-channel add after the folded conv (the
        literal conv -> pool order would pool it)."""
        return self.foldable() and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0

    def forward(self, x, with_bias=True, mask_in=False):
        """with_bias False (the folded path only, see bias_deferrable): the
        convolution alone, a consumer adds self.conv.bias.  mask_in: x is a
        ReLU output whose producer leaves the mask to this conv's input
        gradient (convops.conv2d)."""
        c = self.conv
        if not with_bias:
            assert self.bias_deferrable(x)
            w4 = self._w4 if self._w4 is not None else fold_pool_weight(c.effective_weight())
            return conv2d(x, w4, None, 2, 1, mask_in=mask_in)
        if self.foldable() and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0:
            # meanpool2(conv3x3(x)) as ONE 4x4 stride-2 conv on the folded
            # weight: same value, a quarter of the output rows, no pool and no
            # upsample in the backward; MIOpen runs fwd / Dx / Dw of it in about
            # half the time of the 3x3 + pool (tools/fold_bench.py, r03 profiles)
            w4 = self._w4 if self._w4 is not None else fold_pool_weight(c.effective_weight())
            return conv2d(x, w4, c.bias, 2, 1, mask_in=mask_in)
        return mean_pool2(c(x, mask_in=mask_in))


class prefolded:
    """Fold every ConvMeanPool filter of a critic in ONE launch (and one
    adjoint launch in the backward) for the duration of one forward.

    The folded weights are reused while the effective weights are the same
    tensors, unmodified (same objects and _version, no FlatAdam step since:
    the library's update does not advance torch's version counters) under the
    same grad mode:
    the critic's calls on the real and the fake batch within one step share
    one fold, and autograd sums both uses' gradients before the single adjoint
    launch.  The fold nodes save no tensors, so reuse never backs through a
    freed buffer; a new SN refresh or an in-place update misses the cache."""

    def __init__(self, net):
        self.net = net
        self.mods = [m for m in net.modules() if isinstance(m, _ConvMeanPool) and m.foldable()]

    def __enter__(self):
        if self.mods and all(m.conv.with_sn and m.conv.w_eff is None and
                             m.conv.w_fold is not None for m in self.mods):
            # the SN bank already wrote every folded filter (smmd_sn_layer.fold)
            for m in self.mods:
                m._w4 = m.conv.w_fold
            return self
        if self.mods:
            ws = [m.conv.effective_weight() for m in self.mods]
            key = (torch.is_grad_enabled(),
                   tuple((w._version, _optim.param_epoch(w), w.requires_grad) for w in ws))
            cache = getattr(self.net, '_fold_cache', None) if CACHE_FOLDS else None
            if (cache is not None and cache[0] == key
                    and all(a is b for a, b in zip(cache[1], ws))):
                ws4 = cache[2]
            else:
                ws4 = fold_pool_weights(ws)
                self.net._fold_cache = (key, ws, ws4)
            for m, w4 in zip(self.mods, ws4):
                m._w4 = w4
        return self

    def __exit__(self, *a):
        for m in self.mods:
            m._w4 = None
        return False


class _MeanPoolConv(nn.Module):
    """block.py:69-73."""

    def __init__(self, cin, cout, k, bias, **sn):
        super().__init__()
        self.conv = Conv2d(cin, cout, k, 1, bias=bias, init='glorot_uniform', **sn)

    def forward(self, x):
        return self.conv(mean_pool2(x))


class ResidualBlock(nn.Module):
    """block.py:9-50: shortcut + conv_2(relu(norm(conv_1(relu(norm(x))))))."""

    def __init__(self, cin, cout, k=3, resample=None, mode='', with_sn=False,
                 with_learnable_sn_scale=False):
        super().__init__()
        sn = dict(with_sn=with_sn, with_learnable_sn_scale=with_learnable_sn_scale)
        if resample == 'down':
            short = _MeanPoolConv
            self.conv_1 = Conv2d(cin, cin, k, 1, bias=False, init='glorot_uniform', **sn)
            self.conv_2 = _ConvMeanPool(cin, cout, k, True, **sn)
            n1, n2 = cin, cin
        elif resample == 'up':
            short = _Up
            self.conv_1 = _Up(cin, cout, k, False, **sn)
            self.conv_2 = Conv2d(cout, cout, k, 1, bias=True, init='glorot_uniform', **sn)
            n1, n2 = cin, cout
        elif resample is None:
            short = None
            self.conv_1 = Conv2d(cin, cin, k, 1, bias=False, init='glorot_uniform', **sn)
            self.conv_2 = Conv2d(cin, cout, k, 1, bias=True, init='glorot_uniform', **sn)
            n1, n2 = cin, cin
        else:
            raise ValueError('invalid resample value')
        if cin == cout and resample is None:
            self.shortcut = None
        elif short is None:
            self.shortcut = Conv2d(cin, cout, 1, 1, bias=True, init='glorot_uniform', **sn)
        else:
            self.shortcut = short(cin, cout, 1, True, **sn)
        use_bn = mode == 'batchnorm'                     # Normalize, block.py:76-86
        self.bn1 = _bn_or_id(use_bn, n1)
        self.bn2 = _bn_or_id(use_bn, n2)
        # a critic down block: relu(x) (main path) and the shortcut's mean pool
        # of x read the input in one pass (convops.relu_pool)
        self._relu_pool = resample == 'down' and not use_bn
        # an up block: the shortcut's upsample, both conv biases and the sum
        # in one pass (convops.up_add)
        self._up_add = resample == 'up' and isinstance(self.shortcut, _Up)

    def down_parts(self, x, y=None, slope_p=1.0, bx=None, by=None, defer_bias=False):
        """(shortcut, main path, their biases) of a critic down block, not yet
        added, whose input is u = (x + bx) + (y + by) (None terms absent), or
        lrelu(x) when slope_p is 0.2: the input is never written
        (convops.relu_pool reads x and y once and adds the biases).  With
        defer_bias the two convolutions leave their biases to the consumer
        (the next block's relu_pool) and return them; otherwise (None, None)."""
        r, p = convops.relu_pool(x, y, slope_p, bx, by)
        # norm off: the ReLU in conv_1's epilogue, and its mask in conv_2's
        # input gradient (h1's only consumer; convops.conv2d_relu)
        fuse = isinstance(self.bn2, _Identity)
        if fuse:
            h1 = self.conv_1(r, relu=True, consumer_masks=True)
        else:
            h1 = F.relu(self.bn2(self.conv_1(r)))
        sc = self.shortcut.conv
        if defer_bias and self.conv_2.bias_deferrable(h1) and sc.bias is not None \
                and self.conv_2.conv.bias is not None:
            s = sc(p, with_bias=False)                   # _MeanPoolConv on the pooled input
            h = self.conv_2(h1, with_bias=False, mask_in=fuse)
            return s, h, sc.bias, self.conv_2.conv.bias
        return sc(p), self.conv_2(h1, mask_in=fuse), None, None

    def forward(self, x):
        if self._relu_pool and convops.relu_pool_applicable(x):
            s, h, _, _ = self.down_parts(x)
            return s + h
        if self._up_add and convops.UP_ADD and FOLD_UP and x.is_cuda and \
                self.shortcut.conv.k == 1 and self.shortcut.conv.stride == 1:
            sc = self.shortcut.conv
            s = sc(x, with_bias=False)                   # 1x1 conv before the upsample
            h = self.conv_1(bn_relu(self.bn1, x))
            h = self.conv_2(bn_relu(self.bn2, h), with_bias=False)
            return convops.up_add(s, sc.bias, h, self.conv_2.bias)
        s = x if self.shortcut is None else self.shortcut(x)
        h = self.conv_1(bn_relu(self.bn1, x))
        h = self.conv_2(bn_relu(self.bn2, h))
        return s + h


# ---------------------------------------------------------------------------
# generators
# ---------------------------------------------------------------------------
class SNGANGenerator(nn.Module):
    """architecture.py:211-230."""

    def __init__(self, dim, c_dim, output_size, use_batch_norm, z_dim=128):
        super().__init__()
        s1, s2, s4, s8, _ = conv_sizes(output_size, 4)
        self.dim, self.s8 = dim, s8
        self.h0_lin = Linear(z_dim, dim * 8 * s8 * s8)
        self.bn0 = _bn_or_id(use_batch_norm, dim * 8)
        self.h1 = Deconv2d(dim * 8, dim * 4)
        self.bn1 = _bn_or_id(use_batch_norm, dim * 4)
        self.h2 = Deconv2d(dim * 4, dim * 2)
        self.bn2 = _bn_or_id(use_batch_norm, dim * 2)
        self.h3 = Deconv2d(dim * 2, dim)
        self.bn3 = _bn_or_id(use_batch_norm, dim)
        self.h4 = Deconv2d(dim, c_dim, 3, 1)

    def forward(self, z):
        h = self.h0_lin(z).view(-1, self.dim * 8, self.s8, self.s8)
        h = bn_relu(self.bn0, h)
        h = bn_relu(self.bn1, self.h1(h))
        h = bn_relu(self.bn2, self.h2(h))
        h = bn_relu(self.bn3, self.h3(h))
        return torch.sigmoid(self.h4(h))


class DCGANGenerator(nn.Module):
    """architecture.py:103-124 (layers=4) and DCGAN5Generator :127-149 (layers=5)."""

    def __init__(self, dim, c_dim, output_size, use_batch_norm, z_dim=128, layers=4):
        super().__init__()
        s = conv_sizes(output_size, layers)
        mult = 8 if layers == 4 else 16
        self.top, self.s0 = dim * mult, s[-1]
        self.h0_lin = Linear(z_dim, self.top * s[-1] * s[-1])
        self.bn0 = _bn_or_id(use_batch_norm, self.top)
        chans = [self.top // (2 ** i) for i in range(layers)] + [c_dim]
        self.deconvs = nn.ModuleList(Deconv2d(chans[i], chans[i + 1]) for i in range(layers))
        self.bns = nn.ModuleList(_bn_or_id(use_batch_norm, chans[i + 1])
                                 for i in range(layers - 1))

    def forward(self, z):
        h = bn_relu(self.bn0, self.h0_lin(z).view(-1, self.top, self.s0, self.s0))
        for i, dc in enumerate(self.deconvs):
            h = dc(h)
            if i < len(self.bns):
                h = bn_relu(self.bns[i], h)
        return torch.sigmoid(h)


class ResNetGenerator(nn.Module):
    """architecture.py:152-175 (g-resnet5): blocks with mode='' (no BN), final
    Batchnorm + relu + deconv 5x5/2 + sigmoid."""

    def __init__(self, dim, c_dim, output_size, use_batch_norm, z_dim=128):
        super().__init__()
        s = conv_sizes(output_size, 5)
        self.dim, self.s32 = dim, s[5]
        self.h0_lin = Linear(z_dim, dim * 16 * s[5] * s[5])
        self.res = nn.Sequential(ResidualBlock(16 * dim, 8 * dim, 3, 'up'),
                                 ResidualBlock(8 * dim, 4 * dim, 3, 'up'),
                                 ResidualBlock(4 * dim, 2 * dim, 3, 'up'),
                                 ResidualBlock(2 * dim, dim, 3, 'up'))
        self.bn4 = batch_norm(dim)
        self.h5 = Deconv2d(dim, c_dim)

    def forward(self, z):
        h = self.h0_lin(z).view(-1, self.dim * 16, self.s32, self.s32)
        h = bn_relu(self.bn4, self.res(h))
        return torch.sigmoid(self.h5(h))


class SNResNetGenerator(nn.Module):
    """architecture.py:178-208: mode='batchnorm' blocks; 64 px starts at 4x4."""

    def __init__(self, dim, c_dim, output_size, use_batch_norm, z_dim=128):
        super().__init__()
        s = conv_sizes(output_size, 5)
        s32 = 4 if output_size == 64 else s[5]
        self.dim, self.s32 = dim, s32
        self.h0_lin = Linear(z_dim, dim * 16 * s32 * s32)
        blocks = []
        if output_size != 64:
            blocks.append(ResidualBlock(16 * dim, 16 * dim, 3, 'up', 'batchnorm'))
        blocks += [ResidualBlock(16 * dim, 8 * dim, 3, 'up', 'batchnorm'),
                   ResidualBlock(8 * dim, 4 * dim, 3, 'up', 'batchnorm'),
                   ResidualBlock(4 * dim, 2 * dim, 3, 'up', 'batchnorm'),
                   ResidualBlock(2 * dim, dim, 3, 'up', 'batchnorm')]
        self.res = nn.Sequential(*blocks)
        self.bn4 = batch_norm(dim)
        self.h5 = Deconv2d(dim, c_dim, 3, 1)

    def forward(self, z):
        h = self.h0_lin(z).view(-1, self.dim * 16, self.s32, self.s32)
        h = bn_relu(self.bn4, self.res(h))
        return torch.sigmoid(self.h5(h))


# ---------------------------------------------------------------------------
# critics
# ---------------------------------------------------------------------------
class SNGANDiscriminator(nn.Module):
    """architecture.py:395-407 (final linear is always SN, :406)."""

    def __init__(self, dim, o_dim, use_batch_norm, with_sn=False, with_learnable_sn_scale=False,
                 input_size=32):
        super().__init__()
        sn = dict(with_sn=with_sn, with_learnable_sn_scale=with_learnable_sn_scale)
        spec = [(3, 64, 3, 1), (64, 128, 4, 2), (128, 128, 3, 1), (128, 256, 4, 2),
                (256, 256, 3, 1), (256, 512, 4, 2), (512, 512, 3, 1)]
        self.convs = nn.ModuleList(Conv2d(ci, co, k, s, stddev=0.02, **sn) for ci, co, k, s in spec)
        final = input_size // 8
        self.l4 = Linear(512 * final * final, o_dim, with_sn=True, stddev=0.02)

    def forward(self, x, return_layers=False):
        layers = {}
        h = x
        for i, c in enumerate(self.convs):
            h = lrelu(c(h))
            layers['h%d' % i] = h
        hF = self.l4(h.reshape(h.shape[0], -1))
        layers['hF'] = hF
        return layers if return_layers else hF


class DCGANDiscriminator(nn.Module):
    """architecture.py:323-343 (DCGAN: 4 convs, DCGAN5: 5 convs), 5x5/2 SAME."""

    def __init__(self, dim, o_dim, use_batch_norm, with_sn=False, with_learnable_sn_scale=False,
                 input_size=64, layers=4):
        super().__init__()
        sn = dict(with_sn=with_sn, with_learnable_sn_scale=with_learnable_sn_scale)
        chans = [3] + [dim * (2 ** i) for i in range(layers)]
        self.convs = nn.ModuleList(Conv2d(chans[i], chans[i + 1], 5, 2, **sn)
                                   for i in range(layers))
        self.bns = nn.ModuleList(_bn_or_id(use_batch_norm and i > 0, chans[i + 1])
                                 for i in range(layers))
        final = conv_sizes(input_size, layers)[-1]
        o = o_dim if o_dim > 0 else chans[-1]
        self.lin = Linear(chans[-1] * final * final, o, **sn)

    def forward(self, x, return_layers=False):
        layers = {}
        h = x
        for i, (c, bn) in enumerate(zip(self.convs, self.bns)):
            h = lrelu(bn(c(h)))
            layers['h%d' % i] = h
        hF = self.lin(h.reshape(h.shape[0], -1))
        layers['hF'] = hF
        return layers if return_layers else hF


class SNResNetDiscriminator(nn.Module):
    """architecture.py:410-434."""

    def __init__(self, dim, o_dim, use_batch_norm, with_sn=False, with_learnable_sn_scale=False,
                 input_size=64):
        super().__init__()
        sn = dict(with_sn=with_sn, with_learnable_sn_scale=with_learnable_sn_scale)
        self.h0 = Conv2d(3, dim, 3, 1, init='glorot_uniform', **sn)
        blocks = [ResidualBlock(dim, 2 * dim, 3, 'down', **sn),
                  ResidualBlock(2 * dim, 4 * dim, 3, 'down', **sn),
                  ResidualBlock(4 * dim, 8 * dim, 3, 'down', **sn),
                  ResidualBlock(8 * dim, 16 * dim, 3, 'down', **sn)]
        if input_size != 64:
            blocks.append(ResidualBlock(16 * dim, 16 * dim, 3, None, **sn))
        self.res = nn.ModuleList(blocks)
        self.h5_lin = Linear(16 * dim, o_dim, **sn)

    def forward(self, x, return_layers=False):
        with prefolded(self):
            return self._forward(x, return_layers)

    def _forward(self, x, return_layers):
        if not return_layers:
            return self._forward_chained(x)
        layers = {}
        h = lrelu(self.h0(x))
        layers['h0'] = h
        for i, b in enumerate(self.res):
            h = b(h)
            layers['h%d' % (i + 1)] = h
        h = lrelu(h).sum(dim=(2, 3))
        hF = self.h5_lin(h)
        layers['hF'] = hF
        return layers if return_layers else hF

    def _forward_chained(self, x):
        """The same network with each down block's input kept as the pieces
        that make it -- the first conv's pre-activation (its lrelu fused into
        the block's input ops), then the previous block's two paths and their
        conv biases (the add and the bias adds fused) -- so no block input is
        written or read twice."""
        u, v, bu, bv, slope = self.h0(x), None, None, None, 0.2
        n = len(self.res)
        for i, b in enumerate(self.res):
            if b._relu_pool and convops.relu_pool_applicable(u, v):
                nxt = self.res[i + 1] if i + 1 < n else None
                defer = DEFER_BIAS and nxt is not None and nxt._relu_pool and convops.RELU_POOL
                u, v, bu, bv = b.down_parts(u, v, slope, bu, bv, defer_bias=defer)
                slope = 1.0
                continue
            u, v, bu, bv, slope = b(self._join(u, v, bu, bv, slope)), None, None, None, 1.0
        if bu is None and bv is None and slope == 1.0:
            # the last block's two paths, their add, lrelu and the pixel sum
            # in one launch (convops.lrelu_rowsum)
            return self.h5_lin(convops.lrelu_rowsum(u, v, 0.2))
        h = self._join(u, v, bu, bv, slope)
        return self.h5_lin(lrelu(h).sum(dim=(2, 3)))

    @staticmethod
    def _join(u, v, bu, bv, slope):
        """(u + bu) + (v + bv), then lrelu unless slope is 1: the block
        output exactly as the unfused ops form it."""
        if bu is not None:
            u = u + bu.view(1, -1, 1, 1)
        if v is not None:
            u = u + (v if bv is None else v + bv.view(1, -1, 1, 1))
        return u if slope == 1.0 else lrelu(u, slope)


class ResNetDiscriminator(nn.Module):
    """architecture.py:358-375 (no SN)."""

    def __init__(self, dim, o_dim, use_batch_norm, with_sn=False, with_learnable_sn_scale=False,
                 input_size=64):
        super().__init__()
        self.h0 = Conv2d(3, dim, 3, 1, init='glorot_uniform')
        self.res = nn.ModuleList([ResidualBlock(dim, 2 * dim, 3, 'down'),
                                  ResidualBlock(2 * dim, 4 * dim, 3, 'down'),
                                  ResidualBlock(4 * dim, 8 * dim, 3, 'down'),
                                  ResidualBlock(8 * dim, 8 * dim, 3, 'down')])
        self.h5_lin = Linear(4 * 4 * 8 * dim, o_dim)

    def forward(self, x, return_layers=False):
        with prefolded(self):
            return self._forward(x, return_layers)

    def _forward(self, x, return_layers):
        layers = {}
        h = lrelu(self.h0(x))
        layers['h0'] = h
        for i, b in enumerate(self.res):
            h = b(h)
            layers['h%d' % (i + 1)] = h
        hF = self.h5_lin(h.reshape(h.shape[0], -1))
        layers['hF'] = hF
        return layers if return_layers else hF


def get_networks(architecture):
    """architecture.py:437-459 -> (Generator factory, Discriminator factory)."""
    gd = {
        'dcgan': (lambda *a, **k: DCGANGenerator(*a, layers=4, **k),
                  lambda *a, **k: DCGANDiscriminator(*a, layers=4, **k)),
        'dcgan5': (lambda *a, **k: DCGANGenerator(*a, layers=5, **k),
                   lambda *a, **k: DCGANDiscriminator(*a, layers=5, **k)),
        'sngan': (SNGANGenerator, SNGANDiscriminator),
        'sngan-dcgan5': (SNGANGenerator, lambda *a, **k: DCGANDiscriminator(*a, layers=5, **k)),
        'snresnet': (SNResNetGenerator, SNResNetDiscriminator),
        'resnet5': (ResNetGenerator, ResNetDiscriminator),
    }
    if architecture in gd:
        return gd[architecture]
    if 'g-resnet5' in architecture:
        return ResNetGenerator, lambda *a, **k: DCGANDiscriminator(*a, layers=5, **k)
    if architecture in ('cond_snresnet', 'd-fullconv5', 'dc64', 'dcgan64', 'dc128'):
        raise NotImplementedError('architecture %r is outside this build (SURVEY.md section 2)'
                                  % architecture)
    raise ValueError('Wrong architecture: "%s"' % architecture)
