"""Independent CPU restatement of the reference's networks -- TEST / BASELINE
INFRASTRUCTURE ONLY (the TF-graph mirror oracle/tf_mirror.py runs on it).

The three BASELINE architectures written straight from the reference's
TensorFlow code, on plain torch.nn.functional primitives, with the weights in
the reference's variable layout and names:

  snresnet   SNResNetGenerator / SNResNetDiscriminator  (architecture.py:178-208, :410-434)
  sngan      SNGANGenerator / SNGANDiscriminator        (architecture.py:211-230, :395-407)
  g-resnet5  ResNetGenerator / DCGAN5Discriminator      (architecture.py:152-175, :334-343)

Building blocks follow gan/core/resnet/block.py:9-86 literally: ConvMeanPool is
a SAME 3x3 conv then the add_n of the four strided slices / 4 (:63-66);
MeanPoolConv the same slices, then the conv (:69-73); UpsampleConv a 4x
channel concat + depth_to_space(2) in NHWC, then the conv (:53-60).  Convs are
TF 'SAME' (asymmetric padding, gan/core/resnet/ops/conv2d.py:29-36,
snops.py:69-101), deconvs tf.nn.conv2d_transpose's SAME form (snops.py:104-139),
linears x @ Matrix + bias (snops.py:169-205), batch norm in training mode
(tf.layers.batch_normalization, resnet/ops/batchnorm.py:8-18, snops.py:10-40).

Nothing here imports the product's network modules: ``bind`` only reads the
product's parameters (checking each against the shape the reference code
implies) so the mirror can start from the same weights.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


# ---------------------------------------------------------------------------
# TF ops in NCHW
# ---------------------------------------------------------------------------
def _same(n, k, s):
    """TF 'SAME': output ceil(n / s); total pad, before = total // 2."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2, total - total // 2


def conv2d_same(x, w_hwio, b, stride):
    """tf.nn.conv2d(x, w [kh, kw, in, out], strides, 'SAME', NCHW) (+ bias_add)."""
    kh, kw = w_hwio.shape[0], w_hwio.shape[1]
    _, pt, pb = _same(x.shape[2], kh, stride)
    _, pl, pr = _same(x.shape[3], kw, stride)
    y = F.conv2d(F.pad(x, (pl, pr, pt, pb)), w_hwio.permute(3, 2, 0, 1), None, stride)
    if b is not None:
        y = y + b.view(1, -1, 1, 1)
    return y


def deconv2d_same(x, w_hwoi, b, out_hw, stride):
    """tf.nn.conv2d_transpose(x, w [kh, kw, out, in], output_shape, strides,
    'SAME'): the adjoint of the SAME conv that maps out_hw -> x's size, i.e.
    out[j] = sum over (i, k) with i s + k - pad_before = j of x[i] w[k]."""
    kh, kw = w_hwoi.shape[0], w_hwoi.shape[1]
    H, W = out_hw
    _, pt, _ = _same(H, kh, stride)
    _, pl, _ = _same(W, kw, stride)
    full = F.conv_transpose2d(x, w_hwoi.permute(3, 2, 0, 1), None, stride)
    y = full[:, :, pt:pt + H, pl:pl + W]
    if b is not None:
        y = y + b.view(1, -1, 1, 1)
    return y


def linear(x, M, b):
    """snops.linear: x @ Matrix [in, out] + bias."""
    return x @ M + b


def batchnorm_train(x, gamma, beta, eps=1e-5):
    """tf.layers.batch_normalization(axis=1, training=True): batch mean and
    biased batch variance over (N, H, W)."""
    mean = x.mean(dim=(0, 2, 3), keepdim=True)
    var = ((x - mean) ** 2).mean(dim=(0, 2, 3), keepdim=True)
    return (x - mean) / torch.sqrt(var + eps) * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)


def lrelu(x, leak=0.2):
    """snops.lrelu: tf.maximum(x, leak * x)."""
    return torch.maximum(x, leak * x)


def slice_mean(x):
    """tf.add_n of the four strided slices / 4 (block.py:65, :71)."""
    return (x[:, :, ::2, ::2] + x[:, :, 1::2, ::2] + x[:, :, ::2, 1::2] + x[:, :, 1::2, 1::2]) / 4.


def depth_to_space_nchw(x, r=2):
    """block.py:55-57: transpose to NHWC, tf.depth_to_space(r), back to NCHW.
    NHWC [b, h, w, r r c] -> [b, h r, w r, c] with
    out[b, r i + di, r j + dj, c'] = in[b, i, j, (di r + dj) c + c']."""
    b, crr, h, w = x.shape
    c = crr // (r * r)
    t = x.permute(0, 2, 3, 1).reshape(b, h, w, r, r, c)          # (di, dj, c')
    t = t.permute(0, 1, 3, 2, 4, 5).reshape(b, h * r, w * r, c)
    return t.permute(0, 3, 1, 2)


def conv_sizes(size, layers, stride=2):
    """gan/utils/misc.py:228-232."""
    s = [int(size)]
    for _ in range(layers):
        s.append(int(math.ceil(float(s[-1]) / float(stride))))
    return s


# ---------------------------------------------------------------------------
# layer catalogue: every variable of every architecture in reference naming,
# with the shape the reference code gives it
# ---------------------------------------------------------------------------
class Var:
    __slots__ = ('name', 'shape', 'kind', 'sn', 'trainable')

    def __init__(self, name, shape, kind, sn=False, trainable=True):
        self.name, self.shape, self.kind, self.sn, self.trainable = name, tuple(shape), kind, sn, \
            trainable


def _conv_vars(out, name, k, cin, cout, sn, learn, bias=True):
    out.append(Var(name + '/w', (k, k, cin, cout), 'conv', sn=sn))
    if sn:
        out.append(Var(name + '/s', (1,), 'scale', trainable=learn))
    if bias:
        out.append(Var(name + '/biases', (cout,), 'bias'))


def _deconv_vars(out, name, k, cin, cout):
    out.append(Var(name + '/w', (k, k, cout, cin), 'deconv'))
    out.append(Var(name + '/biases', (cout,), 'bias'))


def _lin_vars(out, name, fin, fout, sn=False, learn=False):
    out.append(Var(name + '/Matrix', (fin, fout), 'linear', sn=sn))
    if sn:
        out.append(Var(name + '/s', (1,), 'scale', trainable=learn))
    out.append(Var(name + '/bias', (fout,), 'bias'))


def _bn_vars(out, name, c):
    out.append(Var(name + '/gamma', (c,), 'gamma'))
    out.append(Var(name + '/beta', (c,), 'beta'))


def _block_vars(out, name, cin, cout, resample, bn, sn=False, learn=False):
    """block.py:9-50 (filter_size 3)."""
    if not (cout == cin and resample is None):
        _conv_vars(out, name + '.Shortcut', 1, cin, cout, sn, learn, bias=True)
    if bn:
        _bn_vars(out, name + '.BN1', cin)
    c1_out = cout if resample == 'up' else cin
    _conv_vars(out, name + '.Conv1', 3, cin, c1_out, sn, learn, bias=False)
    if bn:
        _bn_vars(out, name + '.BN2', c1_out)
    _conv_vars(out, name + '.Conv2', 3, c1_out, cout, sn, learn, bias=True)


def critic_vars(arch, dim, o_dim, size, sn, learn, use_bn=False):
    out = []
    if arch == 'snresnet':                          # architecture.py:410-434
        _conv_vars(out, 'd_h0_conv', 3, 3, dim, sn, learn)
        chans = [dim, 2 * dim, 4 * dim, 8 * dim, 16 * dim]
        for i in range(4):
            _block_vars(out, 'd_res%d' % (i + 1), chans[i], chans[i + 1], 'down', False, sn, learn)
        if size != 64:
            _block_vars(out, 'd_res4_bis', 16 * dim, 16 * dim, None, False, sn, learn)
        _lin_vars(out, 'd_h5_lin', 16 * dim, o_dim, sn, learn)
    elif arch == 'sngan':                           # architecture.py:395-407
        spec = [('d_c0_0', 3, 64, 3), ('d_c0_1', 64, 128, 4), ('d_c1_0', 128, 128, 3),
                ('d_c1_1', 128, 256, 4), ('d_c2_0', 256, 256, 3), ('d_c2_1', 256, 512, 4),
                ('d_c3_0', 512, 512, 3)]
        for name, ci, co, k in spec:
            _conv_vars(out, name, k, ci, co, sn, learn)
        final = conv_sizes(size, 3)[-1]
        _lin_vars(out, 'd_l4', 512 * final * final, o_dim, sn=True, learn=False)   # :406
    elif arch == 'g-resnet5':                       # DCGAN5Discriminator :334-343
        chans = [3, dim, 2 * dim, 4 * dim, 8 * dim, 16 * dim]
        for i in range(5):
            _conv_vars(out, 'd_h%d_conv' % i, 5, chans[i], chans[i + 1], sn, learn)
            if use_bn and i > 0:
                _bn_vars(out, 'd_bn%d' % i, chans[i + 1])
        final = conv_sizes(size, 5)[-1]
        o = o_dim if o_dim > 0 else 16 * dim
        _lin_vars(out, 'd_h6_lin', 16 * dim * final * final, o, sn, learn)
    else:
        raise ValueError(arch)
    return out


def generator_vars(arch, dim, c_dim, size, use_bn, z_dim=128):
    out = []
    if arch == 'snresnet':                          # architecture.py:178-208
        s32 = 4 if size == 64 else conv_sizes(size, 5)[5]
        _lin_vars(out, 'g_h0_lin', z_dim, dim * 16 * s32 * s32)
        blocks = [] if size == 64 else [('g_res0_bis', 16 * dim, 16 * dim)]
        blocks += [('g_res1', 16 * dim, 8 * dim), ('g_res2', 8 * dim, 4 * dim),
                   ('g_res3', 4 * dim, 2 * dim), ('g_res4', 2 * dim, dim)]
        for name, ci, co in blocks:
            _block_vars(out, name, ci, co, 'up', True)
        _bn_vars(out, 'g_h4', dim)
        _deconv_vars(out, 'g_g_h5', 3, dim, c_dim)
    elif arch == 'sngan':                           # architecture.py:211-230
        s8 = conv_sizes(size, 4)[3]
        _lin_vars(out, 'g_h0_lin', z_dim, dim * 8 * s8 * s8)
        if use_bn:
            _bn_vars(out, 'g_bn0', dim * 8)
        for i, (ci, co) in enumerate([(8 * dim, 4 * dim), (4 * dim, 2 * dim), (2 * dim, dim)]):
            _deconv_vars(out, 'g_h%d' % (i + 1), 5, ci, co)
            if use_bn:
                _bn_vars(out, 'g_bn%d' % (i + 1), co)
        _deconv_vars(out, 'g_h4', 3, dim, c_dim)
    elif arch == 'g-resnet5':                       # ResNetGenerator :152-175
        s32 = conv_sizes(size, 5)[5]
        _lin_vars(out, 'g_h0_lin', z_dim, dim * 16 * s32 * s32)
        for name, ci, co in [('g_res1', 16 * dim, 8 * dim), ('g_res2', 8 * dim, 4 * dim),
                             ('g_res3', 4 * dim, 2 * dim), ('g_res4', 2 * dim, dim)]:
            _block_vars(out, name, ci, co, 'up', False)
        _bn_vars(out, 'g_h4', dim)
        _deconv_vars(out, 'g_g_h5', 5, dim, c_dim)
    else:
        raise ValueError(arch)
    return out


# ---------------------------------------------------------------------------
# forward passes (P: name -> tensor in the reference layout; conv / linear
# weights of SN layers are already s * W / sigma)
# ---------------------------------------------------------------------------
def _conv(P, name, x, stride=1):
    return conv2d_same(x, P[name + '/w'], P.get(name + '/biases'), stride)


def _block(P, name, x, resample, bn):
    """block.py:9-50."""
    has_short = (name + '.Shortcut/w') in P
    if resample == 'down':
        short = _conv(P, name + '.Shortcut', slice_mean(x)) if has_short else x
    elif resample == 'up':
        short = _conv(P, name + '.Shortcut', depth_to_space_nchw(torch.cat([x] * 4, 1))) \
            if has_short else x
    else:
        short = _conv(P, name + '.Shortcut', x) if has_short else x
    h = x
    if bn:
        h = batchnorm_train(h, P[name + '.BN1/gamma'], P[name + '.BN1/beta'])
    h = F.relu(h)
    if resample == 'up':
        h = depth_to_space_nchw(torch.cat([h] * 4, 1))
    h = _conv(P, name + '.Conv1', h)
    if bn:
        h = batchnorm_train(h, P[name + '.BN2/gamma'], P[name + '.BN2/beta'])
    h = F.relu(h)
    h = _conv(P, name + '.Conv2', h)
    if resample == 'down':
        h = slice_mean(h)
    return short + h


def critic_forward(arch, P, x, return_layers=False):
    L = {}
    if arch == 'snresnet':
        h = lrelu(_conv(P, 'd_h0_conv', x))
        L['h0'] = h
        names = ['d_res1', 'd_res2', 'd_res3', 'd_res4']
        for i, n in enumerate(names):
            h = _block(P, n, h, 'down', False)
            L['h%d' % (i + 1)] = h
        if 'd_res4_bis.Conv1/w' in P:
            h = _block(P, 'd_res4_bis', h, None, False)
        hF = linear(lrelu(h).sum(dim=(2, 3)), P['d_h5_lin/Matrix'], P['d_h5_lin/bias'])
    elif arch == 'sngan':
        h = x
        spec = [('d_c0_0', 1), ('d_c0_1', 2), ('d_c1_0', 1), ('d_c1_1', 2), ('d_c2_0', 1),
                ('d_c2_1', 2), ('d_c3_0', 1)]
        for i, (n, s) in enumerate(spec):
            h = lrelu(_conv(P, n, h, s))
            L['h%d' % i] = h
        hF = linear(h.reshape(h.shape[0], -1), P['d_l4/Matrix'], P['d_l4/bias'])
    elif arch == 'g-resnet5':
        h = x
        for i in range(5):
            h = _conv(P, 'd_h%d_conv' % i, h, 2)
            if i > 0 and ('d_bn%d/gamma' % i) in P:
                h = batchnorm_train(h, P['d_bn%d/gamma' % i], P['d_bn%d/beta' % i])
            h = lrelu(h)
            L['h%d' % i] = h
        hF = linear(h.reshape(h.shape[0], -1), P['d_h6_lin/Matrix'], P['d_h6_lin/bias'])
    else:
        raise ValueError(arch)
    L['hF'] = hF
    return L if return_layers else hF


def generator_forward(arch, P, z, dim, c_dim, size):
    n = z.shape[0]
    if arch in ('snresnet', 'g-resnet5'):
        s32 = 4 if (arch == 'snresnet' and size == 64) else conv_sizes(size, 5)[5]
        h = linear(z, P['g_h0_lin/Matrix'], P['g_h0_lin/bias']).reshape(n, dim * 16, s32, s32)
        bn = arch == 'snresnet'
        names = ['g_res1', 'g_res2', 'g_res3', 'g_res4']
        if 'g_res0_bis.Conv1/w' in P:
            names = ['g_res0_bis'] + names
        for nm in names:
            h = _block(P, nm, h, 'up', bn)
        h = F.relu(batchnorm_train(h, P['g_h4/gamma'], P['g_h4/beta']))
        stride = 1 if arch == 'snresnet' else 2        # k3 s1 (:207) / k5 s2 (:174)
        out = deconv2d_same(h, P['g_g_h5/w'], P['g_g_h5/biases'], (size, size), stride)
        return torch.sigmoid(out)
    if arch == 'sngan':
        s = conv_sizes(size, 4)
        h = linear(z, P['g_h0_lin/Matrix'], P['g_h0_lin/bias']).reshape(n, dim * 8, s[3], s[3])

        def bn(h, name):
            return batchnorm_train(h, P[name + '/gamma'], P[name + '/beta']) \
                if (name + '/gamma') in P else h
        h = F.relu(bn(h, 'g_bn0'))
        h = F.relu(bn(deconv2d_same(h, P['g_h1/w'], P['g_h1/biases'], (s[2], s[2]), 2), 'g_bn1'))
        h = F.relu(bn(deconv2d_same(h, P['g_h2/w'], P['g_h2/biases'], (s[1], s[1]), 2), 'g_bn2'))
        h = F.relu(bn(deconv2d_same(h, P['g_h3/w'], P['g_h3/biases'], (s[0], s[0]), 2), 'g_bn3'))
        return torch.sigmoid(deconv2d_same(h, P['g_h4/w'], P['g_h4/biases'], (s[0], s[0]), 1))
    raise ValueError(arch)


# ---------------------------------------------------------------------------
# binding to the product's parameters (reading only): the product stores
# conv weights [out, in, kh, kw], deconv [in, out, kh, kw], linear [out, in]
# ---------------------------------------------------------------------------
TO_REF = {'conv': (2, 3, 1, 0), 'deconv': (2, 3, 1, 0), 'linear': (1, 0)}


def _product_params(arch, G, D):
    """(name -> product tensor) for every variable of ``critic_vars`` /
    ``generator_vars``, found by walking the product modules in the
    reference's order."""
    out = {}

    def conv(name, m, bias_ok=True):
        out[name + '/w'] = m.weight
        if getattr(m, 'with_sn', False):
            out[name + '/s'] = m.sn_scale
        if m.bias is not None and bias_ok:
            out[name + '/biases'] = m.bias

    def lin(name, m):
        out[name + '/Matrix'] = m.weight
        if getattr(m, 'with_sn', False):
            out[name + '/s'] = m.sn_scale
        out[name + '/bias'] = m.bias

    def bn(name, m):
        out[name + '/gamma'] = m.weight
        out[name + '/beta'] = m.bias

    def block(name, b):
        if b.shortcut is not None:
            conv(name + '.Shortcut', getattr(b.shortcut, 'conv', b.shortcut))
        if hasattr(b.bn1, 'weight'):
            bn(name + '.BN1', b.bn1)
            bn(name + '.BN2', b.bn2)
        conv(name + '.Conv1', getattr(b.conv_1, 'conv', b.conv_1))
        conv(name + '.Conv2', getattr(b.conv_2, 'conv', b.conv_2))

    if arch == 'snresnet':
        conv('d_h0_conv', D.h0)
        for i, b in enumerate(D.res):
            block('d_res%d' % (i + 1) if i < 4 else 'd_res4_bis', b)
        lin('d_h5_lin', D.h5_lin)
        lin('g_h0_lin', G.h0_lin)
        names = ['g_res1', 'g_res2', 'g_res3', 'g_res4']
        if len(G.res) == 5:
            names = ['g_res0_bis'] + names
        for nm, b in zip(names, G.res):
            block(nm, b)
        bn('g_h4', G.bn4)
        conv('g_g_h5', G.h5)
    elif arch == 'sngan':
        for name, c in zip(['d_c0_0', 'd_c0_1', 'd_c1_0', 'd_c1_1', 'd_c2_0', 'd_c2_1', 'd_c3_0'],
                           D.convs):
            conv(name, c)
        lin('d_l4', D.l4)
        lin('g_h0_lin', G.h0_lin)
        for i, nm in enumerate(['g_bn0', 'g_bn1', 'g_bn2', 'g_bn3']):
            m = getattr(G, 'bn%d' % i)
            if hasattr(m, 'weight'):
                bn(nm, m)
        for i in range(1, 5):
            conv('g_h%d' % i, getattr(G, 'h%d' % i))
    elif arch == 'g-resnet5':
        for i, c in enumerate(D.convs):
            conv('d_h%d_conv' % i, c)
        for i, m in enumerate(D.bns):
            if hasattr(m, 'weight'):
                bn('d_bn%d' % i, m)
        lin('d_h6_lin', D.lin)
        lin('g_h0_lin', G.h0_lin)
        for nm, b in zip(['g_res1', 'g_res2', 'g_res3', 'g_res4'], G.res):
            block(nm, b)
        bn('g_h4', G.bn4)
        conv('g_g_h5', G.h5)
    return out


def bind(arch, G, D, dim_g, dim_d, o_dim, size, sn, learn, g_bn, d_bn=False, c_dim=3,
         z_dim=128):
    """Copies of the product's weights in the reference layout, checked
    against the reference's variable list (name, shape, trainability).
    Returns (critic Vars, generator Vars, {name: tensor}, {name: product
    tensor}) -- the last for mapping gradients back."""
    cv = critic_vars(arch, dim_d, o_dim, size, sn, learn, d_bn)
    gv = generator_vars(arch, dim_g, c_dim, size, g_bn, z_dim)
    prod = _product_params(arch, G, D)
    P = {}
    for v in cv + gv:
        if v.name not in prod:
            raise AssertionError('product has no variable for %s' % v.name)
        t = prod[v.name].detach().cpu()
        if v.kind in TO_REF:
            t = t.permute(*TO_REF[v.kind])
        t = t.reshape(v.shape) if v.kind in ('scale',) else t
        if tuple(t.shape) != v.shape:
            raise AssertionError('%s: product shape %s, reference %s'
                                 % (v.name, tuple(t.shape), v.shape))
        P[v.name] = t.clone().float().requires_grad_(v.trainable)
    extra = set(prod) - {v.name for v in cv + gv}
    if extra:
        raise AssertionError('product variables the reference does not have: %s'
                             % sorted(extra))
    return cv, gv, P, prod
