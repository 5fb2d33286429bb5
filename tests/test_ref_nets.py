"""The oracle's network restatement (oracle/ref_nets.py) against the product's
networks, on CPU.

* variable list: every reference variable (name, shape, trainability) of
  the three BASELINE architectures has exactly one product parameter and vice
  versa; critic sizes equal SURVEY.md section 8(a) a7 (SNResNet-64 10.10 M
  weights in 14 SN layers, SNGAN-32 5.86 M in 8) to the parameter;
* forward: the product's G and D (folded ConvMeanPool / UpsampleConv, its
  own SAME padding) give the reference nets' outputs, layer by layer, on the
  same weights -- a structural difference in either would show here.
"""
import argparse
import math

import pytest

torch = pytest.importorskip('torch')


def _nets(arch, size, gdim, ddim, g_bn=True, d_bn=False, learn=True):
    from gan.core.architecture import get_networks
    G_cls, D_cls = get_networks(arch)
    G = G_cls(gdim, 3, size, g_bn, z_dim=128)
    D = D_cls(ddim, 1, d_bn, with_sn=True, with_learnable_sn_scale=learn, input_size=size)
    return G, D


@pytest.mark.parametrize('arch,size,d_total,n_sn,sn_w', [
    ('snresnet', 64, 10_103_311, 14, 10_099_392),
    ('sngan', 32, 5_860_873, 8, 5_859_008),
    ('g-resnet5', 160, 17_440_391, 6, 17_438_400),
    ('snresnet', 128, 28_978_705, 16, 28_973_760)])
def test_reference_variables_match_product(arch, size, d_total, n_sn, sn_w):
    from oracle import ref_nets as R
    from gan.core.snops import sn_modules
    G, D = _nets(arch, size, 64, 64)
    cv, gv, P, prod = R.bind(arch, G, D, 64, 64, 1, size, True, True, True)
    assert sum(math.prod(v.shape) for v in cv) == d_total
    assert sum(v.sn for v in cv) == n_sn == len(sn_modules(D))
    assert sum(math.prod(v.shape) for v in cv if v.sn) == sn_w
    assert sum(p.numel() for p in D.parameters()) == d_total
    assert sum(p.numel() for p in G.parameters()) == sum(math.prod(v.shape) for v in gv)
    for v in cv + gv:
        assert prod[v.name].requires_grad == v.trainable, v.name


def test_sngan_final_linear_scale_not_trainable():
    """architecture.py:406: d_l4 is always SN, with the default fixed s."""
    from oracle import ref_nets as R
    G, D = _nets('sngan', 32, 16, 64)
    cv, _, _, prod = R.bind('sngan', G, D, 16, 64, 1, 32, True, True, True)
    s = next(v for v in cv if v.name == 'd_l4/s')
    assert not s.trainable and not prod['d_l4/s'].requires_grad
    assert next(v for v in cv if v.name == 'd_c0_0/s').trainable


@pytest.mark.parametrize('arch,size,gdim,ddim,d_bn', [
    ('sngan', 32, 16, 64, False),
    ('snresnet', 64, 8, 8, False),
    ('snresnet', 32, 8, 8, False),          # res0_bis / res4_bis
    ('g-resnet5', 64, 8, 8, False),
    ('g-resnet5', 64, 8, 8, True),          # DCGAN5 critic with d_bn1..4
    ('g-resnet5', 160, 4, 4, False)])       # the celebA size
def test_product_forward_matches_reference_nets(arch, size, gdim, ddim, d_bn):
    from oracle import ref_nets as R
    from oracle.tf_mirror import TFMirrorStep
    torch.manual_seed(0)
    G, D = _nets(arch, size, gdim, ddim, d_bn=d_bn)
    with torch.no_grad():           # non-trivial BN affine parameters and biases
        for m in list(G.modules()) + list(D.modules()):
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
            elif getattr(m, 'bias', None) is not None:
                m.bias.uniform_(-0.05, 0.05)
    cfg = argparse.Namespace(architecture=arch, output_size=size, gf_dim=gdim, df_dim=ddim,
                             dof_dim=1, c_dim=3, z_dim=128, batch_norm=True,
                             # dbn = batch_norm & (gp <= 0) (model.py:270)
                             gradient_penalty=0.0 if d_bn else 1.0, with_sn=True, with_learnable_sn_scale=True,
                             learning_rate=1e-4, beta1=0.5, beta2=0.9, scaling_coeff=10.)
    mirror = TFMirrorStep(cfg, G, D)
    Q = mirror.sn_weights()
    from gan.core.snops import sn_modules
    by_weight = {id(mirror.prod[k]): k for k in mirror.prod}
    for m in sn_modules(D):
        m.w_eff = mirror.to_product(by_weight[id(m.weight)], Q[by_weight[id(m.weight)]]).detach()
    g = torch.Generator().manual_seed(3)
    z = torch.empty(4, 128).uniform_(-1, 1, generator=g)
    with torch.no_grad():
        x_ref = mirror.generator(z)
        x = G(z)
        assert x.shape == x_ref.shape == (4, 3, size, size)
        torch.testing.assert_close(x, x_ref, rtol=1e-4, atol=1e-5)
        L_ref = mirror.critic(Q, x_ref, return_layers=True)
        L = D(x_ref, return_layers=True)
    for k in L_ref:
        torch.testing.assert_close(L[k], L_ref[k], rtol=1e-4, atol=1e-5, msg=k)


def test_depth_to_space_is_nearest_upsample():
    """block.py:55-57 concat x4 + depth_to_space(2) in NHWC = nearest x2."""
    from oracle import ref_nets as R
    x = torch.randn(2, 3, 4, 5)
    up = R.depth_to_space_nchw(torch.cat([x] * 4, 1))
    torch.testing.assert_close(up, torch.nn.functional.interpolate(x, scale_factor=2))


def test_tf_deconv_same_is_conv_adjoint():
    """conv2d_transpose(SAME) = adjoint of conv2d(SAME) for odd and even sizes."""
    from oracle import ref_nets as R
    torch.manual_seed(0)
    for H, k, s in ((16, 5, 2), (5, 5, 2), (10, 3, 1), (80, 5, 2)):
        w = torch.randn(k, k, 3, 4, dtype=torch.float64)        # [kh, kw, out=3, in=4]
        y = torch.randn(2, 3, H, H, dtype=torch.float64)
        x = torch.randn(2, 4, -(-H // s), -(-H // s), dtype=torch.float64)
        lhs = (R.deconv2d_same(x, w, None, (H, H), s) * y).sum()
        rhs = (x * R.conv2d_same(y, w, None, s)).sum()        # conv w as [kh, kw, in=3, out=4]
        assert float(lhs) == pytest.approx(float(rhs), rel=1e-10)
