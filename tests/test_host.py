"""Host-side logic on CPU: config surface (YAML overrides CLI), network
shapes/parameter counts, TF SAME padding, D/G schedule, the oracle's CPU
mirror step."""
import os

import numpy as np
import pytest

torch = pytest.importorskip('torch')

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, 'scaled-mmd-gan_amd', 'configs')


def test_yaml_overrides_cli():
    from gan.main import make_flags
    f = make_flags(argv=['-config_file', os.path.join(CFG, 'imagenet_smmd.yml'),
                         '-batch_size', '32', '-kernel', 'mix_rq'])
    assert f.batch_size == 64 and f.kernel == 'rbf'      # YAML wins (gan/main.py:23-24)
    assert f.architecture == 'snresnet' and f.with_scaling is True
    assert f.scaling_coeff == 10.0 and f.learning_rate_D == -1
    g = make_flags(argv=['-kernel', 'mix_rq', '-with_sn', 'true'])
    assert g.kernel == 'mix_rq' and g.with_sn is True


@pytest.mark.parametrize('name', ['cifar10_smmd.yml', 'celebA_smmd.yml', 'imagenet_smmd.yml'])
def test_configs_load(name):
    from gan.main import load_yaml
    c = load_yaml(os.path.join(CFG, name))
    assert c['model'] == 'smmd' and c['kernel'] == 'rbf' and c['dof_dim'] == 1


def test_same_padding():
    from gan.core.snops import same_pad
    assert same_pad(32, 3, 1) == (1, 1)
    assert same_pad(32, 4, 2) == (1, 1)
    assert same_pad(64, 5, 2) == (1, 2)
    assert same_pad(7, 5, 2) == (2, 2)


def _set_w_eff(net):
    from gan.core.snops import sn_modules
    for m in sn_modules(net):
        m.w_eff = m.weight * 1.0


def _count(net):
    return sum(p.numel() for p in net.parameters())


@pytest.mark.parametrize('arch,size,n_sn,d_params', [
    ('snresnet', 64, 14, 10_101_000), ('sngan', 32, 8, 5_860_000), ('g-resnet5', 64, 6, None)])
def test_networks_shapes(arch, size, n_sn, d_params):
    from gan.core.architecture import get_networks
    from gan.core.snops import sn_modules
    G_cls, D_cls = get_networks(arch)
    G = G_cls(64, 3, size, True, z_dim=128)
    D = D_cls(64, 1, False, with_sn=True, with_learnable_sn_scale=True, input_size=size)
    assert len(sn_modules(D)) == n_sn
    if d_params:
        w = sum(m.weight.numel() for m in sn_modules(D))
        assert abs(w - d_params) / d_params < 0.01
    _set_w_eff(D)
    with torch.no_grad():
        x = G(torch.rand(2, 128) * 2 - 1)
        assert x.shape == (2, 3, size, size)
        assert float(x.min()) >= 0 and float(x.max()) <= 1
        assert D(x).shape == (2, 1)


def test_deconv_matches_tf_same_semantics():
    """conv2d_transpose(SAME, k=5, s=2) = adjoint of conv2d(SAME): <deconv(x), y> = <x, conv(y)>."""
    from gan.core.snops import Conv2d, Deconv2d
    torch.manual_seed(0)
    dc = Deconv2d(4, 3, 5, 2, bias=False)
    cv = Conv2d(3, 4, 5, 2, bias=False)
    with torch.no_grad():
        cv.weight.copy_(dc.weight)              # same [4(in of deconv), 3, 5, 5] tensor
        x = torch.randn(1, 4, 8, 8)
        y = torch.randn(1, 3, 16, 16)
        lhs = (dc(x) * y).sum()
        rhs = (x * cv(y)).sum()
    assert float(lhs) == pytest.approx(float(rhs), rel=1e-5)


def test_counters_match_oracle():
    from oracle import smmd_oracle as O
    import argparse
    from gan.core.model import MMD_GAN
    o = O.Counters()
    m = MMD_GAN.__new__(MMD_GAN)
    m.config = argparse.Namespace(dsteps=5, gsteps=1, start_dsteps=10)
    m.d_counter = m.g_counter = 0
    step = 0
    for _ in range(200):
        is_g = o.update(step)
        m.set_counters(step)
        assert (m.d_counter == 0) == is_g
        if is_g:
            step += 1


def test_cpu_mirror_step_runs():
    from gan.core.architecture import get_networks
    from gan.core.snops import sn_modules
    from oracle.tf_mirror import TFMirrorStep, rbf_mmd2_tf
    from oracle import smmd_oracle as O
    torch.manual_seed(0)
    G_cls, D_cls = get_networks('sngan')
    G = G_cls(16, 3, 32, True)
    D = D_cls(16, 1, False, with_sn=True, with_learnable_sn_scale=True, input_size=32)
    st = TFMirrorStep(G, D, sn_modules(D))
    loss = st.step(torch.rand(4, 3, 32, 32))
    assert np.isfinite(loss)
    X, Y = torch.randn(9, 1, dtype=torch.float64), torch.randn(7, 1, dtype=torch.float64)
    assert float(rbf_mmd2_tf(X, Y)) == pytest.approx(O.mmd2(O.kernel_spec('rbf'), X.numpy(),
                                                            Y.numpy()), rel=1e-10)
