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
    import argparse
    from gan.core.architecture import get_networks
    from gan.main import default_flags
    from oracle.tf_mirror import TFMirrorStep, TFMirrorTrainer, rbf_mmd2_tf
    from oracle import smmd_oracle as O
    torch.manual_seed(0)
    cfg = argparse.Namespace(**default_flags())
    cfg.__dict__.update(architecture='sngan', gf_dim=16, df_dim=16, output_size=32,
                        batch_norm=True, with_sn=True, with_learnable_sn_scale=True, dof_dim=1)
    G_cls, D_cls = get_networks('sngan')
    G = G_cls(16, 3, 32, True)
    D = D_cls(16, 1, False, with_sn=True, with_learnable_sn_scale=True, input_size=32)
    st = TFMirrorStep(cfg, G, D)
    before = {n: p.clone() for n, p in zip(st.d_names, st.params)}
    loss = st.step(torch.rand(4, 3, 32, 32))
    assert np.isfinite(loss)
    assert all(not torch.equal(before[n], p) for n, p in zip(st.d_names, st.params)
               if not n.endswith('d_l4/bias'))
    tr = TFMirrorTrainer(cfg, G, D)
    kinds = ''.join(tr.train_step(torch.rand(4, 3, 32, 32)) for _ in range(12))
    assert kinds == 'D' * 10 + 'GD'          # start_dsteps 10 while step < 20
    X, Y = torch.randn(9, 1, dtype=torch.float64), torch.randn(7, 1, dtype=torch.float64)
    assert float(rbf_mmd2_tf(X, Y)) == pytest.approx(O.mmd2(O.kernel_spec('rbf'), X.numpy(),
                                                            Y.numpy()), rel=1e-10)


def test_conv_second_order_rule_matches_autograd():
    """convops.conv2d: value, first and second derivatives equal F.conv2d's
    (CPU, float64) incl. the weight term of the double backward."""
    from gan.core.convops import conv2d, mean_pool2
    torch.manual_seed(0)
    for stride, pad in ((1, 1), (2, 1), (1, 0)):
        x = torch.randn(3, 4, 9, 9, dtype=torch.float64, requires_grad=True)
        w = torch.randn(5, 4, 3, 3, dtype=torch.float64, requires_grad=True)
        b = torch.randn(5, dtype=torch.float64, requires_grad=True)
        outs = []
        for fn in (lambda: conv2d(x, w, b, stride, pad),
                   lambda: torch.nn.functional.conv2d(x, w, b, stride, pad)):
            y = fn()
            g, = torch.autograd.grad(torch.tanh(y).sum(), x, create_graph=True)
            L = (g * g).sum() + y.pow(2).mean()
            outs.append((y.detach(),) + torch.autograd.grad(L, (x, w, b)))
        for a, c in zip(*outs):
            assert torch.allclose(a, c, rtol=1e-9, atol=1e-10)
    t = torch.randn(2, 3, 8, 6, dtype=torch.float64)
    assert torch.allclose(mean_pool2(t), torch.nn.functional.avg_pool2d(t, 2))
    assert torch.autograd.gradcheck(lambda a, c: conv2d(a, c, None, 1, 1),
                                    (torch.randn(1, 2, 5, 5, dtype=torch.float64, requires_grad=True),
                                     torch.randn(3, 2, 3, 3, dtype=torch.float64, requires_grad=True)))
    assert torch.autograd.gradgradcheck(lambda a, c: conv2d(a, c, None, 2, 1),
                                        (torch.randn(1, 2, 5, 5, dtype=torch.float64, requires_grad=True),
                                         torch.randn(3, 2, 3, 3, dtype=torch.float64, requires_grad=True)))


def test_input_grad_only_pass_keeps_second_order_exact():
    """The Jacobian pass under input_grad_only skips weight gradients but the
    double backward through it still yields the exact parameter gradient."""
    from gan.core.convops import conv2d, input_grad_only
    torch.manual_seed(1)
    x = torch.randn(2, 3, 6, 6, dtype=torch.float64, requires_grad=True)
    w1 = torch.randn(4, 3, 3, 3, dtype=torch.float64, requires_grad=True)
    w2 = torch.randn(1, 4, 3, 3, dtype=torch.float64, requires_grad=True)
    res = []
    for ctxmgr, conv in ((input_grad_only, conv2d), (None, torch.nn.functional.conv2d)):
        y = conv(torch.nn.functional.leaky_relu(conv(x, w1, None, 1, 1), 0.2), w2, None, 1, 1).sum()
        if ctxmgr:
            with ctxmgr():
                g, = torch.autograd.grad(y, x, create_graph=True)
        else:
            g, = torch.autograd.grad(y, x, create_graph=True)
        L = (g * g).sum() * y
        res.append(torch.autograd.grad(L, (x, w1, w2)))
    for a, b in zip(*res):
        assert torch.allclose(a, b, rtol=1e-9, atol=1e-10)


def test_mean_pool2_first_and_second_order():
    from gan.core.convops import mean_pool2
    x = torch.randn(2, 3, 6, 8, dtype=torch.float64, requires_grad=True)
    assert torch.allclose(mean_pool2(x), torch.nn.functional.avg_pool2d(x, 2))
    assert torch.autograd.gradcheck(mean_pool2, (x,))
    assert torch.autograd.gradgradcheck(mean_pool2, (x,))


def test_folded_conv_mean_pool_first_and_second_order():
    """ConvMeanPool as one 4x4 stride-2 conv on the folded weight equals the
    literal conv3x3 -> mean pool (block.py:63-66) in value, input gradient and
    the parameter gradient of a gradient penalty through it (float64)."""
    from gan.core import architecture
    torch.manual_seed(2)
    blk = architecture._ConvMeanPool(3, 5, 3, True).double()
    x = torch.randn(2, 3, 8, 6, dtype=torch.float64, requires_grad=True)
    res = []
    saved = architecture.FOLD_POOL
    try:
        for fold in (True, False):
            architecture.FOLD_POOL = fold
            y = blk(x)
            g, = torch.autograd.grad(torch.tanh(y).sum(), x, create_graph=True)
            L = (g * g).sum() + y.pow(2).mean()
            res.append((y.detach(),) + torch.autograd.grad(
                L, (x, blk.conv.weight, blk.conv.bias)))
    finally:
        architecture.FOLD_POOL = saved
    assert res[0][0].shape == (2, 5, 4, 3)
    for a, c in zip(*res):
        assert torch.allclose(a, c, rtol=1e-9, atol=1e-11)


def test_folded_upsample_conv_matches_literal():
    """UpsampleConv (block.py:53-60) as one 4x4 stride-2 transposed conv on the
    folded weight (3x3) and as conv1x1 -> upsample (1x1) equals the literal
    upsample -> conv in value and first / second-order gradients (float64)."""
    from gan.core import architecture
    torch.manual_seed(3)
    for k, bias in ((3, False), (3, True), (1, True)):
        blk = architecture._Up(4, 3, k, bias).double()
        x = torch.randn(2, 4, 5, 3, dtype=torch.float64, requires_grad=True)
        params = [p for p in blk.parameters()]
        res = []
        saved = architecture.FOLD_UP
        try:
            for fold in (True, False):
                architecture.FOLD_UP = fold
                y = blk(x)
                g, = torch.autograd.grad(torch.tanh(y).sum(), x, create_graph=True)
                L = (g * g).sum() + y.pow(2).mean()
                res.append((y.detach(),) + torch.autograd.grad(L, [x] + params))
        finally:
            architecture.FOLD_UP = saved
        assert res[0][0].shape == (2, 3, 10, 6)
        for a, c in zip(*res):
            assert torch.allclose(a, c, rtol=1e-9, atol=1e-11)


def test_three_sample_lr_scheduler_logic(monkeypatch):
    """gan/utils/scorer.py:119-162 decision rules on scripted statistics:
    p = Phi(stat) > .1 for MMD_sdlr_num_test consecutive scorings -> decay."""
    import argparse
    import numpy as np
    from gan.utils import scorer as S
    stats = iter([-3.0, 2.0, 2.0, 2.0, 2.0])          # p ~ 0.001, then p ~ 0.98 x 4
    kids = iter([0.5, 0.4, 0.6, 0.3, 0.7, 0.7, 0.7, 0.7, 0.7, 0.7])
    monkeypatch.setattr(S.cs, 'polynomial_mmd_averages',
                        lambda *a, **k: np.full(2, next(kids)))

    def fake_diff(X, Y, saved):
        if saved is None:
            return ('sums',)
        return 0.0, next(stats), ('sums',)
    monkeypatch.setattr(S.mmd, 'np_diff_polynomial_mmd2_and_ratio_with_saving', fake_diff)

    class Gan:
        config = argparse.Namespace(MMD_sdlr_freq=1, MMD_sdlr_past_sample=2, MMD_sdlr_num_test=3,
                                    with_scaling=True)
        lr, sc, decays = 1e-4, 10.0, 0

        def decay_ops(self):
            self.decays += 1
            self.lr *= .8
    gan = Gan()
    best = []
    sc = S.Scorer(np.zeros((10, 4)), n_subsets=2, subset_size=5)
    for step in range(6):
        sc.compute(gan, step, np.zeros((10, 4)), save_checkpoint=lambda: best.append(step))
    # scorings 0,1 fill the memory; 2: p small -> keep; 3,4,5: p > .1 three times -> decay
    assert gan.decays == 1 and abs(gan.lr - 0.8e-4) < 1e-12
    assert sc.three_sample_chances == 0
    assert best == [1, 3]                      # KID improved at scorings 1 and 3


def test_miopen_db_install(monkeypatch):
    """The committed MIOpen find db is copied to a writable per-process dir
    and MIOPEN_USER_DB_PATH points at it; a user setting is left alone."""
    import os
    from gan.core import miopen_db
    monkeypatch.delenv('MIOPEN_USER_DB_PATH', raising=False)
    monkeypatch.delenv('SMMD_MIOPEN_DB', raising=False)
    d = miopen_db.install()
    assert d and os.environ['MIOPEN_USER_DB_PATH'] == d
    names = sorted(os.listdir(d))
    assert any(n.endswith('.ufdb.txt') for n in names), names
    assert all(n.startswith('gfx950') for n in names)
    monkeypatch.setenv('MIOPEN_USER_DB_PATH', '/somewhere/else')
    assert miopen_db.install() is None
    assert os.environ['MIOPEN_USER_DB_PATH'] == '/somewhere/else'


def test_oracle_fold_pins_to_literal_conv_mean_pool():
    """The oracle's fold (and its adjoint) against the reference's literal
    conv3x3 SAME -> mean of the four strided slices (block.py:63-66), float64."""
    from oracle import smmd_oracle as O
    F = torch.nn.functional
    rng = np.random.default_rng(4)
    x = torch.tensor(rng.standard_normal((2, 3, 10, 8)))
    W = rng.standard_normal((5, 3, 3, 3))
    y = F.conv2d(x, torch.tensor(W), None, 1, 1)
    lit = (y[:, :, ::2, ::2] + y[:, :, 1::2, ::2] + y[:, :, ::2, 1::2] + y[:, :, 1::2, 1::2]) / 4.
    fol = F.conv2d(x, torch.tensor(O.fold_pool_weight(W)), None, 2, 1)
    assert torch.allclose(lit, fol, rtol=1e-12, atol=1e-12)
    G = rng.standard_normal((5, 3, 4, 4))
    assert abs(float((O.fold_pool_weight(W) * G).sum())
               - float((W * O.fold_pool_weight_adjoint(G)).sum())) < 1e-10


def test_prefold_cache_reuse_and_invalidation():
    """A critic's ConvMeanPool folds are shared by calls on the same effective
    weights and recomputed after an in-place update (SN off: W_eff is W)."""
    from gan.core import architecture
    torch.manual_seed(5)
    D = architecture.ResNetDiscriminator(4, 1, False).double()
    x1 = torch.randn(2, 3, 64, 64, dtype=torch.float64)
    x2 = torch.randn(2, 3, 64, 64, dtype=torch.float64)
    (D(x1).sum() + D(x2).sum()).backward()
    c1 = D._fold_cache
    D(x1)
    assert D._fold_cache is c1                       # same weights: reused
    g_shared = [p.grad.clone() for p in D.parameters()]
    saved = architecture.FOLD_POOL
    try:
        architecture.FOLD_POOL = False
        D.zero_grad()
        (D(x1).sum() + D(x2).sum()).backward()
    finally:
        architecture.FOLD_POOL = saved
    for a, b in zip(g_shared, [p.grad for p in D.parameters()]):
        assert torch.allclose(a, b, rtol=1e-9, atol=1e-12)
    with torch.no_grad():
        for p in D.parameters():
            p.add_(0.01)
    D(x1)
    assert D._fold_cache is not c1                   # in-place update: refolded


def test_run_dirs_and_log_redirect(tmp_path):
    """model.py:62-120: the run's description and out_dir/<x>_dir/name/desc
    folders; -log sends stdout and stderr to <sample_dir>/log.txt and the
    streams come back afterwards."""
    import sys
    from gan.main import LogRedirect, description, make_flags, run_dirs
    f = make_flags(argv=['-config_file', os.path.join(CFG, 'imagenet_smmd.yml'),
                         '-dataset', 'imagenet', '-out_dir', str(tmp_path), '-name', 'exp'])
    d = description(f, 64)
    assert d == 'imagenet64x64_snresnet_dc_rbfd5-10-1_64_64_lr0.00020000_bn'
    dirs = run_dirs(f, 64)
    assert dirs['sample'] == os.path.join(str(tmp_path), 'sample', 'exp', d)
    assert all(os.path.isdir(p) for p in dirs.values())
    out, err = sys.stdout, sys.stderr
    with pytest.raises(KeyError):
        with LogRedirect(dirs['sample']):
            print('hello from the run')
            print('to stderr', file=sys.stderr)
            raise KeyError('boom')
    assert sys.stdout is out and sys.stderr is err
    text = open(os.path.join(dirs['sample'], 'log.txt')).read()
    assert 'Execution start time' in text and 'hello from the run' in text
    assert 'to stderr' in text and 'KeyError' in text
    with LogRedirect(str(tmp_path / 'nowhere'), on=False):
        pass                                          # -log false: nothing opened
    assert not os.path.exists(tmp_path / 'nowhere')
