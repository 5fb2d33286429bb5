"""The SN refresh leaves W_eff unwritten for the layers the Winograd kernels
consume (sn.SpectralNormBank.set_lazy): their filter
transforms form W_eff = (W / sigma) s -- and the ConvMeanPool fold of it --
from the raw weight (smmd_wino3x3_filter_sn, smmd_wino4x4s2(t)_filter_sn).
Checked: those transforms are bit-identical to transforming a written W_eff;
materialize() writes the same bits the refresh would have; a critic update
with lazy layers equals one without (SMMD_SN_LAZY=0)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _bank(shapes, fold_flags, seed=0):
    from gan.core.sn import SpectralNormBank
    g = torch.Generator(device=DEV).manual_seed(seed)
    mods = []
    for (co, ci, k), fold in zip(shapes, fold_flags):
        m = torch.nn.Module()
        m.weight = torch.nn.Parameter(torch.randn(co, ci, k, k, device=DEV, generator=g) * 0.05)
        m.sn_scale = torch.nn.Parameter(torch.full((1,), 1.3, device=DEV))
        m.sn_fold = fold
        mods.append(m)
    return SpectralNormBank(mods)


@pytest.mark.parametrize('fold', [False, True])
def test_filter_sn_bit_identical(fold):
    """The SN-aware filter transforms equal the plain ones applied to the
    W_eff / W' the refresh writes, bit for bit."""
    from gan.core import _lib, convops
    shapes = [(128, 64, 3), (64, 128, 3)]
    bank = _bank(shapes, [fold, fold])
    outs = bank.refresh(update_u=True)       # written (no lazy set)
    L = _lib.lib()
    st = _lib.stream_handle()
    for e, w in zip(bank.entries, outs):
        co, ci = w.shape[0], w.shape[1]
        if not fold:
            for mode in (0, 1):
                kc = (co, ci) if mode == 0 else (ci, co)
                nb = L.smmd_wino3x3_filter_bytes(*kc)
                a = torch.empty(nb // 4, device=DEV)
                b = torch.empty(nb // 4, device=DEV)
                assert L.smmd_wino3x3_filter(_lib.ptr(w), kc[0], kc[1], mode, _lib.ptr(a), nb,
                                             st) == 0
                assert L.smmd_wino3x3_filter_sn(_lib.ptr(e.weight), _lib.ptr(e.sigma),
                                                _lib.ptr(e.scale), kc[0], kc[1], mode, _lib.ptr(b),
                                                nb, st) == 0
                assert torch.equal(a, b)
        else:
            assert tuple(w.shape[2:]) == (4, 4)
            nb = L.smmd_wino4x4s2_filter_bytes(co, ci)
            for plain, sn in ((L.smmd_wino4x4s2_filter, L.smmd_wino4x4s2_filter_sn),
                              (L.smmd_wino4x4s2t_filter, L.smmd_wino4x4s2t_filter_sn)):
                a = torch.empty(nb // 4, device=DEV)
                b = torch.empty(nb // 4, device=DEV)
                assert plain(_lib.ptr(w), co, ci, _lib.ptr(a), nb, st) == 0
                assert sn(_lib.ptr(e.weight), _lib.ptr(e.sigma), _lib.ptr(e.scale), 1, co, ci,
                          _lib.ptr(b), nb, st) == 0
                assert torch.equal(a, b)
    torch.cuda.synchronize()


@pytest.mark.parametrize('fold', [False, True])
def test_lazy_refresh_and_materialize(fold):
    """With the layers lazy the refresh does not write W_eff (sigma, u, v as
    before); materialize() then writes what it would have, bit for bit."""
    from gan.core import convops
    shapes = [(128, 64, 3), (64, 64, 3)]
    ref = _bank(shapes, [fold, fold], seed=3)
    bank = _bank(shapes, [fold, fold], seed=3)
    for e, f in zip(bank.entries, ref.entries):
        e.u.copy_(f.u)
    want = [w.clone() for w in ref.refresh(update_u=True)]
    bank.set_lazy([0, 1])
    outs = bank.refresh(update_u=True)
    for e, f in zip(bank.entries, ref.entries):
        assert torch.equal(e.sigma, f.sigma) and torch.equal(e.u, f.u)
    for w, ww in zip(outs, want):
        assert convops._lazy(w) is not None
        convops.materialize(w)
        assert convops._lazy(w) is None
        assert torch.equal(w, ww)


def test_critic_step_lazy_equals_written(monkeypatch):
    """One critic update of the ImageNet SNResNet-64 critic (batch 8) with
    the Winograd-fed SN layers lazy and with every W_eff written: same loss,
    same updated parameters (MIOpen's weight gradients of the 1x1 shortcuts
    are not bitwise deterministic, and Adam's first step, lr * g / (|g| + eps),
    turns a rounding difference of a near-zero gradient into up to 2 lr: the
    gradients are compared through Adam's first moment, m = (1 - beta1) g,
    to 1e-5 of its max, the parameters to 2 lr)."""
    import bench
    from gan.core import convops, miopen_db
    from gan.core.smmd import SMMD
    miopen_db.install()
    res = []
    for lazy in ('1', '0'):
        monkeypatch.setenv('SMMD_SN_LAZY', lazy)
        convops.clear_wino_cache()
        cfg = bench.imagenet_config(8)
        torch.manual_seed(2)
        model = SMMD(cfg, device=torch.device(DEV))
        assert bool(model.sn_D.lazy) == (lazy == '1')
        if lazy == '1':
            assert len(model.sn_D.lazy) == 8        # 4 conv_1 + 4 ConvMeanPool folds
        g = torch.Generator(device=DEV).manual_seed(0)
        imgs = torch.rand(8, 3, 64, 64, device=DEV, generator=g)
        torch.manual_seed(5)
        g_loss, d_loss, _ = model.d_step(imgs)
        params = torch.cat([p.detach().reshape(-1) for p in model.d_vars])
        res.append((float(d_loss), params, model.d_optim.m.clone(),
                    model.d_optim.lr))
    (l1, p1, m1, lr), (l0, p0, m0, _) = res
    assert l1 == l0
    assert ((m1 - m0).abs().max() / m0.abs().max()).item() < 1e-5
    assert (p1 - p0).abs().max().item() <= 2.0001 * lr


def test_critic_step_lazy_channels_last(monkeypatch):
    """With channels_last weights no layer is registered lazy --
    the _filter_sn transforms read W as OIHW -- and a critic update with
    SMMD_SN_LAZY=1 equals one with 0: the same loss; the two runs take the
    same code path, so Adam's first moment differs only by MIOpen's
    nondeterministic NHWC weight gradients (measured 9e-4 of its max; the
    channels_last mirror test's 5e-3)."""
    import bench
    from gan.core import convops, miopen_db
    from gan.core.smmd import SMMD
    miopen_db.install()
    res = []
    for lazy in ('1', '0'):
        monkeypatch.setenv('SMMD_SN_LAZY', lazy)
        convops.clear_wino_cache()
        cfg = bench.imagenet_config(8)
        torch.manual_seed(2)
        model = SMMD(cfg, device=torch.device(DEV), channels_last=True)
        g = torch.Generator(device=DEV).manual_seed(0)
        imgs = torch.rand(8, 3, 64, 64, device=DEV, generator=g).contiguous(
            memory_format=torch.channels_last)
        with torch.no_grad():
            outs = model.sn_D.refresh(update_u=False)
        assert not any(convops.is_lazy(w) for w in outs)
        torch.manual_seed(5)
        g_loss, d_loss, _ = model.d_step(imgs)
        res.append((float(d_loss), model.d_optim.m.clone()))
    (l1, m1), (l0, m0) = res
    assert abs(l1 - l0) <= 1e-6 * max(1.0, abs(l0))
    assert ((m1 - m0).abs().max() / m0.abs().max()).item() < 5e-3


def test_stale_lazy_weight_raises():
    """A lazy W_eff read after its layer's next refresh (or an update of W)
    raises instead of being formed from the new W, sigma and s."""
    from gan.core import convops
    bank = _bank([(128, 64, 3)], [False], seed=4)
    bank.set_lazy([0])
    old = bank.refresh(update_u=True)[0]
    assert convops.is_lazy(old) and convops._lazy(old) is not None
    new = bank.refresh(update_u=True)[0]
    assert convops._lazy(new) is not None
    with pytest.raises(convops.StaleLazyWeight):
        convops._lazy(old)
    with pytest.raises(convops.StaleLazyWeight):
        convops.materialize(old)
    with torch.no_grad():
        bank.entries[0].weight.mul_(1.5)          # an in-place update of W
    with pytest.raises(convops.StaleLazyWeight):
        convops._wino_filter(new, 128, 64, 0)


def test_refresh_w_eff_writers_bit_exact():
    """W_eff is written by R2's launch for small plain layers (the tile forms
    sigma itself with the layer block's code) and by P3 for the rest (larger
    ones, fold layers): both are bit for bit (W / sigma) * s with the sigma
    the refresh stored, also with the Winograd-fed layers lazy.  Shapes: the
    SNResNet-64 critic's non-lazy layers (thin input conv, 1x1 shortcuts, the
    linear layer), a wide plain layer over R2's redundancy bound, a fold layer."""
    from gan.core.sn import SpectralNormBank
    g = torch.Generator(device=DEV).manual_seed(5)
    specs = [((64, 3, 3, 3), False), ((128, 64, 1, 1), False), ((512, 256, 1, 1), False),
             ((1024, 512, 1, 1), False), ((1, 1024), False), ((1024, 4608), False),
             ((256, 128, 3, 3), True), ((128, 128, 3, 3), False)]
    mods = []
    for shape, fold in specs:
        m = torch.nn.Module()
        m.weight = torch.nn.Parameter(torch.randn(*shape, device=DEV, generator=g) * 0.05)
        m.sn_scale = torch.nn.Parameter(torch.full((1,), 1.7, device=DEV))
        m.sn_fold = fold
        mods.append(m)
    bank = SpectralNormBank(mods)
    bank.set_lazy([7])                       # a Winograd-fed layer: not written
    for _ in range(3):
        with torch.no_grad():
            outs = bank.refresh(update_u=True)
        for i, (e, w) in enumerate(zip(bank.entries, outs)):
            if i == 7:
                continue
            ref = (e.weight.detach() / e.sigma) * e.scale.detach()
            if e.fold:
                from gan.core.convops import fold_pool_weight
                ref = fold_pool_weight(ref)
            assert torch.equal(w, ref), i
        with torch.no_grad():
            for m in mods:
                m.weight.add_(torch.randn(m.weight.shape, device=DEV, generator=g) * 0.01)
