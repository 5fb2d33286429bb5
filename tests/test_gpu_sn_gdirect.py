"""The G-direct critic update against the path that forms dL/dW.

With the bank armed (``SpectralNormBank.arm_gdirect``, what ``MMD_GAN.d_step``
does in one process) the SN backward runs ``smmd_sn_grad_stats`` instead of
``smmd_sn_weight_bwd``: no dL/dW is written or accumulated, dL/ds goes
straight into the scale's gradient, and ``smmd_adam_flat_sn2`` forms
dL/dW = (s G)/sigma - coef u' v^T tile by tile from G (the adjoint of the
pool fold on ConvMeanPool layers), clipped by the analytic norm of the
stats record.  Reference: sn.py:42-51 / snops.py:82-84 (the SN weight's TF
autodiff), model.py:444-468 (clip_by_norm + Adam).

Tolerances: dL/ds to 1e-5 (the same partials summed in another fixed
order); the Adam
moments m, v (= (1-b) clipped g) within 1e-5 of their max + 1e-4 relative
(g differs from the formed dL/dW by rounding, the clip factor by the analytic
norm's ~1e-7); parameters within 1e-3 of the step size on all but 1e-4 of the
elements (Adam's first steps are lr * sign(m): a gradient that cancels to its
rounding level may flip)."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu

PLAIN = [(256, 1152), (64, 27), (1, 300), (130, 1000)]
FOLD = [(128, 64), (64, 7), (33, 40)]         # (N, C) of [N, C, 3, 3] ConvMeanPool weights


def _net(dev, seed):
    from gan.core import sn
    from gan.core.optim import FlatAdam
    rng = np.random.default_rng(seed)
    mods, params = [], []
    shapes = [(s, False) for s in PLAIN] + [(s, True) for s in FOLD]
    for (N, K), fold in shapes:
        m = torch.nn.Module()
        shape = (N, K, 3, 3) if fold else (N, K)
        m.weight = torch.nn.Parameter(torch.tensor(rng.standard_normal(shape) * 0.05,
                                                   dtype=torch.float32, device=dev))
        m.sn_scale = torch.nn.Parameter(torch.tensor([rng.uniform(0.5, 2.0)],
                                                     dtype=torch.float32, device=dev))
        m.bias = torch.nn.Parameter(torch.tensor(rng.standard_normal(N) * 0.1,
                                                 dtype=torch.float32, device=dev))
        m.sn_fold = fold
        mods.append(m)
        params += [m.bias, m.weight, m.sn_scale]
    bank = sn.SpectralNormBank(mods)
    g = torch.Generator().manual_seed(seed)
    for e in bank.entries:
        e.u.copy_(torch.randn(e.N, generator=g))
    opt = FlatAdam(params, 2e-3, 0.5, 0.9, clip_norm=1.0, name='D')
    assert opt.attach_sn(bank)
    return mods, bank, opt


def _backward(mods, bank, opt, seed, scale, gdirect):
    """loss = sum_i <W_eff_i, R_i> + <bias_i, r_i> through the bank's autograd."""
    opt.zero_grad()
    outs = bank.refresh(update_u=True)
    g = torch.Generator().manual_seed(seed)
    loss = 0.0
    for m, w in zip(mods, outs):
        R = (torch.randn(w.shape, generator=g) * scale).to(w.device)
        r = torch.randn(m.bias.shape, generator=g).to(w.device)
        loss = loss + (w * R).sum() + (m.bias * r).sum()
    bank.arm_gdirect(gdirect)
    try:
        loss.backward()
    finally:
        bank.arm_gdirect(False)


@pytest.mark.parametrize('scale', [0.01, 3.0])       # clip inactive / active
def test_gdirect_update_matches_formed_gradient(dev, scale):
    ma, bank_a, opt_a = _net(dev, 21)
    mb, bank_b, opt_b = _net(dev, 21)
    for step in range(3):
        _backward(ma, bank_a, opt_a, 50 + step, scale, True)
        _backward(mb, bank_b, opt_b, 50 + step, scale, False)
        assert bank_a._gd_pending is not None and bank_b._gd_pending is None
        # the SN weights' ranges of the flat gradient stay unwritten; dense_grad
        # forms them from the kept G as the other path did
        ga, gb = opt_a.dense_grad(), opt_b.flat_grad.clone()
        sg = float(gb.abs().max())
        assert torch.allclose(ga, gb, rtol=1e-4, atol=1e-6 * sg), step
        for m_a, m_b in zip(ma, mb):
            # dL/ds: the same partials, summed in another fixed order
            assert torch.allclose(m_a.sn_scale.grad, m_b.sn_scale.grad, rtol=1e-5,
                                  atol=1e-7), step
        p0 = opt_a.flat_param.clone()
        opt_a.step()
        opt_b.step()
        torch.cuda.synchronize()
        for x, y, what in ((opt_a.m, opt_b.m, 'm'), (opt_a.v, opt_b.v, 'v')):
            lim = 1e-5 * float(y.abs().max()) + 1e-4 * y.abs()
            assert bool(((x - y).abs() <= lim).all()), (what, step,
                                                       float((x - y).abs().max()))
        lr_t = opt_a.lr_t()
        dp = (opt_a.flat_param - opt_b.flat_param).abs()
        bad = int((dp > 1e-3 * lr_t).sum())
        assert bad <= max(1, opt_a.numel // 10000), (step, bad, float(dp.max()))
        assert float((opt_a.flat_param - p0).abs().max()) > 0


def test_gdirect_pending_cleared(dev):
    """The kept G is consumed by the step and dropped by zero_grad: a later
    step never reads a freed tensor."""
    ma, bank, opt = _net(dev, 4)
    _backward(ma, bank, opt, 1, 1.0, True)
    assert bank._gd_pending is not None
    opt.zero_grad()
    assert bank._gd_pending is None
    _backward(ma, bank, opt, 2, 1.0, True)
    opt.step()
    assert bank._gd_pending is None
    torch.cuda.synchronize()
