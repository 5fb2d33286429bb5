"""SN-fused optimizer step against the unfused pair.

``FlatAdam.attach_sn`` turns a step into ``smmd_adam_flat_sn`` (the SN weights
updated tile by tile with the first pass of the next power iteration) and the
next ``SpectralNormBank.refresh`` into ``smmd_sn_power_iter_ex(...,
SMMD_SN_P1_READY)``.  The pair must give the same bits as ``smmd_adam_flat``
followed by ``smmd_sn_power_iter``, step after step, and the refresh must still
match the oracle's power iteration (sn.py:16-59, model.py:444-468)."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

from oracle import smmd_oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

# vec interior tiles, ragged rows/cols, K % 4 != 0, one row, several row tiles
SHAPES = [(256, 1152), (64, 27), (1, 300), (130, 1000), (96, 64)]


def _net(dev, seed, num_iters):
    from gan.core import sn
    from gan.core.optim import FlatAdam
    rng = np.random.default_rng(seed)
    mods, params = [], []
    for N, K in SHAPES:
        m = torch.nn.Module()
        m.weight = torch.nn.Parameter(torch.tensor(rng.standard_normal((N, K)) * 0.05,
                                                   dtype=torch.float32, device=dev))
        m.bias = torch.nn.Parameter(torch.tensor(rng.standard_normal(N) * 0.1,
                                                 dtype=torch.float32, device=dev))
        mods.append(m)
        params += [m.bias, m.weight]          # SN weights interleaved with plain tensors
    bank = sn.SpectralNormBank(mods, num_iters=num_iters)
    g = torch.Generator().manual_seed(seed)
    for e in bank.entries:                    # same u in every copy
        e.u.copy_(torch.randn(e.N, generator=g))
    opt = FlatAdam(params, 2e-3, 0.5, 0.9, clip_norm=1.0, name='D')
    return mods, bank, opt


def _grads(opt, seed):
    g = torch.Generator().manual_seed(seed)
    gr = torch.randn(opt.numel, generator=g) * 0.3
    opt.zero_grad()
    opt.flat_grad.copy_(gr.to(opt.flat_grad.device))


@pytest.mark.parametrize('clip', [True, False])
@pytest.mark.parametrize('num_iters', [1, 2])
@pytest.mark.parametrize('groups', ['1', '2', '4'])
def test_fused_step_same_bits_as_unfused(dev, monkeypatch, clip, num_iters, groups):
    monkeypatch.setenv('SMMD_SN_ADAM_H', groups)      # row groups of the fused tile
    _, bank_a, opt_a = _net(dev, 5, num_iters)
    _, bank_b, opt_b = _net(dev, 5, num_iters)
    assert opt_a.attach_sn(bank_a)
    bank_a.refresh(update_u=True)
    bank_b.refresh(update_u=True)
    for step in range(4):
        for opt in (opt_a, opt_b):
            _grads(opt, 100 + step)
            opt.step(grad_scale=0.5 if not clip else 1.0, clip=clip)
        assert bank_a._p1_token is not None and bank_b._p1_token is None
        outs_a = bank_a.refresh(update_u=True)
        outs_b = bank_b.refresh(update_u=True)
        torch.cuda.synchronize()
        for x, y, what in ((opt_a.flat_param, opt_b.flat_param, 'param'), (opt_a.m, opt_b.m, 'm'),
                           (opt_a.v, opt_b.v, 'v')):
            assert torch.equal(x, y), (what, step)
        for i, (ea, eb) in enumerate(zip(bank_a.entries, bank_b.entries)):
            assert torch.equal(ea.u, eb.u), ('u', i, step)
            assert torch.equal(ea.v, eb.v), ('v', i, step)
            assert torch.equal(ea.sigma, eb.sigma), ('sigma', i, step)
            assert torch.equal(outs_a[i], outs_b[i]), ('W_eff', i, step)


def test_fused_refresh_vs_oracle(dev, monkeypatch):
    """After fused steps the refresh is still the oracle's power iteration on
    the updated weights from the u the previous refresh left."""
    mods, bank, opt = _net(dev, 8, 1)
    assert opt.attach_sn(bank)
    bank.refresh(update_u=True)
    for step in range(3):
        _grads(opt, 7 + step)
        opt.step()
        u0 = [e.u.cpu().numpy().astype(np.float64) for e in bank.entries]
        outs = bank.refresh(update_u=True)
        for i, (m, e) in enumerate(zip(mods, bank.entries)):
            W = m.weight.detach().cpu().numpy().astype(np.float64)
            sigma, u1, v1 = O.spectral_norm_rows(W, u0[i], 1)
            np.testing.assert_allclose(e.sigma.item(), sigma, rtol=1e-4)
            np.testing.assert_allclose(e.u.cpu().numpy(), u1, rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(e.v.cpu().numpy(), v1, rtol=1e-4, atol=1e-6)
            weff = W / sigma
            np.testing.assert_allclose(outs[i].detach().cpu().numpy(), weff, rtol=1e-4,
                                       atol=1e-6 * np.abs(weff).max())


def test_torch_write_between_step_and_refresh(dev, monkeypatch):
    """A weight or u written through torch after the fused step (a checkpoint
    load, a manual edit) bumps its version: the refresh recomputes the pass
    instead of using the partials of the old weights."""
    mods, bank, opt = _net(dev, 11, 1)
    assert opt.attach_sn(bank)
    bank.refresh(update_u=True)
    for edit in ('weight', 'u'):
        _grads(opt, 3)
        opt.step()
        with torch.no_grad():
            if edit == 'weight':
                mods[3].weight.mul_(-1.5)
            else:
                bank.entries[3].u.copy_(torch.randn_like(bank.entries[3].u))
        u0 = bank.entries[3].u.cpu().numpy().astype(np.float64)
        bank.refresh(update_u=True)
        W = mods[3].weight.detach().cpu().numpy().astype(np.float64)
        sigma, u1, _ = O.spectral_norm_rows(W, u0, 1)
        np.testing.assert_allclose(bank.entries[3].sigma.item(), sigma, rtol=1e-4)
        np.testing.assert_allclose(bank.entries[3].u.cpu().numpy(), u1, rtol=1e-4, atol=1e-6)


def test_attach_rejects_foreign_weights(dev, monkeypatch):
    from gan.core.optim import FlatAdam
    _, bank, opt = _net(dev, 2, 1)
    other = FlatAdam([torch.nn.Parameter(torch.zeros(8, device=dev))], 1e-3)
    assert not other.attach_sn(bank)
    monkeypatch.setenv('SMMD_SN_FUSE_P1', '0')
    assert not opt.attach_sn(bank)
