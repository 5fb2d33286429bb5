"""The reference's model hooks on the trainer, twice: on the CPU with the
library replaced by the oracle (tests/fake_lib.py), and on the GPU through
libsmmd_hip (the `gpu`-marked parameter).

Reference: MMD_GAN.set_loss / add_gradient_penalty / add_l2_penalty /
add_scaling (gan/core/model.py:313-403), SMMD.set_loss / apply_scaling
(gan/core/smmd.py:10-23), SWGAN (smmd.py:26-42).  A subclass overriding only
``apply_scaling(scale)`` must train and see the scale the reference computes.
"""
import argparse
import os
import sys

import numpy as np
import pytest

torch = pytest.importorskip('torch')

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


DEV = ['cpu']


@pytest.fixture(params=['cpu', pytest.param('cuda', marks=pytest.mark.gpu)])
def fake(request, monkeypatch):
    """'cpu': the oracle stands in for the library; 'cuda': the real HIP path."""
    if request.param == 'cuda':
        if not torch.cuda.is_available():
            pytest.skip('no GPU')
        monkeypatch.setattr(sys.modules[__name__], 'DEV', ['cuda'])
        return None
    import fake_lib
    from gan.core import _lib
    f = fake_lib.FakeLib()
    monkeypatch.setattr(_lib, '_lib', f)
    monkeypatch.setattr(_lib, 'lib', lambda: f)
    monkeypatch.setattr(_lib, 'require_cuda', lambda *t: None)
    monkeypatch.setattr(_lib, 'stream_handle', lambda device=None: None)
    monkeypatch.setattr(_lib, 'workspace', lambda tag, nbytes, device: torch.zeros(
        max(int(nbytes), 256), dtype=torch.uint8))
    return f


def cfg(**kw):
    from gan.main import default_flags
    c = default_flags()
    c.update(dict(batch_size=6, output_size=16, architecture='dcgan', kernel='rbf',
                  model='smmd', batch_norm=False, with_sn=False, with_scaling=True,
                  dof_dim=1, df_dim=4, gf_dim=4, learning_rate=1e-4, dataset='cifar10'))
    c.update(kw)
    return argparse.Namespace(**c)


def build(cls, c, seed=0):
    """The model on the CPU; critic weights x8 so that the scale is far from 1
    (the 0.02-std init gives J ~ 1e-11 on this tiny critic)."""
    torch.manual_seed(seed)
    m = cls(c, device=torch.device(DEV[0]))
    with torch.no_grad():
        for p in m.d_vars:
            p.mul_(8.0)
    return m


def one_critic_loss(model, seed=1, need=True):
    g = torch.Generator().manual_seed(seed)
    images = torch.rand(6, 3, 16, 16, generator=g).to(DEV[0])
    z = torch.empty(6, model.z_dim).uniform_(-1, 1, generator=g).to(DEV[0])
    with torch.no_grad():
        fake = model.generator(z)
    model.d_optim.zero_grad()
    g_loss, d_loss, aux = model.set_tower_loss(images, fake, need_critic_grad=need)
    return g_loss, d_loss, images, fake


def critic_grads(model, d_loss):
    grads = torch.autograd.grad(d_loss, model.d_vars, allow_unused=True)
    return [torch.zeros_like(p) if g is None else g for p, g in zip(model.d_vars, grads)]


def test_apply_scaling_override_matches_fused(fake):
    from gan.core.smmd import SMMD

    class Unfused(SMMD):
        def apply_scaling(self, scale):
            self.seen_scale = scale
            self.g_loss = self.g_loss * scale
            self.d_loss = -self.g_loss

    a, b = build(SMMD, cfg()), build(Unfused, cfg())
    assert a._fused_scaling() == 'mul' and b._fused_scaling() is None
    ga, da, *_ = one_critic_loss(a)
    gb, db, *_ = one_critic_loss(b)
    # SMMD's own apply_scaling: mmd2 and the scaled loss in one launch
    # (smmd_smmd_loss_fwd); the override: mmd2, then scale, then its product
    assert a.fused_loss and not b.fused_loss
    assert float(gb) == pytest.approx(float(ga), rel=1e-6, abs=1e-9)
    assert float(b.seen_scale) == pytest.approx(float(a.aux[2]), rel=1e-6)
    for x, y in zip(critic_grads(a, da), critic_grads(b, db)):
        np.testing.assert_allclose(y.cpu().numpy(), x.cpu().numpy(), rtol=1e-4,
                                   atol=1e-5 * float(x.abs().max()) + 1e-12)


def test_swgan_override_matches_fused(fake):
    from gan.core.smmd import SWGAN

    class Unfused(SWGAN):
        def apply_scaling(self, scale):
            self.g_loss = self.g_loss * torch.sqrt(scale)
            self.d_loss = -self.g_loss

    c = cfg(model='swgan')
    a, b = build(SWGAN, c), build(Unfused, cfg(model='swgan'))
    ga, da, *_ = one_critic_loss(a)
    gb, db, *_ = one_critic_loss(b)
    assert float(gb) == pytest.approx(float(ga), rel=1e-6, abs=1e-9)
    for x, y in zip(critic_grads(a, da), critic_grads(b, db)):
        np.testing.assert_allclose(y.cpu().numpy(), x.cpu().numpy(), rtol=1e-4,
                                   atol=1e-5 * float(x.abs().max()) + 1e-12)


def test_custom_apply_scaling_trains_with_reference_scale(fake):
    """Only apply_scaling overridden (as SWGAN does): the hook receives the
    reference's scale 1/(sc J + 1) and its loss drives the update."""
    from gan.core.smmd import SMMD
    from oracle import smmd_oracle as O

    class Squared(SMMD):
        def apply_scaling(self, scale):
            self.seen = scale
            self.g_loss = self.g_loss * scale * scale
            self.d_loss = -self.g_loss

    m = build(Squared, cfg())
    g_loss, d_loss, images, fake_imgs = one_critic_loss(m)
    # J from plain autograd on the same critic
    x = images.clone().requires_grad_(True)
    gx, = torch.autograd.grad(m.discriminator(x).sum(), x)
    J = float((gx.double() ** 2).sum(dim=(1, 2, 3)).mean())
    assert float(m.seen) == pytest.approx(O.scale_factor(J, 10.0), rel=1e-5)
    base = g_loss / m.seen ** 2
    assert float(g_loss) == pytest.approx(float(base) * float(m.seen) ** 2, rel=1e-6)
    before = m.d_optim.flat_param.clone()
    for _ in range(3):
        m.train_step(images)
    assert np.isfinite(m.check_finite()).all()
    assert not torch.equal(before, m.d_optim.flat_param)


def test_gaussian_noise_scaling(fake):
    """use_gaussian_noise (model.py:367-370): J is taken at N(0, 10^2) inputs
    through one more critic call, not at the real batch."""
    from gan.core.smmd import SMMD
    from oracle import smmd_oracle as O

    class Probe(SMMD):
        def apply_scaling(self, scale):
            self.seen = scale
            super().apply_scaling(scale)

    m = build(Probe, cfg(use_gaussian_noise=True))
    torch.manual_seed(7)
    calls = []
    orig = m.discriminator.forward

    def fwd(x, *a, **k):
        calls.append(x)
        return orig(x, *a, **k)
    m.discriminator.forward = fwd
    g_loss, d_loss, images, _ = one_critic_loss(m)
    assert len(calls) == 3                       # real, fake, noise
    noise = calls[2].detach()
    assert 5.0 < float(noise.std()) < 20.0
    x = noise.clone().requires_grad_(True)
    gx, = torch.autograd.grad(orig(x).sum(), x)
    J = float((gx.double() ** 2).sum(dim=(1, 2, 3)).mean())
    assert float(m.seen) == pytest.approx(O.scale_factor(J, 10.0), rel=1e-5)
    # the real batch's Jacobian gives a different scale
    xr = images.clone().requires_grad_(True)
    gr, = torch.autograd.grad(orig(xr).sum(), xr)
    Jr = float((gr.double() ** 2).sum(dim=(1, 2, 3)).mean())
    assert abs(O.scale_factor(Jr, 10.0) - float(m.seen)) > 1e-6 * O.scale_factor(Jr, 10.0)
    critic_grads(m, d_loss)                      # differentiable through the noise call


def test_l2_discriminator_penalty(fake):
    """add_l2_penalty (model.py:352-364)."""
    from gan.core.smmd import get_model
    coeff = 0.01
    c = cfg(model='mmd', with_scaling=False, L2_discriminator_penalty=coeff)
    m = build(get_model('mmd'), c)
    g_loss, d_loss, images, fake_imgs = one_critic_loss(m)
    pen = 0.0
    for x in (fake_imgs, images):
        for layer in m.discriminator(x, return_layers=True).values():
            pen = pen + (layer.double() ** 2).reshape(layer.shape[0], -1).mean(1)
    expect = -float(g_loss) + coeff * float(pen.mean())
    assert float(d_loss) == pytest.approx(expect, rel=1e-5)
    assert 'L2 dp' in m.optim_name
    critic_grads(m, d_loss)
    # without the penalty d_loss = -g_loss exactly
    m2 = build(get_model('mmd'), cfg(model='mmd', with_scaling=False))
    g2, d2, *_ = one_critic_loss(m2)
    assert float(d2) == -float(g2)


def test_set_loss_override_sees_reference_attributes(fake):
    """A subclass replacing set_loss (as SMMD / SWGAN do) gets the critic
    outputs as arguments and the reference's attributes on self."""
    from gan.core import mmd
    from gan.core.smmd import SMMD

    class Custom(SMMD):
        def set_loss(self, G, images):
            assert G is self.d_G and images is self.d_images
            assert self.images.shape == self.G.shape
            kernel = getattr(mmd, '_%s_kernel' % self.config.kernel)
            self.g_loss = mmd.mmd2(kernel(G, images), biased=True)
            self.d_loss = -self.g_loss
            self.add_scaling()

    m = build(Custom, cfg())
    g_loss, d_loss, *_ = one_critic_loss(m)
    assert np.isfinite(float(g_loss)) and float(d_loss) == -float(g_loss)


def test_kernel_spec_roundtrip():
    from gan.core import mmd
    for name in mmd.KERNEL_NAMES:
        fn = mmd.get_kernel(name)
        assert mmd.spec_of(fn) == mmd.get_kernel_spec(name)
    assert mmd.spec_of(lambda X, Y, K_XY_only=False: None) is None
