"""Thin 3x3 convolutions on the GPU (`smmd_conv3x3_thin*`, csrc/smmd_thin.hip):
the critics' 3-channel input conv and the generators' 3-channel output layer
(snops.conv2d / snops.deconv2d at stride 1 SAME, gan/core/snops.py:69-90,
:109-121), their input gradient (mode 1) and weight gradient, against the
oracle's TF-SAME ops (oracle/ref_nets.py conv2d_same / deconv2d_same) and
torch's float64 conv gradients on the same fp32 inputs; then through
convops' autograd to second order (the scaling regulariser's double backward)
against the MIOpen path.  Tolerance: |d| <= 1e-5 * sum_terms |a x| per output
(the float64 op on |a|, |x|), an fp32-accumulation bound."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

from oracle import ref_nets as R  # noqa: E402

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'

# (N, ci, co, H, W): thin input side, thin output side, the configs' shapes
SHAPES = [(64, 3, 64, 64, 64), (64, 3, 64, 32, 32), (5, 3, 16, 13, 17), (4, 1, 8, 7, 64),
          (3, 4, 5, 9, 33), (2, 2, 3, 1, 1),
          (64, 64, 3, 64, 64), (64, 64, 3, 32, 32), (5, 16, 3, 13, 17), (3, 37, 2, 5, 64),
          (2, 7, 4, 6, 1), (1, 300, 1, 3, 4),
          # a 4-channel thin side at W % 4 == 0 (9 * 4 taps > one 32-column MFMA tile)
          (4, 4, 64, 32, 32), (4, 64, 4, 32, 32)]


def _data(N, ci, co, H, W, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, ci, H, W, generator=g)
    w = torch.randn(co, ci, 3, 3, generator=g) * 0.2
    b = torch.randn(co, generator=g)
    gy = torch.randn(N, co, H, W, generator=g)
    return x, w, b, gy


def _check(got, ref, absum, k=1e-5):
    got = got.double().cpu()
    err = (got - ref).abs()
    lim = k * absum + 1e-30
    bad = (err > lim).sum().item()
    assert bad == 0, 'max err %.3e, max ratio %.3f' % (err.max().item(),
                                                        (err / lim).max().item())


@pytest.mark.parametrize('N,ci,co,H,W', SHAPES)
def test_thin_forward_matches_oracle(N, ci, co, H, W):
    from gan.core import convops
    x, w, b, _ = _data(N, ci, co, H, W, 11 + ci + co)
    y = convops._thin_conv(x.to(DEV), w.to(DEV), b.to(DEV), 0)
    hwio = w.double().permute(2, 3, 1, 0)
    ref = R.conv2d_same(x.double(), hwio, b.double(), 1)
    absum = R.conv2d_same(x.double().abs(), hwio.abs(), b.double().abs(), 1)
    assert y.shape == (N, co, H, W)
    _check(y, ref, absum)


@pytest.mark.parametrize('N,ci,co,H,W', SHAPES)
def test_thin_input_gradient_matches_torch(N, ci, co, H, W):
    """mode 1: gx = Dx(gy, w) of y = conv(x, w), i.e. conv2d_transpose."""
    from gan.core import convops
    x, w, _, gy = _data(N, ci, co, H, W, 23 + ci + co)
    gx = convops._thin_conv(gy.to(DEV), w.to(DEV), None, 1)
    ref = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), padding=1)
    absum = torch.nn.grad.conv2d_input(x.shape, w.double().abs(), gy.double().abs(), padding=1)
    assert gx.shape == x.shape
    _check(gx, ref, absum)
    # the same op as the oracle's TF SAME conv2d_transpose (w as [kh, kw, out, in])
    tf = R.deconv2d_same(gy.double(), w.double().permute(2, 3, 1, 0), None, (H, W), 1)
    assert torch.allclose(ref, tf, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize('N,ci,co,H,W', SHAPES)
def test_thin_weight_gradient_matches_torch(N, ci, co, H, W):
    from gan.core import convops
    x, w, _, gy = _data(N, ci, co, H, W, 37 + ci + co)
    gw = convops._thin_wgrad(gy.to(DEV), x.to(DEV))
    ref = torch.nn.grad.conv2d_weight(x.double(), w.shape, gy.double(), padding=1)
    absum = torch.nn.grad.conv2d_weight(x.double().abs(), w.shape, gy.double().abs(), padding=1)
    assert gw.shape == w.shape
    _check(gw, ref, absum)


def test_thin_kernels_deterministic():
    from gan.core import convops
    x, w, b, gy = [t.to(DEV) for t in _data(64, 3, 64, 64, 64, 5)]
    a = [convops._thin_conv(x, w, b, 0), convops._thin_conv(gy, w, None, 1),
         convops._thin_wgrad(gy, x)]
    c = [convops._thin_conv(x, w, b, 0), convops._thin_conv(gy, w, None, 1),
         convops._thin_wgrad(gy, x)]
    for u, v in zip(a, c):
        assert torch.equal(u, v)


def test_thin_rejects_unsupported():
    from gan.core import _lib
    L = _lib.lib()
    t = torch.zeros(4096, device=DEV)
    p = _lib.ptr(t)
    # both sides wide
    assert L.smmd_conv3x3_thin(p, p, None, p, 1, 8, 8, 4, 4, 0, None) == 4
    # a thin output side wider than one wave of columns
    assert L.smmd_conv3x3_thin(p, p, None, p, 1, 8, 3, 4, 65, 0, None) == 4
    assert L.smmd_conv3x3_thin_wgrad(p, p, p, 1, 3, 8, 4, 65, p, 4096 * 4, None) == 4
    # bad mode / negative sizes
    assert L.smmd_conv3x3_thin(p, p, None, p, 1, 3, 8, 4, 4, 2, None) == 1
    assert L.smmd_conv3x3_thin(p, p, None, p, -1, 3, 8, 4, 4, 0, None) == 1
    # workspace too small
    need = L.smmd_conv3x3_thin_wgrad_workspace_bytes(2, 3, 8, 4, 4)
    assert need == 2 * 1 * 8 * 3 * 9 * 4
    assert L.smmd_conv3x3_thin_wgrad(p, p, p, 2, 3, 8, 4, 4, p, need - 4, None) == 3
    torch.cuda.synchronize()


@pytest.mark.parametrize('ci,co', [(3, 64), (64, 3)])
def test_thin_conv_second_order_matches_miopen(ci, co):
    """convops.conv2d to second order (the Jacobian's double backward of the
    scaling regulariser) on the thin kernels vs the same graph on MIOpen."""
    from gan.core import convops
    N, H, W = 8, 16, 16
    x, w, b, _ = _data(N, ci, co, H, W, 3 + ci)

    def run(thin):
        old = convops.THIN
        convops.THIN = thin
        try:
            xx = x.to(DEV).requires_grad_(True)
            ww = w.to(DEV).requires_grad_(True)
            bb = b.to(DEV).requires_grad_(True)
            y = convops.conv2d(xx, ww, bb, 1, 1)
            f = torch.tanh(y).sum(dim=(1, 2, 3))
            jx, = torch.autograd.grad(f.sum(), xx, create_graph=True)
            loss = (jx * jx).sum() + (y * y).mean()
            gx, gw, gb = torch.autograd.grad(loss, (xx, ww, bb))
            return [t.detach().double().cpu() for t in (y, jx, gx, gw, gb)]
        finally:
            convops.THIN = old

    a, m = run(True), run(False)
    for u, v in zip(a, m):
        scale = v.abs().max().item() + 1e-12
        assert (u - v).abs().max().item() <= 2e-4 * scale


def test_deconv_stride1_routes_to_thin_and_matches_transpose():
    """Deconv2d(dim, 3, 3, 1) (the generators' output layer) = conv with the
    flipped, transposed filter on the thin kernels; equal to the oracle's TF
    SAME conv2d_transpose."""
    from gan.core.snops import Deconv2d
    torch.manual_seed(0)
    layer = Deconv2d(64, 3, 3, 1).to(DEV)
    with torch.no_grad():
        layer.bias.normal_()
    x = torch.randn(16, 64, 32, 32, device=DEV)
    y = layer(x)
    w = layer.weight.detach().double().cpu()           # [in, out, kh, kw]
    ref = R.deconv2d_same(x.double().cpu(), w.permute(2, 3, 1, 0), layer.bias.detach()
                          .double().cpu(), (32, 32), 1)
    absum = R.deconv2d_same(x.double().cpu().abs(), w.abs().permute(2, 3, 1, 0),
                            layer.bias.detach().double().cpu().abs(), (32, 32), 1)
    _check(y, ref, absum)
    # gradients reach the transposed-conv weight and bias
    y.square().sum().backward()
    assert layer.weight.grad is not None and layer.weight.grad.abs().sum() > 0
    assert layer.bias.grad is not None
