"""The residual shortcuts' 1x1 convolutions on the library (`smmd_conv1x1*`,
csrc/smmd_conv1x1.hip, ABI 11; LDS-DMA forms since r15): forward (+ bias), input gradient and weight
gradient against torch's float64 convolutions at the SNResNet-64 critic's and
generator's shortcut shapes and smaller ones (one image per column tile, tiles
across images, many weight-gradient slices), the convops dispatch (MIOpen not
called for them), and the double backward through convops' conv node."""
import pytest

torch = pytest.importorskip('torch')
import torch.nn.functional as F  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'

# (N, C, K, H): x [N, C, H, H], W [K, C, 1, 1]
SHAPES = [(64, 64, 128, 32), (64, 128, 256, 16), (64, 256, 512, 8), (64, 512, 1024, 4),
          (64, 1024, 512, 4), (4, 64, 64, 4), (2, 128, 192, 8), (3, 64, 64, 16),
          # pixels per image dividing a 32-column chunk (the LDS-DMA weight
          # gradient spans images), and neither dividing nor a multiple of it
          # (the register-staged weight gradient)
          (32, 512, 1024, 2), (64, 128, 256, 6)]


def _ref(x, w, b, gy):
    xd, wd, gd = x.double(), w.double(), gy.double()
    y = F.conv2d(xd, wd, None if b is None else b.double())
    gx = torch.nn.grad.conv2d_input(x.shape, wd, gd)
    gw = torch.nn.grad.conv2d_weight(xd, w.shape, gd)
    return y, gx, gw


def _close(a, ref, tol, what):
    err = float((a.double() - ref).abs().max())
    scale = float(ref.abs().max()) + 1e-30
    assert err <= tol * scale, '%s: max err %.3g of max %.3g' % (what, err, scale)


@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('bias', [False, True])
def test_conv1x1_vs_float64(shape, bias):
    from gan.core import convops
    N, C, K, H = shape
    g = torch.Generator(device=DEV).manual_seed(N * 7 + C + K + H)
    x = torch.randn(N, C, H, H, device=DEV, generator=g)
    w = torch.randn(K, C, 1, 1, device=DEV, generator=g) * 0.05
    b = torch.randn(K, device=DEV, generator=g) if bias else None
    gy = torch.randn(N, K, H, H, device=DEV, generator=g)
    assert convops._is_c1(x, w, [1, 1], [0, 0])
    y = convops._c1_fwd(x, w, b)
    gx = convops._c1_dx(gy, w)
    gw = convops._c1_wgrad(gy, x)
    assert y is not None and gx is not None and gw is not None
    yr, gxr, gwr = _ref(x, w, b, gy)
    _close(y, yr, 2e-6, 'forward')
    _close(gx, gxr, 2e-6, 'input gradient')
    _close(gw, gwr, 1e-5, 'weight gradient')        # sums over N H W terms
    # deterministic
    assert torch.equal(convops._c1_wgrad(gy, x), gw)
    assert torch.equal(convops._c1_fwd(x, w, b), y)


def test_conv1x1_routes_to_library():
    """conv2d with a 1x1 weight: forward, input and weight gradient on the
    library (timing keys), none through MIOpen's convolution."""
    from gan.core import _lib, convops
    x = torch.randn(8, 64, 8, 8, device=DEV, requires_grad=True)
    w = torch.randn(128, 64, 1, 1, device=DEV, requires_grad=True)
    _lib.reset_timing()
    _lib.enable_timing(True)
    try:
        y = convops.conv2d(x, w)
        y.square().sum().backward()
    finally:
        _lib.enable_timing(False)
    tm = _lib.timing_ms()
    assert tm['smmd_conv1x1'][0] == 2 and tm['smmd_conv1x1_wgrad'][0] == 1


def test_conv1x1_double_backward_vs_float64():
    """The scaling regulariser's pattern through convops' conv node: the
    input-gradient pass with create_graph, then the gradient of its squared
    norm w.r.t. the weight and the input, against float64 autograd."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(3)
    x0 = torch.randn(4, 64, 8, 8, device=DEV, generator=g)
    w0 = torch.randn(128, 64, 1, 1, device=DEV, generator=g) * 0.1

    def run(conv, x0, w0):
        x = x0.clone().requires_grad_(True)
        w = w0.clone().requires_grad_(True)
        y = conv(x, w)
        jx, = torch.autograd.grad(y.tanh().sum(), x, create_graph=True)
        loss = jx.square().sum()
        return torch.autograd.grad(loss, (x, w))

    got = run(lambda x, w: convops.conv2d(x, w), x0, w0)
    ref = run(lambda x, w: F.conv2d(x, w), x0.double(), w0.double())
    for a, r, what in zip(got, ref, ('dx', 'dw')):
        _close(a, r, 1e-5, what)


@pytest.mark.parametrize('N,C,K,H', [(64, 64, 128, 32), (64, 512, 1024, 4), (64, 128, 256, 16),
                                     (4, 256, 512, 8), (4, 64, 128, 4)])
def test_transposed_weight_gemm_equals_copy(N, C, K, H):
    """smmd_conv1x1_t (ABI 16: the input gradient straight from W [K, C]) is
    bit-identical to smmd_conv1x1 on the W^T copy, split-K slabs included."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(N + C + K + H)
    w = torch.randn(K, C, 1, 1, device=DEV, generator=g) * 0.05
    gy = torch.randn(N, K, H, H, device=DEV, generator=g)
    wm = w.reshape(K, C)
    a = convops._c1_gemm(wm, gy, None, C, ta=True)
    b = convops._c1_gemm(wm.t().contiguous(), gy, None, C)
    assert a is not None and b is not None
    assert torch.equal(a, b)
    ref = torch.nn.functional.conv_transpose2d(gy.double(), w.double())
    err = float((a.double() - ref).abs().max())
    assert err <= 2e-6 * float(ref.abs().max()) + 1e-30


@pytest.mark.parametrize('N,H', [(6, 4), (8, 2), (2, 4)])
def test_bwd_into_partial_library_shape_counts_dw_once(N, H):
    """N*H*W % 64 == 32: the weight gradient tiles on the library (32-column
    chunks) but the input-gradient GEMM (64-column tiles) does not.  `_bwd`
    with gw_into must return base + dW, not base + 2 dW (the *_wgrad_acc
    kernel's sum must not be followed by aten's dW of the same term), and
    aten's dx alone."""
    from gan.core import _lib, convops
    C, K = 64, 128
    L = _lib.lib()
    assert L.smmd_conv1x1_wgrad_supported(N, C, K, H * H)
    assert not L.smmd_conv1x1_supported(N, K, C, H * H)
    g = torch.Generator(device=DEV).manual_seed(N * 31 + H)
    x = torch.randn(N, C, H, H, device=DEV, generator=g)
    w = torch.randn(K, C, 1, 1, device=DEV, generator=g) * 0.05
    gy = torch.randn(N, K, H, H, device=DEV, generator=g)
    base = torch.randn(K, C, 1, 1, device=DEV, generator=g)
    into = base.clone()
    gx, gw = convops._bwd(gy, x, w, [1, 1], [0, 0], (True, True), gw_into=into)
    _, gxr, gwr = _ref(x, w, None, gy)
    _close(gx, gxr, 2e-6, 'input gradient')
    _close(gw - base, gwr, 1e-5, 'accumulated weight gradient')
    # without `into` the same shape gives the plain dW
    gx2, gw2 = convops._bwd(gy, x, w, [1, 1], [0, 0], (True, True))
    _close(gw2, gwr, 1e-5, 'weight gradient')
    assert torch.equal(gx2, gx)
