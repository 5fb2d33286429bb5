"""GPU parity of the polyphase Winograd F(2x2, 2x2) kernels for 4x4 stride-2
convolutions (csrc/smmd_wino_s2.hip, `smmd_wino4x4s2*`): the critics' folded
ConvMeanPool layers (gan/core/resnet/block.py:63-66) and their input gradient,
which also serves the generators' folded UpsampleConv (block.py:53-60), through
the C ABI and through convops' autograd rules, against float64 on the host.
Tolerance 2e-6 of max|ref| (measured 1-5e-7)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'
TOL = 2e-6


@pytest.fixture(autouse=True)
def s2_on():
    """The stride-2 kernels on for these tests, whatever SMMD_WINO_S2 says."""
    from gan.core import convops
    saved = convops.WINO_S2
    convops.WINO_S2 = True
    yield
    convops.WINO_S2 = saved


def _rel(a, ref):
    a = a.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return ((a - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()


# (N, C, K, H, W) of the stride-2 conv x [N, C, H, W] -> [N, K, H/2, W/2]:
# a 4 x 4 image, a row wider than a wave (W = 264: the edge kernels), a split
# reduction (C = 512), the SNResNet-64 critic's four fold layers at batch 4
SHAPES = [(2, 2, 64, 4, 4), (3, 8, 64, 8, 12), (2, 64, 128, 16, 16), (1, 64, 64, 4, 264),
          (4, 512, 64, 8, 8), (2, 6, 128, 12, 8), (4, 64, 128, 64, 64), (4, 128, 256, 32, 32),
          (4, 256, 512, 16, 16), (4, 512, 1024, 8, 8)]


@pytest.mark.parametrize('shape', SHAPES)
def test_s2_conv_and_transposed_vs_float64(shape):
    from gan.core import convops
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(N * 7 + C + K + H + W)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    w = torch.randn(K, C, 4, 4, device=DEV, generator=g)
    b = torch.randn(K, device=DEV, generator=g)
    assert convops._is_s2(x, w, 2, 1)
    y = convops._s2_conv(x, w, b)
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), stride=2, padding=1)
    assert _rel(y, ref) < TOL
    if C % 64 == 0:
        gy = torch.randn(N, K, H // 2, W // 2, device=DEV, generator=g)
        assert convops._is_s2t(gy, w, 2, 1)
        gx = convops._s2t_conv(gy, w, None)
        refx = torch.nn.grad.conv2d_input((N, C, H, W), w.double().cpu(), gy.double().cpu(),
                                          stride=2, padding=1)
        assert _rel(gx, refx) < TOL


@pytest.mark.parametrize('shape', [(2, 2, 64, 4, 4), (1, 64, 64, 4, 264), (4, 512, 64, 8, 8),
                                   (4, 64, 128, 64, 64), (4, 512, 1024, 8, 8)])
def test_s2_pair_conv_vs_float64(shape):
    """smmd_wino4x4s2_conv2: conv(x, w) + conv(x2, w2) (stride 2) in one launch
    against the float64 sum (edge kernel, split reductions over both inputs)."""
    from gan.core import convops
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(N + C + K + H + W)
    x, x2 = (torch.randn(N, C, H, W, device=DEV, generator=g) for _ in range(2))
    w, w2 = (torch.randn(K, C, 4, 4, device=DEV, generator=g) for _ in range(2))
    y = convops._fwd2(x, w, x2, w2, [2, 2], [1, 1])
    assert y is not None
    ref = (F.conv2d(x.double().cpu(), w.double().cpu(), stride=2, padding=1) +
           F.conv2d(x2.double().cpu(), w2.double().cpu(), stride=2, padding=1))
    assert _rel(y, ref) < TOL


@pytest.mark.parametrize('shape', [(2, 64, 64, 8, 8), (3, 128, 64, 12, 4), (4, 64, 64, 8, 8),
                                   (2, 32, 64, 32, 32)])
def test_s2_double_backward_vs_float64(shape):
    """The critic's ConvMeanPool conv through the double backward: conv, Dx,
    Dw and their second-order terms against float64 autograd."""
    from gan.core import convops
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(21)
    t = {k: torch.randn(*s, device=DEV, generator=g) for k, s in
         dict(x=(N, C, H, W), w=(K, C, 4, 4), b=(K,), A=(N, K, H // 2, W // 2),
              B=(N, C, H, W), D=(K, C, 4, 4)).items()}

    def run(dev, dtype, fn):
        v = {k: t[k].to(dev, dtype).requires_grad_(k in ('x', 'w', 'A')) for k in t}
        y = fn(v['x'], v['w'], v['b'])
        loss = (y * v['A']).sum()
        gx, gw = torch.autograd.grad(loss, (v['x'], v['w']), create_graph=True)
        second = (gx * v['B']).sum() + (gw * v['D']).sum()
        hx, hw, hA = torch.autograd.grad(second, (v['x'], v['w'], v['A']))
        return y, gx, gw, hx, hw, hA

    got = run(DEV, torch.float32, lambda x, w, b: convops.conv2d(x, w, b, 2, 1))
    ref = run('cpu', torch.float64, lambda x, w, b: F.conv2d(x, w, b, 2, 1))
    for n, a, r in zip(('y', 'gx', 'gw', 'hx', 'hw', 'hA'), got, ref):
        assert _rel(a, r) < (2e-5 if n in ('gw', 'hx', 'hw') else TOL), n


def test_conv_transpose_s2_autograd_vs_float64():
    """The generator's folded UpsampleConv: forward, grad_x (the stride-2
    conv kernel), grad_w and grad_b against float64."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(8)
    x = torch.randn(4, 128, 8, 8, device=DEV, generator=g)
    w = torch.randn(128, 64, 4, 4, device=DEV, generator=g)
    b = torch.randn(64, device=DEV, generator=g)
    A = torch.randn(4, 64, 16, 16, device=DEV, generator=g)
    outs = []
    for dev, dt, fn in ((DEV, torch.float32, convops.conv_transpose_s2),
                        ('cpu', torch.float64,
                         lambda x, w, b: F.conv_transpose2d(x, w, b, stride=2, padding=1))):
        xx, ww, bb = (t.to(dev, dt).requires_grad_(True) for t in (x, w, b))
        y = fn(xx, ww, bb)
        gx, gw, gb = torch.autograd.grad((y * A.to(dev, dt)).sum(), (xx, ww, bb))
        outs.append((y, gx, gw, gb))
    for n, a, r in zip(('y', 'gx', 'gw', 'gb'), *outs):
        assert _rel(a, r) < (2e-5 if n in ('gw', 'gb') else TOL), n


# the critic's four folded ConvMeanPool layers (SNResNet-64: 64 -> 128 at 64 x 64
# ... 512 -> 1024 at 8 x 8) at small batches, other tile grids, and shapes the
# kernel does not tile (MIOpen then): (x [n, ci, h, w], co)
S2_WGRAD_SHAPES = [(2, 64, 128, 64, 64), (2, 128, 256, 32, 32), (4, 256, 512, 16, 16),
                   (4, 512, 1024, 8, 8), (3, 16, 64, 32, 64), (2, 32, 64, 16, 32),
                   (8, 16, 64, 16, 16), (2, 64, 64, 8, 8), (1, 16, 64, 12, 20)]


@pytest.mark.parametrize('shape', S2_WGRAD_SHAPES)
def test_s2_wgrad_vs_float64(shape):
    """smmd_wino4x4s2_wgrad (through convops' dispatch) against torch's float64
    conv2d_weight: sums over N * H/2 * W/2 terms in fp32, bound 1e-5 of
    max|ref|; deterministic."""
    from gan.core import _lib, convops
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(N + C + K + H + W)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    gy = torch.randn(N, K, H // 2, W // 2, device=DEV, generator=g)
    w = torch.empty(K, C, 4, 4, device=DEV)
    tiled = convops._s2_wgrad_ok(x, gy, K)
    assert tiled == bool(_lib.lib().smmd_wino4x4s2_wgrad_supported(N, C, K, H, W))
    gw = convops._s2_weight_grad(gy, x, w, [2, 2], [1, 1])
    ref = torch.nn.grad.conv2d_weight(x.double().cpu(), (K, C, 4, 4), gy.double().cpu(),
                                      stride=2, padding=1)
    assert _rel(gw, ref) < 1e-5
    if tiled:
        assert torch.equal(gw, convops._s2_weight_grad(gy, x, w, [2, 2], [1, 1]))


def test_s2_wgrad_routes_to_library():
    from gan.core import _lib, convops
    x = torch.randn(2, 64, 32, 32, device=DEV)
    gy = torch.randn(2, 128, 16, 16, device=DEV)
    _lib.reset_timing()
    _lib.enable_timing(True)
    try:
        convops._s2_weight_grad(gy, x, torch.empty(128, 64, 4, 4, device=DEV), [2, 2], [1, 1])
        assert 'smmd_wino4x4s2_wgrad' in _lib.timing_ms()
    finally:
        _lib.enable_timing(False)
        _lib.reset_timing()


def test_s2_off_matches_on():
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(8, 128, 32, 32, device=DEV, generator=g)
    w = torch.randn(256, 128, 4, 4, device=DEV, generator=g) / 45.0
    y1 = convops.conv2d(x, w, None, 2, 1)
    saved = convops.WINO_S2
    convops.WINO_S2 = False
    try:
        y0 = convops.conv2d(x, w, None, 2, 1)
    finally:
        convops.WINO_S2 = saved
    assert _rel(y1, y0) < 5e-6
