"""GPU parity of the fused Winograd F(2x2, 3x3) MFMA convolution
(csrc/smmd_wino.hip, `smmd_wino3x3_*`): the wide 3x3 stride-1 SAME layers of
the critics and generators (gan/core/resnet/block.py:38-50, snops.py:69-90),
forward and input gradient, through the C ABI and through convops' autograd
rules (first and second order), against float64 convolutions on the host.

Tolerance: Winograd reorders the sums (input / filter / output transforms in
fp32 around exact-f32 MFMA fma chains); the measured error is 1-10e-7 of the
output's max, the bound 2e-6 of max|ref|."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'
TOL = 2e-6


def _rel(a, ref):
    a = a.detach().double().cpu()
    ref = ref.detach().double().cpu()
    return ((a - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()


def _abi_conv(x, w, b, mode):
    from gan.core import _lib
    L = _lib.lib()
    N, C, H, W = x.shape
    K = w.shape[0] if mode == 0 else w.shape[1]
    u = torch.empty(L.smmd_wino3x3_filter_bytes(K, C) // 4, device=DEV)
    st = L.smmd_wino3x3_filter(_lib.ptr(w), K, C, mode, _lib.ptr(u), u.numel() * 4,
                               _lib.stream_handle())
    assert st == 0
    y = torch.empty(N, K, H, W, device=DEV)
    nb = L.smmd_wino3x3_workspace_bytes(N, C, K, H, W)
    ws = torch.empty(max(nb // 4, 1), device=DEV)
    st = L.smmd_wino3x3_conv(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, C, K, H, W,
                             _lib.ptr(ws) if nb else None, nb, _lib.stream_handle())
    assert st == 0
    return y, nb


# (N, C, K, H, W): odd tile counts, a row wider than a wave (W = 130: the edge
# kernel), split input channels (512 -> 64 at 8 x 8), a 2 x 2 image, the
# SNResNet-64 critic's four 3x3 layers at a small batch
SHAPES = [(2, 8, 64, 6, 6), (1, 16, 64, 4, 10), (3, 64, 128, 8, 8), (2, 8, 64, 2, 2),
          (1, 8, 64, 130, 4), (1, 8, 64, 4, 130), (4, 512, 64, 8, 8), (2, 256, 128, 4, 6),
          (4, 64, 64, 64, 64), (4, 128, 128, 32, 32), (4, 256, 256, 16, 16), (8, 512, 512, 8, 8)]


@pytest.mark.parametrize('shape', SHAPES)
def test_wino_forward_and_input_grad_vs_float64(shape):
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(N * 1000 + C + K + H * 7 + W)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    w = torch.randn(K, C, 3, 3, device=DEV, generator=g)
    b = torch.randn(K, device=DEV, generator=g)
    y, _ = _abi_conv(x, w, b, 0)
    ref = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
    assert _rel(y, ref) < TOL
    # mode 1: the input gradient of a conv with weight w2 [C, K, 3, 3] at upstream x
    w2 = torch.randn(C, K, 3, 3, device=DEV, generator=g)
    gx, _ = _abi_conv(x, w2, None, 1)
    ref1 = torch.nn.grad.conv2d_input((N, K, H, W), w2.double().cpu(), x.double().cpu(),
                                      padding=1)
    assert _rel(gx, ref1) < TOL


@pytest.mark.parametrize('shape', SHAPES)
def test_wino_eight_wave_form_bit_identical(shape, monkeypatch):
    """The 8-wave kernel (two waves per SIMD splitting the 16 points) and the
    4-wave one accumulate every point in the same order and share the output
    transform's arithmetic: the same bits, both modes, relu too."""
    from gan.core import _lib
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(N * 31 + C + K + H + W)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    w = torch.randn(K, C, 3, 3, device=DEV, generator=g)
    b = torch.randn(K, device=DEV, generator=g)
    out = {}
    for form in ('0', '1'):
        monkeypatch.setenv('SMMD_WINO8', form)
        y0, _ = _abi_conv(x, w, b, 0)
        y1, _ = _abi_conv(x, w.transpose(0, 1).contiguous(), None, 1) if C == K else (None, 0)
        L = _lib.lib()
        u = torch.empty(L.smmd_wino3x3_filter_bytes(K, C) // 4, device=DEV)
        assert L.smmd_wino3x3_filter(_lib.ptr(w), K, C, 0, _lib.ptr(u), u.numel() * 4,
                                     _lib.stream_handle()) == 0
        yr = torch.empty(N, K, H, W, device=DEV)
        nb = L.smmd_wino3x3_workspace_bytes(N, C, K, H, W)
        ws = torch.empty(max(nb // 4, 1), device=DEV)
        assert L.smmd_wino3x3_conv_relu(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(yr), N, C,
                                        K, H, W, _lib.ptr(ws) if nb else None, nb,
                                        _lib.stream_handle()) == 0
        out[form] = (y0, y1, yr)
    monkeypatch.delenv('SMMD_WINO8')
    for a, c in zip(out['0'], out['1']):
        if a is not None:
            assert torch.equal(a, c)
    assert (out['1'][2] >= 0).all()


def test_wino_split_channels_deterministic():
    """The split-input-channel path (workspace + fixed-order add) gives the
    same bits run to run."""
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(16, 512, 8, 8, device=DEV, generator=g)
    w = torch.randn(512, 512, 3, 3, device=DEV, generator=g)
    y0, nb = _abi_conv(x, w, None, 0)
    assert nb > 0
    y1, _ = _abi_conv(x, w, None, 0)
    assert torch.equal(y0, y1)


def test_convops_routes_wide_3x3_to_wino():
    from gan.core import _lib, convops
    x = torch.randn(2, 64, 8, 8, device=DEV)
    w = torch.randn(64, 64, 3, 3, device=DEV)
    assert convops.wino_applicable(x, 64, 64, 3, 1, 1)
    assert not convops.wino_applicable(x, 64, 64, 3, 2, 1)
    assert not convops.wino_applicable(x.to(memory_format=torch.channels_last), 64, 64, 3, 1, 1)
    _lib.reset_timing()
    _lib.enable_timing(True)
    try:
        convops.conv2d(x, w, None, 1, 1)
        assert 'smmd_wino3x3_conv' in _lib.timing_ms()
    finally:
        _lib.enable_timing(False)
        _lib.reset_timing()


@pytest.mark.parametrize('shape', [(2, 64, 64, 8, 8), (3, 128, 64, 6, 4)])
def test_convops_wino_double_backward_vs_float64(shape):
    """loss = <conv(x, w) + b, A>; first-order gx, gw with create_graph, then
    the gradient of <gx, B> + <gw, D> w.r.t. x, w and A: every conv of the
    critic's double backward (conv, Dx, Dw and their second-order terms) on
    the same inputs as float64 autograd on the host."""
    from gan.core import convops
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(11)
    t = {k: torch.randn(*s, device=DEV, generator=g) for k, s in
         dict(x=(N, C, H, W), w=(K, C, 3, 3), b=(K,), A=(N, K, H, W), B=(N, C, H, W),
              D=(K, C, 3, 3)).items()}

    def run(dev, dtype, fn):
        v = {k: t[k].to(dev, dtype).requires_grad_(k in ('x', 'w', 'A')) for k in t}
        y = fn(v['x'], v['w'], v['b'])
        loss = (y * v['A']).sum()
        gx, gw = torch.autograd.grad(loss, (v['x'], v['w']), create_graph=True)
        second = (gx * v['B']).sum() + (gw * v['D']).sum()
        hx, hw, hA = torch.autograd.grad(second, (v['x'], v['w'], v['A']))
        return y, gx, gw, hx, hw, hA

    got = run(DEV, torch.float32, lambda x, w, b: convops.conv2d(x, w, b, 1, 1))
    ref = run('cpu', torch.float64, lambda x, w, b: F.conv2d(x, w, b, 1, 1))
    names = ('y', 'gx', 'gw', 'hx', 'hw', 'hA')
    for n, a, r in zip(names, got, ref):
        if r is None or (r.abs().max() == 0):
            continue
        # gw / hw are MIOpen weight gradients (fp32 sums over N*H*W terms)
        assert _rel(a, r) < (2e-5 if n in ('gw', 'hx', 'hw') else TOL), n


# the pair form: odd tiles, the edge kernel, split reductions over the two
# inputs (512 -> 64 at 8 x 8; 64 -> 64 at batch 1), the critic's layers
PAIR_SHAPES = [(2, 8, 64, 6, 6), (1, 8, 64, 4, 130), (4, 512, 64, 8, 8), (1, 64, 64, 8, 8),
               (3, 128, 128, 32, 32), (2, 256, 256, 16, 16)]


@pytest.mark.parametrize('shape', PAIR_SHAPES)
def test_wino_pair_conv_vs_float64(shape):
    """smmd_wino3x3_conv2: conv(x, w) + conv(x2, w2) in one launch against the
    float64 sum of the two convolutions, through convops (the double
    backward's conv(ggx, w) + conv(x, ggw))."""
    from gan.core import convops
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(N + C + K + H + W)
    x, x2 = (torch.randn(N, C, H, W, device=DEV, generator=g) for _ in range(2))
    w, w2 = (torch.randn(K, C, 3, 3, device=DEV, generator=g) for _ in range(2))
    y = convops._fwd2(x, w, x2, w2, [1, 1], [1, 1])
    assert y is not None
    ref = (F.conv2d(x.double().cpu(), w.double().cpu(), padding=1) +
           F.conv2d(x2.double().cpu(), w2.double().cpu(), padding=1))
    assert _rel(y, ref) < TOL
    assert torch.equal(y, convops._fwd2(x, w, x2, w2, [1, 1], [1, 1]))    # deterministic


def test_wino_pair_off_matches_on(monkeypatch):
    """SMMD_CONV_PAIR=0 (two launches and an add) agrees with the pair launch
    through a critic-shaped double backward."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(4, 128, 16, 16, device=DEV, generator=g, requires_grad=True)
    w = (torch.randn(128, 128, 3, 3, device=DEV, generator=g) / 34.0).requires_grad_(True)
    A = torch.randn(4, 128, 16, 16, device=DEV, generator=g, requires_grad=True)
    B = torch.randn(4, 128, 16, 16, device=DEV, generator=g)
    D = torch.randn(128, 128, 3, 3, device=DEV, generator=g)
    res = []
    for on in (True, False):
        monkeypatch.setattr(convops, 'CONV_PAIR', on)
        y = convops.conv2d(x, w, None, 1, 1)
        gx, gw = torch.autograd.grad((y * A).sum(), (x, w), create_graph=True)
        hA, = torch.autograd.grad((gx * B).sum() + (gw * D).sum(), (A,))
        res.append(hA)
    assert _rel(res[0], res[1]) < 1e-6


def test_wino_off_matches_on():
    """SMMD_WINO=0 (MIOpen) and the Winograd path agree on a critic-shaped layer."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(8, 128, 32, 32, device=DEV, generator=g)
    w = torch.randn(128, 128, 3, 3, device=DEV, generator=g) / 34.0
    b = torch.randn(128, device=DEV, generator=g)
    y1 = convops.conv2d(x, w, b, 1, 1)
    saved = convops.WINO
    convops.WINO = False
    try:
        y0 = convops.conv2d(x, w, b, 1, 1)
    finally:
        convops.WINO = saved
    assert _rel(y1, y0) < 5e-6


@pytest.fixture
def wgrad_on():
    from gan.core import convops
    saved = convops.WINO_WGRAD
    convops.WINO_WGRAD = True
    yield convops
    convops.WINO_WGRAD = saved


# the r11 kernel's chunk shapes: 16-tile rows with halo columns (W 64, 128),
# whole 16-tile rows (W 32), two 8-tile rows (W 16), four 4-tile rows (W 8);
# shapes it does not tile (6 x 8, 4 x 12, 2 x 4, W 8 with H % 8 != 0) take the
# first form
WGRAD_SHAPES = [(2, 64, 64, 6, 8), (3, 64, 128, 8, 8), (4, 128, 64, 4, 12), (2, 64, 64, 2, 4),
                (8, 64, 64, 64, 64), (8, 512, 512, 8, 8), (2, 64, 128, 32, 32),
                (3, 128, 64, 16, 16), (1, 64, 64, 8, 128), (2, 64, 64, 12, 8),
                (4, 128, 128, 32, 32), (16, 256, 256, 16, 16)]


@pytest.mark.parametrize('shape', WGRAD_SHAPES)
def test_wino_wgrad_vs_float64(wgrad_on, shape):
    """smmd_wino3x3_wgrad against torch's float64 conv2d_weight (the sums run
    over N*H*W terms in fp32: bound 1e-5 of max|ref|)."""
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(N + C + K + H + W)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    gy = torch.randn(N, K, H, W, device=DEV, generator=g)
    gw = wgrad_on._wino_wgrad(x, gy)
    ref = torch.nn.grad.conv2d_weight(x.double().cpu(), (K, C, 3, 3), gy.double().cpu(),
                                      padding=1)
    assert _rel(gw, ref) < 1e-5


@pytest.mark.parametrize('shape', [(8, 64, 64, 64, 64), (3, 128, 64, 16, 16), (4, 128, 64, 8, 8)])
def test_wino_wgrad_forms_agree_and_deterministic(wgrad_on, shape, monkeypatch):
    """The coalesced form (default) and the first form (SMMD_WINO_WGRAD_V1=1,
    read per call by the library) agree to rounding; each gives the same bits
    run to run."""
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(N, C, H, W, device=DEV, generator=g)
    gy = torch.randn(N, K, H, W, device=DEV, generator=g)
    a0 = wgrad_on._wino_wgrad(x, gy)
    a1 = wgrad_on._wino_wgrad(x, gy)
    monkeypatch.setenv('SMMD_WINO_WGRAD_V1', '1')
    b0 = wgrad_on._wino_wgrad(x, gy)
    b1 = wgrad_on._wino_wgrad(x, gy)
    monkeypatch.delenv('SMMD_WINO_WGRAD_V1')
    assert torch.equal(a0, a1) and torch.equal(b0, b1)
    assert _rel(a0, b0) < 1e-5


def test_wino_wgrad_double_backward_vs_float64(wgrad_on):
    test_convops_wino_double_backward_vs_float64((2, 64, 64, 8, 8))


@pytest.mark.parametrize('shape', [(2, 64, 64, 8, 8), (3, 512, 512, 8, 8)])
def test_conv2d_relu_double_backward_vs_float64(shape):
    """convops.conv2d_relu (the ReLU in the Winograd epilogue; the 512-channel
    case takes the split-input-channel path, ReLU in the slice add) through
    the critic's double backward against float64 relu(conv2d)."""
    from gan.core import convops
    N, C, K, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(31)
    t = {k: torch.randn(*s, device=DEV, generator=g) for k, s in
         dict(x=(N, C, H, W), w=(K, C, 3, 3), b=(K,), A=(N, K, H, W), B=(N, C, H, W),
              D=(K, C, 3, 3)).items()}
    t['w'] = t['w'] / (9 * C) ** 0.5

    def run(dev, dtype, fn):
        v = {k: t[k].to(dev, dtype).requires_grad_(k in ('x', 'w', 'A')) for k in t}
        y = fn(v['x'], v['w'], v['b'])
        loss = (y * v['A']).sum()
        gx, gw = torch.autograd.grad(loss, (v['x'], v['w']), create_graph=True)
        second = (gx * v['B']).sum() + (gw * v['D']).sum()
        hx, hw, hA = torch.autograd.grad(second, (v['x'], v['w'], v['A']))
        return y, gx, gw, hx, hw, hA

    assert convops._is_wino(t['x'], t['w'], [1, 1], [1, 1], 0)
    got = run(DEV, torch.float32, lambda x, w, b: convops.conv2d_relu(x, w, b, 1, 1))
    # the reference takes the ReLU's mask from the fp32 output, so an
    # activation within rounding of 0 cannot flip between the two
    mask = (got[0] > 0).double().cpu()
    ref = run('cpu', torch.float64, lambda x, w, b: F.conv2d(x, w, b, 1, 1) * mask)
    for n, a, r in zip(('y', 'gx', 'gw', 'hx', 'hw', 'hA'), got, ref):
        assert _rel(a, r) < (2e-5 if n in ('gw', 'hx', 'hw') else 1e-5), n
