"""ConvMeanPool filter fold on the GPU (`smmd_fold_pool_weight`,
csrc/smmd_fold.hip) against the float64 oracle (oracle.smmd_oracle
fold_pool_weight / _adjoint, block.py:63-66), on the SNResNet-64 critic's
ConvMeanPool filter counts and ragged counts (not a multiple of the 256-filter
block), plus the folded conv block end to end against the literal
conv3x3 -> mean pool (first and second order)."""
import numpy as np
import pytest

torch = pytest.importorskip('torch')

from oracle import smmd_oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

SHAPES = [(128, 64), (1024, 512), (3, 5), (1, 1), (257, 3), (7, 300)]


def test_fold_and_adjoint_match_oracle():
    """All SHAPES as the layers of ONE launch each way (ragged block splits)."""
    from gan.core.convops import _FoldPool, _FoldPoolAdj
    rng = np.random.default_rng(7)
    Ws = [rng.standard_normal((co, ci, 3, 3)).astype(np.float32) for co, ci in SHAPES]
    Gs = [rng.standard_normal((co, ci, 4, 4)).astype(np.float32) for co, ci in SHAPES]
    dev = torch.device('cuda:0')
    w4s = _FoldPool.apply(*[torch.tensor(W, device=dev) for W in Ws])
    g3s = _FoldPoolAdj.apply(*[torch.tensor(G, device=dev) for G in Gs])
    torch.cuda.synchronize()
    for (co, ci), W, G, w4, g3 in zip(SHAPES, Ws, Gs, w4s, g3s):
        assert w4.shape == (co, ci, 4, 4) and g3.shape == (co, ci, 3, 3)
        np.testing.assert_allclose(w4.cpu().numpy(), O.fold_pool_weight(W), rtol=1e-6,
                                   atol=1e-7)
        np.testing.assert_allclose(g3.cpu().numpy(), O.fold_pool_weight_adjoint(G),
                                   rtol=1e-6, atol=1e-7)
        # <fold(W), G> == <W, fold^T(G)>
        lhs = float((O.fold_pool_weight(W) * G).sum())
        rhs = float((W * g3.cpu().numpy().astype(np.float64)).sum())
        assert abs(lhs - rhs) <= 1e-4 * (1 + abs(lhs))


@pytest.mark.parametrize('cout,cin', SHAPES)
def test_fold_single_layer_matches_oracle(cout, cin):
    from gan.core.convops import fold_pool_weight
    rng = np.random.default_rng(cout * 1000 + cin)
    W = rng.standard_normal((cout, cin, 3, 3)).astype(np.float32)
    w4 = fold_pool_weight(torch.tensor(W, device='cuda:0'))
    np.testing.assert_allclose(w4.cpu().numpy(), O.fold_pool_weight(W), rtol=1e-6, atol=1e-7)


def test_fold_rejects_bad_arguments():
    from gan.core import _lib
    import ctypes
    L = _lib.lib()
    nf = (ctypes.c_int64 * 1)(-1)
    P = ctypes.c_void_p * 1
    assert L.smmd_fold_pool_weights(P(None), P(None), nf, 1, 0, None) == 1      # EINVAL
    assert L.smmd_fold_pool_weights(P(None), P(None), nf, 17, 0, None) == 1
    nf0 = (ctypes.c_int64 * 1)(0)
    assert L.smmd_fold_pool_weights(P(None), P(None), nf0, 1, 0, None) == 0     # empty: OK
    x = torch.zeros(64, device='cuda:0')
    w4 = (ctypes.c_int64 * 1)(1)
    # misaligned 4x4 side
    assert L.smmd_fold_pool_weights(P(x.data_ptr()), P(x.data_ptr() + 4), w4, 1, 0, None) == 1


def test_fold_autograd_second_order_on_device():
    from gan.core.convops import fold_pool_weight
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    w = torch.randn(6, 5, 3, 3, device=dev, requires_grad=True)
    c = torch.randn(6, 5, 4, 4, device=dev)
    y = (fold_pool_weight(w) * c).pow(2).sum()
    g, = torch.autograd.grad(y, w, create_graph=True)
    gg, = torch.autograd.grad(g.pow(2).sum(), w)
    wc = w.detach().cpu().double().requires_grad_(True)
    from gan.core.convops import _fold_torch
    y2 = (_fold_torch(wc) * c.cpu().double()).pow(2).sum()
    g2, = torch.autograd.grad(y2, wc, create_graph=True)
    gg2, = torch.autograd.grad(g2.pow(2).sum(), wc)
    assert torch.allclose(g.cpu().double(), g2, rtol=1e-4, atol=1e-5)
    assert torch.allclose(gg.cpu().double(), gg2, rtol=1e-4, atol=1e-4)


def test_folded_conv_mean_pool_block_on_device():
    """_ConvMeanPool (folded, HIP fold + MIOpen stride-2 conv) vs the literal
    conv3x3 -> mean pool on the same device: value, input gradient and the
    parameter gradients of a gradient penalty through it."""
    from gan.core import architecture
    dev = torch.device('cuda:0')
    torch.manual_seed(1)
    blk = architecture._ConvMeanPool(16, 32, 3, True).to(dev)
    x = torch.randn(4, 16, 16, 16, device=dev, requires_grad=True)
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
    for a, c in zip(*res):
        tol = 1e-4 * float(c.abs().max()) + 1e-6
        assert float((a - c).abs().max()) <= tol


@pytest.mark.parametrize('k,bias', [(3, False), (1, True)])
def test_folded_upsample_conv_on_device(k, bias):
    """_Up (UpsampleConv, block.py:53-60) folded (4x4 stride-2 transposed conv /
    1x1 before the upsample, MIOpen) vs the literal upsample -> conv on the same
    device: value and the first-order gradients the generator step uses."""
    from gan.core import architecture
    dev = torch.device('cuda:0')
    torch.manual_seed(2)
    blk = architecture._Up(32, 16, k, bias).to(dev)
    x = torch.randn(4, 32, 8, 8, device=dev, requires_grad=True)
    params = list(blk.parameters())
    res = []
    saved = architecture.FOLD_UP
    try:
        for fold in (True, False):
            architecture.FOLD_UP = fold
            y = blk(x)
            L = (torch.tanh(y) * torch.arange(y.numel(), device=dev).view_as(y).sin()).sum()
            res.append((y.detach(),) + torch.autograd.grad(L, [x] + params))
    finally:
        architecture.FOLD_UP = saved
    assert res[0][0].shape == (4, 16, 16, 16)
    for a, c in zip(*res):
        tol = 1e-4 * float(c.abs().max()) + 1e-6
        assert float((a - c).abs().max()) <= tol


@pytest.mark.parametrize('shape', [(64, 64, 64, 64), (64, 128, 32, 32), (64, 1024, 4, 4),
                                   (3, 5, 3, 3), (7, 1, 1, 1), (2, 2000, 2, 2), (0, 4, 2, 2)])
def test_channel_sum_matches_oracle(shape):
    """smmd_channel_sum (conv bias gradient, BiasAddGrad of snops.py:89-90)
    against a float64 sum over (N, H, W); odd HW takes the scalar path."""
    from gan.core.convops import bias_grad
    rng = np.random.default_rng(sum(shape))
    g = rng.standard_normal(shape).astype(np.float32)
    with torch.no_grad():
        out = bias_grad(torch.tensor(g, device='cuda:0'))
    torch.cuda.synchronize()
    ref = g.astype(np.float64).sum(axis=(0, 2, 3))
    tol = 1e-5 * np.sqrt(shape[0] * shape[2] * shape[3] + 1) + 1e-6
    assert out.shape == (shape[1],)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=0, atol=tol)
    if shape[0]:
        with torch.no_grad():
            b2 = bias_grad(torch.tensor(g, device='cuda:0'))
        assert torch.equal(out, b2)           # fixed order: bit-identical


def test_channel_sum_shape_sequence_shared_workspace():
    """Calls of different channel counts back to back through the one cached
    workspace (C < 512 takes the two-stage path, C >= 512 the direct one; wide
    and short rows, batched loads): every result against float64, and repeated
    calls give the same bits."""
    from gan.core.convops import bias_grad
    rng = np.random.default_rng(7)
    shapes = [(64, 64, 16, 16), (64, 256, 8, 8), (64, 3, 8, 8), (64, 1024, 4, 4),
              (32, 128, 4, 4), (64, 64, 16, 16)]
    xs = [torch.tensor(rng.standard_normal(sh).astype(np.float32), device='cuda:0')
          for sh in shapes]
    with torch.no_grad():
        first = [bias_grad(x) for x in xs]
        second = [bias_grad(x) for x in reversed(xs)][::-1]
    torch.cuda.synchronize()
    for sh, x, a, b in zip(shapes, xs, first, second):
        ref = x.cpu().numpy().astype(np.float64).sum(axis=(0, 2, 3))
        tol = 1e-5 * np.sqrt(sh[0] * sh[2] * sh[3] + 1) + 1e-6
        np.testing.assert_allclose(a.cpu().numpy(), ref, rtol=0, atol=tol)
        assert torch.equal(a, b)


def test_fold_caches_follow_flat_adam_updates():
    """The prefold (critic) and folded-UpsampleConv (generator) caches must
    miss after a FlatAdam step: the library writes the parameters without
    advancing torch's version counters (optim.param_epoch keys the caches)."""
    from gan.core import architecture
    from gan.core.optim import FlatAdam
    dev = torch.device('cuda:0')
    torch.manual_seed(3)
    D = architecture.ResNetDiscriminator(4, 1, False).to(dev)       # no SN: W_eff is W
    up = architecture._Up(8, 4, 3, False).to(dev)
    x = torch.rand(2, 3, 64, 64, device=dev)
    z = torch.randn(2, 8, 4, 4, device=dev)
    opt_d = FlatAdam(list(D.parameters()), 1e-2, name='D')
    opt_g = FlatAdam(list(up.parameters()), 1e-2, name='G')
    for _ in range(2):
        with torch.no_grad():
            D(x)
            up(z)                                    # fill the caches
        for p in list(D.parameters()) + list(up.parameters()):
            p.grad.normal_()
        opt_d.step()
        opt_g.step()
        with torch.no_grad():
            d_c, u_c = D(x), up(z)
            saved = architecture.FOLD_POOL, architecture.FOLD_UP
            try:
                architecture.FOLD_POOL = architecture.FOLD_UP = False
                d_l, u_l = D(x), up(z)
            finally:
                architecture.FOLD_POOL, architecture.FOLD_UP = saved
        assert torch.allclose(d_c, d_l, rtol=1e-4, atol=1e-5 * float(d_l.abs().max()) + 1e-6)
        assert torch.allclose(u_c, u_l, rtol=1e-4, atol=1e-5 * float(u_l.abs().max()) + 1e-6)


@pytest.mark.parametrize('offset', [1, 2, 3])
def test_channel_sum_misaligned_base(offset):
    """A contiguous view with a storage offset (not 16-B aligned, e.g. a
    narrow/split backward) takes the kernel's scalar-load path: same sums."""
    from gan.core.convops import bias_grad
    shape = (8, 16, 8, 8)
    rng = np.random.default_rng(offset)
    flat = rng.standard_normal(int(np.prod(shape)) + offset).astype(np.float32)
    base = torch.tensor(flat, device='cuda:0')
    gy = base[offset:].view(shape)
    assert gy.is_contiguous() and gy.data_ptr() % 16 != 0
    with torch.no_grad():
        out = bias_grad(gy)
    ref = flat[offset:].reshape(shape).astype(np.float64).sum(axis=(0, 2, 3))
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=0, atol=1e-4)


def test_upsample_fold_two_backwards_without_step():
    """Two generator backwards with grad enabled and no optimizer step in
    between: the folded UpsampleConv filter is not reused across graphs
    (a cached K would back through a freed graph)."""
    from gan.core import architecture
    dev = torch.device('cuda:0')
    torch.manual_seed(4)
    up = architecture._Up(8, 4, 3, False).to(dev)
    z = torch.randn(2, 8, 4, 4, device=dev)
    for _ in range(2):
        up(z).square().sum().backward()
    assert up.conv.weight.grad is not None and torch.isfinite(up.conv.weight.grad).all()


@pytest.mark.parametrize('shape', SHAPES + [(512, 1024)])
def test_fold_up_weight_and_adjoint_match_oracle(shape):
    """UpsampleConv fold on the library (`smmd_fold_up_weight`, ABI 11): K =
    flip(4 fold(W)) transposed against the float64 oracle's fold, its adjoint
    against the transpose of that linear map, and the double backward (the
    adjoint's backward is the fold again)."""
    from gan.core.convops import fold_up_weight
    co, ci = shape
    rng = np.random.default_rng(co * 7 + ci)
    W = rng.standard_normal((co, ci, 3, 3)).astype(np.float32)
    G = rng.standard_normal((ci, co, 4, 4)).astype(np.float32)
    dev = torch.device('cuda:0')
    w = torch.tensor(W, device=dev, requires_grad=True)
    k = fold_up_weight(w)
    assert k.shape == (ci, co, 4, 4) and k.is_contiguous()
    ref = np.flip(4.0 * O.fold_pool_weight(W.astype(np.float64)), (2, 3)).transpose(1, 0, 2, 3)
    np.testing.assert_allclose(k.detach().cpu().numpy(), ref, rtol=1e-6, atol=1e-6)
    g = torch.tensor(G, device=dev)
    gw, = torch.autograd.grad(k, w, g, create_graph=True)
    gref = 4.0 * O.fold_pool_weight_adjoint(np.flip(G.astype(np.float64), (2, 3))
                                            .transpose(1, 0, 2, 3))
    np.testing.assert_allclose(gw.detach().cpu().numpy(), gref, rtol=1e-6, atol=1e-6)
    # second order: d/dG <gw, V> = fold_up(V) (the adjoint's backward)
    v = torch.randn(co, ci, 3, 3, device=dev)
    gt = g.clone().requires_grad_(True)
    gw2, = torch.autograd.grad(fold_up_weight(w), w, gt, create_graph=True)
    h, = torch.autograd.grad((gw2 * v).sum(), gt)
    np.testing.assert_allclose(h.cpu().numpy(), fold_up_weight(v).cpu().numpy(), rtol=1e-6,
                               atol=1e-6)
