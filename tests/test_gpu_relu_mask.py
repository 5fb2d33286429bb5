"""The critic's conv-ReLU mask moved into its consumer's input gradient
(smmd_wino4x4s2t_conv_mask, ABI 12; convops conv2d_relu(consumer_masks) +
conv2d(mask_in), ResidualBlock.down_parts): the masked transposed conv is
bit-identical to the transposed conv followed by threshold_backward, with and
without the split-K slab sum, and the block's gradients -- first order and
through the scaling regulariser's double backward -- are bit-identical to the
unfused path (the ReLU's own threshold_backward) and match float64.  In the
double backward the consumer's mask of its upstream gradient moves into the
producing 3x3 Winograd conv's epilogue (smmd_wino3x3_conv_mask, ABI 14;
convops _ConvBackward gy_mask), again bit-identical."""
import pytest

torch = pytest.importorskip('torch')
import torch.nn.functional as F  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'

# (N, K, C, Hg): gy [N, K, Hg, Hg] -> dx [N, C, 2 Hg, 2 Hg]; the fold layers'
# input gradients at batch 64 and small ones (the deep ones take slices)
S2T = [(64, 128, 64, 32), (64, 512, 256, 8), (64, 512, 512, 4), (4, 64, 64, 8), (2, 128, 192, 6)]


@pytest.mark.parametrize('shape', S2T)
def test_s2t_mask_equals_threshold_after(shape):
    from gan.core import convops
    N, K, C, Hg = shape
    g = torch.Generator(device=DEV).manual_seed(K + C + Hg)
    gy = torch.randn(N, K, Hg, Hg, device=DEV, generator=g)
    w = torch.randn(K, C, 4, 4, device=DEV, generator=g) / (16 * K) ** 0.5
    m = torch.randn(N, C, 2 * Hg, 2 * Hg, device=DEV, generator=g)
    m[0, 0, :3] = 0.0                       # threshold_backward's (mask <= 0) boundary
    assert convops._is_s2t(gy, w, [2, 2], [1, 1])
    fused = convops._s2t_conv(gy, w, None, mask=m)
    plain = torch.ops.aten.threshold_backward(convops._s2t_conv(gy, w, None), m, 0.0)
    assert torch.equal(fused, plain)
    assert int((fused[m <= 0] != 0).sum()) == 0


def _block(fuse, x0, w1, w2, t1, t2, order):
    from gan.core import convops
    x = x0.clone().requires_grad_(True)
    a = w1.clone().requires_grad_(True)
    b = w2.clone().requires_grad_(True)
    h1 = convops.conv2d_relu(x, a, None, 1, 1, consumer_masks=fuse)
    h = convops.conv2d(h1, b, None, 2, 1, mask_in=fuse)
    if order == 1:
        return torch.autograd.grad((h * t1).sum(), (x, a, b))
    # the scaling regulariser's pattern: the input gradient with create_graph,
    # then a loss of it and of the output, differentiated w.r.t. everything
    jx, = torch.autograd.grad((h * t1).sum(), x, create_graph=True)
    loss = jx.square().sum() + (h * t2).sum()
    return torch.autograd.grad(loss, (x, a, b))


def _block64(x0, w1, w2, t1, t2, order):
    x = x0.double().requires_grad_(True)
    a = w1.double().requires_grad_(True)
    b = w2.double().requires_grad_(True)
    h = F.conv2d(F.relu(F.conv2d(x, a, None, 1, 1)), b, None, 2, 1)
    if order == 1:
        return torch.autograd.grad((h * t1.double()).sum(), (x, a, b))
    jx, = torch.autograd.grad((h * t1.double()).sum(), x, create_graph=True)
    loss = jx.square().sum() + (h * t2.double()).sum()
    return torch.autograd.grad(loss, (x, a, b))


@pytest.mark.parametrize('order', [1, 2])
@pytest.mark.parametrize('shape', [(4, 64, 128, 16), (2, 128, 64, 8)])
def test_block_grads_fused_equal_unfused(shape, order):
    from gan.core import convops
    N, C, K, H = shape
    g = torch.Generator(device=DEV).manual_seed(C + K + H + order)
    x0 = torch.randn(N, C, H, H, device=DEV, generator=g)
    w1 = torch.randn(C, C, 3, 3, device=DEV, generator=g) / (9 * C) ** 0.5
    w2 = torch.randn(K, C, 4, 4, device=DEV, generator=g) / (16 * C) ** 0.5
    t1 = torch.randn(N, K, H // 2, H // 2, device=DEV, generator=g)
    t2 = torch.randn(N, K, H // 2, H // 2, device=DEV, generator=g)
    assert convops._is_wino(x0, w1, [1, 1], [1, 1], 0)
    fused = _block(True, x0, w1, w2, t1, t2, order)
    plain = _block(False, x0, w1, w2, t1, t2, order)
    for f, p, what in zip(fused, plain, ('dx', 'dw1', 'dw2')):
        assert torch.equal(f, p), what
    ref = _block64(x0, w1, w2, t1, t2, order)
    for f, r, what in zip(fused, ref, ('dx', 'dw1', 'dw2')):
        err = float((f.double() - r).abs().max())
        assert err <= 2e-5 * (float(r.abs().max()) + 1e-30), (what, err)


def test_fused_path_skips_threshold_kernel():
    """With the fusion the first-order backward of conv-ReLU -> stride-2 conv
    runs no threshold_backward (torch profiler op names)."""
    from gan.core import convops
    from torch.profiler import ProfilerActivity, profile
    x = torch.randn(4, 64, 16, 16, device=DEV, requires_grad=True)
    w1 = torch.randn(64, 64, 3, 3, device=DEV, requires_grad=True)
    w2 = torch.randn(128, 64, 4, 4, device=DEV, requires_grad=True)
    h = convops.conv2d(convops.conv2d_relu(x, w1, None, 1, 1, consumer_masks=True), w2, None, 2,
                       1, mask_in=True)
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        h.square().sum().backward()
    names = {e.name for e in prof.events()}
    assert 'aten::threshold_backward' not in names


def _tail_run(fn, u0, v0, t, order):
    u = u0.clone().requires_grad_(True)
    v = v0.clone().requires_grad_(True)
    y = fn(u, v)
    if order == 1:
        return (y,) + torch.autograd.grad((y * t).sum(), (u, v))
    gu, = torch.autograd.grad((y * t).sum(), u, create_graph=True)
    loss = (gu * u0.sin()).sum() + (y * t).square().sum()
    return (y,) + torch.autograd.grad(loss, (u, v))


@pytest.mark.parametrize('order', [1, 2])
def test_critic_tail_vs_torch(order):
    """convops.lrelu_rowsum (smmd_row_lrelu_sum / _bcast: the critic's last
    add + lrelu + pixel sum) against torch's ops in float64, first order and
    through a double backward; its backward is bit-identical to torch's."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(5 + order)
    u0 = torch.randn(64, 1024, 4, 4, device=DEV, generator=g)
    v0 = torch.randn(64, 1024, 4, 4, device=DEV, generator=g)
    t = torch.randn(64, 1024, device=DEV, generator=g)
    assert convops._tail_ok(u0, v0)
    got = _tail_run(lambda u, v: convops.lrelu_rowsum(u, v, 0.2), u0, v0, t, order)
    ref = _tail_run(lambda u, v: F.leaky_relu(u + v, 0.2).sum(dim=(2, 3)), u0.double(),
                    v0.double(), t.double(), order)
    for a, r, what in zip(got, ref, ('y', 'du', 'dv')):
        err = float((a.double() - r).abs().max())
        assert err <= 1e-5 * (float(r.abs().max()) + 1e-30), (what, err)
    if order == 1:
        plain = _tail_run(lambda u, v: F.leaky_relu(u + v, 0.2).sum(dim=(2, 3)), u0, v0, t, 1)
        assert torch.equal(got[1], plain[1]) and torch.equal(got[2], plain[2])


# (N, C, K, H): conv(x [N, C, H, H], w [K, C, 3, 3]) masked by m [N, K, H, H]:
# the critic's 64- and 128-channel first convs at batch 64 (one launch), the
# deep ones (split-C slabs: the mask in the slab reduction), a tile row that
# does not divide the wave (the EDGE kernel)
WINO_MASK = [(64, 64, 64, 64), (64, 128, 128, 32), (64, 512, 512, 8), (4, 64, 64, 16),
             (2, 64, 64, 12)]


@pytest.mark.parametrize('shape', WINO_MASK)
def test_wino_conv_mask_equals_threshold_after(shape):
    from gan.core import convops
    N, C, K, H = shape
    g = torch.Generator(device=DEV).manual_seed(N + C + K + H)
    x = torch.randn(N, C, H, H, device=DEV, generator=g)
    w = torch.randn(K, C, 3, 3, device=DEV, generator=g) / (9 * C) ** 0.5
    b = torch.randn(K, device=DEV, generator=g)
    m = torch.randn(N, K, H, H, device=DEV, generator=g)
    m[0, 0, :2] = 0.0                       # threshold_backward's (mask <= 0) boundary
    assert convops._is_wino(x, w, [1, 1], [1, 1], 0)
    for bias in (None, b):
        fused = convops._wino_conv(x, w, bias, 0, mask=m)
        plain = torch.ops.aten.threshold_backward(convops._wino_conv(x, w, bias, 0), m, 0.0)
        assert torch.equal(fused, plain)
    # the dispatcher's route (convops._fwd ymask) is the fused launch
    assert torch.equal(convops._fwd(x, w, b, [1, 1], [1, 1], ymask=m), fused)


def _count_thresholds(fn):
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        out = fn()
    return out, sum(1 for e in prof.events() if e.name == 'aten::threshold_backward')


@pytest.mark.parametrize('shape', [(4, 64, 128, 16), (64, 64, 128, 64)])
def test_double_backward_mask_moves_to_producer(shape, monkeypatch):
    """The scaling regulariser's double backward through conv-ReLU -> stride-2
    conv: with the upstream mask in the producer's epilogue the gradients are
    bit-identical to the consumer masking it, with one threshold_backward
    fewer."""
    from gan.core import convops
    N, C, K, H = shape
    g = torch.Generator(device=DEV).manual_seed(N + C + K + H + 9)
    x0 = torch.randn(N, C, H, H, device=DEV, generator=g)
    w1 = torch.randn(C, C, 3, 3, device=DEV, generator=g) / (9 * C) ** 0.5
    w2 = torch.randn(K, C, 4, 4, device=DEV, generator=g) / (16 * C) ** 0.5
    t1 = torch.randn(N, K, H // 2, H // 2, device=DEV, generator=g)
    t2 = torch.randn(N, K, H // 2, H // 2, device=DEV, generator=g)
    on, n_on = _count_thresholds(lambda: _block(True, x0, w1, w2, t1, t2, 2))
    monkeypatch.setattr(convops, 'GGX_MASK_FUSE', False)
    off, n_off = _count_thresholds(lambda: _block(True, x0, w1, w2, t1, t2, 2))
    for a, b, what in zip(on, off, ('dx', 'dw1', 'dw2')):
        assert torch.equal(a, b), what
    assert n_on == n_off - 1, (n_on, n_off)


def _two_blocks(x0, t, on, monkeypatch):
    """Two critic down blocks (the second reading the first's two paths
    through relu_pool, so its gu feeds both of the first block's convs), the
    scaling regulariser's pattern: the input gradient with create_graph, then
    a loss of it and of the output, differentiated in an armed backward."""
    from gan.core import convops
    from gan.core.architecture import ResidualBlock
    monkeypatch.setattr(convops, 'GY_ACC', on)
    torch.manual_seed(3)
    b1 = ResidualBlock(64, 128, 3, 'down').to(DEV)
    b2 = ResidualBlock(128, 256, 3, 'down').to(DEV)
    x = x0.clone().requires_grad_(True)
    s, h = b1.down_parts(x)[:2]
    s2, h2 = b2.down_parts(s, h)[:2]
    out = s2 + h2
    jx, = torch.autograd.grad((out * t).sum(), x, create_graph=True)
    loss = jx.square().sum() + (out * t).sum()
    params = list(b1.parameters()) + list(b2.parameters())
    n0 = convops._late['gy_acc']
    convops.arm_late_wgrad_sums(True)
    try:
        grads = torch.autograd.grad(loss, params + [x], allow_unused=True)
    finally:
        convops.arm_late_wgrad_sums(False)
    return grads, convops._late['gy_acc'] - n0


@pytest.mark.parametrize('N,H', [(4, 16), (64, 32)])
def test_shared_gy_contributions_summed_in_kernel(N, H, monkeypatch):
    """The double backward's two gradients of one block-output gradient (main
    path's stride-2 conv and shortcut's 1x1 conv, both fed _ReluPool's gu):
    the second computed into the first (smmd_wino4x4s2_conv_acc, ABI 15) gives
    the gradients autograd's own sum gives, bit for bit."""
    g = torch.Generator(device=DEV).manual_seed(N + H)
    x0 = torch.randn(N, 64, H, H, device=DEV, generator=g)
    t = torch.randn(N, 256, H // 4, H // 4, device=DEV, generator=g)
    on, n_on = _two_blocks(x0, t, True, monkeypatch)
    off, n_off = _two_blocks(x0, t, False, monkeypatch)
    assert n_on > 0 and n_off == 0, (n_on, n_off)
    for i, (a, b) in enumerate(zip(on, off)):
        assert (a is None) == (b is None), i
        if a is not None:
            assert torch.equal(a, b), i
