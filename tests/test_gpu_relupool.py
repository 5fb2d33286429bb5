"""GPU parity of the fused input ops of a critic down block (csrc/smmd_relupool.hip,
convops.relu_pool): relu(x) of the main path (gan/core/resnet/block.py:44) and
the shortcut's 2x2 mean pool (block.py:69-71), forward, backward and double
backward, against the torch composition they replace.  The kernels keep that
composition's operation order, so values and gradients are compared for
equality (not a tolerance)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'


def _ref(x):
    from gan.core.convops import mean_pool2
    return F.relu(x), mean_pool2(x)


@pytest.fixture
def relu_pool_off():
    from gan.core import convops
    saved = convops.RELU_POOL
    yield convops
    convops.RELU_POOL = saved


@pytest.mark.parametrize('shape', [(64, 64, 64, 64), (4, 128, 32, 32), (3, 5, 8, 4), (2, 1, 2, 4)])
def test_relu_pool_forward_equals_torch(shape):
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(sum(shape))
    x = torch.randn(shape, device=DEV, generator=g)
    assert convops.relu_pool_applicable(x)
    r, p = convops.relu_pool(x)
    rr, pr = _ref(x)
    assert torch.equal(r, rr) and torch.equal(p, pr)


@pytest.mark.parametrize('use', ['both', 'relu', 'pool'])
def test_relu_pool_backward_equals_torch(use):
    """The input gradient when the block uses both outputs (their sum), or
    only one (the other arrives as None)."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(8, 16, 16, 16, device=DEV, generator=g)
    A = torch.randn(8, 16, 16, 16, device=DEV, generator=g)
    B = torch.randn(8, 16, 8, 8, device=DEV, generator=g)
    grads = []
    for fn in (convops.relu_pool, _ref):
        xx = x.clone().requires_grad_(True)
        r, p = fn(xx)
        L = {'both': (r * A).sum() + (p * B).sum(), 'relu': (r * A).sum(),
             'pool': (p * B).sum()}[use]
        gx, = torch.autograd.grad(L, xx)
        grads.append(gx)
    assert torch.equal(grads[0], grads[1])


def _tiny_critic(x, w1, w2, w3, fn):
    """x -> (relu, pool) -> 3x3 conv of the relu branch + 1x1 conv of the
    pooled branch (a down block's two paths), reduced to one feature per image."""
    r, p = fn(x)
    h = F.conv2d(r, w1, padding=1)
    h = F.avg_pool2d(F.relu(h), 2)
    s = F.conv2d(p, w2)
    out = F.conv2d(F.relu(h + s), w3)
    return out.mean(dim=(1, 2, 3))


def test_relu_pool_double_backward_matches_torch():
    """The scaling regulariser's pattern: the Jacobian of the features with
    respect to the input (create_graph), then the gradient of its squared
    norm with respect to the weights, through the fused ops."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(4, 8, 16, 16, device=DEV, generator=g)
    w1 = torch.randn(8, 8, 3, 3, device=DEV, generator=g) * 0.2
    w2 = torch.randn(8, 8, 1, 1, device=DEV, generator=g) * 0.2
    w3 = torch.randn(1, 8, 1, 1, device=DEV, generator=g) * 0.2
    res = []
    for fn in (convops.relu_pool, _ref):
        xx = x.clone().requires_grad_(True)
        ws = [w.clone().requires_grad_(True) for w in (w1, w2, w3)]
        feat = _tiny_critic(xx, *ws, fn)
        jac, = torch.autograd.grad(feat.sum(), xx, create_graph=True)
        J = (jac * jac).sum()
        gws = torch.autograd.grad(J + feat.sum(), ws)
        res.append([jac.detach()] + list(gws))
    for a, b in zip(*res):
        tol = 1e-5 * float(b.abs().max()) + 1e-7
        assert float((a - b).abs().max()) <= tol


def test_relu_pool_third_order_runs():
    """Each kernel's backward is the other one: a third differentiation (the
    witness penalty's second order through a critic Jacobian) stays defined."""
    from gan.core import convops
    x = torch.randn(2, 4, 8, 8, device=DEV, requires_grad=True)
    A = torch.randn(2, 4, 8, 8, device=DEV)
    r, p = convops.relu_pool(x)
    L = (r * A).sum() + (p * p).sum()
    gx, = torch.autograd.grad(L, x, create_graph=True)
    ggx, = torch.autograd.grad((gx * gx).sum(), x, create_graph=True)
    assert torch.isfinite(ggx).all()


def test_residual_down_block_fused_equals_unfused(relu_pool_off):
    """An SNResNet critic down block (block.py:9-50, resample 'down') with the
    fused input ops against the same block on relu + mean_pool2: output, the
    input gradient and the parameter gradients of a scaled Jacobian loss."""
    convops = relu_pool_off
    from gan.core.architecture import ResidualBlock
    torch.manual_seed(3)
    blk = ResidualBlock(16, 32, 3, 'down').to(DEV)
    x0 = torch.randn(8, 16, 32, 32, device=DEV)
    out = []
    for on in (True, False):
        convops.RELU_POOL = on
        x = x0.clone().requires_grad_(True)
        y = blk(x)
        feat = y.mean(dim=(1, 2, 3))
        jac, = torch.autograd.grad(feat.sum(), x, create_graph=True)
        L = feat.sum() + 10.0 * (jac * jac).sum()
        gp = torch.autograd.grad(L, list(blk.parameters()))
        out.append([y.detach(), jac.detach()] + [t.detach() for t in gp])
    for a, b in zip(*out):
        tol = 1e-5 * float(b.abs().max()) + 1e-7
        assert float((a - b).abs().max()) <= tol


def test_mask_pool_abi_rejects_bad_shapes():
    from gan.core import _lib
    L = _lib.lib()
    x = torch.zeros(1, 1, 4, 6, device=DEV)
    o = torch.empty_like(x)
    s = _lib.stream_handle(x.device)
    P = _lib.ptr
    b = torch.zeros(3, device=DEV)
    args = lambda H, W, om, op, C=1, bx=None: (P(x), None, P(bx), None, C, None, 0.0, 1.0, 1,
                                              H, W, om, op, s)
    assert L.smmd_mask_pool2(*args(4, 6, P(o), None)) != 0          # W % 4
    assert L.smmd_mask_pool2(*args(3, 4, P(o), None)) != 0          # H odd
    assert L.smmd_mask_pool2(*args(4, 4, None, None)) != 0          # no output
    assert L.smmd_mask_pool2(*args(4, 4, P(o), None, 3, b)) != 0    # planes % C
    assert L.smmd_mask_pool2_adj(None, None, P(x), 0.0, 1.0, 1, 4, 4, P(o), s) != 0     # no term
    assert L.smmd_mask_pool2_adj(P(x), None, None, 0.0, 1.0, 1, 4, 4, P(o), s) != 0     # no mask
    torch.cuda.synchronize()
    np.testing.assert_array_equal(o.shape, x.shape)


def _ref_general(x, y, slope):
    from gan.core.convops import mean_pool2
    u = x if y is None else x + y
    if slope != 1.0:
        u = F.leaky_relu(u, slope)
    return F.relu(u), mean_pool2(u)


@pytest.mark.parametrize('variant', ['add', 'lrelu', 'add_lrelu'])
def test_relu_pool_fused_add_and_lrelu_equal_torch(variant):
    """The chained critic's block inputs: u = x + y (the previous block's two
    paths, block.py:50) or lrelu(x) (the first conv's pre-activation,
    architecture.py:393): outputs and the gradients of x and y, bit for bit."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(21)
    x = torch.randn(8, 16, 16, 16, device=DEV, generator=g)
    y = torch.randn(8, 16, 16, 16, device=DEV, generator=g) if 'add' in variant else None
    slope = 0.2 if 'lrelu' in variant else 1.0
    A = torch.randn(8, 16, 16, 16, device=DEV, generator=g)
    B = torch.randn(8, 16, 8, 8, device=DEV, generator=g)
    res = []
    for fn in (convops.relu_pool, _ref_general):
        xx = x.clone().requires_grad_(True)
        yy = y.clone().requires_grad_(True) if y is not None else None
        r, p = fn(xx, yy, slope)
        ins = [xx] + ([yy] if yy is not None else [])
        grads = torch.autograd.grad((r * A).sum() + (p * B).sum(), ins)
        res.append([r.detach(), p.detach()] + list(grads))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_relu_pool_with_deferred_biases_equals_torch():
    """The previous block's two conv biases added inside the fused pass:
    u = (x + bx) + (y + by); outputs and the gradients of x, y, bx, by against
    the broadcast adds of the unfused convolutions, bit for bit."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(31)
    x = torch.randn(8, 16, 16, 16, device=DEV, generator=g)
    y = torch.randn(8, 16, 16, 16, device=DEV, generator=g)
    bx = torch.randn(16, device=DEV, generator=g)
    by = torch.randn(16, device=DEV, generator=g)
    A = torch.randn(8, 16, 16, 16, device=DEV, generator=g)
    B = torch.randn(8, 16, 8, 8, device=DEV, generator=g)

    def ref(x, y, bx, by):
        return _ref_general(x + bx.view(1, -1, 1, 1), y + by.view(1, -1, 1, 1), 1.0)

    res = []
    for fn in (lambda *a: convops.relu_pool(a[0], a[1], 1.0, a[2], a[3]), ref):
        ins = [t.clone().requires_grad_(True) for t in (x, y, bx, by)]
        r, p = fn(*ins)
        grads = torch.autograd.grad((r * A).sum() + (p * B).sum(), ins)
        res.append([r.detach(), p.detach()] + list(grads))
    for a, b in zip(res[0][:4], res[1][:4]):
        assert torch.equal(a, b)
    for a, b in zip(res[0][4:], res[1][4:]):            # bias gradients: channel sums
        tol = 1e-5 * float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= tol


def test_relu_pool_lrelu_double_backward_matches_torch():
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(23)
    x = torch.randn(4, 8, 16, 16, device=DEV, generator=g)
    w1 = torch.randn(8, 8, 3, 3, device=DEV, generator=g) * 0.2
    w2 = torch.randn(8, 8, 1, 1, device=DEV, generator=g) * 0.2
    w3 = torch.randn(1, 8, 1, 1, device=DEV, generator=g) * 0.2
    res = []
    for fn in (lambda t: convops.relu_pool(t, None, 0.2), lambda t: _ref_general(t, None, 0.2)):
        xx = x.clone().requires_grad_(True)
        ws = [w.clone().requires_grad_(True) for w in (w1, w2, w3)]
        feat = _tiny_critic(xx, *ws, fn)
        jac, = torch.autograd.grad(feat.sum(), xx, create_graph=True)
        gws = torch.autograd.grad((jac * jac).sum() + feat.sum(), ws)
        res.append([jac.detach()] + list(gws))
    for a, b in zip(*res):
        tol = 1e-5 * float(b.abs().max()) + 1e-7
        assert float((a - b).abs().max()) <= tol


def test_snresnet_critic_chained_equals_layerwise(relu_pool_off):
    """The SNResNet-64 critic (architecture.py:410-434) with its block inputs
    chained through the fused ops against the same critic on the unfused
    composition: features, the input Jacobian and the parameter gradients of
    a scaling-regulariser loss."""
    convops = relu_pool_off
    from gan.core.architecture import SNResNetDiscriminator
    torch.manual_seed(4)
    D = SNResNetDiscriminator(16, 1, False, input_size=64).to(DEV)
    x0 = torch.rand(8, 3, 64, 64, device=DEV)
    out = []
    for on in (True, False):
        convops.RELU_POOL = on
        x = x0.clone().requires_grad_(True)
        feat = D(x)
        jac, = torch.autograd.grad(feat.sum(), x, create_graph=True)
        L = feat.sum() + 10.0 * (jac * jac).sum()
        gp = torch.autograd.grad(L, list(D.parameters()))
        out.append([feat.detach(), jac.detach()] + [t.detach() for t in gp])
    # same ops in the same order, but MIOpen's convolutions are not bitwise
    # reproducible run to run, so the comparison carries a tolerance
    for a, b in zip(*out):
        tol = 1e-5 * float(b.abs().max()) + 1e-7
        assert float((a - b).abs().max()) <= tol


def test_up_add_equals_torch():
    """A generator up block's output up(s + bs) + (h + bh) (block.py:50,
    :53-60): value and the gradients of s, bs, h, bh against the unfused
    bias adds, nearest upsample and add."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(41)
    s = torch.randn(8, 32, 8, 8, device=DEV, generator=g)
    h = torch.randn(8, 32, 16, 16, device=DEV, generator=g)
    bs = torch.randn(32, device=DEV, generator=g)
    bh = torch.randn(32, device=DEV, generator=g)
    A = torch.randn(8, 32, 16, 16, device=DEV, generator=g)

    def ref(s, bs, h, bh):
        return (F.interpolate(s + bs.view(1, -1, 1, 1), scale_factor=2, mode='nearest')
                + (h + bh.view(1, -1, 1, 1)))

    res = []
    for fn in (convops.up_add, ref):
        ins = [t.clone().requires_grad_(True) for t in (s, bs, h, bh)]
        out = fn(*ins)
        grads = torch.autograd.grad((out * A).sum(), ins)
        res.append([out.detach()] + list(grads))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][3], res[1][3])
    for a, b in ((res[0][2], res[1][2]), (res[0][4], res[1][4])):   # bias grads
        tol = 1e-5 * float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= tol


def test_snresnet_generator_up_add_equals_unfused():
    """The SNResNet-64 generator (architecture.py:178-208) with its up blocks'
    outputs on smmd_up_add against SMMD_UP_ADD off: images and the parameter
    gradients."""
    from gan.core import convops
    from gan.core.architecture import SNResNetGenerator
    saved = convops.UP_ADD
    torch.manual_seed(6)
    G = SNResNetGenerator(16, 3, 64, True).to(DEV)
    z = torch.rand(8, 128, device=DEV) * 2 - 1
    out = []
    try:
        for on in (True, False):
            convops.UP_ADD = on
            img = G(z)
            gp = torch.autograd.grad((img * img).sum(), list(G.parameters()))
            out.append([img.detach()] + [t.detach() for t in gp])
    finally:
        convops.UP_ADD = saved
    # conv biases in front of a batch norm have a zero gradient in exact
    # arithmetic (rounding noise in both runs), so the bound is relative to
    # the largest gradient of the network, not to each tensor's own
    assert float((out[0][0] - out[1][0]).abs().max()) <= 1e-5 * float(out[1][0].abs().max())
    scale = max(float(t.abs().max()) for t in out[1][1:])
    for a, b in zip(out[0][1:], out[1][1:]):
        assert float((a - b).abs().max()) <= 1e-5 * scale


@pytest.mark.parametrize('shape,mul,add', [((64, 64, 64, 64), 3, 1), ((64, 512, 8, 8), 3, 1),
                                           ((8, 1024, 4, 4), 3, 1), ((3, 7, 4, 4), 3, 1),
                                           # |mean| >> std: the variance must not cancel
                                           ((64, 64, 64, 64), 0.01, 50), ((8, 256, 8, 8), 0.01, 50)])
def test_bn_relu_no_grad_matches_torch(shape, mul, add):
    """smmd_bn_relu_fwd (the generator's batch norm + ReLU in a critic step,
    resnet/block.py:42-47) against training-mode batch norm + relu in float64
    on the module's own state: output and the updated moving averages."""
    from gan.core import snops
    from gan.core.snops import batch_norm, bn_relu
    saved, snops.BN_RELU = snops.BN_RELU, True
    g = torch.Generator(device=DEV).manual_seed(sum(shape))
    x = torch.randn(shape, device=DEV, generator=g) * mul + add
    bns = [batch_norm(shape[1]).to(DEV) for _ in range(2)]
    with torch.no_grad():
        for bn in bns:
            bn.weight.copy_(torch.rand(shape[1], device=DEV, generator=g) + 0.5)
            bn.bias.copy_(torch.randn(shape[1], device=DEV, generator=g))
        bns[1].load_state_dict(bns[0].state_dict())
        try:
            y = bn_relu(bns[0], x)
        finally:
            snops.BN_RELU = saved
        # float64 reference: MIOpen's fp32 training-mode batch norm itself
        # cancels on the |mean| >> std inputs (its outputs reach 25 there)
        b1 = bns[1]
        rm, rv = b1.running_mean.double(), b1.running_var.double()
        ref = torch.relu(torch.nn.functional.batch_norm(
            x.double(), rm, rv, b1.weight.double(), b1.bias.double(), training=True,
            momentum=b1.momentum, eps=b1.eps))
    assert float((y.double() - ref).abs().max()) <= 2e-5 * float(ref.abs().max()) + 1e-6
    a = bns[0]
    assert int(a.state_dict()['num_batches_tracked']) == 1     # counted on the host, added here
    for got, want in ((a.running_mean, rm), (a.running_var, rv)):
        assert float((got.double() - want).abs().max()) <= 1e-5 * float(want.abs().max()) + 1e-7


@pytest.mark.parametrize('shape,mul,add', [((64, 64, 64, 64), 3, 1), ((64, 512, 8, 8), 3, 1),
                                           ((8, 1024, 4, 4), 1, 0), ((3, 7, 4, 4), 3, 1),
                                           ((16, 32, 16, 16), 0.01, 50)])
def test_bn_relu_backward_matches_float64(shape, mul, add):
    """The generator step's batch norm + ReLU with a gradient (snops._BNReLU:
    smmd_bn_relu_fwd_save + smmd_bn_relu_bwd; resnet/block.py:42-47) against
    torch's training-mode batch norm + relu in float64 on the same state:
    output, the moving averages, dx, dgamma, dbeta."""
    from gan.core import snops
    from gan.core.snops import batch_norm, bn_relu
    g = torch.Generator(device=DEV).manual_seed(sum(shape) + 1)
    x = torch.randn(shape, device=DEV, generator=g) * mul + add
    gy = torch.randn(shape, device=DEV, generator=g)
    bn = batch_norm(shape[1]).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(shape[1], device=DEV, generator=g) + 0.5)
        bn.bias.copy_(torch.randn(shape[1], device=DEV, generator=g))
    w64 = bn.weight.detach().double().requires_grad_(True)
    b64 = bn.bias.detach().double().requires_grad_(True)
    rm, rv = bn.running_mean.double().clone(), bn.running_var.double().clone()
    x64 = x.double().requires_grad_(True)
    ref = torch.relu(torch.nn.functional.batch_norm(x64, rm, rv, w64, b64, training=True,
                                                    momentum=bn.momentum, eps=bn.eps))
    ref.backward(gy.double())
    saved = snops.BN_RELU, snops.BN_RELU_GRAD
    snops.BN_RELU = snops.BN_RELU_GRAD = True
    try:
        xx = x.clone().requires_grad_(True)
        y = bn_relu(bn, xx)
        assert y.grad_fn is not None and 'BNReLU' in type(y.grad_fn).__name__
        y.backward(gy)
    finally:
        snops.BN_RELU, snops.BN_RELU_GRAD = saved
    assert float((y.double() - ref).abs().max()) <= 2e-5 * float(ref.abs().max()) + 1e-6
    for got, want in ((bn.running_mean, rm), (bn.running_var, rv)):
        assert float((got.double() - want).abs().max()) <= 1e-5 * float(want.abs().max()) + 1e-7
    for got, want, what in ((xx.grad, x64.grad, 'dx'), (bn.weight.grad, w64.grad, 'dgamma'),
                            (bn.bias.grad, b64.grad, 'dbeta')):
        err = float((got.double() - want).abs().max())
        assert err <= 1e-4 * float(want.abs().max()) + 1e-6, (what, err)


def test_bn_relu_double_backward_is_differentiable():
    """create_graph through _BNReLU (a critic with batch norm inside the
    scaling regulariser's double backward): the second-order gradient equals
    torch's composition."""
    from gan.core import snops
    from gan.core.snops import batch_norm, bn_relu
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(6, 5, 4, 4, device=DEV, generator=g)
    outs = []
    for lib in (True, False):
        bn = batch_norm(5).to(DEV)
        with torch.no_grad():
            bn.weight.fill_(1.3)
            bn.bias.fill_(0.2)
        saved = snops.BN_RELU, snops.BN_RELU_GRAD
        snops.BN_RELU = snops.BN_RELU_GRAD = lib
        try:
            xx = x.clone().requires_grad_(True)
            y = bn_relu(bn, xx)
            gx, = torch.autograd.grad((y * y.detach().cos()).sum(), xx, create_graph=True)
            gw, = torch.autograd.grad((gx * gx).sum(), bn.weight)
        finally:
            snops.BN_RELU, snops.BN_RELU_GRAD = saved
        outs.append((gx.detach(), gw.detach()))
    for a, b in zip(*outs):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max()))
