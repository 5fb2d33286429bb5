"""The weight gradients' accumulating entry points (ABI 13:
smmd_conv3x3_thin_wgrad_acc, smmd_wino3x3_wgrad_acc, smmd_wino4x4s2_wgrad_acc,
smmd_conv1x1_wgrad_acc): each adds the weight gradient into the output
buffer instead of overwriting it, bit-identical to the plain entry followed by
one fp32 add (convops._late_gw computes an SN weight's later contributions
straight into its first one this way)."""
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


def _check(fn, shape_w, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    base = torch.randn(*shape_w, device=DEV, generator=g)
    plain = fn(None)
    acc = base.clone()
    got = fn(acc)
    assert got is acc
    assert torch.equal(got, base + plain)
    # twice: the second call adds onto the first sum
    again = fn(acc)
    assert again is acc and torch.equal(acc, (base + plain) + plain)


# (N, ci, co, H): the generator's / critic's first layers at batch 64, small
THIN = [(64, 3, 64, 64), (4, 3, 64, 16), (64, 64, 3, 64)]
WINO = [(64, 64, 64, 32), (64, 512, 512, 8), (4, 128, 64, 16), (2, 64, 128, 8)]
S2 = [(64, 64, 128, 64), (64, 512, 512, 8), (4, 64, 128, 16)]
C1 = [(64, 64, 128, 32), (64, 512, 1024, 4), (4, 128, 256, 8)]


@pytest.mark.parametrize('shape', THIN)
def test_thin_wgrad_acc(shape):
    from gan.core import convops
    N, ci, co, H = shape
    g = torch.Generator(device=DEV).manual_seed(ci + co + H)
    x = torch.randn(N, ci, H, H, device=DEV, generator=g)
    gy = torch.randn(N, co, H, H, device=DEV, generator=g)
    assert convops._is_thin(x, torch.empty(co, ci, 3, 3, device=DEV), [1, 1], [1, 1])
    _check(lambda into: convops._thin_wgrad(gy, x, into), (co, ci, 3, 3), H)


@pytest.mark.parametrize('shape', WINO)
def test_wino_wgrad_acc(shape):
    from gan.core import convops
    N, ci, co, H = shape
    g = torch.Generator(device=DEV).manual_seed(ci + co + H + 1)
    x = torch.randn(N, ci, H, H, device=DEV, generator=g)
    gy = torch.randn(N, co, H, H, device=DEV, generator=g)
    _check(lambda into: convops._wino_wgrad(x, gy, into), (co, ci, 3, 3), H + 1)


@pytest.mark.parametrize('shape', S2)
def test_s2_wgrad_acc(shape):
    from gan.core import convops
    N, ci, co, H = shape
    g = torch.Generator(device=DEV).manual_seed(ci + co + H + 2)
    x = torch.randn(N, ci, H, H, device=DEV, generator=g)
    gy = torch.randn(N, co, H // 2, H // 2, device=DEV, generator=g)
    assert convops._s2_wgrad_ok(x, gy, co)
    _check(lambda into: convops._s2_wgrad(x, gy, into), (co, ci, 4, 4), H + 2)


@pytest.mark.parametrize('shape', C1)
def test_c1_wgrad_acc(shape):
    from gan.core import convops
    N, ci, co, H = shape
    g = torch.Generator(device=DEV).manual_seed(ci + co + H + 3)
    x = torch.randn(N, ci, H, H, device=DEV, generator=g)
    gy = torch.randn(N, co, H, H, device=DEV, generator=g)
    assert convops._c1_wgrad(gy, x) is not None
    _check(lambda into: convops._c1_wgrad(gy, x, into), (co, ci, 1, 1), H + 3)


def test_bwd_gw_into_on_library_fallback():
    """_bwd(gw_into=) where no accumulating kernel runs (MIOpen's weight
    gradient): the result is added into gw_into and gw_into returned."""
    from gan.core import convops
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(2, 8, 9, 9, device=DEV, generator=g)
    w = torch.randn(16, 8, 4, 4, device=DEV, generator=g)
    gy = torch.randn(2, 16, 4, 4, device=DEV, generator=g)
    _, plain = convops._bwd(gy, x, w, [2, 2], [1, 1], (False, True, False))
    base = torch.randn(16, 8, 4, 4, device=DEV, generator=g)
    into = base.clone()
    _, got = convops._bwd(gy, x, w, [2, 2], [1, 1], (False, True, False), gw_into=into)
    assert got is into and torch.equal(got, base + plain)
