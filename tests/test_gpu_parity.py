"""GPU parity: libsmmd_hip (through the C ABI, via the gan.core API) against the
float64 CPU oracle (oracle/smmd_oracle.py) on the same seeded inputs.

Tolerances (fp32 kernels vs float64 oracle on identical fp32 inputs):
  mmd2 / sums / kernel values:  |d| <= 1e-5 + 1e-4 |ref|
  gradients:                     |d| <= 1e-4 max|ref| + 1e-3 |ref|   (elementwise)
  spectral norm sigma, u, v:     rtol 1e-4 ; W_eff, dW: rtol 1e-4, atol 1e-6 max|ref|
"""
import zlib

import numpy as np
import pytest

torch = pytest.importorskip('torch')

from oracle import smmd_oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


def _close(got, ref, atol, rtol, what):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref)
    lim = atol + rtol * np.abs(ref)
    bad = err > lim
    assert not bad.any(), '%s: max err %.3e (worst at %s: got %r ref %r)' % (
        what, err.max(), np.argmax(err - lim), got.flat[np.argmax(err - lim)],
        ref.flat[np.argmax(err - lim)])


def _grad_close(got, ref, what):
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-12)
    _close(got, ref, 1e-4 * scale, 1e-3, what)


def _feats(m, n, d, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    X = (rng.standard_normal((m, d)) * scale).astype(np.float32)
    Y = (rng.standard_normal((n, d)) * scale + 0.3).astype(np.float32)
    return X, Y


SHAPES = [(4, 4, 1), (32, 32, 1), (64, 64, 1), (256, 256, 1), (64, 48, 3), (33, 70, 16),
          (17, 9, 32), (130, 127, 2)]


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('biased', [False, True])
def test_mmd2_fused_vs_oracle(dev, name, shape, biased):
    from gan.core import mmd
    m, n, d = shape
    X, Y = _feats(m, n, d, seed=zlib.crc32(repr((name, shape)).encode()))
    spec = O.kernel_spec(name)
    # the distance kernel's gradient -ms'(raw)(z_i - z_j) amplifies the fp32
    # rounding of the Gram expansion for near-coincident points, exactly as
    # in the reference's fp32 graph: check it against the oracle with the
    # Gram pieces formed in fp32 (oracle gram32), everything else float64
    g32 = spec.kind == 'distance'
    ref = O.mmd2(spec, X, Y, biased, gram32=g32)
    rdx, rdy = O.mmd2_grad(spec, X, Y, biased, gram32=g32)
    Xt = torch.tensor(X, device=dev, requires_grad=True)
    Yt = torch.tensor(Y, device=dev, requires_grad=True)
    val, sums = mmd.mmd2_fused(Xt, Yt, name, biased=biased, return_sums=True)
    val.backward()
    _close(val.item(), ref, 1e-5, 1e-4, 'mmd2 %s %s' % (name, shape))
    rs = O.mmd2_sums(spec, X, Y, gram32=g32)
    _close(sums[:5].cpu().numpy(), rs, 1e-4, 1e-4, 'sums')
    _grad_close(Xt.grad.cpu().numpy(), rdx, 'dX %s %s' % (name, shape))
    _grad_close(Yt.grad.cpu().numpy(), rdy, 'dY %s %s' % (name, shape))


# MFMA Gram path (smmd_gram.hip): every d > 32; features scaled by 1/sqrt(d)
# so D2 = O(1) and the kernels are not saturated at 0
GRAM_SHAPES = [(64, 64, 40), (100, 37, 128), (33, 70, 300)]


def _gfeats(m, n, d, seed):
    """N(0, 1/d) rows, Y shifted by 0.3/sqrt(d) per coordinate: D2 = O(1)."""
    X, Y = _feats(m, n, d, seed, scale=1.0 / np.sqrt(d))
    return X, (Y - np.float32(0.3) + np.float32(0.3 / np.sqrt(d))).astype(np.float32)


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
@pytest.mark.parametrize('shape', GRAM_SHAPES)
@pytest.mark.parametrize('tile', ['64', '128'])
def test_mmd2_gram_vs_oracle(dev, monkeypatch, name, shape, tile):
    """Both block tilings of the Gram path (64 x 64 with one 32 x 32 MFMA tile
    per wave; 128 x 128 with 2 x 2 per wave), forced by SMMD_GRAM_TILE on
    ragged shapes (partial row and column tiles, padded K)."""
    from gan.core import mmd
    monkeypatch.setenv('SMMD_GRAM_TILE', tile)
    m, n, d = shape
    X, Y = _gfeats(m, n, d, seed=zlib.crc32(repr(('gram', name, shape)).encode()))
    spec = O.kernel_spec(name)
    g32 = spec.kind == 'distance'          # see test_mmd2_fused_vs_oracle
    ref = O.mmd2(spec, X, Y, False, gram32=g32)
    rdx, rdy = O.mmd2_grad(spec, X, Y, False, gram32=g32)
    Xt = torch.tensor(X, device=dev, requires_grad=True)
    Yt = torch.tensor(Y, device=dev, requires_grad=True)
    val, sums = mmd.mmd2_fused(Xt, Yt, name, return_sums=True)
    val.backward()
    _close(val.item(), ref, 1e-5, 1e-4, 'mmd2 %s %s' % (name, shape))
    _close(sums[:5].cpu().numpy(), O.mmd2_sums(spec, X, Y, gram32=g32), 1e-4, 1e-4, 'sums')
    _grad_close(Xt.grad.cpu().numpy(), rdx, 'dX %s %s' % (name, shape))
    _grad_close(Yt.grad.cpu().numpy(), rdy, 'dY %s %s' % (name, shape))


@pytest.mark.parametrize('biased', [False, True])
@pytest.mark.parametrize('shape', [(256, 256, 1024), (1100, 1000, 200)])
def test_mmd2_gram_wide(dev, biased, shape):
    """d = 1024 (SURVEY 8d MFMA sweep) at N = 2 x 256, and 2100 rows (the
    128 x 128 tiling's own choice, a partial last tile) at d = 200, rbf."""
    from gan.core import mmd
    m, n, d = shape
    X, Y = _gfeats(m, n, d, seed=21)
    spec = O.kernel_spec('rbf')
    Xt = torch.tensor(X, device=dev, requires_grad=True)
    Yt = torch.tensor(Y, device=dev, requires_grad=True)
    val = mmd.mmd2_fused(Xt, Yt, 'rbf', biased=biased)
    val.backward()
    _close(val.item(), O.mmd2(spec, X, Y, biased), 1e-5, 1e-4, 'mmd2 wide')
    rdx, rdy = O.mmd2_grad(spec, X, Y, biased)
    _grad_close(Xt.grad.cpu().numpy(), rdx, 'dX wide')
    _grad_close(Yt.grad.cpu().numpy(), rdy, 'dY wide')


@pytest.mark.parametrize('name', ['rbf', 'mix_rq_dot', 'distance', 'dot', 'tanh_mix_rq'])
@pytest.mark.parametrize('shape', [(64, 64, 1), (33, 70, 16), (17, 9, 32), (130, 127, 2)])
def test_mmd2_gram_matches_row_sweep(dev, monkeypatch, name, shape):
    """SMMD_MMD_GRAM=1 forces the MFMA path where the row-sweep kernel also
    applies: the dot products are the same k-ordered fma chain, so the two
    paths agree to the order of their final sums."""
    from gan.core import mmd
    m, n, d = shape
    X, Y = _gfeats(m, n, d, seed=zlib.crc32(repr(('g-vs-f', name, shape)).encode()))
    out = {}
    for path in ('0', '1'):
        monkeypatch.setenv('SMMD_MMD_GRAM', path)
        Xt = torch.tensor(X, device=dev, requires_grad=True)
        Yt = torch.tensor(Y, device=dev, requires_grad=True)
        val, sums = mmd.mmd2_fused(Xt, Yt, name, return_sums=True)
        val.backward()
        out[path] = (val.item(), sums[:6].cpu().numpy(), Xt.grad.cpu().numpy(),
                     Yt.grad.cpu().numpy())
    a, b = out['1'], out['0']
    _close(a[0], b[0], 1e-6, 1e-5, 'mmd2 gram vs sweep')
    _close(a[1], b[1], 1e-5, 1e-5, 'sums gram vs sweep')
    # the gradient is formed as (sum_j c_ij) z_i - sum_j c_ij z_j on the MFMA
    # path and as sum_j c_ij (z_i - z_j) on the row sweep: the same tolerance
    # as against the oracle (small entries lose digits to the cancellation)
    for ga, gb, what in ((a[2], b[2], 'dX'), (a[3], b[3], 'dY')):
        _grad_close(ga, gb, what + ' gram vs sweep')


@pytest.mark.parametrize('shape', [(600, 500, 16), (300, 300, 32), (600, 500, 8)])
def test_mmd2_default_path_choice(dev, monkeypatch, shape):
    """Without SMMD_MMD_GRAM the library picks the path by size (the Gram path
    for d >= 16 from 1024 rows and d = 32 from 512 rows, else the row sweep):
    each choice against the oracle."""
    from gan.core import mmd
    monkeypatch.delenv('SMMD_MMD_GRAM', raising=False)
    m, n, d = shape
    X, Y = _gfeats(m, n, d, seed=zlib.crc32(repr(('auto', shape)).encode()))
    spec = O.kernel_spec('mix_rbf')
    Xt = torch.tensor(X, device=dev, requires_grad=True)
    Yt = torch.tensor(Y, device=dev, requires_grad=True)
    val = mmd.mmd2_fused(Xt, Yt, 'mix_rbf')
    val.backward()
    _close(val.item(), O.mmd2(spec, X, Y), 1e-5, 1e-4, 'mmd2 auto %s' % (shape,))
    rdx, rdy = O.mmd2_grad(spec, X, Y)
    _grad_close(Xt.grad.cpu().numpy(), rdx, 'dX auto')
    _grad_close(Yt.grad.cpu().numpy(), rdy, 'dY auto')


def test_mmd2_reference_api_path(dev):
    """mmd.mmd2(mmd._rbf_kernel(X, Y)) -- the exact call of SMMD.set_loss."""
    from gan.core import mmd
    X, Y = _feats(64, 64, 1, seed=7)
    Xt, Yt = torch.tensor(X, device=dev), torch.tensor(Y, device=dev)
    got = mmd.mmd2(mmd._rbf_kernel(Xt, Yt)).item()
    _close(got, O.mmd2(O.kernel_spec('rbf'), X, Y), 1e-5, 1e-4, 'api')
    # materialised tuple then the explicit-matrix estimator
    K = mmd._mix_rq_kernel(Xt, Yt)
    KXX, KXY, KYY, c = K
    rK = O.kernel_matrices(O.kernel_spec('mix_rq'), X, Y)
    for a, b in zip((KXX, KXY, KYY), rK[:3]):
        _close(a.cpu().numpy(), b, 1e-5, 1e-4, 'kmat')
    assert c == 3.0
    _close(mmd.mmd2((KXX, KXY, KYY, c)).item(), O.mmd2_from_K(*rK), 1e-5, 1e-4, 'tuple')


def test_mmd2_deterministic(dev):
    from gan.core import mmd
    X, Y = _feats(256, 256, 4, seed=3)
    Xt, Yt = torch.tensor(X, device=dev), torch.tensor(Y, device=dev)
    a = [mmd.mmd2_fused(Xt, Yt, 'mix_rbf').item() for _ in range(5)]
    assert len(set(a)) == 1


# ---------------------------------------------------------------------------
# The 2-D tiled path (csrc/smmd_mmd_tile.hip, d <= 8): the configs' global
# batch sizes (C4: 8 GPUs x 64 = 512 rows per side; C5: 8 x 256 = 2048) and
# ragged shapes (partial row tiles, chunks straddling the X | Y boundary).
# ---------------------------------------------------------------------------
TILE_NAMES = ['rbf', 'mix_rbf', 'mix_rq_dot', 'distance', 'dot', 'tanh_mix_rq']


@pytest.mark.parametrize('name', TILE_NAMES)
@pytest.mark.parametrize('shape', [(512, 512, 1), (2048, 2048, 1), (1000, 777, 3),
                                   (65, 4100, 2), (129, 64, 8)])
def test_mmd2_tile_large_vs_oracle(dev, name, shape):
    from gan.core import mmd
    m, n, d = shape
    X, Y = _feats(m, n, d, seed=zlib.crc32(repr(('tile', name, shape)).encode()))
    spec = O.kernel_spec(name)
    g32 = spec.kind == 'distance'          # see test_mmd2_fused_vs_oracle
    Xt = torch.tensor(X, device=dev, requires_grad=True)
    Yt = torch.tensor(Y, device=dev, requires_grad=True)
    val, sums = mmd.mmd2_fused(Xt, Yt, name, return_sums=True)
    val.backward()
    _close(val.item(), O.mmd2(spec, X, Y, gram32=g32), 1e-5, 1e-4, 'mmd2 %s %s' % (name, shape))
    _close(sums[:5].cpu().numpy(), O.mmd2_sums(spec, X, Y, gram32=g32), 1e-4 * max(m, n) / 64,
           1e-4, 'sums')
    rdx, rdy = O.mmd2_grad(spec, X, Y, gram32=g32)
    _grad_close(Xt.grad.cpu().numpy(), rdx, 'dX %s %s' % (name, shape))
    _grad_close(Yt.grad.cpu().numpy(), rdy, 'dY %s %s' % (name, shape))


def _abi_mmd2_rows(dev, spec_name, X, Y, xb, xe, yb, ye, ws):
    """One smmd_mmd2_fwd call through the C ABI on the row slices
    [xb, xe) of X and [yb, ye) of Y against all columns: (sums[8], dX rows,
    dY rows)."""
    from gan.core import _lib, mmd
    L = _lib.lib()
    m, d = X.shape
    n = Y.shape[0]
    sums = torch.empty(8, device=dev)
    out = torch.empty(1, device=dev)
    gx = torch.empty(max(xe - xb, 1), d, device=dev)
    gy = torch.empty(max(ye - yb, 1), d, device=dev)
    _lib.check(L.smmd_mmd2_fwd(mmd.get_kernel_spec(spec_name).desc(), _lib.ptr(X), m, _lib.ptr(Y),
                               n, d, 0, xb, xe, yb, ye, _lib.ptr(sums), _lib.ptr(out),
                               _lib.ptr(gx), _lib.ptr(gy), _lib.ptr(ws), ws.numel(),
                               _lib.stream_handle(dev)), 'smmd_mmd2_fwd')
    return sums, gx[:xe - xb], gy[:ye - yb]


@pytest.mark.parametrize('name', ['rbf', 'mix_rq', 'distance'])
@pytest.mark.parametrize('per_rank', [64, 256])
def test_mmd2_row_sharded_8way(dev, name, per_rank):
    """The all-gather mode of 8 ranks emulated on one device:
    8 calls on rank r's row slices of X and Y against all 8 * per_rank
    columns, the 8 sums vectors added, then smmd_mmd2_combine -- equal to the
    one-process oracle on the concatenated batch (C4: 8 x 64, C5: 8 x 256),
    and each call's row gradients equal that process's rows."""
    from gan.core import _lib, mmd
    world = 8
    N = world * per_rank
    X, Y = _feats(N, N, 1, seed=zlib.crc32(repr(('shard', name, per_rank)).encode()))
    spec = O.kernel_spec(name)
    g32 = spec.kind == 'distance'
    Xd, Yd = torch.tensor(X, device=dev), torch.tensor(Y, device=dev)
    L = _lib.lib()
    ws = torch.zeros(L.smmd_mmd2_workspace_bytes(N, N, 1), dtype=torch.uint8, device=dev)
    total = torch.zeros(8, device=dev, dtype=torch.float64)
    gxs, gys = [], []
    for r in range(world):
        s, gx, gy = _abi_mmd2_rows(dev, name, Xd, Yd, r * per_rank, (r + 1) * per_rank,
                                   r * per_rank, (r + 1) * per_rank, ws)
        total += s.double()
        gxs.append(gx.cpu().numpy())
        gys.append(gy.cpu().numpy())
    out = torch.empty(1, device=dev)
    _lib.check(L.smmd_mmd2_combine(mmd.get_kernel_spec(name).desc(),
                                   _lib.ptr(total.float().contiguous()), N, N, 0, _lib.ptr(out),
                                   _lib.stream_handle(dev)), 'smmd_mmd2_combine')
    _close(out.item(), O.mmd2(spec, X, Y, gram32=g32), 1e-5, 1e-4, 'sharded mmd2')
    rdx, rdy = O.mmd2_grad(spec, X, Y, gram32=g32)
    _grad_close(np.concatenate(gxs), rdx, 'sharded dX')
    _grad_close(np.concatenate(gys), rdy, 'sharded dY')


@pytest.mark.parametrize('name', ['rbf', 'mix_rq_dot', 'distance', 'dot', 'tanh_mix_rq'])
@pytest.mark.parametrize('shape', [(64, 64, 1), (300, 200, 2), (2048, 2048, 1)])
def test_mmd2_tile_matches_row_sweep(dev, monkeypatch, name, shape):
    """SMMD_MMD_TILE=0 selects the round-1 row sweep: both paths agree to the
    order of their sums."""
    from gan.core import mmd
    m, n, d = shape
    X, Y = _feats(m, n, d, seed=zlib.crc32(repr(('t-vs-s', name, shape)).encode()))
    out = {}
    for path in ('0', '1'):
        monkeypatch.setenv('SMMD_MMD_TILE', path)
        Xt = torch.tensor(X, device=dev, requires_grad=True)
        Yt = torch.tensor(Y, device=dev, requires_grad=True)
        val, sums = mmd.mmd2_fused(Xt, Yt, name, return_sums=True)
        val.backward()
        out[path] = (val.item(), sums[:6].cpu().numpy(), Xt.grad.cpu().numpy(),
                     Yt.grad.cpu().numpy())
    a, b = out['1'], out['0']
    _close(a[0], b[0], 1e-6, 1e-5, 'mmd2 tile vs sweep')
    _close(a[1], b[1], 1e-4 * max(m, n) / 64, 1e-5, 'sums tile vs sweep')
    for ga, gb, what in ((a[2], b[2], 'dX'), (a[3], b[3], 'dY')):
        _grad_close(ga, gb, what + ' tile vs sweep')


def test_mmd2_tile_deterministic_and_shared_workspace(dev, monkeypatch):
    """Bit-identical repeats, and one workspace shared by the three paths in
    turn (Gram, tiled, row sweep): every path leaves the counter header at
    rest for the next."""
    from gan.core import mmd
    X, Y = _feats(2048, 2048, 1, seed=5)
    Xt, Yt = torch.tensor(X, device=dev), torch.tensor(Y, device=dev)
    first = mmd.mmd2_fused(Xt, Yt, 'rbf').item()
    ref = O.mmd2(O.kernel_spec('rbf'), X, Y)
    Xw, Yw = _gfeats(300, 300, 64, seed=6)
    Xw, Yw = torch.tensor(Xw, device=dev), torch.tensor(Yw, device=dev)
    for k in range(6):
        if k % 3 == 1:
            mmd.mmd2_fused(Xw, Yw, 'rbf').item()                 # Gram path
        if k % 3 == 2:
            monkeypatch.setenv('SMMD_MMD_TILE', '0')              # row sweep
            v = mmd.mmd2_fused(Xt, Yt, 'rbf').item()
            _close(v, ref, 1e-5, 1e-4, 'row sweep after tile')
            monkeypatch.delenv('SMMD_MMD_TILE')
        assert mmd.mmd2_fused(Xt, Yt, 'rbf').item() == first
        # every arrival counter back at rest (forward-only and gradient calls)
        from gan.core import _lib
        hdr = _lib.workspace('mmd2', 0, dev)[:16384]
        assert int(hdr.count_nonzero()) == 0
    Xg, Yg = Xt.clone().requires_grad_(True), Yt.clone().requires_grad_(True)
    v = mmd.mmd2_fused(Xg, Yg, 'rbf')
    v.backward()
    from gan.core import _lib
    assert int(_lib.workspace('mmd2', 0, dev)[:16384].count_nonzero()) == 0


@pytest.mark.parametrize('name', ['rbf', 'mix_rq_dot', 'distance', 'dot', 'tanh_mix_rq'])
def test_kernel_matrix_backward(dev, name):
    from gan.core import mmd
    A, B = _feats(19, 70, 3, seed=11)
    spec = O.kernel_spec(name)
    rng = np.random.default_rng(5)
    G = rng.standard_normal((19, 70))
    At = torch.tensor(A, device=dev, requires_grad=True)
    Bt = torch.tensor(B, device=dev, requires_grad=True)
    K = mmd.kernel_matrix(At, Bt, name)
    (K * torch.tensor(G, device=dev, dtype=torch.float32)).sum().backward()
    A1, B1 = (np.tanh(A.astype(np.float64)), np.tanh(B.astype(np.float64))) if spec.tanh else (A, B)
    A1, B1 = np.asarray(A1, np.float64), np.asarray(B1, np.float64)
    g32 = spec.kind == 'distance'          # see test_mmd2_fused_vs_oracle
    AB, sa, sb = O._gram(A1, B1, g32)
    rdA, rdB = O._block_grads(spec, A1, B1, AB, sa, sb, G, g32)
    if spec.tanh:
        rdA = rdA * (1 - A1 ** 2)
        rdB = rdB * (1 - B1 ** 2)
    _close(K.detach().cpu().numpy(), O.kernel_matrices(spec, A, B, K_XY_only=True, gram32=g32),
           1e-5, 1e-4, 'K')
    _grad_close(At.grad.cpu().numpy(), rdA, 'gA')
    _grad_close(Bt.grad.cpu().numpy(), rdB, 'gB')


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
def test_witness_forward(dev, name):
    from gan.core import mmd
    rng = np.random.default_rng(21)
    H = rng.standard_normal((40, 2)).astype(np.float32)
    R = rng.standard_normal((40, 2)).astype(np.float32)
    F = (rng.standard_normal((40, 2)) + 0.5).astype(np.float32)
    spec = O.kernel_spec(name)
    g32 = spec.kind == 'distance'          # see test_mmd2_fused_vs_oracle
    dH, w = mmd.witness_and_grad(*(torch.tensor(a, device=dev) for a in (H, R, F)), kernel=name)
    _close(w.cpu().numpy(), O.witness(spec, H, R, F, g32), 1e-5, 1e-4, 'witness')
    _grad_close(dH.cpu().numpy(), O.witness_grad_H(spec, H, R, F, g32), 'dH')


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
def test_witness_second_order(dev, name):
    """d <g, dH>/d(H, R, F) against central differences of the float64 oracle,
    for every kernel (incl. distance / dot and the tanh-input ones)."""
    from gan.core import mmd
    rng = np.random.default_rng(4)
    H = rng.standard_normal((12, 2))
    R = rng.standard_normal((10, 2))
    F = rng.standard_normal((9, 2)) + 0.5
    g = rng.standard_normal((12, 2))
    spec = O.kernel_spec(name)
    ts = [torch.tensor(a, device=dev, dtype=torch.float32, requires_grad=True) for a in (H, R, F)]
    dH, _ = mmd.witness_and_grad(*ts, kernel=name)
    (dH * torch.tensor(g, device=dev, dtype=torch.float32)).sum().backward()
    H32, R32, F32 = (np.asarray(a, np.float32).astype(np.float64) for a in (H, R, F))

    def f(Hh, Rr, Ff):
        return np.sum(O.witness_grad_H(spec, Hh, Rr, Ff) * g)

    for idx, arr in enumerate((H32, R32, F32)):
        num = np.zeros_like(arr)
        for k in np.ndindex(arr.shape):
            e = 1e-5
            ap, am = arr.copy(), arr.copy()
            ap[k] += e
            am[k] -= e
            args_p = [H32, R32, F32]
            args_m = [H32, R32, F32]
            args_p[idx], args_m[idx] = ap, am
            num[k] = (f(*args_p) - f(*args_m)) / (2 * e)
        _close(ts[idx].grad.cpu().numpy(), num, 2e-3 * max(np.abs(num).max(), 1e-6), 2e-3,
               'witness 2nd order arg %d' % idx)


SN_SHAPES = [(64, 27), (128, 576), (256, 1152), (1, 1024), (1024, 4608), (7, 13), (130, 300)]

def _sn_bank(dev, shapes, seed, num_iters=1, fold=()):
    """SN bank over plain modules; shapes (N, K), or (N, C, 3, 3) for a conv,
    with fold[i] marking a ConvMeanPool conv (the bank then writes its
    pool-folded 4 x 4 filter, smmd_sn_layer.fold)."""
    from gan.core import sn
    rng = np.random.default_rng(seed)
    mods = []
    for i, shp in enumerate(shapes):
        m = torch.nn.Module()
        m.weight = torch.nn.Parameter(torch.tensor(rng.standard_normal(shp) * 0.05,
                                                   dtype=torch.float32, device=dev))
        m.sn_scale = torch.nn.Parameter(torch.tensor([1.3], device=dev))
        m.sn_fold = bool(fold[i]) if i < len(fold) else False
        mods.append(m)
    return mods, sn.SpectralNormBank(mods, num_iters=num_iters), rng


def _check_sn(mods, bank, u0, outs, Gs, num_iters=1):
    for i, (m, e) in enumerate(zip(mods, bank.entries)):
        W4d = m.weight.detach().cpu().numpy().astype(np.float64)
        W = W4d.reshape(W4d.shape[0], -1)
        sigma, u1, v1 = O.spectral_norm_rows(W, u0[i], num_iters)
        _close(e.sigma.item(), sigma, 0, 1e-4, 'sigma %d' % i)
        _close(e.u.cpu().numpy(), u1, 1e-6, 1e-4, 'u %d' % i)
        _close(e.v.cpu().numpy(), v1, 1e-6, 1e-4, 'v %d' % i)
        weff = W4d / sigma * 1.3
        if e.fold:
            weff = O.fold_pool_weight(weff)
        _close(outs[i].detach().cpu().numpy(), weff, 1e-6 * np.abs(weff).max(), 1e-4, 'Weff')
        if Gs is None:
            continue
        G = O.fold_pool_weight_adjoint(Gs[i]) if e.fold else Gs[i]
        gW, gs = O.sn_weight_backward(W, 1.3, sigma, u1, v1, G.reshape(W.shape))
        _close(m.weight.grad.cpu().numpy().reshape(W.shape), gW, 1e-4 * np.abs(gW).max(), 1e-3,
               'gW %d' % i)
        _close(m.sn_scale.grad.item(), gs, 1e-4 * abs(gs), 1e-3, 'gs %d' % i)


def _sn_roundtrip(dev, shapes, seed, fold=()):
    mods, bank, rng = _sn_bank(dev, shapes, seed, fold=fold)
    u0 = [e.u.cpu().numpy().astype(np.float64) for e in bank.entries]
    outs = bank.refresh(update_u=True)
    Gs = [rng.standard_normal(tuple(o.shape)) for o in outs]
    loss = sum((o * torch.tensor(G, device=dev, dtype=torch.float32)).sum()
               for o, G in zip(outs, Gs))
    loss.backward()
    _check_sn(mods, bank, u0, outs, Gs)
    return mods, bank, outs


def test_sn_bank_vs_oracle(dev):
    _sn_roundtrip(dev, SN_SHAPES, 2)


SN_FOLD_SHAPES = [(128, 64, 3, 3), (256, 128, 3, 3), (64, 3, 3, 3), (7, 5, 3, 3),
                  (130, 300), (1024, 512, 3, 3)]


def test_sn_bank_fold_layers_vs_oracle(dev):
    """ConvMeanPool layers (fold = 1): the bank writes the pool-folded filter
    of s W / sigma directly and its backward takes dL/dW' (the fold's
    adjoint applied in the same pass), mixed with plain layers in one call."""
    mods, bank, outs = _sn_roundtrip(dev, SN_FOLD_SHAPES, 3, fold=(1, 1, 0, 1, 0, 1))
    assert [tuple(o.shape) for o in outs] == [(128, 64, 4, 4), (256, 128, 4, 4), (64, 3, 3, 3),
                                             (7, 5, 4, 4), (130, 300), (1024, 512, 4, 4)]


def test_sn_fold_matches_separate_fold_launch(dev, monkeypatch):
    """The fused path equals W_eff followed by smmd_fold_pool_weights (the
    SMMD_SN_FOLD=0 path): the same arithmetic in the same order."""
    from gan.core import convops, sn
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(sn, 'SN_FOLD', fused)
        torch.manual_seed(0)
        mods, bank, rng = _sn_bank(dev, SN_FOLD_SHAPES[:2], 5, fold=(1, 1))
        outs = bank.refresh(update_u=True)
        if not fused:
            outs = convops.fold_pool_weights(outs)
        G = [torch.tensor(rng.standard_normal(tuple(o.shape)), device=dev, dtype=torch.float32)
             for o in outs]
        torch.autograd.backward(outs, G)
        res[fused] = ([o.detach().cpu().numpy() for o in outs],
                      [m.weight.grad.cpu().numpy() for m in mods])
    for a, b in zip(res[True][0], res[False][0]):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(res[True][1], res[False][1]):
        _close(a, b, 1e-6 * np.abs(b).max(), 1e-5, 'gW fused vs separate')


def test_sn_num_iters(dev):
    """num_iters > 1 (sn.py:24-35)."""
    shapes = [(64, 27), (256, 1152), (33, 70)]
    mods, bank, rng = _sn_bank(dev, shapes, 5, num_iters=3)
    u0 = [e.u.cpu().numpy().astype(np.float64) for e in bank.entries]
    outs = bank.refresh(update_u=True)
    _check_sn(mods, bank, u0, outs, None, num_iters=3)


def test_sn_snresnet64_critic_layers(dev):
    """the SNResNet-64 critic (df_dim 64) has exactly 14 SN
    layers, 10,099,392 SN weights, in the reference's layer order and shapes
    (architecture.py:410-434); its 4 ConvMeanPool convs take the fused fold.
    The whole bank runs forward + backward against the oracle."""
    from gan.core.architecture import SNResNetDiscriminator
    from gan.core.snops import sn_modules
    D = SNResNetDiscriminator(64, 1, False, with_sn=True, with_learnable_sn_scale=True)
    layers = sn_modules(D)
    shapes = [tuple(m.weight.shape) for m in layers]
    assert len(shapes) == 14
    assert sum(int(np.prod(s)) for s in shapes) == 10_099_392
    expect = [(64, 3, 3, 3)]                          # d_h0_conv
    for ci, co in ((64, 128), (128, 256), (256, 512), (512, 1024)):
        # d_res{i}: .Conv1, .Conv2 (ConvMeanPool), .Shortcut (1 x 1, MeanPoolConv)
        expect += [(ci, ci, 3, 3), (co, ci, 3, 3), (co, ci, 1, 1)]
    expect.append((1, 1024))                          # d_h5_lin
    assert shapes == expect
    folds = [bool(getattr(m, 'sn_fold', False)) for m in layers]
    assert folds == [False] + [False, True, False] * 4 + [False]
    _sn_roundtrip(dev, shapes, 11, fold=folds)


def test_sn_repeated_calls_track_weights(dev):
    """Workspace state carried between calls (slabs, u') never leaks into the
    next call: new weights each call, checked against the oracle from the u
    the previous call left."""
    shapes = [(1024, 4608), (64, 27), (1, 1024), (130, 300), (2048, 9216)]
    mods, bank, rng = _sn_bank(dev, shapes, 21)
    for _ in range(4):
        with torch.no_grad():
            for m in mods:
                m.weight.add_(torch.randn_like(m.weight) * 0.01)
        u0 = [e.u.cpu().numpy().astype(np.float64) for e in bank.entries]
        outs = bank.refresh(update_u=True)
        _check_sn(mods, bank, u0, outs, None)


def test_sn_reference_layout(dev):
    """spectral_normed_weight on a TF-layout conv weight [kh, kw, Cin, Cout]."""
    from gan.core import sn
    rng = np.random.default_rng(9)
    W = rng.standard_normal((3, 3, 16, 32)).astype(np.float32)
    u = O.np.asarray(rng.standard_normal((1, 32)), np.float32)
    Wb, sigma, u1, _ = O.spectral_normed_weight(W, u)
    ut = torch.tensor(u, device=dev)
    got, s = sn.spectral_normed_weight(torch.tensor(W, device=dev), u=ut, with_sigma=True)
    _close(s.item(), sigma, 0, 1e-4, 'sigma')
    _close(got.cpu().numpy(), Wb, 1e-6, 1e-4, 'W_bar')
    _close(ut.cpu().numpy(), u1, 1e-6, 1e-4, 'u assign')


@pytest.mark.parametrize('variant', ['grad', 'value_and_grad'])
@pytest.mark.parametrize('sqrt_scale', [False, True])
def test_scaled_loss_vs_oracle(dev, variant, sqrt_scale):
    from gan.core import ops
    rng = np.random.default_rng(13)
    b = 24
    jac = rng.standard_normal((2, b, 3, 9, 7)).astype(np.float32) * 0.1
    feat = rng.standard_normal((b, 2)).astype(np.float32)
    base = np.float32(0.37)
    jt = torch.tensor(jac, device=dev, requires_grad=True)
    ft = torch.tensor(feat, device=dev, requires_grad=True)
    bt = torch.tensor(base, device=dev, requires_grad=True)
    g, aux = ops.scaled_loss(bt, jt, ft, sc=10.0, variant=variant, sqrt_scale=sqrt_scale)
    J = np.mean(sum(O.squared_norm_per_sample(jac[c]) for c in range(2)))
    nD = np.mean(feat.astype(np.float64) ** 2)
    sc_ = O.scale_factor(J, 10.0, nD, variant)
    f = np.sqrt(sc_) if sqrt_scale else sc_
    _close(aux[3].item(), J, 0, 1e-5, 'J')
    _close(aux[2].item(), sc_, 0, 1e-5, 'scale')
    _close(g.item(), base * f, 0, 1e-5, 'g_loss')
    g.backward()
    fp = 0.5 / np.sqrt(sc_) if sqrt_scale else 1.0
    coefq = base * fp * (-10.0 * sc_ ** 2)
    _close(bt.grad.item(), f, 0, 1e-5, 'd base')
    _grad_close(jt.grad.cpu().numpy(), coefq * 2.0 / b * jac.astype(np.float64), 'd jac')
    if variant == 'value_and_grad':
        _grad_close(ft.grad.cpu().numpy(), coefq * 2.0 / (b * 2) * feat.astype(np.float64),
                    'd feat')


@pytest.mark.parametrize('variant', ['grad', 'value_and_grad'])
def test_scaled_loss_batch256_vs_oracle(dev, variant):
    """BASELINE configs[4]'s per-GPU size: the Jacobian of 256 real images at
    3x64x64 (12.6 MB), J / scale / g_loss and the backward against the
    float64 oracle (ops.py:228-233, model.py:366-403)."""
    from gan.core import ops
    rng = np.random.default_rng(29)
    b = 256
    jac = rng.standard_normal((1, b, 3, 64, 64)).astype(np.float32) * 0.05
    feat = rng.standard_normal((b, 1)).astype(np.float32)
    base = np.float32(0.21)
    jt = torch.tensor(jac, device=dev, requires_grad=True)
    ft = torch.tensor(feat, device=dev, requires_grad=True)
    bt = torch.tensor(base, device=dev, requires_grad=True)
    g, aux = ops.scaled_loss(bt, jt, ft, sc=10.0, variant=variant)
    J = np.mean(O.squared_norm_per_sample(jac[0]))
    nD = np.mean(feat.astype(np.float64) ** 2)
    sc_ = O.scale_factor(J, 10.0, nD, variant)
    _close(aux[3].item(), J, 0, 1e-5, 'J')
    _close(aux[2].item(), sc_, 0, 1e-5, 'scale')
    _close(g.item(), base * sc_, 0, 1e-5, 'g_loss')
    g.backward()
    coefq = base * (-10.0 * sc_ ** 2)
    _close(bt.grad.item(), sc_, 0, 1e-5, 'd base')
    _grad_close(jt.grad.cpu().numpy(), coefq * 2.0 / b * jac.astype(np.float64), 'd jac')
    if variant == 'value_and_grad':
        _grad_close(ft.grad.cpu().numpy(), coefq * 2.0 / b * feat.astype(np.float64), 'd feat')


@pytest.mark.parametrize('kernel,variant,b,both', [
    ('rbf', 'grad', 64, False), ('rbf', 'value_and_grad', 64, False), ('rbf', 'grad', 64, True),
    ('mix_rq_dot', 'grad', 32, False), ('mix_rbf', 'value_and_grad', 24, True),
    ('tanh_mix_rq', 'value_and_grad', 16, False), ('distance', 'grad', 20, False),
    ('rbf', 'grad', 256, False)])
def test_smmd_loss_fused_vs_oracle(dev, kernel, variant, b, both):
    """The SMMD loss in one launch (smmd_smmd_loss_fwd / _bwd, through
    mmd.pending_scale + mmd.mmd2 as set_tower_loss runs it): mmd2, J, scale,
    g_loss = mmd2 * scale and the gradients w.r.t. the features (X = d_G, Y =
    d_images, which is also nD's feature) and the Jacobian, against the float64
    oracle (smmd.py:10-23, model.py:366-403).  ``both``: mmd2 and g_loss both
    feed the backward."""
    from gan.core import mmd
    rng = np.random.default_rng(31 + b)
    X = rng.standard_normal((b, 1)).astype(np.float32)
    Y = (rng.standard_normal((b, 1)) * 0.7 + 0.3).astype(np.float32)
    jac = rng.standard_normal((1, b, 3, 16, 16)).astype(np.float32) * 0.05
    Xt = torch.tensor(X, device=dev, requires_grad=True)
    Yt = torch.tensor(Y, device=dev, requires_grad=True)
    jt = torch.tensor(jac, device=dev, requires_grad=True)
    p = mmd.ScalePending(jt, Yt, 10.0, variant)
    with mmd.pending_scale(p):
        val = mmd.mmd2(mmd.get_kernel(kernel)(Xt, Yt))
    assert p.result is not None and p.result[0] is val
    _, g, out = p.result
    spec = O.kernel_spec(kernel)
    mm = O.mmd2(spec, X, Y)
    J = np.mean(O.squared_norm_per_sample(jac[0]))
    nD = np.mean(Y.astype(np.float64) ** 2)
    sc_ = O.scale_factor(J, 10.0, nD, variant)
    _close(val.item(), mm, 1e-5, 1e-4, 'mmd2')
    _close(out[3].item(), J, 0, 1e-5, 'J')
    _close(out[2].item(), sc_, 0, 1e-5, 'scale')
    _close(g.item(), mm * sc_, 1e-6, 1e-4, 'g_loss')
    (g + val if both else g).backward()
    dX, dY = O.mmd2_grad(spec, X, Y)
    w = sc_ + (1.0 if both else 0.0)
    coefq = mm * (-10.0 * sc_ ** 2)
    gy_ref = w * dY
    if variant == 'value_and_grad':
        gy_ref = gy_ref + coefq * 2.0 / b * Y.astype(np.float64)
    _grad_close(Xt.grad.cpu().numpy(), w * dX, 'dX')
    _grad_close(Yt.grad.cpu().numpy(), gy_ref, 'dY')
    _grad_close(jt.grad.cpu().numpy(), coefq * 2.0 / b * jac.astype(np.float64), 'd jac')


def test_smmd_loss_fused_without_jacobian_grad(dev):
    """A generator step: the Jacobian is a constant, so the backward writes
    only the feature gradients (gjac NULL) and they are the same."""
    from gan.core import mmd
    rng = np.random.default_rng(5)
    X = rng.standard_normal((64, 1)).astype(np.float32)
    Y = rng.standard_normal((64, 1)).astype(np.float32)
    jac = rng.standard_normal((1, 64, 3, 8, 8)).astype(np.float32) * 0.1
    grads = []
    for need in (True, False):
        Xt = torch.tensor(X, device=dev, requires_grad=True)
        jt = torch.tensor(jac, device=dev, requires_grad=need)
        p = mmd.ScalePending(jt, None, 10.0, 'grad')
        with mmd.pending_scale(p):
            mmd.mmd2(mmd._rbf_kernel(Xt, torch.tensor(Y, device=dev)))
        p.result[1].backward()
        grads.append(Xt.grad.clone())
    assert torch.equal(grads[0], grads[1])


class _GatherEmulation:
    """A StepExchange of rank ``rank`` whose all-gather is emulated: every
    rank's packed [X; Y; stats] row built from the given per-rank tensors."""

    def __init__(self, rank, rows):
        self.world, self.rank, self.rows = len(rows), rank, rows
        self.used = False

    def gather_packed(self, X, Y):
        self.used = True
        allp = torch.stack(self.rows)
        ml, nl, d = X.shape[0], Y.shape[0], X.shape[1]
        Xa = allp[:, :ml * d].reshape(self.world * ml, d)
        Ya = allp[:, ml * d:(ml + nl) * d].reshape(self.world * nl, d)
        return allp, Xa, Ya


@pytest.mark.parametrize('world,variant', [(2, 'grad'), (8, 'grad'), (4, 'value_and_grad')])
def test_smmd_loss_gathered_vs_oracle(dev, world, variant):
    """The all-gather mode's fused loss through the ABI (smmd_smmd_loss_fwd_gathered
    + smmd_smmd_loss_bwd_ex, mmd._SMMDLossGathered) with the all-gather emulated:
    every rank gets mmd2, J, scale and g_loss of the global batch (the float64
    oracle on the concatenated batch), bit-identical across ranks, and the
    gradients of its own rows and Jacobian (normaliser: the global batch)."""
    from gan.core import mmd, ops
    b = 16
    B = world * b
    rng = np.random.default_rng(7 + world)
    X = rng.standard_normal((B, 1)).astype(np.float32)
    Y = (rng.standard_normal((B, 1)) * 0.7 + 0.3).astype(np.float32)
    jac = rng.standard_normal((1, B, 3, 8, 8)).astype(np.float32) * 0.05
    v = {'grad': 0, 'value_and_grad': 1}[variant]
    ranks, rows = [], []
    for r in range(world):
        sl = slice(r * b, (r + 1) * b)
        Xt = torch.tensor(X[sl], device=dev, requires_grad=True)
        Yt = torch.tensor(Y[sl], device=dev, requires_grad=True)
        jt = torch.tensor(jac[:, sl], device=dev, requires_grad=True)
        # this rank's (J, nD) shares over the global batch (ops.scaling_partials)
        L = mmd._lib.lib()
        out = torch.empty(8, device=dev)
        ws = mmd._lib.workspace('scaled_loss', L.smmd_scaled_loss_workspace_bytes(b, 3 * 64), dev)
        assert L.smmd_scaled_loss_fwd(mmd._lib.ptr(jt.detach()), 1, b, B, 3 * 64,
                                      mmd._lib.ptr(Yt.detach()), 1, None, 0.0, v, 0,
                                      mmd._lib.ptr(out), None, mmd._lib.ptr(ws), ws.numel(),
                                      mmd._lib.stream_handle(dev)) == 0
        rows.append(torch.cat([Xt.detach().reshape(-1), Yt.detach().reshape(-1), out[3:5]]))
        ranks.append((Xt, Yt, jt))
    spec = O.kernel_spec('rbf')
    mm = O.mmd2(spec, X, Y)
    J = np.mean(O.squared_norm_per_sample(jac[0]))
    nD = np.mean(Y.astype(np.float64) ** 2)
    sc_ = O.scale_factor(J, 10.0, nD, variant)
    dX, dY = O.mmd2_grad(spec, X, Y)
    coefq = mm * (-10.0 * sc_ ** 2)
    outs = []
    for r, (Xt, Yt, jt) in enumerate(ranks):
        ex = _GatherEmulation(r, rows)
        val, g, _, out = mmd._SMMDLossGathered.apply(Xt, Yt, jt, Yt if v else None,
                                                     mmd.get_kernel_spec("rbf"), False, 10.0,
                                                     v, ex)
        outs.append(out.clone())
        _close(val.item(), mm, 1e-5, 1e-4, 'mmd2')
        _close(out[3].item(), J, 0, 1e-5, 'J')
        _close(out[2].item(), sc_, 0, 1e-5, 'scale')
        _close(g.item(), mm * sc_, 1e-6, 1e-4, 'g_loss')
        g.backward()
        sl = slice(r * b, (r + 1) * b)
        gy_ref = sc_ * dY[sl]
        if v:
            gy_ref = gy_ref + coefq * 2.0 / B * Y[sl].astype(np.float64)
        _grad_close(Xt.grad.cpu().numpy(), sc_ * dX[sl], 'dX')
        _grad_close(Yt.grad.cpu().numpy(), gy_ref, 'dY')
        _grad_close(jt.grad.cpu().numpy(), coefq * 2.0 / B * jac[:, sl].astype(np.float64),
                    'd jac')
    assert all(torch.equal(o, outs[0]) for o in outs)     # the same bits on every rank


def test_scaled_loss_workspace_reuse(dev):
    """The squared-norm pass elects its finalizing block by a ticket at a fixed
    offset of the cached workspace; calls with fewer rows reuse the buffer
    (whose partial slab then holds an earlier call's values) and must still
    finalize once, correctly."""
    from gan.core import ops
    rng = np.random.default_rng(17)
    for b, per in ((24, (3, 64, 64)), (5, (3, 9, 7)), (64, (3, 32, 32)), (1, (3, 4, 4))):
        jac = rng.standard_normal((1, b) + per).astype(np.float32) * 0.1
        jt = torch.tensor(jac, device=dev)
        bt = torch.tensor(np.float32(0.5), device=dev)
        g, aux = ops.scaled_loss(bt, jt, None, sc=10.0)
        J = np.mean(O.squared_norm_per_sample(jac[0]))
        _close(aux[3].item(), J, 0, 1e-5, 'J b=%d' % b)
        _close(g.item(), 0.5 * O.scale_factor(J, 10.0, 0.0, 'grad'), 0, 1e-5, 'g_loss b=%d' % b)


def test_smmd_objective_end_to_end(dev):
    """SMMD generator loss through a tanh-MLP critic: value vs the oracle and
    d loss / d critic params (double backward through jac) vs central
    differences of the float64 oracle."""
    from gan.core import mmd, ops
    rng = np.random.default_rng(17)
    P, Hd = 12, 6
    xf = rng.uniform(0, 1, (16, P))
    xr = rng.uniform(0, 1, (16, P))
    W1 = rng.standard_normal((P, Hd)) * 0.5
    W2 = rng.standard_normal((Hd, 1)) * 0.5
    ref, _, _ = O.smmd_objective(O.kernel_spec('rbf'), xf.astype(np.float32),
                                 xr.astype(np.float32), W1.astype(np.float32),
                                 W2.astype(np.float32))
    t = lambda a, g=False: torch.tensor(a, device=dev, dtype=torch.float32, requires_grad=g)
    W1t, W2t = t(W1, True), t(W2, True)
    xft, xrt = t(xf), t(xr, True)
    dG = torch.tanh(xft @ W1t) @ W2t
    dI = torch.tanh(xrt @ W1t) @ W2t
    m2 = mmd.mmd2(mmd._rbf_kernel(dG, dI))
    jac = ops.jacobian_columns(dI, xrt)
    g_loss, aux = ops.scaled_loss(m2, jac, None, sc=10.0)
    _close(g_loss.item(), ref, 1e-6, 1e-4, 'smmd g_loss')
    g_loss.backward()
    W1_32, W2_32 = W1.astype(np.float32).astype(np.float64), W2.astype(np.float32).astype(np.float64)
    xf32, xr32 = xf.astype(np.float32).astype(np.float64), xr.astype(np.float32).astype(np.float64)
    for which, arr, got in ((0, W1_32, W1t.grad), (1, W2_32, W2t.grad)):
        num = np.zeros_like(arr)
        for k in np.ndindex(arr.shape):
            e = 1e-6
            ap, am = arr.copy(), arr.copy()
            ap[k] += e
            am[k] -= e
            if which == 0:
                fp = O.smmd_objective(O.kernel_spec('rbf'), xf32, xr32, ap, W2_32)[0]
                fm = O.smmd_objective(O.kernel_spec('rbf'), xf32, xr32, am, W2_32)[0]
            else:
                fp = O.smmd_objective(O.kernel_spec('rbf'), xf32, xr32, W1_32, ap)[0]
                fm = O.smmd_objective(O.kernel_spec('rbf'), xf32, xr32, W1_32, am)[0]
            num[k] = (fp - fm) / (2 * e)
        _close(got.cpu().numpy(), num, 2e-3 * np.abs(num).max(), 2e-3, 'dparam %d' % which)


def test_clip_adam_vs_oracle(dev):
    from gan.core import optim
    rng = np.random.default_rng(23)
    sizes = [5, 70000, 1, 33000, 0, 128]
    shapes = [(s,) for s in sizes]
    params = [torch.nn.Parameter(torch.tensor(rng.standard_normal(s), dtype=torch.float32,
                                              device=dev)) for s in shapes]
    opt = optim.FlatAdam(params, lr=2e-4, beta1=0.5, beta2=0.9, clip_norm=1.0)
    ref_p = [p.detach().cpu().numpy().astype(np.float64) for p in params]
    ref_m = [np.zeros_like(p) for p in ref_p]
    ref_v = [np.zeros_like(p) for p in ref_p]
    for step in range(1, 4):
        grads = [rng.standard_normal(s).astype(np.float32) * (3.0 if i % 2 else 0.1)
                 for i, s in enumerate(shapes)]
        opt.zero_grad()
        for p, g in zip(params, grads):
            p.grad.copy_(torch.tensor(g, device=dev))
        opt.step()
        for i, g in enumerate(grads):
            gc = O.clip_by_norm(g, 1.0) if g.size else g.astype(np.float64)
            ref_p[i], ref_m[i], ref_v[i] = O.adam_step(ref_p[i], ref_m[i], ref_v[i], gc, step,
                                                       2e-4)
    for p, r in zip(params, ref_p):
        _close(p.detach().cpu().numpy(), r, 1e-6, 1e-5, 'adam param')


def test_missing_inputs_fail_loudly(dev):
    from gan.core import mmd, _lib
    with pytest.raises(_lib.SmmdError):
        mmd.mmd2_fused(torch.zeros(4, 1), torch.zeros(4, 1))   # CPU tensors: no CPU path


# ---- polynomial-kernel MMD: KID scorer and 3-sample test -------------------
def _codes(n, dim, seed, scale=1.0):
    """Synthetic pool3-like codes: |N(0, 1)| (Inception is unavailable offline)."""
    rng = np.random.default_rng(seed)
    return (np.abs(rng.standard_normal((n, dim))) * scale).astype(np.float32)


@pytest.mark.parametrize('na,nb,dim', [(100, 100, 64), (257, 130, 2048), (64, 64, 33)])
def test_poly_kernel_sums_vs_oracle(dev, na, nb, dim):
    from gan.core import mmd
    A, B = _codes(na, dim, 1), _codes(nb, dim, 2, 1.1)
    s = mmd.polynomial_kernel_sums(torch.tensor(A, device=dev), torch.tensor(B, device=dev))
    K = O.polynomial_kernel(A, B)
    d = np.diagonal(K)
    # each K is an fp32 dot over dim features then cubed (as the reference's
    # float32 sklearn call): ~3e-6 relative per element at dim 2048; the
    # double sums average that down
    _close(s.diag.cpu().numpy(), d, 0, 2e-5, 'diag')
    _close(s.rows.cpu().numpy(), K.sum(1), 0, 1e-5, 'rows')
    _close(s.cols.cpu().numpy(), K.sum(0), 0, 1e-5, 'cols')
    _close(s.stats.cpu().numpy(), [K.sum(), (K * K).sum(), d.sum(), (d * d).sum()], 0, 1e-5,
           'stats')


@pytest.mark.parametrize('mmd_est', ['unbiased', 'biased', 'u-statistic'])
def test_polynomial_mmd_vs_oracle(dev, mmd_est):
    """KID of gan/compute_scores.py:232-335 at 512 x 2048 codes."""
    from gan import compute_scores as cs
    from gan.core import mmd
    X, Y = _codes(512, 2048, 3), _codes(512, 2048, 4, 1.05)
    Kxx, Kyy, Kxy = (O.polynomial_kernel(a, b) for a, b in ((X, X), (Y, Y), (X, Y)))
    ref_m, ref_v = O.mmd2_and_variance(Kxx, Kxy, Kyy, mmd_est=mmd_est, var_at_m=1000)
    Xt, Yt = torch.tensor(X, device=dev), torch.tensor(Y, device=dev)
    sums = [mmd.polynomial_kernel_sums(a, b) for a, b in ((Xt, Xt), (Yt, Yt), (Xt, Yt))]
    got = mmd.poly_mmd2_and_variance(*sums, var_at_m=1000, mmd_est=mmd_est).cpu().numpy()
    scale = Kxy.mean()              # the estimator is a difference of O(mean K) terms
    _close(got[0], ref_m, 1e-6 * scale, 1e-4, 'mmd2 %s' % mmd_est)
    _close(got[1], ref_v, 1e-6 * abs(ref_v) + 1e-9 * scale ** 2, 1e-2, 'var %s' % mmd_est)
    if mmd_est == 'unbiased':
        m2, v2 = cs.polynomial_mmd(X, Y, var_at_m=1000)
        _close([m2, v2], got, 0, 1e-12, 'polynomial_mmd')
        # the materialised-matrix entry point on the same matrices
        m3, v3 = cs._mmd2_and_variance(Kxx.astype(np.float32), Kxy.astype(np.float32),
                                       Kyy.astype(np.float32), var_at_m=1000)
        _close(m3, ref_m, 1e-6 * scale, 1e-4, '_mmd2_and_variance')


def test_polynomial_mmd_averages_subsets(dev):
    from gan import compute_scores as cs
    G, R = _codes(1500, 2048, 5), _codes(1200, 2048, 6)
    np.random.seed(0)
    got = cs.polynomial_mmd_averages(G, R, n_subsets=3, subset_size=1000, ret_var=False)
    np.random.seed(0)
    for i in range(3):
        g = G[np.random.choice(len(G), 1000, replace=False)]
        r = R[np.random.choice(len(R), 1000, replace=False)]
        Ks = [O.polynomial_kernel(a, b) for a, b in ((g, g), (g, r), (r, r))]
        ref = O.mmd2_and_variance(*Ks, var_at_m=1200, ret_var=False)
        _close(got[i], ref, 1e-6 * Ks[1].mean(), 1e-4, 'subset %d' % i)


def test_three_sample_diff_and_ratio(dev):
    """gan/core/mmd.py:429-512 as the LR scheduler calls it (gan/utils/scorer.py:124-162)."""
    from gan.core import mmd
    X, Y, Z = _codes(300, 2048, 7), _codes(300, 2048, 8, 1.02), _codes(300, 2048, 9, 1.08)
    saved = mmd.np_diff_polynomial_mmd2_and_ratio_with_saving(X, Z, None)
    diff, ratio, _ = mmd.np_diff_polynomial_mmd2_and_ratio_with_saving(X, Y, saved)
    K = lambda a, b: O.polynomial_kernel(a, b)
    ref = O.diff_mmd2_and_ratio_from_sums(O.np_get_sums(K(X, Y), K(Y, Y)),
                                          O.np_get_sums(K(X, Z), K(Z, Z)), 300)
    scale = K(X, Y).mean()
    _close(diff, ref[0], 1e-6 * scale, 1e-4, 'mmd2_diff')
    _close(ratio, ref[1], 1e-3 * abs(ref[1]) + 1e-3, 1e-3, 'ratio')
