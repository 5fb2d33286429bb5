"""Pin the float64 oracle (parity unpinned by the reference: no reference tests,
fixtures or runnable TF exist -- SURVEY.md K7) with analytic known answers,
central finite differences of its own forward, and the committed golden
vectors (regression)."""
import math
import os

import numpy as np
import pytest

from oracle import smmd_oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _fd(f, x, e=1e-6):
    g = np.zeros_like(x)
    for k in np.ndindex(x.shape):
        xp, xm = x.copy(), x.copy()
        xp[k] += e
        xm[k] -= e
        g[k] = (f(xp) - f(xm)) / (2 * e)
    return g


def test_rbf_two_point_closed_form():
    # mmd.py:55-82 + :208-218 with m = n = 2, D = 1, sigma = 1
    a, b, c, d = 0.3, -1.2, 0.9, 2.0
    k = lambda p, q: math.exp(-(p - q) ** 2 / 2)
    ref = (2 * k(a, b) / 2 + 2 * k(c, d) / 2 - 2 * (k(a, c) + k(a, d) + k(b, c) + k(b, d)) / 4)
    got = O.mmd2(O.kernel_spec('rbf'), np.array([[a], [b]]), np.array([[c], [d]]))
    assert got == pytest.approx(ref, rel=1e-12)


def test_const_diag_and_trace_conventions():
    assert O.kernel_spec('rbf').const_diag == 1.0
    assert O.kernel_spec('mix_rbf').const_diag == 6.0
    assert O.kernel_spec('mix_rq_dot').const_diag == 3.0    # quirk mmd.py:182-188
    assert O.kernel_spec('mix_rq_dot').add_dot == 0.1
    assert O.kernel_spec('distance').const_diag is None
    assert O.kernel_spec('dot').const_diag is None
    # distance kernel diagonal: 2 sqrt(|x|^2 + eps) - sqrt(eps)
    X = np.array([[1.5], [-0.5]])
    KXX = O.kernel_matrices(O.kernel_spec('distance'), X, X)[0]
    assert KXX[0, 0] == pytest.approx(2 * math.sqrt(2.25 + 1e-5) - math.sqrt(1e-5))


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
def test_biased_zero_when_equal(name):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((9, 3))
    assert abs(O.mmd2(O.kernel_spec(name), X, X, biased=True)) < 1e-10


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
def test_symmetry_and_permutation(name):
    rng = np.random.default_rng(1)
    X, Y = rng.standard_normal((7, 2)), rng.standard_normal((7, 2))
    s = O.kernel_spec(name)
    v = O.mmd2(s, X, Y)
    assert O.mmd2(s, Y, X) == pytest.approx(v, rel=1e-10, abs=1e-12)
    p = rng.permutation(7)
    assert O.mmd2(s, X[p], Y[::-1]) == pytest.approx(v, rel=1e-10, abs=1e-12)


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
@pytest.mark.parametrize('biased', [False, True])
def test_mmd2_grad_matches_fd(name, biased):
    rng = np.random.default_rng(2)
    X, Y = rng.standard_normal((6, 2)), rng.standard_normal((5, 2)) + 0.4
    s = O.kernel_spec(name)
    dX, dY = O.mmd2_grad(s, X, Y, biased)
    np.testing.assert_allclose(dX, _fd(lambda x: O.mmd2(s, x, Y, biased), X), rtol=1e-5,
                               atol=1e-8)
    np.testing.assert_allclose(dY, _fd(lambda y: O.mmd2(s, X, y, biased), Y), rtol=1e-5,
                               atol=1e-8)


@pytest.mark.parametrize('name', O.KERNEL_NAMES)
def test_witness_grad_matches_fd(name):
    rng = np.random.default_rng(3)
    H, R, F = rng.standard_normal((5, 2)), rng.standard_normal((4, 2)), rng.standard_normal((6, 2))
    s = O.kernel_spec(name)
    g = O.witness_grad_H(s, H, R, F)
    np.testing.assert_allclose(g, _fd(lambda h: O.witness(s, h, R, F).sum(), H), rtol=1e-5,
                               atol=1e-8)


def test_spectral_norm_converges_to_top_singular_value():
    rng = np.random.default_rng(4)
    W = rng.standard_normal((20, 12))
    u = rng.standard_normal((1, 12))
    _, sigma, _, _ = O.spectral_normed_weight(W, u, num_iters=200)
    assert sigma == pytest.approx(np.linalg.svd(W, compute_uv=False)[0], rel=1e-8)


def test_spectral_norm_layout_invariance():
    """Reference layout [kh,kw,Cin,Cout] vs this build's [Cout, Cin*kh*kw]."""
    rng = np.random.default_rng(5)
    W = rng.standard_normal((3, 3, 4, 8))
    u = rng.standard_normal((1, 8))
    _, sigma, u1, _ = O.spectral_normed_weight(W, u)
    Wt = W.transpose(3, 2, 0, 1).reshape(8, -1)
    sigma2, u2, _ = O.spectral_norm_rows(Wt, u[0])
    assert sigma2 == pytest.approx(sigma, rel=1e-12)
    np.testing.assert_allclose(u2, u1[0], rtol=1e-12)


def test_sn_backward_matches_fd():
    rng = np.random.default_rng(6)
    W = rng.standard_normal((5, 7))
    u = rng.standard_normal(5)
    G = rng.standard_normal((5, 7))
    s = 1.7
    sigma, u1, v1 = O.spectral_norm_rows(W, u)

    def L(Wp):
        sig = float(v1 @ Wp.T @ u1)             # u, v stopped (sn.py:32-34)
        return np.sum(G * s * Wp / sig)
    gW, gs = O.sn_weight_backward(W, s, sigma, u1, v1, G)
    np.testing.assert_allclose(gW, _fd(L, W), rtol=1e-6, atol=1e-9)
    assert gs == pytest.approx(np.sum(G * W) / sigma)


def test_clip_and_adam_known_answers():
    g = np.array([3.0, 4.0])
    np.testing.assert_allclose(O.clip_by_norm(g, 1.0), [0.6, 0.8])
    np.testing.assert_allclose(O.clip_by_norm(g * 0.1, 1.0), g * 0.1)
    var, m, v = O.adam_step(np.array([1.0]), np.zeros(1), np.zeros(1), np.array([0.5]), 1,
                            lr=1e-3)
    # first step moves by ~lr * sign(g)
    assert var[0] == pytest.approx(1.0 - 1e-3, rel=1e-6)


def test_counters_schedule():
    c = O.Counters()
    seq = [c.update(step) for step in range(0, 30)]
    # steps < 20: 10 D updates then a G update (model.py:474-478)
    assert seq[:11] == [False] * 10 + [True]
    c = O.Counters()
    gsteps = sum(c.update(s) for s in range(100, 160))
    assert gsteps == 10          # 5 D + 1 G per cycle


def test_mlp_jacobian_matches_fd():
    rng = np.random.default_rng(7)
    x = rng.uniform(0, 1, (3, 5))
    W1, W2 = rng.standard_normal((5, 4)), rng.standard_normal((4, 2))
    got = O.mlp_critic_sq_jac(x, W1, W2)
    for b in range(3):
        tot = 0.0
        for i in range(2):
            gi = _fd(lambda xx: O.mlp_critic(xx[None], W1, W2)[0][0, i], x[b].copy())
            tot += np.sum(gi ** 2)
        assert got[b] == pytest.approx(tot, rel=1e-6)


def test_golden_mmd_regression():
    z = np.load(os.path.join(GOLDEN, 'mmd2_cases.npz'))
    keys = sorted({k.rsplit('__', 1)[0] for k in z.files})
    assert len(keys) >= 100
    for key in keys:
        kname, shape, b = key.split('__')
        s = O.kernel_spec(kname)
        X, Y = z[key + '__X'], z[key + '__Y']
        assert O.mmd2(s, X, Y, b == 'b1') == pytest.approx(float(z[key + '__mmd2']), rel=1e-12,
                                                           abs=1e-15)
        if shape.startswith('4_'):
            dX, dY = O.mmd2_grad(s, X, Y, b == 'b1')
            np.testing.assert_allclose(dX, z[key + '__dX'], rtol=1e-12, atol=1e-15)


def test_golden_sn_regression():
    z = np.load(os.path.join(GOLDEN, 'sn_cases.npz'))
    keys = sorted({k.rsplit('__', 1)[0] for k in z.files})
    for key in keys:
        sigma, u1, _ = O.spectral_norm_rows(z[key + '__W'], z[key + '__u'])
        assert sigma == pytest.approx(float(z[key + '__sigma']), rel=1e-12)
        np.testing.assert_allclose(u1, z[key + '__u1'], rtol=1e-12, atol=1e-15)


# ---- polynomial-kernel MMD (KID scorer / 3-sample scheduler) --------------
def test_polynomial_kernel_matches_sklearn():
    """The reference calls sklearn's polynomial_kernel (compute_scores.py:237-239)."""
    from sklearn.metrics.pairwise import polynomial_kernel as sk
    rng = np.random.default_rng(0)
    X, Y = rng.standard_normal((7, 5)), rng.standard_normal((4, 5))
    np.testing.assert_allclose(O.polynomial_kernel(X, Y), sk(X, Y), rtol=1e-12)
    np.testing.assert_allclose(O.polynomial_kernel(X, Y, degree=2, gamma=.3, coef0=.5),
                               sk(X, Y, degree=2, gamma=.3, coef0=.5), rtol=1e-12)


def test_poly_mmd2_known_answers():
    rng = np.random.default_rng(1)
    X, Y = np.abs(rng.standard_normal((9, 6))), np.abs(rng.standard_normal((9, 6))) * 1.3
    Kxx, Kyy, Kxy = (O.polynomial_kernel(a, b) for a, b in ((X, X), (Y, Y), (X, Y)))
    # biased MMD^2 of a sample with itself is 0
    assert abs(O.mmd2_and_variance(Kxx, Kxx, Kxx, mmd_est='biased', ret_var=False)) < 1e-12
    # unbiased: off-diagonal means minus twice the cross mean, by brute force
    m = 9
    off = lambda K: sum(K[i, j] for i in range(m) for j in range(m) if i != j) / (m * (m - 1))
    ref = off(Kxx) + off(Kyy) - 2 * Kxy.mean()
    mmd2, var = O.mmd2_and_variance(Kxx, Kxy, Kyy)
    assert abs(mmd2 - ref) < 1e-12 and var > 0
    # the 3-sample difference equals the difference of the two unbiased MMDs
    Z = np.abs(rng.standard_normal((9, 6))) * 0.8
    Kzz, Kxz = O.polynomial_kernel(Z, Z), O.polynomial_kernel(X, Z)
    diff, ratio = O.diff_mmd2_and_ratio_from_sums(O.np_get_sums(Kxy, Kyy),
                                                  O.np_get_sums(Kxz, Kzz), m)
    d_ref = (O.mmd2_and_variance(Kxx, Kxy, Kyy, ret_var=False)
             - O.mmd2_and_variance(Kxx, Kxz, Kzz, ret_var=False))
    assert abs(diff - d_ref) < 1e-10 and np.isfinite(ratio)
