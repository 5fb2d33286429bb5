"""CPU oracle for the Scaled-MMD-GAN hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product path
(``scaled-mmd-gan_amd/``) never imports it and fails loudly when the HIP
library is missing.

What it is
    A float64 NumPy restatement of the reference's TensorFlow-1.x graph for
    the hot path, op by op, including TF's autodiff tie rules:

    * kernel family          gan/core/mmd.py:12 (mysqrt), :18-188
    * unbiased/biased MMD^2  gan/core/mmd.py:194-220
    * safer_norm             gan/core/ops.py:203-206
    * squared_norm_jacobian  gan/core/ops.py:228-233
    * scaling regulariser    gan/core/model.py:366-403, gan/core/smmd.py:21-23, :40-42
    * witness GP             gan/core/model.py:327-350
    * spectral norm          gan/core/sn.py:12-59, gan/core/snops.py:81-84
    * clip + average + Adam  gan/core/model.py:233-266, :405-412, :444-456
                             (tf.clip_by_norm / tf.train.AdamOptimizer semantics)

Parity status: **parity unpinned**.  The reference ships no tests, fixtures or
golden vectors and imports TensorFlow 1.6 at module
top (gan/core/mmd.py:8), which is not installed and cannot be installed
offline, so neither "reference golden vectors" nor "outputs of the reference
run here" exist.  This oracle is instead pinned by analytic known-answer
tests and by central finite differences of its own float64 forward
(tests/test_oracle.py); tests/golden/*.npz are generated from it by
oracle/gen_golden.py.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

EPS = 1.0e-5          # gan/core/mmd.py:6  (_eps)
SN_EPS = 1.0e-12      # gan/core/sn.py:12  (_l2normalize eps)


# --------------------------------------------------------------------------
# kernel registry: reference kernel name -> parameters
# --------------------------------------------------------------------------
@dataclass
class KernelSpec:
    """Parameters of one reference kernel (gan/core/mmd.py:18-188).

    kind: 'rbf' (sum of Gaussians), 'rq' (sum of rational quadratics, optional
    add_dot * <x,y>), 'distance', 'dot'.  const_diag is None when the
    reference returns ``False`` (trace is used in _mmd2, mmd.py:212-213).
    """
    kind: str
    params: list = field(default_factory=list)   # sigmas (rbf) or alphas (rq)
    wts: list = field(default_factory=list)
    add_dot: float = 0.0
    tanh: bool = False
    const_diag: float | None = None


def kernel_spec(name: str, **kw) -> KernelSpec:
    """Map ``config.kernel`` (gan/core/smmd.py:11) to a KernelSpec."""
    if name == 'rbf':                              # mmd.py:55-82
        sigma = kw.get('sigma', 1.0)
        wt = kw.get('wt', 1.0)
        return KernelSpec('rbf', [sigma], [wt], const_diag=wt)
    if name == 'mix_rbf':                          # mmd.py:85-116
        sigmas = kw.get('sigmas', [2.0, 5.0, 10.0, 20.0, 40.0, 80.0])
        wts = kw.get('wts') or [1] * len(sigmas)
        return KernelSpec('rbf', list(sigmas), list(wts), const_diag=float(sum(wts)))
    rq_dot = {'mix_rq': 0.0, 'mix_rq_dot': .1, 'mix_rq_1dot': 1., 'mix_rq_10dot': 10.,
              'mix_rq_01dot': .1, 'mix_rq_001dot': .01, 'tanh_mix_rq': 0.0}
    if name in rq_dot:                             # mmd.py:119-188
        alphas = kw.get('alphas', [.1, 1., 10.])
        wts = kw.get('wts') or [1.] * len(alphas)
        add_dot = kw.get('add_dot', rq_dot[name])
        # quirk: const diag = sum(wts) even with add_dot > 0 (mmd.py:182-188)
        return KernelSpec('rq', list(alphas), list(wts), add_dot=add_dot,
                          tanh=(name == 'tanh_mix_rq'), const_diag=float(sum(wts)))
    if name in ('distance', 'tanh_distance'):      # mmd.py:18-41
        return KernelSpec('distance', tanh=(name == 'tanh_distance'), const_diag=None)
    if name == 'dot':                              # mmd.py:44-52
        return KernelSpec('dot', const_diag=None)
    raise ValueError('unknown kernel %r' % name)


KERNEL_NAMES = ['rbf', 'mix_rbf', 'mix_rq', 'mix_rq_dot', 'mix_rq_1dot', 'mix_rq_10dot',
                'mix_rq_01dot', 'mix_rq_001dot', 'tanh_mix_rq', 'distance',
                'tanh_distance', 'dot']


def _mysqrt(x):
    """mysqrt = sqrt(max(x + eps, 0))  (gan/core/mmd.py:12)."""
    return np.sqrt(np.maximum(x + EPS, 0.0))


def _mysqrt_grad(x):
    # d/dx sqrt(max(x+eps,0)); tf.maximum passes the gradient to its first
    # argument on ties (x+eps >= 0).
    xe = x + EPS
    with np.errstate(divide='ignore'):
        return np.where(xe >= 0, 0.5 / np.sqrt(np.maximum(xe, 0.0)), 0.0)


def _block(spec: KernelSpec, A, B, AB, sa, sb, gram32=False):
    """Kernel block K(A,B) from the Gram pieces, and dK/d(raw), dK/dAB,
    dK/dsa, dK/dsb as elementwise factors (float64)."""
    if gram32:
        raw = _raw32(AB, sa, sb)
    else:
        raw = -2.0 * AB + sa[:, None] + sb[None, :]      # mmd.py:67 (pre-clamp)
    if spec.kind == 'rbf':
        R = np.maximum(raw, 0.0)                          # mmd.py:67
        K = np.zeros_like(R)
        dKdR = np.zeros_like(R)
        for sigma, wt in zip(spec.params, spec.wts):
            gamma = 1.0 / (2.0 * sigma ** 2)              # mmd.py:69
            e = wt * np.exp(-gamma * R)
            K += e
            dKdR += -gamma * e
        dKdraw = dKdR * (raw >= 0)                        # tf.maximum tie rule
        return K, dKdraw, np.zeros_like(K), None, None
    if spec.kind == 'rq':
        R = np.maximum(raw, 0.0)                          # mmd.py:163
        K = np.zeros_like(R)
        dKdR = np.zeros_like(R)
        for alpha, wt in zip(spec.params, spec.wts):
            q = 1.0 + R / (2.0 * alpha)                   # mmd.py:166
            e = wt * np.exp(-alpha * np.log(q))           # mmd.py:167
            K += e
            dKdR += e * (-alpha) / q / (2.0 * alpha)
        dKdAB = np.zeros_like(K)
        if spec.add_dot > 0:                              # mmd.py:168-169
            K = K + spec.add_dot * AB
            dKdAB = np.full_like(K, spec.add_dot)
        dKdraw = dKdR * (raw >= 0)
        return K, dKdraw, dKdAB, None, None
    if spec.kind == 'distance':                           # mmd.py:29
        K = _mysqrt(sa)[:, None] + _mysqrt(sb)[None, :] - _mysqrt(raw)
        dKdraw = -_mysqrt_grad(raw)
        dsa = _mysqrt_grad(sa)[:, None] * np.ones_like(K)
        dsb = _mysqrt_grad(sb)[None, :] * np.ones_like(K)
        return K, dKdraw, np.zeros_like(K), dsa, dsb
    if spec.kind == 'dot':                                # mmd.py:45
        return AB.copy(), np.zeros_like(AB), np.ones_like(AB), None, None
    raise ValueError(spec.kind)


def _gram(A, B, gram32):
    """A B^T, diag(A A^T), diag(B B^T).  gram32=True forms them in float32 the
    way the reference's fp32 graph does (tf.matmul + diag_part, mmd.py:57-61),
    then widens: the Gram expansion -2ab + |a|^2 + |b|^2 loses the same bits
    as in TF, which matters for the ill-conditioned distance kernel."""
    if not gram32:
        return A @ B.T, np.sum(A * A, 1), np.sum(B * B, 1)
    A32, B32 = A.astype(np.float32), B.astype(np.float32)
    AB = (A32 @ B32.T).astype(np.float32)
    sa = np.sum(A32 * A32, 1, dtype=np.float32)
    sb = np.sum(B32 * B32, 1, dtype=np.float32)
    return AB.astype(np.float64), sa.astype(np.float64), sb.astype(np.float64)


def _raw32(AB, sa, sb):
    """(-2 AB + sa) + sb evaluated in float32 (mmd.py:67 operation order)."""
    r = (np.float32(-2.0) * AB.astype(np.float32) + sa.astype(np.float32)[:, None])
    return (r + sb.astype(np.float32)[None, :]).astype(np.float64)


def kernel_matrices(spec: KernelSpec, X, Y, K_XY_only=False, gram32=False):
    """(K_XX, K_XY, K_YY, const_diag) exactly as mmd._<name>_kernel
    (gan/core/mmd.py:18-188); const_diag None means the reference's False."""
    X = np.asarray(X, np.float64)
    Y = np.asarray(Y, np.float64)
    if spec.tanh:
        X, Y = np.tanh(X), np.tanh(Y)
    XY, sx, sy = _gram(X, Y, gram32)
    XX, _, _ = _gram(X, X, gram32)
    YY, _, _ = _gram(Y, Y, gram32)
    if gram32:
        np.fill_diagonal(XX, sx)
        np.fill_diagonal(YY, sy)
    else:
        sx, sy = np.diag(XX).copy(), np.diag(YY).copy()
    KXY = _block(spec, X, Y, XY, sx, sy, gram32)[0]
    if K_XY_only:
        return KXY
    KXX = _block(spec, X, X, XX, sx, sx, gram32)[0]
    KYY = _block(spec, Y, Y, YY, sy, sy, gram32)[0]
    return KXX, KXY, KYY, spec.const_diag


def mmd2_from_K(KXX, KXY, KYY, const_diag=None, biased=False):
    """_mmd2 (gan/core/mmd.py:199-220)."""
    m, n = KXX.shape[0], KYY.shape[0]
    if biased:
        return KXX.sum() / (m * m) + KYY.sum() / (n * n) - 2 * KXY.sum() / (m * n)
    if const_diag is not None:
        trX, trY = m * const_diag, n * const_diag
    else:
        trX, trY = np.trace(KXX), np.trace(KYY)
    return ((KXX.sum() - trX) / (m * (m - 1)) + (KYY.sum() - trY) / (n * (n - 1))
            - 2 * KXY.sum() / (m * n))


def mmd2(spec: KernelSpec, X, Y, biased=False, gram32=False):
    """mmd.mmd2(kernel(X, Y)) (gan/core/mmd.py:194-196)."""
    KXX, KXY, KYY, c = kernel_matrices(spec, X, Y, gram32=gram32)
    return mmd2_from_K(KXX, KXY, KYY, c, biased)


def mmd2_sums(spec: KernelSpec, X, Y, gram32=False):
    """(sum K_XX, sum K_XY, sum K_YY, trace K_XX, trace K_YY) in float64."""
    KXX, KXY, KYY, _ = kernel_matrices(spec, X, Y, gram32=gram32)
    return np.array([KXX.sum(), KXY.sum(), KYY.sum(), np.trace(KXX), np.trace(KYY)])


def _block_grads(spec, A, B, AB, sa, sb, G, gram32=False):
    """TF-autodiff gradient of sum(G * K(A,B)) w.r.t. A and B, where
    sa = diag(A A^T), sb = diag(B B^T) come from the Gram diagonal
    (mmd.py:60-61), so d sa_i / d a_i = 2 a_i."""
    K, dKdraw, dKdAB, dsa, dsb = _block(spec, A, B, AB, sa, sb, gram32)
    Graw = G * dKdraw
    GAB = -2.0 * Graw + G * dKdAB
    gsa = Graw.sum(1)
    gsb = Graw.sum(0)
    if dsa is not None:
        gsa = gsa + (G * dsa).sum(1)
        gsb = gsb + (G * dsb).sum(0)
    dA = GAB @ B + 2.0 * gsa[:, None] * A
    dB = GAB.T @ A + 2.0 * gsb[:, None] * B
    return dA, dB


def mmd2_grad(spec: KernelSpec, X, Y, biased=False, gram32=False):
    """Analytic d mmd2 / dX, d mmd2 / dY following TF autodiff of
    gan/core/mmd.py:55-220 (tf.maximum ties pass the gradient)."""
    X0 = np.asarray(X, np.float64)
    Y0 = np.asarray(Y, np.float64)
    X1, Y1 = (np.tanh(X0), np.tanh(Y0)) if spec.tanh else (X0, Y0)
    m, n = X1.shape[0], Y1.shape[0]
    if biased:
        gXX = np.full((m, m), 1.0 / (m * m))
        gYY = np.full((n, n), 1.0 / (n * n))
    else:
        gXX = np.full((m, m), 1.0 / (m * (m - 1)))
        gYY = np.full((n, n), 1.0 / (n * (n - 1)))
        if spec.const_diag is None:       # trace subtracted -> diag grads cancel
            np.fill_diagonal(gXX, 0.0)
            np.fill_diagonal(gYY, 0.0)
    gXY = np.full((m, n), -2.0 / (m * n))
    XY, sx, sy = _gram(X1, Y1, gram32)
    XX, _, _ = _gram(X1, X1, gram32)
    YY, _, _ = _gram(Y1, Y1, gram32)
    if gram32:
        np.fill_diagonal(XX, sx)
        np.fill_diagonal(YY, sy)
    else:
        sx, sy = np.diag(XX).copy(), np.diag(YY).copy()
    a, b = _block_grads(spec, X1, X1, XX, sx, sx, gXX, gram32)
    dX = a + b
    a, b = _block_grads(spec, Y1, Y1, YY, sy, sy, gYY, gram32)
    dY = a + b
    a, b = _block_grads(spec, X1, Y1, XY, sx, sy, gXY, gram32)
    dX += a
    dY += b
    if spec.tanh:
        dX *= 1.0 - X1 ** 2
        dY *= 1.0 - Y1 ** 2
    return dX, dY


# --------------------------------------------------------------------------
# witness (K_XY_only row means), gan/core/model.py:327-350
# --------------------------------------------------------------------------
def witness(spec: KernelSpec, H, R, F, gram32=False):
    """witness_i = mean_j K(h_i, r_j) - mean_j K(h_i, f_j)  (model.py:336-338)."""
    return (kernel_matrices(spec, H, R, K_XY_only=True, gram32=gram32).mean(1)
            - kernel_matrices(spec, H, F, K_XY_only=True, gram32=gram32).mean(1))


def witness_grad_H(spec: KernelSpec, H, R, F, gram32=False):
    """d sum_i witness_i / d H  (the inner gradient of model.py:339 at the
    critic-output level), float64 analytic."""
    H0 = np.asarray(H, np.float64)
    out = np.zeros_like(H0)
    for Z, sgn in ((R, 1.0), (F, -1.0)):
        Z0 = np.asarray(Z, np.float64)
        H1, Z1 = (np.tanh(H0), np.tanh(Z0)) if spec.tanh else (H0, Z0)
        G = np.full((H1.shape[0], Z1.shape[0]), sgn / Z1.shape[0])
        HZ, sh, sz = _gram(H1, Z1, gram32)
        dA, _ = _block_grads(spec, H1, Z1, HZ, sh, sz, G, gram32)
        if spec.tanh:
            dA *= 1.0 - H1 ** 2
        out += dA
    return out


def safer_norm(t, axis=None, keep_dims=False, epsilon=EPS):
    """gan/core/ops.py:203-206."""
    t = np.asarray(t, np.float64)
    return np.sqrt(np.sum(t * t, axis=axis, keepdims=keep_dims) + epsilon)


def gp_penalty(grad_xhat):
    """mean((safer_norm(g, axis=1) - 1)^2)  (model.py:341): channel axis only."""
    return np.mean((safer_norm(grad_xhat, axis=1) - 1.0) ** 2)


# --------------------------------------------------------------------------
# scaling regulariser (gan/core/model.py:366-403, ops.py:228-233)
# --------------------------------------------------------------------------
def squared_norm_per_sample(grads):
    """sum over [1,2,3] of grad^2 per sample (ops.py:231) for one output
    column's gradient g [b, C, H, W]; ops.py:232 sums these over columns."""
    g = np.asarray(grads, np.float64)
    return np.sum(g.reshape(g.shape[0], -1) ** 2, axis=1)


def scale_factor(norm2_jac_mean, sc, norm_discriminator=0.0, variant='grad'):
    """scale = 1/(sc*J + 1) ('grad') or 1/(sc*(J + nD) + 1)  (model.py:387-390)."""
    if variant == 'grad':
        return 1.0 / (sc * norm2_jac_mean + 1.0)
    if variant == 'value_and_grad':
        return 1.0 / (sc * (norm2_jac_mean + norm_discriminator) + 1.0)
    raise ValueError(variant)


def smmd_loss(mmd2_value, scale):
    """SMMD.apply_scaling: g_loss = mmd2*scale, d_loss = -g_loss (smmd.py:21-23)."""
    g = mmd2_value * scale
    return g, -g


def swgan_loss(d_G, d_images, scale):
    """SWGAN (smmd.py:31-42): d_loss = mean(G) - mean(images), scaled by sqrt(scale)."""
    d = (np.mean(d_G) - np.mean(d_images)) * math.sqrt(scale)
    return -d, d


# --------------------------------------------------------------------------
# spectral norm (gan/core/sn.py:12-59)
# --------------------------------------------------------------------------
def _l2normalize(v, eps=SN_EPS):
    """v / (||v|| + eps)   (sn.py:12-13)."""
    return v / (np.sqrt(np.sum(v ** 2)) + eps)


def spectral_normed_weight(W, u, num_iters=1):
    """Reference layout: W of any shape, reshaped to [-1, W.shape[-1]]
    (sn.py:18-19); u [1, N].  Returns (W_bar, sigma, u_final, v_final)."""
    W = np.asarray(W, np.float64)
    Wr = W.reshape(-1, W.shape[-1])
    u_i = np.asarray(u, np.float64).reshape(1, -1)
    v_i = np.zeros((1, Wr.shape[0]))
    for _ in range(num_iters):                       # sn.py:24-27
        v_i = _l2normalize(u_i @ Wr.T)
        u_i = _l2normalize(v_i @ Wr)
    sigma = (v_i @ Wr @ u_i.T)[0, 0]                  # sn.py:42
    return (Wr / sigma).reshape(W.shape), sigma, u_i, v_i


def spectral_norm_rows(Wt, u, num_iters=1):
    """Same power iteration on the [N rows = out, K cols] layout this build
    stores (torch conv/linear weights flattened).  Wt = W_r^T up to a
    permutation of K, which leaves sigma and u unchanged."""
    Wt = np.asarray(Wt, np.float64)
    u_i = np.asarray(u, np.float64).reshape(-1)
    v_i = np.zeros(Wt.shape[1])
    for _ in range(num_iters):
        v_i = _l2normalize(u_i @ Wt)
        u_i = _l2normalize(Wt @ v_i)
    sigma = float(v_i @ Wt.T @ u_i)
    return sigma, u_i, v_i


def sn_weight_backward(Wt, s, sigma, u, v, G_eff):
    """Gradient of L(W_eff), W_eff = s * W / sigma(W) with u, v stopped
    (sn.py:32-34, :42-43, snops.py:84): returns dL/dW, dL/ds.
    dsigma/dW = u v^T in the [N, K] layout."""
    Wt = np.asarray(Wt, np.float64)
    G = np.asarray(G_eff, np.float64)
    gWbar = s * G
    dot = np.sum(gWbar * Wt)
    gW = gWbar / sigma - (dot / sigma ** 2) * np.outer(u, v)
    gs = np.sum(G * Wt) / sigma
    return gW, gs


# --------------------------------------------------------------------------
# clip + average + Adam (gan/core/model.py:233-266, :405-412, :444-468)
# --------------------------------------------------------------------------
def clip_by_norm(t, clip_norm=1.0):
    """tf.clip_by_norm: t * clip_norm / max(||t||_2, clip_norm)."""
    t = np.asarray(t, np.float64)
    nrm = np.sqrt(np.sum(t * t))
    return t * clip_norm / max(nrm, clip_norm)


def average_gradients(tower_grads):
    """mean over towers of each variable's gradient (model.py:245-265)."""
    return [np.mean(np.stack(gs), axis=0) for gs in zip(*tower_grads)]


def adam_step(var, m, v, g, step, lr, beta1=0.5, beta2=0.9, eps=1e-8):
    """tf.train.AdamOptimizer update (epsilon-hat form); step is 1-based."""
    lr_t = lr * math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    var = var - lr_t * m / (np.sqrt(v) + eps)
    return var, m, v


# --------------------------------------------------------------------------
# D/G schedule (gan/core/model.py:470-478)
# --------------------------------------------------------------------------
class Counters:
    """Mirror of MMD_GAN.set_counters: 5 D steps then 1 G step; 10 D steps
    while step < 20 or step % 500 == 0."""

    def __init__(self, dsteps=5, gsteps=1, start_dsteps=10):
        self.dsteps, self.gsteps, self.start_dsteps = dsteps, gsteps, start_dsteps
        self.d_counter = 0
        self.g_counter = 0

    def update(self, step):
        if self.g_counter == 0:
            d_steps = self.dsteps
            if step % 500 == 0 or step < 20:
                d_steps = self.start_dsteps
            self.d_counter = (self.d_counter + 1) % (d_steps + 1)
        if self.d_counter == 0:
            self.g_counter = (self.g_counter + 1) % self.gsteps
        return self.d_counter == 0     # True -> generator step


# --------------------------------------------------------------------------
# a tiny differentiable critic for end-to-end loss checks
# --------------------------------------------------------------------------
def mlp_critic(x, W1, W2):
    """h = tanh(x W1); D(x) = h W2.  x [b, P]."""
    h = np.tanh(np.asarray(x, np.float64) @ W1)
    return h @ W2, h


def mlp_critic_sq_jac(x, W1, W2):
    """sum_i ||dD_i/dx||^2 per sample for the tanh MLP (analytic)."""
    _, h = mlp_critic(x, W1, W2)
    out = np.zeros(x.shape[0])
    for i in range(W2.shape[1]):
        # dD_i/dx = W1 diag(1-h^2) W2[:, i]
        J = ((1 - h ** 2) * W2[:, i][None, :]) @ W1.T      # [b, P]
        out += np.sum(J ** 2, axis=1)
    return out


def smmd_objective(spec, x_fake, x_real, W1, W2, sc=10.0, variant='grad', biased=False):
    """Full SMMD generator loss for the tanh-MLP critic (smmd.py:10-19 +
    model.py:366-403): returns (g_loss, mmd2, scale)."""
    dG, _ = mlp_critic(x_fake, W1, W2)
    dI, _ = mlp_critic(x_real, W1, W2)
    m2 = mmd2(spec, dG, dI, biased)
    J = float(np.mean(mlp_critic_sq_jac(x_real, W1, W2)))
    nD = float(np.mean(dI ** 2))
    sc_ = scale_factor(J, sc, nD, variant)
    return m2 * sc_, m2, sc_


# ---------------------------------------------------------------------------
# Polynomial-kernel MMD of the KID scorer and the 3-sample LR scheduler.
# The reference computes these in numpy (float64 sums over float32 kernel
# matrices); restated here in float64 throughout.
# ---------------------------------------------------------------------------
def polynomial_kernel(X, Y=None, degree=3, gamma=None, coef0=1):
    """sklearn.metrics.pairwise.polynomial_kernel (scikit_learn==0.19.1,
    /root/reference requirements.txt:12; called at gan/compute_scores.py:237-239):
    K = (gamma X Y^T + coef0)^degree, gamma None -> 1 / n_features."""
    X = np.asarray(X, np.float64)
    Y = X if Y is None else np.asarray(Y, np.float64)
    g = 1.0 / X.shape[1] if gamma is None else gamma
    return (g * (X @ Y.T) + coef0) ** degree


def _sqn(a):
    f = np.ravel(a)
    return float(f @ f)


def mmd2_and_variance(K_XX, K_XY, K_YY, unit_diagonal=False, mmd_est='unbiased',
                      var_at_m=None, ret_var=True):
    """gan/compute_scores.py:246-335 (_mmd2_and_variance)."""
    m = K_XX.shape[0]
    if var_at_m is None:
        var_at_m = m
    if unit_diagonal:
        diag_X = diag_Y = 1
        sum_diag_X = sum_diag_Y = m
        sum_diag2_X = sum_diag2_Y = m
    else:
        diag_X, diag_Y = np.diagonal(K_XX), np.diagonal(K_YY)
        sum_diag_X, sum_diag_Y = diag_X.sum(), diag_Y.sum()
        sum_diag2_X, sum_diag2_Y = _sqn(diag_X), _sqn(diag_Y)
    Kt_XX_sums = K_XX.sum(axis=1) - diag_X
    Kt_YY_sums = K_YY.sum(axis=1) - diag_Y
    K_XY_sums_0 = K_XY.sum(axis=0)
    K_XY_sums_1 = K_XY.sum(axis=1)
    Kt_XX_sum, Kt_YY_sum, K_XY_sum = Kt_XX_sums.sum(), Kt_YY_sums.sum(), K_XY_sums_0.sum()
    if mmd_est == 'biased':
        mmd2 = ((Kt_XX_sum + sum_diag_X) / (m * m) + (Kt_YY_sum + sum_diag_Y) / (m * m)
                - 2 * K_XY_sum / (m * m))
    else:
        mmd2 = (Kt_XX_sum + Kt_YY_sum) / (m * (m - 1))
        if mmd_est == 'unbiased':
            mmd2 -= 2 * K_XY_sum / (m * m)
        else:
            mmd2 -= 2 * (K_XY_sum - np.trace(K_XY)) / (m * (m - 1))
    if not ret_var:
        return mmd2
    Kt_XX_2_sum = _sqn(K_XX) - sum_diag2_X
    Kt_YY_2_sum = _sqn(K_YY) - sum_diag2_Y
    K_XY_2_sum = _sqn(K_XY)
    dot_XX_XY = Kt_XX_sums.dot(K_XY_sums_1)
    dot_YY_YX = Kt_YY_sums.dot(K_XY_sums_0)
    m1, m2 = m - 1, m - 2
    zeta1 = (1 / (m * m1 * m2) * (_sqn(Kt_XX_sums) - Kt_XX_2_sum + _sqn(Kt_YY_sums) - Kt_YY_2_sum)
             - 1 / (m * m1) ** 2 * (Kt_XX_sum ** 2 + Kt_YY_sum ** 2)
             + 1 / (m * m * m1) * (_sqn(K_XY_sums_1) + _sqn(K_XY_sums_0) - 2 * K_XY_2_sum)
             - 2 / m ** 4 * K_XY_sum ** 2
             - 2 / (m * m * m1) * (dot_XX_XY + dot_YY_YX)
             + 2 / (m ** 3 * m1) * (Kt_XX_sum + Kt_YY_sum) * K_XY_sum)
    zeta2 = (1 / (m * m1) * (Kt_XX_2_sum + Kt_YY_2_sum)
             - 1 / (m * m1) ** 2 * (Kt_XX_sum ** 2 + Kt_YY_sum ** 2)
             + 2 / (m * m) * K_XY_2_sum
             - 2 / m ** 4 * K_XY_sum ** 2
             - 4 / (m * m * m1) * (dot_XX_XY + dot_YY_YX)
             + 4 / (m ** 3 * m1) * (Kt_XX_sum + Kt_YY_sum) * K_XY_sum)
    var_est = (4 * (var_at_m - 2) / (var_at_m * (var_at_m - 1)) * zeta1
               + 2 / (var_at_m * (var_at_m - 1)) * zeta2)
    return mmd2, var_est


def np_get_sums(K_XY, K_YY):
    """gan/core/mmd.py:515-539 (_np_get_sums, const_diagonal=False)."""
    diag_Y = np.diag(K_YY)
    sum_diag2_Y = diag_Y @ diag_Y
    return (K_YY.sum(axis=1) - diag_Y, (K_YY ** 2).sum() - sum_diag2_Y, K_XY.sum(axis=0),
            K_XY.sum(axis=1), (K_XY ** 2).sum())


def diff_mmd2_and_ratio_from_sums(Y_sums, Z_sums, m):
    """gan/core/mmd.py:444-512 (_np_diff_mmd2_and_ratio_from_sums), _eps = 1e-5 (:6)."""
    Kt_YY_sums, Kt_YY_2_sum, K_XY_sums_0, K_XY_sums_1, K_XY_2_sum = Y_sums
    Kt_ZZ_sums, Kt_ZZ_2_sum, K_XZ_sums_0, K_XZ_sums_1, K_XZ_2_sum = Z_sums
    Kt_YY_sum, Kt_ZZ_sum = Kt_YY_sums.sum(), Kt_ZZ_sums.sum()
    K_XY_sum, K_XZ_sum = K_XY_sums_0.sum(), K_XZ_sums_0.sum()
    muY_muY = Kt_YY_sum / (m * (m - 1))
    muZ_muZ = Kt_ZZ_sum / (m * (m - 1))
    muX_muY = K_XY_sum / (m * m)
    muX_muZ = K_XZ_sum / (m * m)
    E_y_muY_sq = (Kt_YY_sums @ Kt_YY_sums - Kt_YY_2_sum) / (m * (m - 1) * (m - 2))
    E_z_muZ_sq = (Kt_ZZ_sums @ Kt_ZZ_sums - Kt_ZZ_2_sum) / (m * (m - 1) * (m - 2))
    E_x_muY_sq = (K_XY_sums_1 @ K_XY_sums_1 - K_XY_2_sum) / (m * m * (m - 1))
    E_x_muZ_sq = (K_XZ_sums_1 @ K_XZ_sums_1 - K_XZ_2_sum) / (m * m * (m - 1))
    E_y_muX_sq = (K_XY_sums_0 @ K_XY_sums_0 - K_XY_2_sum) / (m * m * (m - 1))
    E_z_muX_sq = (K_XZ_sums_0 @ K_XZ_sums_0 - K_XZ_2_sum) / (m * m * (m - 1))
    E_y_muY_y_muX = Kt_YY_sums @ K_XY_sums_0 / (m * m * (m - 1))
    E_z_muZ_z_muX = Kt_ZZ_sums @ K_XZ_sums_0 / (m * m * (m - 1))
    E_x_muY_x_muZ = K_XY_sums_1 @ K_XZ_sums_1 / (m * m * m)
    E_kyy2 = Kt_YY_2_sum / (m * (m - 1))
    E_kzz2 = Kt_ZZ_2_sum / (m * (m - 1))
    E_kxy2 = K_XY_2_sum / (m * m)
    E_kxz2 = K_XZ_2_sum / (m * m)
    mmd2_diff = muY_muY - 2 * muX_muY - muZ_muZ + 2 * muX_muZ
    first_order = 4 * (m - 2) / (m * (m - 1)) * (
        E_y_muY_sq - muY_muY ** 2 + E_x_muY_sq - muX_muY ** 2 + E_y_muX_sq - muX_muY ** 2
        + E_z_muZ_sq - muZ_muZ ** 2 + E_x_muZ_sq - muX_muZ ** 2 + E_z_muX_sq - muX_muZ ** 2
        - 2 * E_y_muY_y_muX + 2 * muY_muY * muX_muY
        - 2 * E_x_muY_x_muZ + 2 * muX_muY * muX_muZ
        - 2 * E_z_muZ_z_muX + 2 * muZ_muZ * muX_muZ)
    second_order = 2 / (m * (m - 1)) * (
        E_kyy2 - muY_muY ** 2 + 2 * E_kxy2 - 2 * muX_muY ** 2 + E_kzz2 - muZ_muZ ** 2
        + 2 * E_kxz2 - 2 * muX_muZ ** 2
        - 4 * E_y_muY_y_muX + 4 * muY_muY * muX_muY
        - 4 * E_x_muY_x_muZ + 4 * muX_muY * muX_muZ
        - 4 * E_z_muZ_z_muX + 4 * muZ_muZ * muX_muZ)
    var_est = first_order + second_order
    return mmd2_diff, mmd2_diff / np.sqrt(max(var_est, 1.0e-5))


def fold_pool_weight(W):
    """ConvMeanPool (gan/core/resnet/block.py:63-66): mean_pool2(conv3x3_same(x, W))
    == conv4x4_stride2_pad1(x, W'), W'[s,t] = 1/4 sum_{a,b in {0,1}} W[s-a, t-b].
    W [..., 3, 3] -> [..., 4, 4], float64."""
    W = np.asarray(W, np.float64)
    out = np.zeros(W.shape[:-2] + (4, 4))
    for a in (0, 1):
        for b in (0, 1):
            out[..., a:a + 3, b:b + 3] += W
    return out * 0.25


def fold_pool_weight_adjoint(G):
    """Adjoint of fold_pool_weight: G [..., 4, 4] -> [..., 3, 3],
    g[u,v] = 1/4 sum_{a,b in {0,1}} G[u+a, v+b] (the gradient w.r.t. W)."""
    G = np.asarray(G, np.float64)
    out = np.zeros(G.shape[:-2] + (3, 3))
    for a in (0, 1):
        for b in (0, 1):
            out += G[..., a:a + 3, b:b + 3]
    return out * 0.25
