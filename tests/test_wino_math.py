"""CPU check of the Winograd algebra the library's convolution kernels run
(csrc/smmd_wino.hip, smmd_wino_s2.hip), restated in float64 NumPy with the
kernels' transform matrices, tile offsets and phase maps, against torch's
conv2d / conv_transpose2d (the TF SAME convs of gan/core/snops.py:69-90 and
the folded ConvMeanPool / UpsampleConv of gan/core/resnet/block.py:53-66).
The GPU tests (tests/test_gpu_wino*.py) check the kernels themselves."""
import numpy as np
import torch
import torch.nn.functional as F


def _wino23(x, w):
    """F(2x2, 3x3): V = B^T d B, U = G g G^T, y = A^T (sum_c U V) A."""
    N, C, H, W = x.shape
    K = w.shape[0]
    xp = np.zeros((N, C, H + 2, W + 2))
    xp[:, :, 1:-1, 1:-1] = x
    BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], float)
    G = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]])
    AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], float)
    U = np.einsum('ia,kcab,jb->kcij', G, w, G)
    y = np.zeros((N, K, H, W))
    for ty in range(H // 2):
        for tx in range(W // 2):
            d = xp[:, :, 2 * ty:2 * ty + 4, 2 * tx:2 * tx + 4]
            V = np.einsum('ia,ncab,jb->ncij', BT, d, BT)
            M = np.einsum('kcij,ncij->nkij', U, V)
            y[:, :, 2 * ty:2 * ty + 2, 2 * tx:2 * tx + 2] = np.einsum('ai,nkij,bj->nkab', AT, M, AT)
    return y


BT2 = np.array([[1, -1, 0], [0, 1, 0], [0, -1, 1]], float)
G2 = np.array([[1, 0], [1, 1], [0, 1]], float)
AT2 = np.array([[1, 1, 0], [0, 1, 1]], float)


def _wino22_s2(x, w):
    """4x4 stride-2 pad-1 conv as polyphase F(2x2, 2x2): phase (pi, pj) tile
    rows 4ty-1+pi+2a, cols 4tx-1+pj+2b; taps g[a][b] = w[2a+pi][2b+pj]."""
    N, C, H, W = x.shape
    K = w.shape[0]
    xp = np.zeros((N, C, H + 8, W + 8))
    xp[:, :, 4:4 + H, 4:4 + W] = x
    y = np.zeros((N, K, H // 2, W // 2))
    for ty in range(H // 4):
        for tx in range(W // 4):
            M = 0
            for pi in (0, 1):
                for pj in (0, 1):
                    r = 4 * ty - 1 + pi + 4 + 2 * np.arange(3)
                    c = 4 * tx - 1 + pj + 4 + 2 * np.arange(3)
                    d = xp[:, :, r][:, :, :, c]
                    g = w[:, :, pi::2, pj::2]
                    M = M + np.einsum('kcij,ncij->nkij', np.einsum('ia,kcab,jb->kcij', G2, g, G2),
                                      np.einsum('ia,ncab,jb->ncij', BT2, d, BT2))
            y[:, :, 2 * ty:2 * ty + 2, 2 * tx:2 * tx + 2] = np.einsum('ai,nkij,bj->nkab', AT2, M, AT2)
    return y


def _wino22_s2t(gy, w):
    """conv_transpose2d(gy, w, stride 2, pad 1): output phase (qi, qj) is an
    F(2x2, 2x2) correlation of gy at rows 2ty-1+qi+a with taps w[3-qi-2a][3-qj-2b]."""
    N, K, Hg, Wg = gy.shape
    C = w.shape[1]
    gp = np.zeros((N, K, Hg + 4, Wg + 4))
    gp[:, :, 2:2 + Hg, 2:2 + Wg] = gy
    dx = np.zeros((N, C, 2 * Hg, 2 * Wg))
    for qi in (0, 1):
        for qj in (0, 1):
            g = w[:, :, [3 - qi, 1 - qi]][:, :, :, [3 - qj, 1 - qj]]
            U = np.einsum('ia,kcab,jb->kcij', G2, g, G2)
            for ty in range(Hg // 2):
                for tx in range(Wg // 2):
                    d = gp[:, :, 2 * ty - 1 + qi + 2:2 * ty + 2 + qi + 2,
                           2 * tx - 1 + qj + 2:2 * tx + 2 + qj + 2]
                    M = np.einsum('kcij,nkij->ncij', U, np.einsum('ia,nkab,jb->nkij', BT2, d, BT2))
                    out = np.einsum('ai,ncij,bj->ncab', AT2, M, AT2)
                    dx[:, :, 4 * ty + qi:4 * ty + 4 + qi:2, 4 * tx + qj:4 * tx + 4 + qj:2] = out
    return dx


def test_f23_matches_conv3x3():
    rng = np.random.default_rng(1)
    x, w = rng.standard_normal((2, 3, 6, 8)), rng.standard_normal((4, 3, 3, 3))
    ref = F.conv2d(torch.tensor(x), torch.tensor(w), padding=1).numpy()
    assert np.abs(_wino23(x, w) - ref).max() < 1e-12


def test_f23_input_gradient_is_flipped_transposed_filter():
    """mode 1 of smmd_wino3x3_filter: the input gradient is the same F(2,3)
    conv with g[a][b] = w[c][k][2-a][2-b]."""
    rng = np.random.default_rng(2)
    gy, w = rng.standard_normal((2, 4, 6, 6)), rng.standard_normal((4, 3, 3, 3))
    ref = torch.nn.grad.conv2d_input((2, 3, 6, 6), torch.tensor(w), torch.tensor(gy),
                                     padding=1).numpy()
    wt = np.ascontiguousarray(w[:, :, ::-1, ::-1].transpose(1, 0, 2, 3))
    assert np.abs(_wino23(gy, wt) - ref).max() < 1e-12


def test_polyphase_f22_matches_stride2_conv():
    rng = np.random.default_rng(3)
    x, w = rng.standard_normal((2, 3, 8, 12)), rng.standard_normal((5, 3, 4, 4))
    ref = F.conv2d(torch.tensor(x), torch.tensor(w), stride=2, padding=1).numpy()
    assert np.abs(_wino22_s2(x, w) - ref).max() < 1e-12


def test_polyphase_f22_matches_stride2_transposed_conv():
    rng = np.random.default_rng(4)
    gy, w = rng.standard_normal((2, 5, 4, 6)), rng.standard_normal((5, 3, 4, 4))
    ref = F.conv_transpose2d(torch.tensor(gy), torch.tensor(w), stride=2, padding=1).numpy()
    assert np.abs(_wino22_s2t(gy, w) - ref).max() < 1e-12
