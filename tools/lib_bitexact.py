"""Bit-for-bit comparison of two library builds on the Winograd convolutions,
for changes that must not move a single bit (block orders, the LDS-DMA wait
placement): python tools/lib_bitexact.py LIB_A LIB_B

Covered: the 3x3 conv over every tests/test_gpu_wino.py shape in both forms
(8-wave default, SMMD_WINO8=0 the 4-wave one), modes 0 and 1 of the filter,
the relu epilogue and the pair form; the stride-2 conv (plain and pair) and
the transposed stride-2 conv over the fold-layer shapes; both weight
gradients (3x3, stride 2) over their test shapes and the bench layers.  `make -C scaled-mmd-gan_amd/csrc conservative` builds
the conservative variant (every filter-stage LDS-DMA piece waited for right
after its issue, -DWN_DMA_SYNC) that this compares with the shipped build."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from gan.core import _lib  # noqa: E402

# (N, C, K, H, W): split reductions, the edge kernel, odd tile counts, the fold layers
S2_SHAPES = [(2, 8, 64, 8, 12), (1, 64, 64, 4, 264), (4, 512, 64, 8, 8), (2, 6, 128, 12, 8),
             (64, 64, 128, 64, 64), (64, 256, 512, 16, 16), (64, 512, 512, 8, 8)]


def _w3_shapes():
    from test_gpu_wino import PAIR_SHAPES, SHAPES
    return SHAPES, PAIR_SHAPES


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib._SIGS.items():
        if hasattr(L, name):
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
    return L


def _ws(nbytes, dev):
    return torch.empty(max(nbytes // 4, 4), device=dev)


def run_s2(L, x, w, b, x2, w2, st):
    N, C, H, W = x.shape
    K = w.shape[0]
    u = torch.empty(L.smmd_wino4x4s2_filter_bytes(K, C) // 4, device=x.device)
    u2 = torch.empty_like(u)
    assert L.smmd_wino4x4s2_filter(_lib.ptr(w), K, C, _lib.ptr(u), u.numel() * 4, st) == 0
    assert L.smmd_wino4x4s2_filter(_lib.ptr(w2), K, C, _lib.ptr(u2), u2.numel() * 4, st) == 0
    y = torch.empty(N, K, H // 2, W // 2, device=x.device)
    nb = L.smmd_wino4x4s2_workspace_bytes(N, C, K, H, W)
    ws = _ws(nb, x.device)
    assert L.smmd_wino4x4s2_conv(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, C, K, H, W,
                                 _lib.ptr(ws), nb, st) == 0
    y2 = torch.empty_like(y)
    nb2 = L.smmd_wino4x4s2_conv2_workspace_bytes(N, C, K, H, W)
    ws2 = _ws(nb2, x.device)
    assert L.smmd_wino4x4s2_conv2(_lib.ptr(x), _lib.ptr(u), _lib.ptr(x2), _lib.ptr(u2), _lib.ptr(b),
                                  _lib.ptr(y2), N, C, K, H, W, _lib.ptr(ws2), nb2, st) == 0
    torch.cuda.synchronize()
    return y.cpu(), y2.cpu()


def run_s2t(L, gy, w, b, st):
    N, K, Hg, Wg = gy.shape
    C = w.shape[1]
    u = torch.empty(L.smmd_wino4x4s2_filter_bytes(K, C) // 4, device=gy.device)
    assert L.smmd_wino4x4s2t_filter(_lib.ptr(w), K, C, _lib.ptr(u), u.numel() * 4, st) == 0
    dx = torch.empty(N, C, 2 * Hg, 2 * Wg, device=gy.device)
    nb = L.smmd_wino4x4s2t_workspace_bytes(N, K, C, Hg, Wg)
    ws = _ws(nb, gy.device)
    assert L.smmd_wino4x4s2t_conv(_lib.ptr(gy), _lib.ptr(u), _lib.ptr(b), _lib.ptr(dx), N, K, C,
                                  Hg, Wg, _lib.ptr(ws), nb, st) == 0
    torch.cuda.synchronize()
    return [dx.cpu()]


def run_wgrad(L, x, gy, s2, st):
    N, C, H, W = x.shape
    K = gy.shape[1]
    kk = 4 if s2 else 3
    gw = torch.empty(K, C, kk, kk, device=x.device)
    fb = L.smmd_wino4x4s2_wgrad_workspace_bytes if s2 else L.smmd_wino3x3_wgrad_workspace_bytes
    fn = L.smmd_wino4x4s2_wgrad if s2 else L.smmd_wino3x3_wgrad
    nb = fb(N, C, K, H, W)
    ws = _ws(nb, x.device)
    assert fn(_lib.ptr(x), _lib.ptr(gy), _lib.ptr(gw), N, C, K, H, W, _lib.ptr(ws), nb, st) == 0
    torch.cuda.synchronize()
    return [gw.cpu()]


def run_w3(L, x, w, b, x2, w2, st, pair):
    """mode-0 conv, mode-1 conv (w read as [ci', co'] = the input gradient's
    filter), relu; the pair form when `pair`."""
    N, C, H, W = x.shape
    K = w.shape[0]
    outs = []
    nb = L.smmd_wino3x3_workspace_bytes(N, C, K, H, W)
    ws = _ws(nb, x.device)
    for mode in ((0,) if pair else (0, 1)):
        u = torch.empty(L.smmd_wino3x3_filter_bytes(K, C) // 4, device=x.device)
        wm = w if mode == 0 else w.reshape(C, K, 3, 3)    # same bytes, other reading
        assert L.smmd_wino3x3_filter(_lib.ptr(wm), K, C, mode, _lib.ptr(u), u.numel() * 4, st) == 0
        y = torch.empty(N, K, H, W, device=x.device)
        if pair:
            u2 = torch.empty_like(u)
            assert L.smmd_wino3x3_filter(_lib.ptr(w2), K, C, 0, _lib.ptr(u2), u2.numel() * 4,
                                         st) == 0
            nb2 = L.smmd_wino3x3_conv2_workspace_bytes(N, C, K, H, W)
            ws2 = _ws(nb2, x.device)
            assert L.smmd_wino3x3_conv2(_lib.ptr(x), _lib.ptr(u), _lib.ptr(x2), _lib.ptr(u2),
                                        _lib.ptr(b), _lib.ptr(y), N, C, K, H, W, _lib.ptr(ws2),
                                        nb2, st) == 0
            outs.append(y)
            continue
        assert L.smmd_wino3x3_conv(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, C, K,
                                   H, W, _lib.ptr(ws), nb, st) == 0
        outs.append(y)
        if mode == 0:
            yr = torch.empty_like(y)
            assert L.smmd_wino3x3_conv_relu(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(yr), N,
                                            C, K, H, W, _lib.ptr(ws), nb, st) == 0
            outs.append(yr)
    torch.cuda.synchronize()
    return [o.cpu() for o in outs]


def main():
    A, B = load(sys.argv[1]), load(sys.argv[2])
    dev = torch.device('cuda:0')
    st = _lib.stream_handle(dev)
    ok = True
    w3, w3pair = _w3_shapes()
    for form in ('1', '0'):
        os.environ['SMMD_WINO8'] = form          # read by the library at every call
        for pair, shapes in ((False, w3), (True, w3pair)):
            for (N, C, K, H, W) in shapes:
                g = torch.Generator(device=dev).manual_seed(N + C + K + H + W)
                x, x2 = (torch.randn(N, C, H, W, device=dev, generator=g) for _ in range(2))
                w, w2 = (torch.randn(K, C, 3, 3, device=dev, generator=g) for _ in range(2))
                b = torch.randn(K, device=dev, generator=g)
                ra = run_w3(A, x, w, b, x2, w2, st, pair)
                rb = run_w3(B, x, w, b, x2, w2, st, pair)
                same = all(torch.equal(p, q) for p, q in zip(ra, rb))
                ok &= same
                print('3x3', 'wino8' if form == '1' else 'wino4', 'pair' if pair else 'conv',
                      (N, C, K, H, W), 'bit-identical' if same else 'DIFFERENT', flush=True)
    os.environ.pop('SMMD_WINO8', None)
    for (N, C, K, H, W) in S2_SHAPES:
        g = torch.Generator(device=dev).manual_seed(N + C + K + H + W)
        x, x2 = (torch.randn(N, C, H, W, device=dev, generator=g) for _ in range(2))
        w, w2 = (torch.randn(K, C, 4, 4, device=dev, generator=g) for _ in range(2))
        b = torch.randn(K, device=dev, generator=g)
        ra, rb = run_s2(A, x, w, b, x2, w2, st), run_s2(B, x, w, b, x2, w2, st)
        same = all(torch.equal(p, q) for p, q in zip(ra, rb))
        ok &= same
        print('s2', (N, C, K, H, W), 'bit-identical' if same else 'DIFFERENT', flush=True)
    for (N, C, K, H, W) in S2_SHAPES:             # the transposed conv: gy [N, K, H/2, W/2]
        if C % 8 or K % 64:
            continue
        g = torch.Generator(device=dev).manual_seed(N + C + K + H + W + 1)
        gy = torch.randn(N, C, H // 2, W // 2, device=dev, generator=g)
        w = torch.randn(C, K, 4, 4, device=dev, generator=g)
        b = torch.randn(K, device=dev, generator=g)
        same = all(torch.equal(p, q) for p, q in zip(run_s2t(A, gy, w, b, st),
                                                      run_s2t(B, gy, w, b, st)))
        ok &= same
        print('s2t', (N, C, K, H, W), 'bit-identical' if same else 'DIFFERENT', flush=True)
    from test_gpu_wino import WGRAD_SHAPES
    from test_gpu_wino_s2 import S2_WGRAD_SHAPES
    for s2, shapes in ((False, WGRAD_SHAPES + [(64, 64, 64, 64, 64), (64, 512, 512, 8, 8)]),
                       (True, S2_WGRAD_SHAPES + [(64, 64, 128, 64, 64), (64, 512, 1024, 8, 8)])):
        sup = A.smmd_wino4x4s2_wgrad_supported if s2 else A.smmd_wino3x3_wgrad_supported
        for (N, C, K, H, W) in shapes:
            if not sup(N, C, K, H, W):
                continue
            g = torch.Generator(device=dev).manual_seed(N + C + K + H + W + 2)
            x = torch.randn(N, C, H, W, device=dev, generator=g)
            d = 2 if s2 else 1
            gy = torch.randn(N, K, H // d, W // d, device=dev, generator=g)
            same = all(torch.equal(p, q) for p, q in zip(run_wgrad(A, x, gy, s2, st),
                                                          run_wgrad(B, x, gy, s2, st)))
            ok &= same
            print('s2 wgrad' if s2 else '3x3 wgrad', (N, C, K, H, W),
                  'bit-identical' if same else 'DIFFERENT', flush=True)
    print('ALL BIT-IDENTICAL' if ok else 'MISMATCH')
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
