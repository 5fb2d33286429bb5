"""Bit-for-bit comparison of two library builds on the stride-2 forward
convolution (plain and pair form), for block-order changes that must not move
a single bit: python tools/lib_bitexact.py LIB_A LIB_B"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))
from gan.core import _lib  # noqa: E402

# (N, C, K, H, W): split reductions, the edge kernel, odd tile counts, the fold layers
SHAPES = [(2, 8, 64, 8, 12), (1, 64, 64, 4, 264), (4, 512, 64, 8, 8), (2, 6, 128, 12, 8),
          (64, 64, 128, 64, 64), (64, 256, 512, 16, 16), (64, 512, 512, 8, 8)]


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib._SIGS.items():
        if hasattr(L, name):
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
    return L


def run(L, x, w, b, x2, w2, st):
    N, C, H, W = x.shape
    K = w.shape[0]
    u = torch.empty(L.smmd_wino4x4s2_filter_bytes(K, C) // 4, device=x.device)
    u2 = torch.empty_like(u)
    assert L.smmd_wino4x4s2_filter(_lib.ptr(w), K, C, _lib.ptr(u), u.numel() * 4, st) == 0
    assert L.smmd_wino4x4s2_filter(_lib.ptr(w2), K, C, _lib.ptr(u2), u2.numel() * 4, st) == 0
    y = torch.empty(N, K, H // 2, W // 2, device=x.device)
    nb = L.smmd_wino4x4s2_workspace_bytes(N, C, K, H, W)
    ws = torch.empty(max(nb // 4, 4), device=x.device)
    assert L.smmd_wino4x4s2_conv(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, C, K, H, W,
                                 _lib.ptr(ws), nb, st) == 0
    y2 = torch.empty_like(y)
    nb2 = L.smmd_wino4x4s2_conv2_workspace_bytes(N, C, K, H, W)
    ws2 = torch.empty(max(nb2 // 4, 4), device=x.device)
    assert L.smmd_wino4x4s2_conv2(_lib.ptr(x), _lib.ptr(u), _lib.ptr(x2), _lib.ptr(u2), _lib.ptr(b),
                                  _lib.ptr(y2), N, C, K, H, W, _lib.ptr(ws2), nb2, st) == 0
    torch.cuda.synchronize()
    return y.cpu(), y2.cpu()


def main():
    A, B = load(sys.argv[1]), load(sys.argv[2])
    dev = torch.device('cuda:0')
    st = _lib.stream_handle(dev)
    ok = True
    for (N, C, K, H, W) in SHAPES:
        g = torch.Generator(device=dev).manual_seed(N + C + K + H + W)
        x, x2 = (torch.randn(N, C, H, W, device=dev, generator=g) for _ in range(2))
        w, w2 = (torch.randn(K, C, 4, 4, device=dev, generator=g) for _ in range(2))
        b = torch.randn(K, device=dev, generator=g)
        ra, rb = run(A, x, w, b, x2, w2, st), run(B, x, w, b, x2, w2, st)
        same = all(torch.equal(p, q) for p, q in zip(ra, rb))
        ok &= same
        print((N, C, K, H, W), 'bit-identical' if same else 'DIFFERENT', flush=True)
    print('ALL BIT-IDENTICAL' if ok else 'MISMATCH')
    sys.exit(0 if ok else 1)


if __name__ == '__main__':
    main()
