"""Polyphase Winograd F(2x2,2x2) for the 4x4 stride-2 convs (smmd_wino4x4s2_*):
parity against float64 on the host and timing against MIOpen on the SNResNet-64
critic's four folded ConvMeanPool layers at batch 64.
python tools/wino_s2_bench.py [--lib PATH] [--iters N]"""
import argparse
import ctypes
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', default=os.path.join(ROOT, 'scaled-mmd-gan_amd', 'lib', 'libsmmd_hip.so'))
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    from gan.core import miopen_db
    miopen_db.install()
    L = ctypes.CDLL(a.lib)
    P, I, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.smmd_wino4x4s2_filter.argtypes = [P, I, I, P, SZ, P]
    L.smmd_wino4x4s2_conv.argtypes = [P, P, P, P, I, I, I, I, I, P, SZ, P]
    L.smmd_wino4x4s2_workspace_bytes.restype = SZ
    L.smmd_wino4x4s2_workspace_bytes.argtypes = [I] * 5
    L.smmd_wino4x4s2t_filter.argtypes = [P, I, I, P, SZ, P]
    L.smmd_wino4x4s2t_conv.argtypes = [P, P, P, P, I, I, I, I, I, P, SZ, P]
    L.smmd_wino4x4s2t_workspace_bytes.restype = SZ
    L.smmd_wino4x4s2t_workspace_bytes.argtypes = [I] * 5
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    dev = torch.device('cuda:0')

    def run(x, w, b):
        N, C, H, W = x.shape
        K = w.shape[0]
        u = torch.empty(36 * K * C, device=dev)
        assert L.smmd_wino4x4s2_filter(w.data_ptr(), K, C, u.data_ptr(), u.numel() * 4, st()) == 0
        nb = L.smmd_wino4x4s2_workspace_bytes(N, C, K, H, W)
        ws = torch.empty(max(nb // 4, 4), device=dev)
        y = torch.empty(N, K, H // 2, W // 2, device=dev)
        f = lambda: L.smmd_wino4x4s2_conv(x.data_ptr(), u.data_ptr(),
                                          b.data_ptr() if b is not None else None, y.data_ptr(),
                                          N, C, K, H, W, ws.data_ptr(), nb, st())
        assert f() == 0
        return y, f

    def runt(gy, w, b):
        """conv_transpose2d(gy, w [K, C, 4, 4], stride 2, padding 1) + b."""
        N, K, Hg, Wg = gy.shape
        C = w.shape[1]
        u = torch.empty(36 * K * C, device=dev)
        assert L.smmd_wino4x4s2t_filter(w.data_ptr(), K, C, u.data_ptr(), u.numel() * 4, st()) == 0
        nb = L.smmd_wino4x4s2t_workspace_bytes(N, K, C, Hg, Wg)
        ws = torch.empty(max(nb // 4, 4), device=dev)
        dx = torch.empty(N, C, 2 * Hg, 2 * Wg, device=dev)
        f = lambda: L.smmd_wino4x4s2t_conv(gy.data_ptr(), u.data_ptr(),
                                           b.data_ptr() if b is not None else None, dx.data_ptr(),
                                           N, K, C, Hg, Wg, ws.data_ptr(), nb, st())
        assert f() == 0
        return dx, f

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters * 1e3

    torch.manual_seed(0)
    for (N, C, K, H, W) in [(2, 2, 64, 4, 4), (3, 8, 64, 8, 12), (2, 64, 128, 16, 16),
                            (1, 4, 64, 4, 264), (4, 512, 64, 8, 8), (2, 6, 128, 12, 8)]:
        x = torch.randn(N, C, H, W, device=dev)
        w = torch.randn(K, C, 4, 4, device=dev)
        b = torch.randn(K, device=dev)
        y, _ = run(x, w, b)
        ref = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), stride=2, padding=1)
        err = ((y.double().cpu() - ref).abs().max() / ref.abs().max()).item()
        gy = torch.randn(N, K, H // 2, W // 2, device=dev)
        w2 = torch.randn(K, 64 if C % 64 else C, 4, 4, device=dev)
        b2 = torch.randn(w2.shape[1], device=dev)
        dx, _ = runt(gy, w2, b2)
        ref2 = F.conv_transpose2d(gy.double().cpu(), w2.double().cpu(), b2.double().cpu(),
                                  stride=2, padding=1)
        err2 = ((dx.double().cpu() - ref2).abs().max() / ref2.abs().max()).item()
        print('parity', N, C, K, H, W, 'fwd %.2e  transposed %.2e' % (err, err2), flush=True)
    for (N, C, K, H) in [(64, 64, 128, 64), (64, 128, 256, 32), (64, 256, 512, 16),
                         (64, 512, 1024, 8)]:
        x = torch.randn(N, C, H, H, device=dev)
        w = torch.randn(K, C, 4, 4, device=dev) / (16 * C) ** 0.5
        b = torch.randn(K, device=dev)
        y, f = run(x, w, b)
        ref = F.conv2d(x, w, b, stride=2, padding=1)
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        t = timed(f)
        tm = timed(lambda: F.conv2d(x, w, b, stride=2, padding=1))
        fl = 2.0 * N * C * K * 16 * (H // 2) ** 2
        gy = torch.randn(N, K, H // 2, H // 2, device=dev)
        dx, ft = runt(gy, w, None)
        refx = torch.nn.grad.conv2d_input(x.shape, w, gy, stride=2, padding=1)
        errx = ((dx - refx).abs().max() / refx.abs().max()).item()
        tt = timed(ft)
        tmx = timed(lambda: torch.nn.grad.conv2d_input(x.shape, w, gy, stride=2, padding=1))
        print(json.dumps({'shape': [N, C, K, H], 'rel_vs_miopen': err, 'wino_us': round(t, 1),
                          'miopen_us': round(tm, 1), 'executed_tflops': round(fl / 1.78 / t / 1e6, 1),
                          'direct_tflops_miopen': round(fl / tm / 1e6, 1),
                          'dgrad_rel_vs_miopen': errx, 'dgrad_wino_us': round(tt, 1),
                          'dgrad_miopen_us': round(tmx, 1)}), flush=True)


if __name__ == '__main__':
    main()
