"""Winograd F(2,3) MFMA conv (smmd_wino3x3_*): parity against MIOpen / float64
and per-shape timing against MIOpen's own pick (find db installed), for the
3x3 stride-1 SAME convolutions of the SNResNet-64 critic and generator.

python tools/wino_bench.py [--lib PATH] [--iters N]
"""
import argparse
import ctypes
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))


def load(path):
    L = ctypes.CDLL(path)
    L.smmd_wino3x3_filter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    L.smmd_wino3x3_conv.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int] * 5 + [
        ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    L.smmd_wino3x3_workspace_bytes.restype = ctypes.c_size_t
    L.smmd_wino3x3_workspace_bytes.argtypes = [ctypes.c_int] * 5
    if hasattr(L, 'smmd_wino3x3_wgrad'):
        L.smmd_wino3x3_wgrad.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 5 + [
            ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        L.smmd_wino3x3_wgrad_workspace_bytes.restype = ctypes.c_size_t
        L.smmd_wino3x3_wgrad_workspace_bytes.argtypes = [ctypes.c_int] * 5
    L.smmd_wino3x3_filter_bytes.restype = ctypes.c_size_t
    L.smmd_wino3x3_filter_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    return L


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def wino(L, x, w, b, mode):
    """mode 0: conv(x, w) + b, w [K, C, 3, 3]; mode 1: the input gradient of a
    conv with weight w [C', K', 3, 3] at upstream x [N, C', H, W]."""
    N, C, H, W = x.shape
    K = w.shape[0] if mode == 0 else w.shape[1]
    u = torch.empty(16 * K * C, device=x.device)
    st = L.smmd_wino3x3_filter(w.data_ptr(), K, C, mode, u.data_ptr(), u.numel() * 4, stream())
    assert st == 0, st
    y = torch.empty((N, K, H, W), device=x.device)
    nb = L.smmd_wino3x3_workspace_bytes(N, C, K, H, W)
    ws = torch.empty(max(nb // 4, 4), device=x.device)
    st = L.smmd_wino3x3_conv(x.data_ptr(), u.data_ptr(), b.data_ptr() if b is not None else None,
                             y.data_ptr(), N, C, K, H, W, ws.data_ptr(), nb, stream())
    assert st == 0, st
    return y, u, ws


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', default=os.path.join(ROOT, 'scaled-mmd-gan_amd', 'lib', 'libsmmd_hip.so'))
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--out', default='')
    a = ap.parse_args()
    from gan.core import miopen_db
    miopen_db.install()
    L = load(a.lib)
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    res = {'parity': [], 'timing': []}
    # parity: small shapes against float64 on the host
    for (N, C, K, H, Wd) in [(2, 8, 64, 6, 6), (1, 16, 64, 4, 10), (3, 64, 128, 8, 8),
                             (2, 8, 64, 2, 2), (1, 8, 64, 130, 4), (1, 8, 64, 4, 130),
                             (4, 512, 64, 8, 8), (2, 256, 128, 4, 6)]:
        x = torch.randn(N, C, H, Wd, device=dev)
        w = torch.randn(K, C, 3, 3, device=dev)
        b = torch.randn(K, device=dev)
        y, _, _ = wino(L, x, w, b, 0)
        ref = F.conv2d(x.double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
        err = ((y.double().cpu() - ref).abs().max() / ref.abs().max()).item()
        # mode 1: gx = conv_transpose(gy, w2), w2 [K2=C', C2=K', 3, 3] forward weight
        w2 = torch.randn(C, K, 3, 3, device=dev)     # forward conv K' = K out... see doc
        gy = x
        gx, _, _ = wino(L, gy, w2, None, 1)
        ref1 = torch.nn.grad.conv2d_input((N, K, H, Wd), w2.double().cpu(), gy.double().cpu(),
                                          padding=1)
        err1 = ((gx.double().cpu() - ref1).abs().max() / ref1.abs().max()).item()
        res['parity'].append({'shape': [N, C, K, H, Wd], 'fwd_rel': err, 'bwd_data_rel': err1})
        print('parity', N, C, K, H, Wd, 'fwd %.2e  dgrad %.2e' % (err, err1), flush=True)
    # timing: the SNResNet-64 3x3 convs at batch 64
    for (N, C, K, H) in [(64, 64, 64, 64), (64, 128, 128, 32), (64, 256, 256, 16),
                         (64, 512, 512, 8)]:
        x = torch.randn(N, C, H, H, device=dev)
        w = torch.randn(K, C, 3, 3, device=dev) * (1.0 / (9 * C) ** 0.5)
        b = torch.randn(K, device=dev)
        y, u, ws = wino(L, x, w, b, 0)
        ref = F.conv2d(x, w, b, padding=1)
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        gy = torch.randn(N, K, H, H, device=dev)
        gx, _, _ = wino(L, gy, w, None, 1)
        refx = torch.nn.grad.conv2d_input(x.shape, w, gy, padding=1)
        errx = ((gx - refx).abs().max() / refx.abs().max()).item()
        t_conv = timed(lambda: L.smmd_wino3x3_conv(x.data_ptr(), u.data_ptr(), b.data_ptr(),
                                                   y.data_ptr(), N, C, K, H, H, ws.data_ptr(),
                                                   ws.numel() * 4, stream()), a.iters)
        t_filt = timed(lambda: L.smmd_wino3x3_filter(w.data_ptr(), K, C, 0, u.data_ptr(),
                                                     u.numel() * 4, stream()), a.iters)
        t_mi = timed(lambda: F.conv2d(x, w, b, padding=1), a.iters)
        t_mi_dx = timed(lambda: torch.nn.grad.conv2d_input(x.shape, w, gy, padding=1), a.iters)
        flops = 2.0 * N * C * K * 9 * H * H
        wg = {}
        if hasattr(L, 'smmd_wino3x3_wgrad'):
            nbw = L.smmd_wino3x3_wgrad_workspace_bytes(N, C, K, H, H)
            wsw = torch.empty(max(nbw // 4, 4), device=dev)
            gw = torch.empty(K, C, 3, 3, device=dev)
            fw = lambda: L.smmd_wino3x3_wgrad(x.data_ptr(), gy.data_ptr(), gw.data_ptr(), N, C, K,
                                              H, H, wsw.data_ptr(), nbw, stream())
            assert fw() == 0
            refw = torch.nn.grad.conv2d_weight(x, (K, C, 3, 3), gy, padding=1)
            wg = {'wgrad_rel_vs_miopen': ((gw - refw).abs().max() / refw.abs().max()).item(),
                  'wgrad_miopen_us': timed(lambda: torch.nn.grad.conv2d_weight(
                      x, (K, C, 3, 3), gy, padding=1), a.iters)}
            # interleaved A/B of the two forms (the library reads
            # SMMD_WINO_WGRAD_V1 per call): default, v1, default, v1
            ab = {'default': [], 'v1': []}
            for arm in ('default', 'v1', 'default', 'v1'):
                if arm == 'v1':
                    os.environ['SMMD_WINO_WGRAD_V1'] = '1'
                ab[arm].append(timed(fw, a.iters))
                os.environ.pop('SMMD_WINO_WGRAD_V1', None)
            wg.update(wgrad_wino_us=min(ab['default']), wgrad_v1_us=min(ab['v1']),
                      wgrad_ab_us=ab,
                      wgrad_executed_tflops=flops / 2.25 / min(ab['default']) / 1e6,
                      wgrad_mfma_frac=flops / 2.25 / min(ab['default']) / 1e6 / 157.3)
        r = {'shape': [N, C, K, H, H], 'fwd_rel_vs_miopen': err, 'dgrad_rel_vs_miopen': errx,
             'wino_us': t_conv, 'filter_us': t_filt, 'miopen_fwd_us': t_mi,
             'miopen_dgrad_us': t_mi_dx, 'direct_tflops_wino': flops / t_conv / 1e6,
             'executed_tflops_wino': flops / 2.25 / t_conv / 1e6,
             'direct_tflops_miopen': flops / t_mi / 1e6, **wg}
        res['timing'].append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
