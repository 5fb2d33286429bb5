"""Launch-only driver for counter passes over the forward Winograd kernels:
the four SNResNet-64 3x3 layers (smmd_wino3x3_conv) and the four folded
stride-2 layers (smmd_wino4x4s2_conv) at batch 64, random data, --iters
launches each, through the stamped library.  Prints per-shape HIP-event
times (no profiler: run it bare for times, under rocprofv3 --pmc for counters).

python tools/wino_pmc.py [--iters N] [--only 3x3|s2|s2t|wgrad|s2w] [--lib PATH]
(--lib: another build of the library, unstamped, for interleaved A/B runs)
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))

SHAPES_3X3 = [(64, 64, 64, 64), (64, 128, 128, 32), (64, 256, 256, 16), (64, 512, 512, 8)]
SHAPES_S2 = [(64, 64, 128, 64), (64, 128, 256, 32), (64, 256, 512, 16), (64, 512, 512, 8)]


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def clock_ghz(L, blocks):
    """Diagnostic builds (-DWN_CLOCK) only: the median in-kernel clock of the
    last launch's blocks, d(s_memtime) / d(s_memrealtime) x 100 MHz, and the
    median block duration in us."""
    if not hasattr(L, 'smmd_diag_wino_clock'):
        return None
    import ctypes
    n = min(blocks, 4096)
    buf = (ctypes.c_ulonglong * (4 * n))()
    torch.cuda.synchronize()
    if L.smmd_diag_wino_clock(buf, n) != 0:
        return None
    ghz, dur = [], []
    for b in range(n):
        t0, t1, r0, r1 = buf[4 * b:4 * b + 4]
        if r1 > r0 and t1 > t0:
            ghz.append((t1 - t0) / (r1 - r0) * 0.1)
            dur.append((r1 - r0) / 100.0)
    ghz.sort()
    dur.sort()
    return [round(ghz[len(ghz) // 2], 3), round(dur[len(dur) // 2], 2)] if ghz else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--only', default='')
    ap.add_argument('--lib', default='')
    a = ap.parse_args()
    from gan.core import _lib
    if a.lib:
        import ctypes
        L = ctypes.CDLL(os.path.abspath(a.lib))
        for name, (res, args) in _lib._SIGS.items():
            if hasattr(L, name):
                getattr(L, name).restype = res
                getattr(L, name).argtypes = args
    else:
        L = _lib.lib()
    dev = torch.device('cuda:0')
    st = _lib.stream_handle(dev)
    torch.manual_seed(0)
    out = {'smmd_source_hash': L.smmd_source_hash().decode(), 'lib': a.lib or 'stamped'}
    if a.only in ('', '3x3'):
        for (N, C, K, H) in SHAPES_3X3:
            x = torch.randn(N, C, H, H, device=dev)
            w = torch.randn(K, C, 3, 3, device=dev) / (9 * C) ** 0.5
            b = torch.randn(K, device=dev)
            u = torch.empty(L.smmd_wino3x3_filter_bytes(K, C) // 4, device=dev)
            assert L.smmd_wino3x3_filter(_lib.ptr(w), K, C, 0, _lib.ptr(u), u.numel() * 4, st) == 0
            y = torch.empty(N, K, H, H, device=dev)
            nb = L.smmd_wino3x3_workspace_bytes(N, C, K, H, H)
            ws = torch.empty(max(nb // 4, 4), device=dev)

            def f():
                s = L.smmd_wino3x3_conv(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, C,
                                        K, H, H, _lib.ptr(ws), nb, st)
                assert s == 0
            us = timed(f, a.iters)
            clk = clock_ghz(L, N * (H // 2) ** 2 // 64 * (K // 64))
            fl = 2.0 * 16 * N * (H // 2) ** 2 * C * K
            out['3x3_%d_%d_%d' % (C, K, H)] = {'us': round(us, 2), 'clock_ghz': clk,
                                               'executed_tflops': round(fl / us / 1e6, 1),
                                               'mfma_frac': round(fl / us / 1e6 / 157.3, 3)}
            print(json.dumps({k: v for k, v in out.items() if k.startswith('3x3_%d_' % C)}),
                  flush=True)
    if a.only in ('', 's2'):
        for (N, C, K, H) in SHAPES_S2:
            x = torch.randn(N, C, H, H, device=dev)
            w = torch.randn(K, C, 4, 4, device=dev) / (16 * C) ** 0.5
            b = torch.randn(K, device=dev)
            u = torch.empty(L.smmd_wino4x4s2_filter_bytes(K, C) // 4, device=dev)
            assert L.smmd_wino4x4s2_filter(_lib.ptr(w), K, C, _lib.ptr(u), u.numel() * 4, st) == 0
            y = torch.empty(N, K, H // 2, H // 2, device=dev)
            nb = L.smmd_wino4x4s2_workspace_bytes(N, C, K, H, H)
            ws = torch.empty(max(nb // 4, 4), device=dev)

            def f():
                s = L.smmd_wino4x4s2_conv(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N,
                                          C, K, H, H, _lib.ptr(ws), nb, st)
                assert s == 0
            us = timed(f, a.iters)
            fl = 2.0 * 9 * N * (H // 4) ** 2 * 4 * C * K
            out['s2_%d_%d_%d' % (C, K, H)] = {'us': round(us, 2),
                                              'executed_tflops': round(fl / us / 1e6, 1),
                                              'mfma_frac': round(fl / us / 1e6 / 157.3, 3)}
            print(json.dumps(out['s2_%d_%d_%d' % (C, K, H)]), flush=True)
    if a.only in ('', 's2t'):
        for (N, C, K, H) in SHAPES_S2:
            # the input gradient of the fold layer: gy [N, K, H/2, H/2] -> dx [N, C, H, H]
            Hg = H // 2
            gy = torch.randn(N, K, Hg, Hg, device=dev)
            w = torch.randn(K, C, 4, 4, device=dev) / (16 * C) ** 0.5
            u = torch.empty(L.smmd_wino4x4s2_filter_bytes(K, C) // 4, device=dev)
            assert L.smmd_wino4x4s2t_filter(_lib.ptr(w), K, C, _lib.ptr(u), u.numel() * 4,
                                            st) == 0
            dx = torch.empty(N, C, H, H, device=dev)
            nb = L.smmd_wino4x4s2t_workspace_bytes(N, K, C, Hg, Hg)
            ws = torch.empty(max(nb // 4, 4), device=dev)

            def f():
                s = L.smmd_wino4x4s2t_conv(_lib.ptr(gy), _lib.ptr(u), None, _lib.ptr(dx), N, K,
                                           C, Hg, Hg, _lib.ptr(ws), nb, st)
                assert s == 0
            us = timed(f, a.iters)
            fl = 2.0 * 9 * 4 * N * (Hg // 2) ** 2 * K * C
            out['s2t_%d_%d_%d' % (C, K, H)] = {'us': round(us, 2),
                                               'executed_tflops': round(fl / us / 1e6, 1),
                                               'mfma_frac': round(fl / us / 1e6 / 157.3, 3)}
            print(json.dumps(out['s2t_%d_%d_%d' % (C, K, H)]), flush=True)
    if a.only in ('', 'wgrad'):
        for (N, C, K, H) in SHAPES_3X3:
            x = torch.randn(N, C, H, H, device=dev)
            gy = torch.randn(N, K, H, H, device=dev)
            gw = torch.empty(K, C, 3, 3, device=dev)
            nb = L.smmd_wino3x3_wgrad_workspace_bytes(N, C, K, H, H)
            ws = torch.empty(max(nb // 4, 4), device=dev)

            def f():
                s = L.smmd_wino3x3_wgrad(_lib.ptr(x), _lib.ptr(gy), _lib.ptr(gw), N, C, K, H, H,
                                         _lib.ptr(ws), nb, st)
                assert s == 0
            us = timed(f, a.iters)
            fl = 2.0 * 16 * N * (H // 2) ** 2 * C * K
            out['wgrad_%d_%d_%d' % (C, K, H)] = {'us': round(us, 2),
                                                 'executed_tflops': round(fl / us / 1e6, 1),
                                                 'mfma_frac': round(fl / us / 1e6 / 157.3, 3)}
            print(json.dumps(out['wgrad_%d_%d_%d' % (C, K, H)]), flush=True)
    if a.only in ('', 's2w'):
        # the critic's folded ConvMeanPool layers: x [64, C, H, H], gy [64, K, H/2, H/2]
        for (N, C, K, H) in ((64, 64, 128, 64), (64, 128, 256, 32), (64, 256, 512, 16),
                             (64, 512, 1024, 8)):
            x = torch.randn(N, C, H, H, device=dev)
            gy = torch.randn(N, K, H // 2, H // 2, device=dev)
            gw = torch.empty(K, C, 4, 4, device=dev)
            nb = L.smmd_wino4x4s2_wgrad_workspace_bytes(N, C, K, H, H)
            ws = torch.empty(max(nb // 4, 4), device=dev)

            def f():
                s = L.smmd_wino4x4s2_wgrad(_lib.ptr(x), _lib.ptr(gy), _lib.ptr(gw), N, C, K, H,
                                           H, _lib.ptr(ws), nb, st)
                assert s == 0
            us = timed(f, a.iters)
            fl = 2.0 * 9 * 4 * N * (H // 4) ** 2 * C * K
            out['s2w_%d_%d_%d' % (C, K, H)] = {'us': round(us, 2),
                                               'executed_tflops': round(fl / us / 1e6, 1),
                                               'mfma_frac': round(fl / us / 1e6 / 157.3, 3)}
            print(json.dumps(out['s2w_%d_%d_%d' % (C, K, H)]), flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
