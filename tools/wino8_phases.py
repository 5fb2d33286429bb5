"""Phase times of the 8-wave forward Winograd kernel from a -DWN_CLOCK build
(tools/build_wino_variant.sh clk smmd_wino.hip -DWN_CLOCK): per 3x3 layer at
batch 64, the median over blocks of the prologue, chunk loop and epilogue
(waves 0 and 4) in us, the in-kernel clock, and the spread of block starts.

python tools/wino8_phases.py --lib tools/hip/v_clk.so
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))
SHAPES_3X3 = [(64, 64, 64, 64), (64, 128, 128, 32), (64, 256, 256, 16), (64, 512, 512, 8)]


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', required=True)
    a = ap.parse_args()
    from gan.core import _lib
    L = ctypes.CDLL(os.path.abspath(a.lib))
    for name, (res, args) in _lib._SIGS.items():
        if hasattr(L, name):
            getattr(L, name).restype = res
            getattr(L, name).argtypes = args
    dev = torch.device('cuda:0')
    st = _lib.stream_handle(dev)
    torch.manual_seed(0)
    out = {}
    for (N, C, K, H) in SHAPES_3X3:
        x = torch.randn(N, C, H, H, device=dev)
        w = torch.randn(K, C, 3, 3, device=dev) / (9 * C) ** 0.5
        b = torch.randn(K, device=dev)
        u = torch.empty(L.smmd_wino3x3_filter_bytes(K, C) // 4, device=dev)
        assert L.smmd_wino3x3_filter(_lib.ptr(w), K, C, 0, _lib.ptr(u), u.numel() * 4, st) == 0
        y = torch.empty(N, K, H, H, device=dev)
        nb = L.smmd_wino3x3_workspace_bytes(N, C, K, H, H)
        ws = torch.empty(max(nb // 4, 4), device=dev)
        for _ in range(5):
            assert L.smmd_wino3x3_conv(_lib.ptr(x), _lib.ptr(u), _lib.ptr(b), _lib.ptr(y), N, C, K,
                                       H, H, _lib.ptr(ws), nb, st) == 0
        torch.cuda.synchronize()
        blocks = min(N * (H // 2) ** 2 // 64 * (K // 64), 4096)
        buf = (ctypes.c_ulonglong * (16 * blocks))()
        assert L.smmd_diag_wino8_clock(buf, blocks) == 0
        res = {}
        starts = []
        for ph in (0, 1):
            ghz, pro, loop, b1, b2, epi, tot = [], [], [], [], [], [], []
            for bk in range(blocks):
                t0, t1, t2, t3, t4, t5, r0, r1 = buf[16 * bk + 8 * ph:16 * bk + 8 * ph + 8]
                if r1 <= r0 or t5 <= t0:
                    continue
                g = (t5 - t0) / (r1 - r0) * 0.1
                ghz.append(g)
                pro.append((t1 - t0) / g / 1e3)
                loop.append((t2 - t1) / g / 1e3)
                b1.append((t3 - t2) / g / 1e3)
                b2.append((t4 - t3) / g / 1e3)
                epi.append((t5 - t4) / g / 1e3)
                tot.append((r1 - r0) / 100.0)
                if ph == 0:
                    starts.append(r0)
            res['ph%d' % ph] = {'ghz': round(med(ghz), 3), 'prologue_us': round(med(pro), 2),
                                'loop_us': round(med(loop), 2), 'to_barrier1_us': round(med(b1), 2),
                                'swap_us': round(med(b2), 2), 'rows_us': round(med(epi), 2),
                                'block_us': round(med(tot), 2)}
        starts.sort()
        res['start_spread_us'] = round((starts[-1] - starts[0]) / 100.0, 2)
        res['blocks'] = blocks
        out['3x3_%d_%d_%d' % (C, K, H)] = res
        print(json.dumps({'3x3_%d_%d_%d' % (C, K, H): res}), flush=True)


if __name__ == '__main__':
    main()
