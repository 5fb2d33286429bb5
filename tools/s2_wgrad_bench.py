"""Stride-2 4x4 weight gradient: smmd_wino4x4s2_wgrad against MIOpen's
(convolution_backward, which adds NCHW<->NHWC transposes around igemm_wrw) on
the SNResNet-64 critic's folded ConvMeanPool layers and the generator's folded
UpsampleConv layers (roles swapped), batch 64.  HIP-event time per call.

    python tools/s2_wgrad_bench.py [--iters N]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))

PEAK = 157.3


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
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    from gan.core import convops, miopen_db
    miopen_db.install()
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)
    aten = torch.ops.aten
    # (name, x [n, ci, h, w], co): critic ConvMeanPool folds; generator UpsampleConv
    # folds as conv(gy_big, .) at upstream x_small
    cases = [('critic_fold%d' % i, (64, c, h, h), 2 * c)
             for i, (c, h) in enumerate([(64, 64), (128, 32), (256, 16), (512, 8)])]
    cases += [('gen_up%d' % i, (64, c, h, h), co)
              for i, (c, h, co) in enumerate([(512, 8, 512), (256, 16, 512), (128, 32, 256),
                                              (64, 64, 128)])]
    for name, (n, ci, h, w), co in cases:
        x = torch.randn(n, ci, h, w, device=dev, generator=g)
        gy = torch.randn(n, co, h // 2, w // 2, device=dev, generator=g)
        wt = torch.empty(co, ci, 4, 4, device=dev)
        ok = convops._s2_wgrad_ok(x, gy, co)
        ref = aten.convolution_backward(gy, x, wt, None, [2, 2], [1, 1], [1, 1], False, [0, 0],
                                        1, [False, True, False])[1]
        row = {'case': name, 'x': [n, ci, h, w], 'co': co, 'tiled': ok}
        t_mi = timed(lambda: aten.convolution_backward(gy, x, wt, None, [2, 2], [1, 1], [1, 1],
                                                       False, [0, 0], 1,
                                                       [False, True, False]), a.iters)
        direct = 2.0 * n * (h // 2) * (w // 2) * co * ci * 16
        row.update(miopen_us=round(t_mi, 1), miopen_direct_tflops=round(direct / t_mi / 1e6, 1))
        if ok:
            gw = convops._s2_wgrad(x, gy)
            t = timed(lambda: convops._s2_wgrad(x, gy), a.iters)
            ex = direct / 16 * 9 / 4 * 4 / 4      # 9 products per (tile, phase column, co)
            ex = 2.0 * 9 * n * (h // 4) * (w // 4) * 4 * ci * co
            row.update(wino_us=round(t, 1), executed_tflops=round(ex / t / 1e6, 1),
                       mfma_frac=round(ex / t / 1e6 / PEAK, 3),
                       rel_err_vs_miopen=float((gw - ref).abs().max() / ref.abs().max()))
        print(json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
