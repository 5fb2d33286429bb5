"""Microbench: conv3x3(SAME) + 2x2 mean pool vs the folded 4x4 stride-2 conv.

meanpool2(conv3x3(x, W)) == conv4x4_s2_p1(x, W'), W'[s,t] = 1/4 sum_{a+u=s, b+v=t} W[u,v]
(gan/core/resnet/block.py:63-66 ConvMeanPool).  Times forward, backward-data and
backward-weights of both forms at the SNResNet-64 critic's ConvMeanPool shapes
(batch 64), in MIOpen immediate mode with the committed find db and, with
--find 1, under cudnn.benchmark.  Prints one JSON line.

  python tools/fold_bench.py [--find 0|1] [--batch 64]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--find', type=int, default=0)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    from gan.core import miopen_db
    miopen_db.install()
    import torch
    import torch.nn.functional as F
    from gan.core.convops import fold_pool_weight
    torch.backends.cudnn.benchmark = bool(a.find)
    dev = torch.device('cuda:0')
    aten = torch.ops.aten
    shapes = [(64, 128, 64), (128, 256, 32), (256, 512, 16), (512, 1024, 8)]
    out = []

    def t(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    for cin, cout, H in shapes:
        x = torch.randn(a.batch, cin, H, H, device=dev)
        w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
        w4 = fold_pool_weight(w)
        y_ref = F.avg_pool2d(F.conv2d(x, w, None, 1, 1), 2)
        y_f = F.conv2d(x, w4, None, 2, 1)
        err = (y_ref - y_f).abs().max().item() / y_ref.abs().max().item()
        gy_full = torch.randn(a.batch, cout, H, H, device=dev)
        gy_half = torch.randn(a.batch, cout, H // 2, H // 2, device=dev)
        r = {'cin': cin, 'cout': cout, 'H': H, 'rel_err': err}
        r['pool_fwd'] = t(lambda: F.avg_pool2d(F.conv2d(x, w, None, 1, 1), 2))
        r['fold_fwd'] = t(lambda: F.conv2d(x, w4, None, 2, 1))
        r['pool_dx'] = t(lambda: aten.convolution_backward(
            F.interpolate(gy_half * 0.25, scale_factor=2, mode='nearest'), x, w, None,
            [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
        r['fold_dx'] = t(lambda: aten.convolution_backward(
            gy_half, x, w4, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]))
        r['pool_dw'] = t(lambda: aten.convolution_backward(
            gy_full, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        r['fold_dw'] = t(lambda: aten.convolution_backward(
            gy_half, x, w4, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        for k in ('pool', 'fold'):
            r[k + '_sum'] = r[k + '_fwd'] + r[k + '_dx'] + r[k + '_dw']
        out.append({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()})
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    print(json.dumps({'find': a.find, 'batch': a.batch, 'rows': out}))


if __name__ == '__main__':
    main()
