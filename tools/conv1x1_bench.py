"""The critic's 1x1 shortcut convolutions (MeanPoolConv: the 1x1 conv on the
pooled block input, gan/core/resnet/block.py:28-40) at bench.py's shapes:
MIOpen (F.conv2d / convolution_backward, what the step runs) against GEMM
forms on NCHW without transposes (torch.matmul -> hipBLASLt batched GEMMs)
and the library's smmd_conv1x1* (lib_*).

    python tools/conv1x1_bench.py [--iters 50]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [(64, 64, 128, 32), (64, 128, 256, 16), (64, 256, 512, 8), (64, 512, 1024, 4)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    args = ap.parse_args()
    from gan.core import miopen_db
    miopen_db.install()
    torch.backends.cudnn.benchmark = False
    dev = torch.device('cuda', 0)
    aten = torch.ops.aten
    res = {}
    for n, c, k, h in SHAPES:
        x = torch.randn(n, c, h, h, device=dev)
        gy = torch.randn(n, k, h, h, device=dev)
        w = torch.randn(k, c, 1, 1, device=dev) * 0.05
        w2 = w.view(k, c)
        x3, gy3 = x.view(n, c, h * h), gy.view(n, k, h * h)
        fl = 2.0 * n * h * h * c * k
        row = {}
        row['miopen_fwd'] = timeit(lambda: F.conv2d(x, w), args.iters)
        row['miopen_dx'] = timeit(lambda: aten.convolution_backward(
            gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False]),
            args.iters)
        row['miopen_dw'] = timeit(lambda: aten.convolution_backward(
            gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False]),
            args.iters)
        row['mm_fwd'] = timeit(lambda: torch.matmul(w2, x3), args.iters)
        row['mm_dx'] = timeit(lambda: torch.matmul(w2.t(), gy3), args.iters)
        row['bmm_dw_sum'] = timeit(lambda: torch.bmm(gy3, x3.transpose(1, 2)).sum(0), args.iters)
        row['einsum_dw'] = timeit(lambda: torch.einsum('nkp,ncp->kc', gy3, x3), args.iters)
        from gan.core import convops
        row['lib_fwd'] = timeit(lambda: convops._c1_fwd(x, w, None), args.iters)
        row['lib_dx'] = timeit(lambda: convops._c1_dx(gy, w), args.iters)
        row['lib_dw'] = timeit(lambda: convops._c1_wgrad(gy, x), args.iters)
        y0 = F.conv2d(x, w)
        y1 = torch.matmul(w2, x3).view_as(y0)
        d0 = aten.convolution_backward(gy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                       [False, True, False])[1].view(k, c)
        d1 = torch.einsum('nkp,ncp->kc', gy3, x3)
        row['fwd_maxdiff'] = float((y0 - y1).abs().max() / y0.abs().max())
        row['lib_fwd_maxdiff'] = float((y0 - convops._c1_fwd(x, w, None)).abs().max()
                                       / y0.abs().max())
        row['lib_dw_maxdiff'] = float((d0 - convops._c1_wgrad(gy, x).view(k, c)).abs().max()
                                      / d0.abs().max())
        row['dw_maxdiff'] = float((d0 - d1).abs().max() / d0.abs().max())
        row = {q: (round(v, 2) if 'diff' not in q else v) for q, v in row.items()}
        row['gflop'] = round(fl / 1e9, 3)
        res['%dx%dx%dx%d' % (n, c, k, h)] = row
        print(json.dumps({'%dx%dx%dx%d' % (n, c, k, h): row}), flush=True)


if __name__ == '__main__':
    main()
