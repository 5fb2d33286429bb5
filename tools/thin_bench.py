"""Microbench of the thin 3x3 convolutions at the ImageNet config's shapes
(critic h0: 3 -> 64 at 64 x 64, batch 64; generator h5: 64 -> 3), library
kernels vs MIOpen, for rocprofv3 --kernel-trace --stats.
usage: python tools/thin_bench.py [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'scaled-mmd-gan_amd'))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from gan.core import convops, miopen_db  # noqa: E402

aten = torch.ops.aten


def timeit(name, fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print('%-28s %8.1f us/call (wall, incl. launch)' % (name, (time.perf_counter() - t0) / reps * 1e6))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    miopen_db.install()         # the committed find db (MIOpen's measured-best solvers)
    dev = 'cuda:0'
    N, H, W = 64, 64, 64
    x3 = torch.randn(N, 3, H, W, device=dev)
    x64 = torch.randn(N, 64, H, W, device=dev)
    w_in = torch.randn(64, 3, 3, 3, device=dev) * 0.1      # conv 3 -> 64
    w_out = torch.randn(3, 64, 3, 3, device=dev) * 0.1     # conv 64 -> 3
    b64 = torch.randn(64, device=dev)
    b3 = torch.randn(3, device=dev)
    gy64 = torch.randn(N, 64, H, W, device=dev)
    gy3 = torch.randn(N, 3, H, W, device=dev)
    cases = [
        ('thin_in fwd', lambda: convops._thin_conv(x3, w_in, b64, 0)),
        ('miopen fwd 3->64', lambda: F.conv2d(x3, w_in, b64, 1, 1)),
        ('thin_out dX (3->64 conv)', lambda: convops._thin_conv(gy64, w_in, None, 1)),
        ('miopen dX (3->64 conv)', lambda: aten.convolution_backward(
            gy64, x3, w_in, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])),
        ('thin wgrad (3->64 conv)', lambda: convops._thin_wgrad(gy64, x3)),
        ('miopen wgrad (3->64 conv)', lambda: aten.convolution_backward(
            gy64, x3, w_in, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])),
        ('thin_out fwd 64->3', lambda: convops._thin_conv(x64, w_out, b3, 0)),
        ('miopen fwd 64->3', lambda: F.conv2d(x64, w_out, b3, 1, 1)),
        ('thin_in dX (64->3 conv)', lambda: convops._thin_conv(gy3, w_out, None, 1)),
        ('thin wgrad (64->3 conv)', lambda: convops._thin_wgrad(gy3, x64)),
        ('miopen wgrad (64->3 conv)', lambda: aten.convolution_backward(
            gy3, x64, w_out, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])),
    ]
    for name, fn in cases:
        timeit(name, fn, reps)


if __name__ == '__main__':
    main()
