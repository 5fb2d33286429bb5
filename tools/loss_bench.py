"""The SMMD loss side alone (no convolutions): the fused launch
(smmd_smmd_loss_fwd / _bwd) and the two-launch path (mmd2 + scaled loss),
batch B features [B, 1] and a [1, B, 3, 64, 64] Jacobian, fwd + bwd, for
kernel-trace timing (tools/gpu_trace_loss.sh).

    rocprofv3 --kernel-trace --stats -- python tools/loss_bench.py --iters 200
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--batch', type=int, nargs='+', default=[64, 256])
    args = ap.parse_args()
    from gan.core import mmd, ops
    dev = torch.device('cuda:0')
    for B in args.batch:
        X = torch.randn(B, 1, device=dev, requires_grad=True)
        Y = torch.randn(B, 1, device=dev, requires_grad=True)
        jac = (torch.randn(1, B, 3, 64, 64, device=dev) * 0.05).requires_grad_(True)
        for fused in (True, False):
            for _ in range(args.iters):
                if fused:
                    p = mmd.ScalePending(jac, Y, 10.0, 'grad')
                    with mmd.pending_scale(p):
                        mmd.mmd2(mmd._rbf_kernel(X, Y))
                    g = p.result[1]
                else:
                    v = mmd.mmd2(mmd._rbf_kernel(X, Y))
                    g, _ = ops.scaled_loss(v, jac, None, sc=10.0)
                torch.autograd.grad(g, (X, Y, jac))
            torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()
