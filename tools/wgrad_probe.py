"""Runs smmd_wino3x3_wgrad on the SNResNet-64 critic's four 3x3 layer shapes
(batch 64) a few times each, for rocprofv3 counter passes and kernel traces
(tools/gpu_wgrad_pmc.sh).  python tools/wgrad_probe.py [--reps N] [--v1]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--v1', action='store_true')
    a = ap.parse_args()
    if a.v1:
        os.environ['SMMD_WINO_WGRAD_V1'] = '1'
    from gan.core import convops
    dev = torch.device('cuda:0')
    g = torch.Generator(device=dev).manual_seed(0)
    for (N, C, K, H) in [(64, 64, 64, 64), (64, 128, 128, 32), (64, 256, 256, 16),
                         (64, 512, 512, 8)]:
        x = torch.randn(N, C, H, H, device=dev, generator=g)
        gy = torch.randn(N, K, H, H, device=dev, generator=g)
        for _ in range(a.reps):
            convops._wino_wgrad(x, gy)
        torch.cuda.synchronize()
    print('done', flush=True)


if __name__ == '__main__':
    main()
