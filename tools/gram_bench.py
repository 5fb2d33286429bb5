"""MFMA Gram path of smmd_mmd2_fwd (d > 32): HIP-event time of the library call
per (N per side, D), for the 64 x 64 and 128 x 128 block tilings
(SMMD_GRAM_TILE), with TFLOP/s against the f32 MFMA peak (157.3 TF).

    python tools/gram_bench.py [--json out.json]

Flops counted as executed: the Gram S = Z Z^T over all (2N)^2 pairs plus
G = C Z, 2 * D * (2N)^2 each (the bench's mmd_sweep counts the reference's
three blocks, P = 3 N^2 pairs, i.e. 3/4 of these)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--json', default='')
    ap.add_argument('--only', default='', help='N,D: one size (PMC passes)')
    ap.add_argument('--tiles', default='64,128')
    ap.add_argument('--paths', action='store_true',
                    help='row sweep vs Gram path (SMMD_MMD_GRAM=0/1) at small d')
    args = ap.parse_args()
    if args.paths:
        return path_sweep(args)
    from gan.core import _lib, mmd
    dev = torch.device('cuda:0')
    rows = []
    sizes = [(512, 128), (512, 1024), (1024, 1024), (2048, 128), (2048, 1024), (4096, 512)]
    if args.only:
        sizes = [tuple(int(v) for v in args.only.split(','))]
    for N, D in sizes:
        rng = np.random.default_rng(1234)
        X = torch.tensor(rng.standard_normal((N, D)) / np.sqrt(D), dtype=torch.float32,
                         device=dev, requires_grad=True)
        Y = torch.tensor(rng.standard_normal((N, D)) / np.sqrt(D), dtype=torch.float32,
                         device=dev, requires_grad=True)
        for tile in args.tiles.split(','):
            os.environ['SMMD_GRAM_TILE'] = tile
            for _ in range(3):
                v = mmd.mmd2_fused(X, Y, 'rbf')
                torch.autograd.grad(v, (X, Y))
            torch.cuda.synchronize()
            _lib.reset_timing()
            _lib.enable_timing(True)
            iters = 10
            for _ in range(iters):
                v = mmd.mmd2_fused(X, Y, 'rbf')
                torch.autograd.grad(v, (X, Y))
            _lib.enable_timing(False)
            ms = _lib.timing_ms()['smmd_mmd2_fwd'][1]
            fl = 4.0 * D * (2 * N) ** 2
            tf = fl / (ms * 1e-3) / 1e12
            rows.append({'N': N, 'D': D, 'tile': int(tile), 'ms': round(ms, 4),
                         'tflops': round(tf, 2), 'mfma_frac': round(tf / PEAK, 4),
                         'mmd2': float(v)})
            print(json.dumps(rows[-1]), flush=True)
    os.environ.pop('SMMD_GRAM_TILE', None)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(rows, f, indent=1)


def path_sweep(args):
    """smmd_mmd2_fwd time, row-sweep kernel vs MFMA Gram path, d <= 32."""
    from gan.core import _lib, mmd
    dev = torch.device('cuda:0')
    rows = []
    for N in (256, 1024, 2048):
        for D in (1, 2, 4, 8, 16, 32):
            rng = np.random.default_rng(1234)
            X = torch.tensor(rng.standard_normal((N, D)) / np.sqrt(D), dtype=torch.float32,
                             device=dev, requires_grad=True)
            Y = torch.tensor(rng.standard_normal((N, D)) / np.sqrt(D), dtype=torch.float32,
                             device=dev, requires_grad=True)
            rec = {'N': N, 'D': D}
            for path in ('0', '1'):
                os.environ['SMMD_MMD_GRAM'] = path
                for _ in range(3):
                    v = mmd.mmd2_fused(X, Y, 'rbf')
                    torch.autograd.grad(v, (X, Y))
                torch.cuda.synchronize()
                _lib.reset_timing()
                _lib.enable_timing(True)
                for _ in range(10):
                    v = mmd.mmd2_fused(X, Y, 'rbf')
                    torch.autograd.grad(v, (X, Y))
                _lib.enable_timing(False)
                rec['sweep_ms' if path == '0' else 'gram_ms'] = round(
                    _lib.timing_ms()['smmd_mmd2_fwd'][1], 4)
            rows.append(rec)
            print(json.dumps(rec), flush=True)
    os.environ.pop('SMMD_MMD_GRAM', None)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
