"""MMD kernel microbenchmark for rocprofv3 kernel traces: smmd_mmd2_fwd (value
+ unit gradient) on X, Y ~ N(0,1) [N, D] (numpy default_rng(1234))
for each (kernel, N, D), `--iters` calls back to back, so the per-kernel
durations of `rocprofv3 --kernel-trace --stats` are the kernels alone (HIP
events around single small calls also time the host's launch gap).

    rocprofv3 --kernel-trace --stats -d out -o run -- python tools/mmd_bench.py
"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--grid', default='rbf:64:1,rbf:512:1,rbf:2048:1,mix_rq:2048:1,'
                                      'mix_rbf:2048:1,rbf:4096:1')
    ap.add_argument('--json', default='')
    args = ap.parse_args()
    from gan.core import _lib, mmd
    dev = torch.device('cuda:0')
    res = []
    for item in args.grid.split(','):
        kern, N, D = item.split(':')
        N, D = int(N), int(D)
        rng = np.random.default_rng(1234)
        X = torch.tensor((rng.standard_normal((N, D)) / np.sqrt(D)).astype(np.float32), device=dev)
        Y = torch.tensor((rng.standard_normal((N, D)) / np.sqrt(D)).astype(np.float32), device=dev)
        spec = mmd.get_kernel_spec(kern)
        desc = spec.desc()
        L = _lib.lib()
        ws = torch.zeros(L.smmd_mmd2_workspace_bytes(N, N, D), dtype=torch.uint8, device=dev)
        sums = torch.empty(8, device=dev)
        out = torch.empty(1, device=dev)
        gx, gy = torch.empty_like(X), torch.empty_like(Y)
        s = _lib.stream_handle(dev)
        args_ = (desc, _lib.ptr(X), N, _lib.ptr(Y), N, D, 0, 0, N, 0, N, _lib.ptr(sums),
                 _lib.ptr(out), _lib.ptr(gx), _lib.ptr(gy), _lib.ptr(ws), ws.numel(), s)
        for _ in range(5):
            _lib.check(L.smmd_mmd2_fwd(*args_), 'smmd_mmd2_fwd')
        torch.cuda.synchronize()
        # a long kernel in front keeps the queue full: the events then time
        # the back-to-back MMD launches, not the host's launch gaps
        big = torch.empty(64 << 20, device=dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        big.fill_(1.0)
        e0.record()
        for _ in range(args.iters):
            L.smmd_mmd2_fwd(*args_)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        P = 3 * N * N
        res.append({'kernel': kern, 'N': N, 'D': D, 'us_per_call': round(ms * 1e3, 2),
                    'pairs_ref': P, 'pair_evals_per_s': round(P / (ms * 1e-3), 1),
                    'mmd2': out.item()})
        print(json.dumps(res[-1]), flush=True)
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
