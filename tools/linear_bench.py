"""Microbenchmark of the step's two Linear layers in alternative formulations
(hipBLASLt addmm vs mm + bias vs broadcast-multiply + reduction), forward and
first / second order backward, HIP-event timed.

    python tools/linear_bench.py
"""
import time

import torch
import torch.nn.functional as F


def timeit(fn, iters=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def forms():
    return {
        'addmm': lambda x, w, b: F.linear(x, w, b),
        'mm+b': lambda x, w, b: torch.mm(x, w.t()) + b,
        'mul_sum': lambda x, w, b: (x.unsqueeze(1) * w.unsqueeze(0)).sum(-1) + b,
        'matmul_T': lambda x, w, b: torch.matmul(w, x.t()).t() + b,
    }


def main():
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    for (m, k, n) in [(64, 1024, 1), (64, 128, 16384)]:
        x = torch.randn(m, k, device=dev, requires_grad=True)
        w = torch.randn(n, k, device=dev, requires_grad=True)
        b = torch.randn(n, device=dev, requires_grad=True)
        ref = F.linear(x, w, b)
        for name, f in forms().items():
            if name == 'mul_sum' and n > 1:
                continue
            y = f(x, w, b)
            err = float((y - ref).abs().max())
            with torch.no_grad():
                t_f = timeit(lambda: f(x, w, b))

            def bwd():
                y = f(x, w, b)
                torch.autograd.grad(y.sum(), (x, w, b))

            def dbl():
                y = f(x, w, b)
                gx, = torch.autograd.grad(y.sum(), x, create_graph=True)
                torch.autograd.grad((gx * gx).sum() + y.sum(), (w, b))

            t_b = timeit(bwd)
            torch.cuda.synchronize()
            time.sleep(0.05)             # segment marker for a kernel trace
            t_d = timeit(dbl, iters=100)
            torch.cuda.synchronize()
            time.sleep(0.05)
            print('%-6s M=%d K=%d N=%d %-9s fwd %7.1f us  fwd+bwd %7.1f us  fwd+jac+dbl %7.1f us  '
                  'max|d| %.2e' % ('', m, k, n, name, t_f, t_b, t_d, err), flush=True)


if __name__ == '__main__':
    main()
