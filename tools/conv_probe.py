"""Find slow convolution calls: run the bench workload's step kinds (lean and
reference schedule, or another --config) with every aten convolution op
synchronised and timed; print each distinct (op, shapes, strides, params)
whose call took longer than --ms, once.

    python tools/conv_probe.py [--schedule reference] [--ms 1.0]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402


def desc(a):
    if isinstance(a, torch.Tensor):
        return 'T%s%s%s' % (list(a.shape), list(a.stride()), '' if a.is_contiguous() else '!nc')
    if isinstance(a, (list, tuple)):
        return '[' + ','.join(desc(x) for x in a) + ']'
    return repr(a)


class Probe(TorchDispatchMode):
    def __init__(self, ms):
        super().__init__()
        self.ms = ms
        self.seen = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if 'convolution' not in str(func):
            return func(*args, **kwargs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = func(*args, **kwargs)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        key = str(func) + ' ' + ' '.join(desc(a) for a in args)
        if dt > self.ms:
            n, tot = self.seen.get(key, (0, 0.0))
            self.seen[key] = (n + 1, tot + dt)
            if n == 0:
                print('%.2f ms  %s' % (dt, key), flush=True)
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--schedule', default='reference')
    ap.add_argument('--config', default='imagenet')
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--steps', type=int, default=14)
    ap.add_argument('--ms', type=float, default=1.0)
    args = ap.parse_args()
    import bench
    from gan.core import miopen_db
    miopen_db.install()
    torch.backends.cudnn.benchmark = False
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    from gan.core.smmd import SMMD
    cfg = bench.CONFIGS[args.config][0](args.batch)
    size = int(cfg.output_size)
    torch.manual_seed(2)
    model = SMMD(cfg, device=dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    images = [torch.rand(args.batch, 3, size, size, device=dev, generator=gen) for _ in range(2)]
    model.schedule = args.schedule
    for i in range(2):                            # MIOpen's first calls (compile, db)
        model.d_step(images[i % len(images)])
        model.g_step(images[i % len(images)])
    torch.cuda.synchronize()
    p = Probe(args.ms)
    with p:
        for i in range(args.steps):
            model.train_step(images[i % len(images)])
    torch.cuda.synchronize()
    print('slow calls:', sum(n for n, _ in p.seen.values()), 'ms total: %.1f' %
          sum(t for _, t in p.seen.values()), flush=True)


if __name__ == '__main__':
    main()
