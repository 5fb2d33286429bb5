"""Where the step's PyTorch elementwise kernels come from: one critic and one
generator step of the bench workload under torch.profiler, every device
kernel of the chosen aten ops attributed to the autograd node (or forward
module call) that issued it, with its input shapes and GPU time.

    python tools/op_sources.py [--ops add,add_,threshold_backward,...] [--top 40]
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def owner(ev):
    """The nearest enclosing autograd node or the top-level forward op."""
    p, chain = ev.cpu_parent, []
    while p is not None:
        chain.append(p.name)
        if p.name.startswith('autograd::engine::evaluate_function'):
            return p.name.split(': ', 1)[-1], chain
        p = p.cpu_parent
    return (chain[-1] if chain else '<top>'), chain


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--ops', default='aten::add,aten::add_,aten::threshold_backward,aten::fill_,'
                                     'aten::zero_,aten::sub,aten::mul,aten::copy_,aten::where,'
                                     'aten::relu,aten::leaky_relu,aten::leaky_relu_backward,'
                                     'aten::cat,aten::sum,aten::avg_pool2d,'
                                     'aten::avg_pool2d_backward,aten::neg')
    ap.add_argument('--top', type=int, default=50)
    ap.add_argument('--batch', type=int, default=64)
    args = ap.parse_args()
    ops = set(args.ops.split(','))
    import bench
    from gan.core import miopen_db
    from gan.core.smmd import SMMD
    miopen_db.install()
    torch.backends.cudnn.benchmark = False
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    cfg = bench.imagenet_config(args.batch)
    torch.manual_seed(2)
    model = SMMD(cfg, device=dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    size = int(cfg.output_size)
    images = [torch.rand(args.batch, 3, size, size, device=dev, generator=gen) for _ in range(4)]
    for _ in range(2):
        model.d_step(images[0])
        model.g_step(images[1])
    model.step = 21
    torch.cuda.synchronize()
    for kind, fn in (('D', lambda: model.d_step(images[2])), ('G', lambda: model.g_step(images[3]))):
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                     record_shapes=True) as prof:
            fn()
            torch.cuda.synchronize()
        agg = collections.defaultdict(lambda: [0, 0.0])
        tot_all = 0.0
        for ev in prof.events():
            t = ev.device_time_total
            if ev.device_type == torch.autograd.DeviceType.CPU and ev.cpu_parent is None:
                tot_all += t
            if ev.name not in ops or t <= 0:
                continue
            # only the op's own launch, not an op nested in another listed op
            p = ev.cpu_parent
            nested = False
            while p is not None:
                if p.name in ops:
                    nested = True
                    break
                p = p.cpu_parent
            if nested:
                continue
            who, _ = owner(ev)
            shapes = tuple(tuple(s) for s in (ev.input_shapes or []) if s)[:2]
            a = agg[(ev.name, who, shapes)]
            a[0] += 1
            a[1] += t
        rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
        s = sum(v[1] for v in agg.values())
        print('== %s step: listed ops %.1f us of %.1f us device time' % (kind, s, tot_all))
        for (name, who, shapes), (n, t) in rows[:args.top]:
            print('%8.1f us %4d  %-28s %-44s %s' % (t, n, name, who[:44], shapes))


if __name__ == '__main__':
    main()
