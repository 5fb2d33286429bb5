"""Per-aten-op GPU time of the bench workload (torch.profiler), to attribute
the non-convolution kernels of the step to the ops that launch them.

    python tools/op_profile.py [--steps 6] [--out gpurun_out/ops.txt]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--out', default='gpurun_out/ops.txt')
    ap.add_argument('--stack', action='store_true',
                    help='also attribute small add_/fill_/add kernels to Python call sites')
    args = ap.parse_args()
    import bench
    from gan.core import miopen_db
    from gan.core.smmd import SMMD
    miopen_db.install()
    dev = torch.device('cuda:0')
    cfg = bench.imagenet_config()
    torch.manual_seed(2)
    model = SMMD(cfg, device=dev)
    images = torch.rand(64, 3, 64, 64, device=dev)
    model.step = 21
    for _ in range(12):
        model.train_step(images)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 record_shapes=True, with_stack=args.stack) as prof:
        for _ in range(args.steps):
            model.train_step(images)
        torch.cuda.synchronize()
    tab = prof.key_averages().table(sort_by='self_cuda_time_total', row_limit=60,
                                    max_name_column_width=60)
    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    with open(args.out, 'w') as f:
        f.write(tab)
    # the elementwise ops by input shape (which tensors the adds accumulate)
    shp = prof.key_averages(group_by_input_shape=True)
    conv = [e for e in shp if e.key in ('aten::miopen_convolution', 'aten::convolution_backward',
                                        'aten::miopen_convolution_transpose',
                                        'aten::cudnn_convolution', 'aten::convolution')]
    conv.sort(key=lambda e: -e.self_device_time_total)
    with open(args.out.replace('.txt', '_convs.txt'), 'w') as f:
        for e in conv[:80]:
            f.write('%-36s %10.1f us total %5d calls %8.1f us/call  %s\n' % (
                e.key, e.self_device_time_total, e.count, e.self_device_time_total / e.count,
                str(e.input_shapes)[:200]))
    rows = [e for e in shp if e.key in ('aten::add_', 'aten::add', 'aten::mul', 'aten::fill_')]
    rows.sort(key=lambda e: -e.self_device_time_total)
    with open(args.out.replace('.txt', '_shapes.txt'), 'w') as f:
        for e in rows[:60]:
            f.write('%-12s %10.1f us total %5d calls  %s\n' % (
                e.key, e.self_device_time_total, e.count, str(e.input_shapes)[:160]))
    if args.stack:
        st = prof.key_averages(group_by_stack_n=6)
        rows = [e for e in st if e.key in ('aten::add_', 'aten::add', 'aten::mul', 'aten::fill_',
                                           'aten::zero_',
                                           'aten::zeros', 'aten::zeros_like', 'aten::copy_')]
        rows.sort(key=lambda e: -e.count)
        with open(args.out.replace('.txt', '_stacks.txt'), 'w') as f:
            for e in rows[:40]:
                f.write('%-14s %5d calls %10.1f us\n    %s\n' % (
                    e.key, e.count, e.self_device_time_total, '\n    '.join(e.stack[:6])))
    print(tab[:6000])


if __name__ == '__main__':
    main()
