"""The bench workload (ImageNet SNResNet-64 SMMD, batch 64, lean schedule)
for profiler passes: prime every step kind, warm up, then run exactly
`--cycles` whole 5 D + 1 G cycles.  Every step ends in exactly one optimizer
update kernel (opt_adam*), so a post-processor (tools/step_flops_pmc.py) cuts
the window as the dispatches after the (updates - 6 cycles)-th update.

    rocprofv3 --pmc ... -- python tools/step_cycle.py --cycles 2
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]

import torch  # noqa: E402

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cycles', type=int, default=2)
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--warmup', type=int, default=6)
    args = ap.parse_args()
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
    model.d_step(images[0])
    model.g_step(images[1])
    model.step = 21
    for i in range(args.warmup):
        model.train_step(images[i % 4])
    model.d_counter = model.g_counter = 0
    torch.cuda.synchronize()
    kinds = []
    for i in range(6 * args.cycles):
        before = model.step
        model.train_step(images[i % 4])
        kinds.append('G' if model.step != before else 'D')
    torch.cuda.synchronize()
    print('steps', ''.join(kinds), flush=True)


if __name__ == '__main__':
    main()
