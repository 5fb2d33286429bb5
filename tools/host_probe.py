"""Host (Python) time per training step against GPU time, on bench.py's
workload: is the GPU queue ever left empty?  For K steps after a warmup:
the host time until train_step returns (no sync inside), the time at which
the GPU finishes (one sync at the end), and per step kind the host time of
the call.  If the host's time per step approaches the GPU's, the GPU runs
dry at the step boundaries (the kernel trace's gaps there).

    python tools/host_probe.py [--steps 60] [--profile]   (--profile: cProfile
    of the host side over the timed steps, top entries by own time)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=60)
    ap.add_argument('--profile', action='store_true')
    args = ap.parse_args()
    import bench
    from gan.core import miopen_db
    from gan.core.smmd import SMMD
    miopen_db.install()
    torch.backends.cudnn.benchmark = False
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    cfg = bench.imagenet_config(64)
    torch.manual_seed(2)
    model = SMMD(cfg, device=dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    images = [torch.rand(64, 3, 64, 64, device=dev, generator=gen) for _ in range(4)]
    model.d_step(images[0])
    model.g_step(images[1])
    model.step = 21
    for i in range(12):
        model.train_step(images[i % 4])
    model.d_counter = model.g_counter = 0
    torch.cuda.synchronize()
    host = {'D': [], 'G': []}
    prof = None
    if args.profile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for i in range(args.steps):
        kind = 'G' if model.d_counter == 0 and model.step >= 0 and False else None
        a = time.perf_counter()
        dc = model.d_counter
        model.train_step(images[i % 4])
        host['G' if model.d_counter == 0 and dc != 0 or (dc == 0) else 'D'].append(
            time.perf_counter() - a)
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    tg = time.perf_counter() - t0
    if prof is not None:
        prof.disable()
    print('steps %d: host %.3f ms/step, until the GPU finished %.3f ms/step (host/GPU %.3f)' % (
        args.steps, th / args.steps * 1e3, tg / args.steps * 1e3, th / tg))
    for k, v in host.items():
        if v:
            print('  host per %s call: mean %.3f ms  min %.3f  max %.3f (n=%d)' % (
                k, sum(v) / len(v) * 1e3, min(v) * 1e3, max(v) * 1e3, len(v)))
    if prof is not None:
        import pstats
        pstats.Stats(prof).sort_stats('tottime').print_stats(40)


if __name__ == '__main__':
    main()
