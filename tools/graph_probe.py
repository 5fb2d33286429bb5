"""Probe: the lean training step as HIP-graph replays (model.enable_graphs)
against eager, on the bench workload.  GPU only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]
import torch  # noqa: E402


def main():
    import bench
    from gan.core import miopen_db
    from gan.core.smmd import SMMD
    miopen_db.install()
    dev = torch.device('cuda:0')
    name = sys.argv[1] if len(sys.argv) > 1 else 'imagenet'
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    cfg = bench.CONFIGS[name][0](batch)
    size = int(cfg.output_size)
    torch.manual_seed(2)
    model = SMMD(cfg, device=dev)
    imgs = [torch.rand(batch, 3, size, size, device=dev) for _ in range(4)]
    print(name, batch, flush=True)
    model.step = 25
    for i in range(12):
        model.train_step(imgs[i % 4])
    torch.cuda.synchronize()

    def timeit(n=60):
        model.d_counter = model.g_counter = 0
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(n):
            model.train_step(imgs[i % 4])
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    print('eager ms/step %.3f' % timeit(), flush=True)
    model.enable_graphs()
    t = time.perf_counter()
    for i in range(12):
        model.train_step(imgs[i % 4])
    torch.cuda.synchronize()
    print('captures + 12 steps %.2f s, kinds %s' % (time.perf_counter() - t,
                                                   sorted(model._graphs.graphs)), flush=True)
    print('graph ms/step %.3f' % timeit(), flush=True)
    print('loss', float(model.last['d_loss']), float(model.last['g_loss']), flush=True)
    model.enable_graphs(False)
    print('eager again ms/step %.3f' % timeit(), flush=True)


if __name__ == '__main__':
    main()
