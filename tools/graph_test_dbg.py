"""Debug: the step-graph parity test body outside pytest, with progress prints."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]
import torch  # noqa: E402


def main():
    from gan.main import default_flags
    from gan.core.smmd import SMMD
    from gan.core import model as M
    c = default_flags()
    c.update(dict(batch_size=8, output_size=32, architecture='sngan', kernel='rbf', model='smmd',
                  batch_norm=True, with_sn=True, with_learnable_sn_scale=True, with_scaling=True,
                  dof_dim=1, learning_rate=1e-4, dataset='cifar10'))
    cfg = argparse.Namespace(**c)
    dev = torch.device('cuda:0')
    two = len(sys.argv) > 1 and sys.argv[1] == 'two'
    torch.manual_seed(0)
    b = SMMD(cfg, device=dev)
    a = SMMD(cfg, device=dev) if two else None
    g = torch.Generator().manual_seed(3)
    imgs = [torch.rand(8, 3, 32, 32, generator=g).to(dev) for _ in range(3)]
    z = torch.empty(8, 128).uniform_(-1, 1, generator=g).to(dev)
    orig = M.StepGraphs._capture

    def cap(self, kind, critic):
        print('capture', kind, flush=True)
        orig(self, kind, critic)
        print('captured', kind, flush=True)
    M.StepGraphs._capture = cap
    for m in [x for x in (a, b) if x is not None]:
        m.sample_z = lambda n: z
        for i in range(12):
            m.train_step(imgs[i % 3])
    torch.cuda.synchronize()
    print('eager done', flush=True)
    b.enable_graphs()
    b.step = 25
    for i in range(14):
        if a is not None:
            a.train_step(imgs[i % 3])
        b.train_step(imgs[i % 3])
        print('step', i, flush=True)
    torch.cuda.synchronize()
    print('ok', float(b.last['d_loss']), flush=True)


if __name__ == '__main__':
    main()
