"""Run-to-run determinism of the critic step by width.

Two SNResNet-64 models from the same seed take one critic update each; the
second under the torch profiler (CPU activity) to list the aten convolution
ops (MIOpen) the step ran.  Prints, per width, the aten conv ops and the max
|difference| of the two flat critic gradients.  At width 16 the channel
counts 16 / 32 fail the library's cout % 64 guards, so MIOpen runs some
convolutions (its weight gradients are not bitwise deterministic); at the
ImageNet config's width 64 every conv is on the library."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd'), os.path.join(ROOT, 'tests')]

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def one(width, batch, prof):
    from gan.core.smmd import SMMD
    from gan.main import default_flags
    c = default_flags()
    c.update(dict(batch_size=batch, output_size=64, architecture='snresnet', kernel='rbf',
                  model='smmd', batch_norm=True, with_sn=True, with_learnable_sn_scale=True,
                  with_scaling=True, dof_dim=1, learning_rate=1e-4, dataset='cifar10',
                  df_dim=width, gf_dim=width))
    torch.manual_seed(0)
    model = SMMD(argparse.Namespace(**c), device='cuda:0')
    images = torch.rand(batch, 3, 64, 64, generator=torch.Generator().manual_seed(1)).cuda()
    z = torch.empty(batch, 128).uniform_(-1, 1, generator=torch.Generator().manual_seed(2)).cuda()
    model.sample_z = lambda n: z
    model.step = 25
    model.d_counter = model.g_counter = 0
    cap = {}
    orig = model.d_optim.step

    def c_(*a, **k):
        cap['g'] = model.d_optim.dense_grad().clone()
        return orig(*a, **k)
    model.d_optim.step = c_
    convs = []
    if prof:
        with profile(activities=[ProfilerActivity.CPU]) as p:
            model.d_step(images)
        convs = sorted({e.name for e in p.events()
                        if e.name.startswith('aten::') and 'conv' in e.name})
    else:
        model.d_step(images)
    torch.cuda.synchronize()
    return cap['g'], convs


def main():
    from gan.core import _lib
    print('library stamp', _lib.lib().smmd_source_hash().decode())
    for width, batch in ((16, 8), (64, 8), (64, 64)):
        a, _ = one(width, batch, False)
        diffs = []
        convs = None
        for rep in range(3):
            b, cv = one(width, batch, rep == 0)
            convs = cv if rep == 0 else convs
            diffs.append(float((a - b).abs().max()))
        print('width %d batch %d: aten conv ops %s; max|g_a - g_b| over 3 repeats %s '
              '(scale %.3g)' % (width, batch, convs or 'none', diffs, float(a.abs().max())))


if __name__ == '__main__':
    main()
