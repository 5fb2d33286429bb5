"""Repeat test_tower_and_global_agree_on_one_gpu's comparison and report the
largest differences (MIOpen weight-gradient nondeterminism vs a real bug)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import torch  # noqa: E402
from test_gpu_model import _cfg  # noqa: E402
from gan.core.smmd import SMMD  # noqa: E402

dev = torch.device('cuda:0')
for rep in range(3):
    outs = []
    for mode in ('tower', 'global', 'tower'):
        torch.manual_seed(0)
        model = SMMD(_cfg(), device=dev, dp_mode=mode)
        cap = {}
        orig = model.d_optim.step

        def step(*a, _o=orig, _c=cap, _m=model, **k):
            _c['g'] = _m.d_optim.flat_grad.clone()
            return _o(*a, **k)
        model.d_optim.step = step
        torch.manual_seed(5)
        images = torch.rand(8, 3, 32, 32, device=dev)
        model.train_step(images)
        outs.append(cap['g'])
    scale = float(outs[0].abs().max())
    for k in (1, 2):
        d = (outs[0] - outs[k]).abs()
        i = int(d.argmax())
        offs = model.d_optim.offsets
        t = max(j for j in range(len(offs) - 1) if int(offs[j]) <= i)
        print('rep %d vs %d: max|d| %.3e (%.2e of scale %.3e) at %d tensor %d shape %s: %.6e vs %.6e; '
              'n(|d| > 1e-5 scale) %d' % (rep, k, float(d.max()), float(d.max()) / scale, scale, i, t,
                                          tuple(model.d_optim.params[t].shape), float(outs[0][i]),
                                          float(outs[k][i]), int((d > 1e-5 * scale).sum())), flush=True)
