"""Graph replay vs eager, step by step (the all-library SNResNet-64 step at
width 64, batch 8): the first step whose parameters differ, per variant.
python tools/graph_diff_probe.py [variant ...]; variants: base, nolazy, nocache"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd'), os.path.join(ROOT, 'tests')]

import torch  # noqa: E402


def run(variant):
    from gan.core import convops, sn
    import test_gpu_model as T
    from gan.core.smmd import SMMD
    if variant == 'nocache':
        convops.arm_capture_cache = lambda on: None
    os.environ['SMMD_SN_LAZY_GRAPH'] = '0' if variant == 'nolazy' else '1'
    dev = torch.device('cuda:0')
    a, images = T._headline_model(dev, batch=8)
    g = torch.Generator().manual_seed(3)
    imgs = [torch.rand(8, 3, 64, 64, generator=g).to(dev) for _ in range(3)]
    for i in range(7):
        a.train_step(imgs[i % 3])
    b = SMMD(a.config, device=dev)
    b.load_state_dict(a.state_dict())
    b.sample_z = a.sample_z
    assert torch.equal(a.d_optim.flat_param, b.d_optim.flat_param)
    bufs = {}

    def hook(m, tag):
        opt = m.d_optim
        orig = opt.step
        buf = bufs[tag] = torch.zeros_like(opt.flat_grad)
        lrb = bufs[tag + 'lr'] = torch.zeros(1, device=dev)

        def st(*a, **k):
            buf.copy_(opt.dense_grad())
            r = orig(*a, **k)
            lrb.copy_(opt.lr_t_dev.view(-1)[:1])
            return r
        opt.step = st
    hook(a, 'a')
    hook(b, 'b')
    b.enable_graphs()
    out = []
    for i in range(13):
        kind = 'D' if a.d_counter != 0 else 'G'
        la = a.train_step(imgs[i % 3])
        lb = b.train_step(imgs[i % 3])
        torch.cuda.synchronize()
        dd = float((a.d_optim.flat_param - b.d_optim.flat_param).abs().max())
        dg = float((a.g_optim.flat_param - b.g_optim.flat_param).abs().max())
        dl = float((la[1] - lb[1]).abs())
        dgr = float((bufs['a'] - bufs['b']).abs().max())
        dlr = float((bufs['alr'] - bufs['blr']).abs().max())
        out.append('%s%d dD %.3g dG %.3g d_loss %.3g dgrad %.3g dlr %.3g' % (kind, i, dd, dg, dl,
                                                                       dgr, dlr))
    print(variant, '|', '; '.join(out), flush=True)


if __name__ == '__main__':
    for v in (sys.argv[1:] or ['base']):
        run(v)
