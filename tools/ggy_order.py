"""Which of the two double-backward nodes that share one first-order gradient
(a critic block's main-path and shortcut convs, both fed _ReluPool's gu) runs
first: one critic step of the bench workload with _ConvBackward.backward
logged (gy pointer, x and w shapes, the order of arrival).

    python tools/ggy_order.py
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]

import torch  # noqa: E402


def main():
    import bench
    from gan.core import convops, miopen_db
    from gan.core.smmd import SMMD
    miopen_db.install()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    cfg = bench.imagenet_config(64)
    torch.manual_seed(2)
    model = SMMD(cfg, device=dev)
    gen = torch.Generator(device=dev).manual_seed(0)
    size = int(cfg.output_size)
    images = [torch.rand(64, 3, size, size, device=dev, generator=gen) for _ in range(3)]
    model.d_step(images[0])
    model.g_step(images[1])
    log = []
    orig = convops._ConvBackward.backward

    def logged(ctx, ggx, ggw):
        x, w, gy, _ = ctx.saved_tensors
        out = orig(ctx, ggx, ggw)
        log.append((gy.data_ptr(), tuple(gy.shape), tuple(x.shape), tuple(w.shape),
                    out[2] is not None))
        return out

    convops._ConvBackward.backward = staticmethod(logged)
    model.d_step(images[2])
    torch.cuda.synchronize()
    convops._ConvBackward.backward = orig
    seen = collections.defaultdict(list)
    for i, (p, gys, xs, ws, has) in enumerate(log):
        seen[p].append((i, gys, xs, ws, has))
    print('%d _ConvBackward.backward calls' % len(log))
    for p, calls in seen.items():
        if len(calls) > 1:
            print('shared gy', calls[0][1])
            for i, gys, xs, ws, has in calls:
                print('   #%3d x %-20s w %-20s g_gy %s' % (i, xs, ws, has))


if __name__ == '__main__':
    main()
