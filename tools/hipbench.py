"""Library-only microbenchmark: the libsmmd_hip launches of one SNResNet-64
SMMD training step at bench.py's sizes, without the convolutions.

    python tools/hipbench.py [--iters 200] [--json out.json]

Times each entry point with HIP events on the compute stream (mean over
iterations after warm-up) and reports algorithmic GB/s and the fraction of the
8 TB/s HBM peak.  Used for kernel A/B work and for the PMC (FETCH_SIZE /
WRITE_SIZE) passes, which crash the profiler when MIOpen is in the process.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--json', default='')
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--no-fuse', action='store_true',
                    help='plain smmd_adam_flat + full refresh (no SN-fused update)')
    args = ap.parse_args()
    from gan.core import _lib, mmd, ops
    from gan.core.architecture import SNResNetDiscriminator
    from gan.core.optim import FlatAdam
    from gan.core.sn import SpectralNormBank
    from gan.core.snops import sn_modules
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    D = SNResNetDiscriminator(64, 1, False, with_sn=True, with_learnable_sn_scale=True,
                              input_size=64).to(dev)
    bank = SpectralNormBank(sn_modules(D))
    opt = FlatAdam([p for p in D.parameters() if p.requires_grad], 2e-4, name='D')
    if not args.no_fuse:     # as MMD_GAN: the critic step of the bench's 5 D + 1 G schedule
        assert opt.attach_sn(bank)
    with torch.no_grad():      # the refresh outputs (pool-folded 4x4 filters for ConvMeanPool)
        Gs = [torch.randn_like(o) for o in bank.refresh(update_u=False)]
    B = args.batch
    X = torch.randn(B, 1, device=dev, requires_grad=True)
    Y = torch.randn(B, 1, device=dev, requires_grad=True)
    jac = torch.randn(1, B, 3, 64, 64, device=dev, requires_grad=True)
    for p in opt.params:
        p.grad.normal_()
    # ConvMeanPool filter fold + adjoint of the critic's 4 down blocks (one
    # launch each way per critic step, as architecture.prefolded runs it)
    from gan.core.architecture import _ConvMeanPool
    from gan.core.convops import _FoldPool, _FoldPoolAdj
    cmp_w = [m.conv.weight.detach() for m in D.modules() if isinstance(m, _ConvMeanPool)]
    cmp_g = [torch.randn(w.shape[0], w.shape[1], 4, 4, device=dev) for w in cmp_w]
    # conv bias gradients: every biased conv output of one critic forward
    # (real and fake batches: two calls per shape per critic step)
    from gan.core.convops import bias_grad
    from gan.core.snops import Conv2d as _SNConv
    shapes = []
    hooks = [m.register_forward_hook(lambda m, i, o: shapes.append(tuple(o.shape)))
             for m in D.modules()
             if (isinstance(m, _SNConv) and m.bias is not None) or isinstance(m, _ConvMeanPool)]
    with torch.no_grad():
        bank.refresh(update_u=False)
        D(torch.rand(B, 3, 64, 64, device=dev))
    for h in hooks:
        h.remove()
    gys = [torch.randn(sh, device=dev) for sh in shapes for _ in range(2)]

    def one():
        outs = bank.refresh(update_u=True)
        torch.autograd.backward(outs, Gs)
        opt.step()
        m2 = mmd.mmd2_fused(X, Y, 'rbf')
        g, _ = ops.scaled_loss(m2, jac, None, sc=10.0)
        g.backward()
        _FoldPool.apply(*cmp_w)
        _FoldPoolAdj.apply(*cmp_g)
        with torch.no_grad():
            for gy in gys:
                bias_grad(gy)

    for _ in range(20):
        one()
    torch.cuda.synchronize()
    _lib.reset_timing()
    _lib.enable_timing(True)
    for _ in range(args.iters):
        one()
    _lib.enable_timing(False)
    tm = _lib.timing_ms()
    tb = _lib.timing_bytes()
    kn = sum(e.N * e.K for e in bank.entries)
    alg = {'smmd_sn_power_iter': kn * 4 * 2, 'smmd_sn_weight_bwd': kn * 4 * 3,
           'smmd_adam_flat[D]': opt.numel * 4 * 8,
           'smmd_adam_flat_sn[D]': opt.numel * 4 * 8,
           'smmd_mmd2_fwd': 2 * B * 4 * 2 + 32,
           'smmd_scaled_loss_fwd': B * 3 * 64 * 64 * 4,
           'smmd_scaled_loss_bwd': 2 * B * 3 * 64 * 64 * 4,
           'smmd_fold_pool_weights': sum(w.shape[0] * w.shape[1] for w in cmp_w) * 25 * 4}
    alg.update({k: int(v) for k, v in tb.items()})
    res = {}
    for k, (n, ms) in sorted(tm.items()):
        b = alg.get(k)
        res[k] = {'calls': n, 'avg_us': round(ms * 1e3, 2)}
        if b:
            gbs = b / (ms * 1e-3) / 1e9
            res[k].update(bytes=b, GB_s=round(gbs, 1), frac=round(gbs / PEAK, 4))
    print(json.dumps(res, indent=1))
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
