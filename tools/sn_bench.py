"""SN launch sets of the SNResNet-64 critic at bench.py's state, timed alone.

    python tools/sn_bench.py [--iters 200] [--json out.json]
    SMMD_HIP_LIB=other.so python tools/sn_bench.py   (an unstamped build, A/B)

One critic update's SN work as MMD_GAN runs it (model.py: the Winograd-fed
layers lazy, the G-direct backward, the SN-fused update writing the next
refresh's first pass): refresh -> smmd_sn_grad_stats -> smmd_adam_flat_sn2,
plus a refresh whose first pass is not ready (the generator step's, and the
critic step after it).  HIP events on the compute stream around each library
call (_lib.timed); rocprofv3 --kernel-trace --stats of the same command gives
the per-kernel split.
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
    args = ap.parse_args()
    from gan.core import _lib
    from gan.core.architecture import SNResNetDiscriminator
    from gan.core.model import _winograd_fed
    from gan.core.optim import FlatAdam
    from gan.core.sn import SpectralNormBank
    from gan.core.snops import sn_modules
    dev = torch.device('cuda:0')
    torch.manual_seed(0)
    D = SNResNetDiscriminator(64, 1, False, with_sn=True, with_learnable_sn_scale=True,
                              input_size=64).to(dev)
    bank = SpectralNormBank(sn_modules(D))
    bank.set_lazy(_winograd_fed(bank))
    opt = FlatAdam([p for p in D.parameters() if p.requires_grad], 2e-4, name='D')
    assert opt.attach_sn(bank)
    with torch.no_grad():
        Gs = [torch.randn_like(o) * 1e-3 for o in bank.refresh(update_u=False)]

    def update(cold):
        if cold:
            bank.invalidate()
        opt.zero_grad()
        opt.flat_grad.normal_(0, 1e-3)
        bank.arm_gdirect(True)
        outs = bank.refresh(update_u=True)
        torch.autograd.backward(outs, Gs)
        bank.arm_gdirect(False)
        opt.step()

    for i in range(20):
        update(i % 6 == 5)
    torch.cuda.synchronize()
    res = {'smmd_source_hash': _lib.lib().smmd_source_hash().decode(),
           'lib': os.environ.get('SMMD_HIP_LIB', 'stamped'),
           'lazy_layers': sorted(bank.lazy)}
    kn = sum(e.N * e.K for e in bank.entries)
    sn_out = sum(e.N * e.K * 16 // 9 if e.fold else e.N * e.K for e in bank.entries)
    written = sum(e.N * e.K * 16 // 9 if e.fold else e.N * e.K
                  for i, e in enumerate(bank.entries) if i not in bank.lazy)
    alg = {'refresh': (kn + written) * 4, 'grad_stats': (sn_out + kn) * 4}
    for tag, cold in (('ready', False), ('cold', True)):
        _lib.reset_timing()
        _lib.enable_timing(True)
        for i in range(args.iters):
            update(cold)
        _lib.enable_timing(False)
        tm = _lib.timing_ms()
        for k, (n, ms) in sorted(tm.items()):
            key = {'smmd_sn_power_iter': 'refresh', 'smmd_sn_grad_stats': 'grad_stats'}.get(k)
            row = {'calls': n, 'avg_us': round(ms * 1e3, 2)}
            if key:
                b = alg[key]
                gbs = b / (ms * 1e-3) / 1e9
                row.update(bytes=b, GB_s=round(gbs, 1), frac=round(gbs / PEAK, 4))
            res['%s/%s' % (tag, k)] = row
    print(json.dumps(res))
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(res, f, indent=1)


if __name__ == '__main__':
    main()
