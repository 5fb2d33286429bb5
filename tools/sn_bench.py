"""Time the SN refresh of the SNResNet-64 critic bank (14 layers, 10.1 M
weights) per call: the launch set (SMMD_SN_P23=0) against the fused kernel,
plus any SMMD_SN_P23_DBG knobs given.  python tools/sn_bench.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..',
                                'scaled-mmd-gan_amd'))
from gan.core.architecture import SNResNetDiscriminator  # noqa: E402
from gan.core.snops import sn_modules  # noqa: E402
from gan.core import sn  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device('cuda:0')
    D = SNResNetDiscriminator(64, 1, False, with_sn=True, with_learnable_sn_scale=True).to(dev)
    bank = sn.SpectralNormBank(sn_modules(D))
    modes = [('0', ''), ('1', ''), ('1', '1'), ('1', '2'), ('1', '3')]
    if len(sys.argv) > 2:                        # one mode, e.g. 1:2
        modes = [tuple(sys.argv[2].split(':'))]
    for p23, dbg in modes * 2:
        os.environ['SMMD_SN_P23'] = p23
        os.environ['SMMD_SN_P23_DBG'] = dbg
        with torch.no_grad():
            for _ in range(5):
                bank.refresh(update_u=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                bank.refresh(update_u=True)
            e1.record()
            torch.cuda.synchronize()
        print('P23=%s DBG=%-2s %.2f us/call' % (p23, dbg, e0.elapsed_time(e1) * 1e3 / reps),
              flush=True)


if __name__ == '__main__':
    main()
