"""Phase timeline of the resident SN power iteration on the SNResNet-64 critic
(block 0 and the last block; s_memrealtime stamps in the workspace header) and
HIP-event time per call for num_iters 1..3 and both launch modes.  GPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = ['start', 'A done', 'bar1', 'A2 done', 'bar2', 'B done', 'bar3', 'R done', 'bar4', 'C done']


def main():
    from gan.core.architecture import SNResNetDiscriminator
    from gan.core.sn import SpectralNormBank
    from gan.core.snops import sn_modules
    dev = torch.device('cuda:0')
    D = SNResNetDiscriminator(64, 1, False, with_sn=True, with_learnable_sn_scale=True).to(dev)
    for coop in ('1', '0'):
        os.environ['SMMD_SN_COOP'] = coop
        for iters in (1, 2, 3):
            bank = SpectralNormBank(sn_modules(D), num_iters=iters)
            for _ in range(10):
                bank.refresh(update_u=False)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50
            e0.record()
            for _ in range(n):
                with torch.no_grad():
                    bank.refresh(update_u=False)
            e1.record()
            torch.cuda.synchronize()
            hdr = bank.ws[:256].cpu().numpy().view(np.uint64)
            b0 = hdr[2:12].astype(np.int64)
            bl = hdr[16:26].astype(np.int64)
            print('coop=%s iters=%d  %.1f us/call (incl. autograd wrapper)' % (
                coop, iters, e0.elapsed_time(e1) * 1e3 / n))
            if iters == 1:
                for name, k in zip(NAMES, range(10)):
                    print('   %-8s blk0 %+8.2f us   last %+8.2f us' % (
                        name, (b0[k] - b0[0]) / 100.0, (bl[k] - b0[0]) / 100.0))


if __name__ == '__main__':
    main()
