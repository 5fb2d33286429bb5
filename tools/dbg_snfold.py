"""Debug: fused SN fold vs W_eff + separate fold launch (positions of any
differences, sigma of both banks).  GPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from gan.core import convops, sn
    dev = torch.device('cuda:0')
    rng = np.random.default_rng(5)
    W = rng.standard_normal((128, 64, 3, 3)) * 0.05
    res = {}
    for fused in (True, False):
        sn.SN_FOLD = fused
        torch.manual_seed(0)
        m = torch.nn.Module()
        m.weight = torch.nn.Parameter(torch.tensor(W, dtype=torch.float32, device=dev))
        m.sn_scale = torch.nn.Parameter(torch.tensor([1.3], device=dev))
        m.sn_fold = True
        bank = sn.SpectralNormBank([m])
        out, = bank.refresh(update_u=True)
        weff = None if fused else out.detach().clone()
        if not fused:
            out, = convops.fold_pool_weights([out])
        res[fused] = (out.detach().cpu().numpy(), bank.entries[0].sigma.item(), weff)
    a, b = res[True][0], res[False][0]
    print('sigma fused %.9g separate %.9g' % (res[True][1], res[False][1]))
    d = a != b
    print('mismatch', d.sum(), 'of', d.size)
    pos = d.reshape(-1, 16).sum(0)
    print('per 4x4 position', pos.reshape(4, 4))
    weff = res[False][2].cpu().numpy()
    sig = res[False][1]
    w32 = W.astype(np.float32)
    k = (w32 / np.float32(sig)).astype(np.float32) * np.float32(1.3)
    print('W_eff from numpy f32 equal to device W_eff:', np.array_equal(k.astype(np.float32), weff))
    print('max |k - weff|', np.abs(k - weff).max())


if __name__ == '__main__':
    main()
