"""Diagnose the resident SN backward: per-tile <G, W> partials (workspace dotp)
against numpy, and the layer sum each path implies.  GPU only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'scaled-mmd-gan_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def al(x):
    return (x + 255) // 256 * 256


def carve(shapes, TR=32, TC=256):
    off = 256
    out = []
    for N, K in shapes:
        nrt, nct = -(-N // TR), -(-K // TC)
        p = off
        p1 = p; p += al(nrt * K * 4)
        vraw = p; p += al(K * 4)
        q2 = p; p += al(nct * N * 4)
        ucur = p; p += al(N * 4)
        dotp = p; p += al(nrt * nct * 4)
        out.append(dict(p1=p1, vraw=vraw, q2=q2, ucur=ucur, dotp=dotp, nrt=nrt, nct=nct))
        off = p
    return out


def main():
    from gan.core import sn
    dev = torch.device('cuda:0')
    shapes = [(64, 27), (128, 576), (256, 1152), (1, 1024), (1024, 4608), (7, 13), (130, 300)]
    rng = np.random.default_rng(2)
    Ws = [rng.standard_normal(s) * 0.05 for s in shapes]
    Gs = [rng.standard_normal(s) for s in shapes]
    for path in ('1', '0'):
        os.environ['SMMD_SN_RESIDENT'] = path
        mods = []
        for W in Ws:
            m = torch.nn.Module()
            m.weight = torch.nn.Parameter(torch.tensor(W, dtype=torch.float32, device=dev))
            m.sn_scale = torch.nn.Parameter(torch.tensor([1.3], device=dev))
            mods.append(m)
        bank = sn.SpectralNormBank(mods)
        outs = bank.refresh(update_u=True)
        torch.autograd.backward(outs, [torch.tensor(G, dtype=torch.float32, device=dev) for G in Gs])
        torch.cuda.synchronize()
        ws = bank.ws.cpu().numpy()
        print('path', path, 'hdr', ws[:16].view(np.uint32))
        lay = carve(shapes)
        for i, (N, K) in enumerate(shapes):
            W32 = Ws[i].astype(np.float32).astype(np.float64)
            G32 = Gs[i].astype(np.float32).astype(np.float64)
            d_ref = float(np.sum(W32 * G32))
            e = bank.entries[i]
            sigma = e.sigma.item()
            u = e.u.cpu().numpy().astype(np.float64)
            v = e.v.cpu().numpy().astype(np.float64)
            gW = mods[i].weight.grad.cpu().numpy().astype(np.float64)
            r1 = 1.3 * G32 / sigma - gW          # = coef u v^T
            coef = float(u @ r1 @ v) / (float(u @ u) * float(v @ v))
            d_impl = coef * sigma * sigma / 1.3
            L = lay[i]
            nt = L['nrt'] * L['nct']
            dotp = ws[L['dotp']:L['dotp'] + nt * 4].view(np.float32).astype(np.float64)
            tiles = np.zeros(nt)
            for rt in range(L['nrt']):
                for ct in range(L['nct']):
                    tiles[rt * L['nct'] + ct] = np.sum(W32[rt * 32:(rt + 1) * 32, ct * 256:(ct + 1) * 256]
                                                      * G32[rt * 32:(rt + 1) * 32, ct * 256:(ct + 1) * 256])
            bad = np.nonzero(np.abs(dotp - tiles) > 1e-3 * (1 + np.abs(tiles)))[0]
            print('layer %d %s d_ref %.4f d_impl %.4f sum(dotp) %.4f badtiles %d %s' % (
                i, (N, K), d_ref, d_impl, dotp.sum(), len(bad), bad[:12].tolist()))
            if len(bad):
                print('   got', dotp[bad[:6]], 'want', tiles[bad[:6]])


if __name__ == '__main__':
    main()
