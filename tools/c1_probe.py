"""Per-launch GPU times of the 1x1 shortcut kernels (smmd_conv1x1 /
smmd_conv1x1_wgrad, csrc/smmd_conv1x1.hip) at the SNResNet-64 step's shapes,
for one or more builds of that source: standalone shared libraries of the one
file (tools/hip/c1_*.so, built by tools/build_c1_variants.sh) or the stamped
library.  Raw ctypes launches on torch's current stream, timed with HIP
events over --iters back-to-back launches (no Python work inside the timed
loop besides the ctypes call), so the numbers are the kernels' own (plus the
split-K sum launch where the call makes one).

    python tools/c1_probe.py [--iters 200] [--libs c1_d1,c1_d3rf,...] [--pmc] [--check]
(--pmc: a single pass of 20 launches per case, for rocprofv3 --pmc runs;
--check: also compare every case's output bit for bit with the first library's)
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))

import torch  # noqa: E402

# (N, C, K, H): the critic's MeanPoolConv shortcuts (C -> 2C at the pooled
# size) and the generator's up-block shortcuts (2C -> C before the upsample)
SHAPES = [(64, 64, 128, 32), (64, 128, 256, 16), (64, 256, 512, 8), (64, 512, 1024, 4),
          (64, 1024, 512, 4), (64, 512, 256, 8), (64, 256, 128, 16), (64, 128, 64, 32),
          (64, 512, 1024, 2), (64, 128, 256, 6)]     # + pixels dividing 32, and neither way


def load(name):
    if name == 'lib':
        from gan.core import _lib
        L = _lib.lib()
    else:
        L = ctypes.CDLL(os.path.join(ROOT, 'tools', 'hip', name + '.so'))
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.smmd_conv1x1.argtypes = [vp, vp, vp, vp, i, i, i, i, vp, sz, vp]
    L.smmd_conv1x1.restype = i
    L.smmd_conv1x1_t.argtypes = [vp, vp, vp, vp, i, i, i, i, vp, sz, vp]
    L.smmd_conv1x1_t.restype = i
    L.smmd_conv1x1_wgrad_acc.argtypes = [vp, vp, vp, i, i, i, i, vp, sz, vp]
    L.smmd_conv1x1_wgrad_acc.restype = i
    L.smmd_conv1x1_workspace_bytes.argtypes = [i, i, i, i]
    L.smmd_conv1x1_workspace_bytes.restype = sz
    L.smmd_conv1x1_wgrad.argtypes = [vp, vp, vp, i, i, i, i, vp, sz, vp]
    L.smmd_conv1x1_wgrad.restype = i
    L.smmd_conv1x1_wgrad_workspace_bytes.argtypes = [i, i, i, i]
    L.smmd_conv1x1_wgrad_workspace_bytes.restype = sz
    return L


def cases(L, dev):
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    out = []
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    for n, c, k, h in SHAPES:
        p = h * h
        x = torch.randn(n, c, h, h, device=dev, generator=g)
        gy = torch.randn(n, k, h, h, device=dev, generator=g)
        w = torch.randn(k, c, device=dev, generator=g) * 0.05
        wt = w.t().contiguous()
        b = torch.randn(k, device=dev, generator=g)
        y = torch.empty(n, k, h, h, device=dev)
        gx = torch.empty(n, c, h, h, device=dev)
        gxt = torch.empty(n, c, h, h, device=dev)
        gw = torch.empty(k, c, device=dev)
        gwa = torch.randn(k, c, device=dev, generator=g)
        gwa0 = gwa.clone()
        keep = [x, gy, w, wt, b, y, gx, gxt, gw, gwa, gwa0]

        def gemm(fn, a, xx, bias, yy, r, m):
            nb = L.smmd_conv1x1_workspace_bytes(n, r, m, p)
            ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            keep.append(ws)
            args = (a.data_ptr(), xx.data_ptr(), bias.data_ptr() if bias is not None else None,
                    yy.data_ptr(), n, r, m, p, ws.data_ptr(), nb, st)
            return lambda: fn(*args)

        nb = L.smmd_conv1x1_wgrad_workspace_bytes(n, c, k, p)
        ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
        keep.append(ws)
        wargs = (gy.data_ptr(), x.data_ptr(), gw.data_ptr(), n, c, k, p, ws.data_ptr(), nb, st)
        aargs = (gy.data_ptr(), x.data_ptr(), gwa.data_ptr(), n, c, k, p, ws.data_ptr(), nb, st)

        def acc_once(a=aargs, gwa=gwa, gwa0=gwa0):
            gwa.copy_(gwa0)
            return L.smmd_conv1x1_wgrad_acc(*a)
        tag = '%dx%dx%dx%d' % (n, c, k, h)

        def refs(x=x, gy=gy, w=w, b=b, gwa0=gwa0, n=n, c=c, k=k, p=p):
            xd = x.double().reshape(n, c, p)
            gd = gy.double().reshape(n, k, p)
            wd = w.double()
            yr = torch.einsum('kc,ncp->nkp', wd, xd) + b.double().view(1, k, 1)
            gxr = torch.einsum('kc,nkp->ncp', wd, gd)
            gwr = torch.einsum('nkp,ncp->kc', gd, xd)
            return {'fwd': yr, 'dx': gxr, 'dxt': gxr, 'dw': gwr, 'dwacc': gwr + gwa0.double()}
        # (keep: every tensor a launch's raw pointers name stays alive)
        out.append((tag, 'fwd', gemm(L.smmd_conv1x1, w, x, b, y, c, k), y, refs, keep))
        out.append((tag, 'dx', gemm(L.smmd_conv1x1, wt, gy, None, gx, k, c), gx, refs, keep))
        out.append((tag, 'dxt', gemm(L.smmd_conv1x1_t, w, gy, None, gxt, k, c), gxt, refs, keep))
        out.append((tag, 'dw', lambda a=wargs: L.smmd_conv1x1_wgrad(*a), gw, refs, keep))
        out.append((tag, 'dwacc', acc_once, gwa, refs, keep, True))
    return out


def run(fn, iters):
    for _ in range(3):
        assert fn() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=200)
    ap.add_argument('--libs', default='lib')
    ap.add_argument('--pmc', action='store_true')
    ap.add_argument('--check', action='store_true')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    res = {}
    ref = {}
    bad = []
    names = args.libs.split(',')
    for name in names:
        L = load(name)
        for case in cases(L, dev):
            tag, op, fn, outt, refs = case[:5]
            key = tag + ' ' + op
            if args.check:
                assert fn() == 0
                torch.cuda.synchronize()
                r = refs()[op].reshape(outt.shape)
                rel = float((outt.double() - r).abs().max()) / (float(r.abs().max()) + 1e-30)
                print('%s %-22s rel err vs float64 %.3g' % (name, key, rel), flush=True)
                if not rel < 1e-5:
                    bad.append('%s %s: rel err vs float64 %.3g' % (name, key, rel))
                if name == names[0]:
                    ref[key] = outt.clone()
                elif not torch.equal(ref[key], outt):
                    bad.append('%s %s: max |diff| %.3g' % (
                        name, key, (ref[key] - outt).abs().max().item()))
            if len(case) > 6:        # the accumulate form: checked, not timed
                continue
            t = run(fn, 20 if args.pmc else args.iters)
            res.setdefault(key, {})[name] = round(t, 2)
    print('%-22s' % 'case' + ''.join('%14s' % nm for nm in names))
    tot = {nm: 0.0 for nm in names}
    for key, r in res.items():
        print('%-22s' % key + ''.join('%14.2f' % r[nm] for nm in names))
        for nm in names:
            tot[nm] += r[nm]
    print('%-22s' % 'sum' + ''.join('%14.2f' % tot[nm] for nm in names))
    if args.check:
        print('bit-identical to %s: %s' % (names[0], 'all cases' if not bad else 'NO'))
        for b in bad:
            print('  DIFFERS', b)
    print(json.dumps(res))
    if bad:
        sys.exit(1)


if __name__ == '__main__':
    main()
