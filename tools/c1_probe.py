"""Per-launch GPU times of the 1x1 shortcut kernels (smmd_conv1x1 /
smmd_conv1x1_wgrad, csrc/smmd_conv1x1.hip) at the SNResNet-64 step's shapes,
for one or more builds of that source: standalone shared libraries of the one
file (tools/hip/c1_*.so, built by tools/build_c1_variants.sh) or the stamped
library.  Raw ctypes launches on torch's current stream, timed with HIP
events over --iters back-to-back launches (no Python work inside the timed
loop besides the ctypes call), so the numbers are the kernels' own (plus the
split-K sum launch where the call makes one).

    python tools/c1_probe.py [--iters 200] [--libs c1_d1,c1_d3rf,...] [--pmc]
(--pmc: a single pass of 20 launches per case, for rocprofv3 --pmc runs)
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
          (64, 1024, 512, 4), (64, 512, 256, 8), (64, 256, 128, 16), (64, 128, 64, 32)]


def load(name):
    if name == 'lib':
        from gan.core import _lib
        L = _lib.lib()
    else:
        L = ctypes.CDLL(os.path.join(ROOT, 'tools', 'hip', name + '.so'))
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.smmd_conv1x1.argtypes = [vp, vp, vp, vp, i, i, i, i, vp, sz, vp]
    L.smmd_conv1x1.restype = i
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
    for n, c, k, h in SHAPES:
        p = h * h
        x = torch.randn(n, c, h, h, device=dev)
        gy = torch.randn(n, k, h, h, device=dev)
        w = torch.randn(k, c, device=dev) * 0.05
        wt = w.t().contiguous()
        b = torch.randn(k, device=dev)
        y = torch.empty(n, k, h, h, device=dev)
        gx = torch.empty(n, c, h, h, device=dev)
        gw = torch.empty(k, c, device=dev)
        keep = [x, gy, w, wt, b, y, gx, gw]

        def gemm(a, xx, bias, yy, r, m):
            nb = L.smmd_conv1x1_workspace_bytes(n, r, m, p)
            ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            keep.append(ws)
            args = (a.data_ptr(), xx.data_ptr(), bias.data_ptr() if bias is not None else None,
                    yy.data_ptr(), n, r, m, p, ws.data_ptr(), nb, st)
            return lambda: L.smmd_conv1x1(*args)

        nb = L.smmd_conv1x1_wgrad_workspace_bytes(n, c, k, p)
        ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
        keep.append(ws)
        wargs = (gy.data_ptr(), x.data_ptr(), gw.data_ptr(), n, c, k, p, ws.data_ptr(), nb, st)
        tag = '%dx%dx%dx%d' % (n, c, k, h)
        out.append((tag, 'fwd', gemm(w, x, b, y, c, k), keep))
        out.append((tag, 'dx', gemm(wt, gy, None, gx, k, c), keep))
        out.append((tag, 'dw', lambda a=wargs: L.smmd_conv1x1_wgrad(*a), keep))
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
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    res = {}
    for name in args.libs.split(','):
        L = load(name)
        for tag, op, fn, _ in cases(L, dev):
            t = run(fn, 20 if args.pmc else args.iters)
            res.setdefault(tag + ' ' + op, {})[name] = round(t, 2)
    names = args.libs.split(',')
    print('%-22s' % 'case' + ''.join('%14s' % nm for nm in names))
    tot = {nm: 0.0 for nm in names}
    for key, r in res.items():
        print('%-22s' % key + ''.join('%14.2f' % r[nm] for nm in names))
        for nm in names:
            tot[nm] += r[nm]
    print('%-22s' % 'sum' + ''.join('%14.2f' % tot[nm] for nm in names))
    print(json.dumps(res))


if __name__ == '__main__':
    main()
