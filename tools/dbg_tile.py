import os, sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/scaled-mmd-gan_amd')
import numpy as np, torch
from gan.core import _lib, mmd
dev = torch.device('cuda:0')
for N in (256, 512):
    rng = np.random.default_rng(0)
    X = torch.tensor(rng.standard_normal((N, 1)).astype(np.float32), device=dev)
    Y = torch.tensor(rng.standard_normal((N, 1)).astype(np.float32) + 0.3, device=dev)
    L = _lib.lib()
    ws = torch.zeros(L.smmd_mmd2_workspace_bytes(N, N, 1), dtype=torch.uint8, device=dev)
    res = {}
    for tile in ('1', '0', '1'):
        os.environ['SMMD_MMD_TILE'] = tile
        sums = torch.empty(8, device=dev); out = torch.empty(1, device=dev)
        gx = torch.full((N, 1), 777.0, device=dev); gy = torch.full((N, 1), 777.0, device=dev)
        _lib.check(L.smmd_mmd2_fwd(mmd.get_kernel_spec('rbf').desc(), _lib.ptr(X), N, _lib.ptr(Y), N, 1, 0, 0, N, 0, N,
                                   _lib.ptr(sums), _lib.ptr(out), _lib.ptr(gx), _lib.ptr(gy), _lib.ptr(ws), ws.numel(),
                                   _lib.stream_handle(dev)), 'fwd')
        torch.cuda.synchronize()
        hdr = ws[:16384].view(torch.int32)
        print(N, 'tile', tile, 'mmd2', out.item(), 'counters nonzero', int((hdr != 0).sum()), hdr[:4].tolist(), hdr[64:68].tolist())
        res.setdefault(tile, []).append((gx.cpu().numpy().ravel(), gy.cpu().numpy().ravel()))
    a, b = res['1'][0], res['0'][0]
    bad = np.where(np.abs(a[0] - b[0]) > 1e-3 * np.abs(b[0]).max())[0]
    print(N, 'bad X rows', len(bad), bad[:20], 'tiles', sorted(set((bad // 64).tolist())))
    print('  tile', a[0][bad[:5]], 'sweep', b[0][bad[:5]])
    bad = np.where(np.abs(a[1] - b[1]) > 1e-3 * np.abs(b[1]).max())[0]
    print(N, 'bad Y rows', len(bad), bad[:20])
