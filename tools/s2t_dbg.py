import ctypes, os, sys, torch
sys.path.insert(0, 'scaled-mmd-gan_amd')
from gan.core import _lib
def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib._SIGS.items():
        if hasattr(L, name):
            getattr(L, name).restype = res; getattr(L, name).argtypes = args
    return L
dev = torch.device('cuda:0'); st = _lib.stream_handle(dev)
N, K, C, Hg, Wg = 2, 128, 64, 8, 8
torch.manual_seed(0)
gy = torch.randn(N, K, Hg, Wg, device=dev); w = torch.randn(K, C, 4, 4, device=dev)
out = {}
for name in ('tools/hip/v_base.so', 'scaled-mmd-gan_amd/lib/libsmmd_hip.so'):
    L = load(name)
    u = torch.empty(L.smmd_wino4x4s2_filter_bytes(K, C) // 4, device=dev)
    assert L.smmd_wino4x4s2t_filter(_lib.ptr(w), K, C, _lib.ptr(u), u.numel() * 4, st) == 0
    dx = torch.full((N, C, 2 * Hg, 2 * Wg), 7.0, device=dev)
    nb = L.smmd_wino4x4s2t_workspace_bytes(N, K, C, Hg, Wg)
    ws = torch.empty(max(nb // 4, 4), device=dev)
    print(name, 'ws', nb)
    assert L.smmd_wino4x4s2t_conv(_lib.ptr(gy), _lib.ptr(u), None, _lib.ptr(dx), N, K, C, Hg, Wg, _lib.ptr(ws), nb, st) == 0
    torch.cuda.synchronize(); out[name] = dx.cpu()
a, b = out.values()
d = (a - b).abs() > 1e-3
print('bad', d.sum().item(), 'of', d.numel())
idx = d.nonzero()
for dim, nm in enumerate('ncyx'):
    print(nm, torch.unique(idx[:, dim]).tolist()[:40])
print(b[0, 0, :4, :8]); print(a[0, 0, :4, :8])
print('odd new', b[0, 1, :2, :8]); print('odd base', a[0, 1, :2, :8]); print('even base c0', a[0, 0, :2, :8])
print('c2 base', a[0, 2, :2, :8])
