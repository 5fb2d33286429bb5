"""Time first/second calls of conv fwd+bwd (MIOpen) vs unfold+GEMM on a fresh box."""
import os, sys, time
import torch
import torch.nn.functional as F
mode = sys.argv[1] if len(sys.argv) > 1 else 'miopen'
torch.backends.cudnn.benchmark = (mode == 'bench')
if mode == 'nocudnn':
    torch.backends.cudnn.enabled = False
dev = torch.device('cuda:0')
shapes = [(64, 3, 64, 64, 64, 3), (64, 64, 64, 64, 64, 3), (64, 64, 32, 32, 128, 3),
          (64, 128, 32, 32, 128, 3), (64, 512, 8, 8, 1024, 3), (64, 64, 32, 32, 128, 1)]
t00 = time.time()
for (b, ci, h, w, co, k) in shapes:
    x = torch.randn(b, ci, h, w, device=dev, requires_grad=True)
    wt = torch.randn(co, ci, k, k, device=dev, requires_grad=True)
    for it in range(3):
        torch.cuda.synchronize(); t0 = time.time()
        y = F.conv2d(x, wt, padding=k // 2)
        g, = torch.autograd.grad(y.sum(), x, create_graph=True)
        (g * g).sum().backward()
        torch.cuda.synchronize()
        print('%s shape=%s it=%d %.3f s (elapsed %.1f)' % (mode, (b, ci, h, w, co, k), it, time.time() - t0, time.time() - t00), flush=True)
