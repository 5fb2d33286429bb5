"""Run a few SMMD steps with MIOpen command logging to list the conv problems."""
import os, sys, time
os.environ.setdefault('MIOPEN_ENABLE_LOGGING_CMD', '1')
os.environ.setdefault('MIOPEN_LOG_LEVEL', '6')
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'scaled-mmd-gan_amd'))
import torch
import bench
from gan.core.smmd import SMMD
dev = torch.device('cuda:0')
cfg = bench.imagenet_config()
model = SMMD(cfg, device=dev)
imgs = torch.rand(64, 3, 64, 64, device=dev)
model.step = 21
for i in range(7):
    model.train_step(imgs)
    torch.cuda.synchronize()
    print('STEP_DONE', i, file=sys.stderr, flush=True)
# per-step timing of D and G steps with the profiler-free path
for kind in ('d', 'g'):
    fn = model.d_step if kind == 'd' else model.g_step
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(5):
        fn(imgs)
    torch.cuda.synchronize()
    print('%s_step ms %.2f' % (kind, (time.perf_counter() - t) / 5 * 1e3), file=sys.stderr, flush=True)
