"""Training-step benchmark: 64x64 ImageNet SMMD (SNResNet G/D), batch 64 per GPU.

    python bench.py --gpus N --steps K --warmup W
    (N > 1 is launched by torch.distributed.run, one rank per GPU over RCCL)

A step is one optimizer update of the reference schedule (5 critic updates,
then 1 generator update; gan/core/model.py:470-478) on a synthetic batch of
images resident in HBM (U[0,1], seed 0; z ~ U(-1,1)); random-init weights.
value = images/s of the whole job = N * batch * K / (max over ranks of the
timed region).  Multi-GPU uses the all-gather ('global') MMD mode: every rank
sees the full (N*64) x (N*64) pairwise kernel (weak scaling).

Extra fields: roofline of the dominant HIP launch set (the clip+Adam update of
the critic, HBM-bound) timed with HIP events on the compute stream, the
fused-MMD kernel's rate, and a CPU baseline (the oracle's op-by-op mirror of
the TF graph, timed on a bounded sample on this host).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'scaled-mmd-gan_amd')
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
BATCH = 64


PMC_TRAFFIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'r01',
                           'pmc_traffic.json')


def pmc_traffic(entry):
    """HBM bytes per call of a library entry point from the committed rocprofv3
    PMC passes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, tools/pmc_traffic.py,
    same kernels and sizes via tools/hipbench.py), or None when not measured."""
    try:
        with open(PMC_TRAFFIC) as f:
            rec = json.load(f).get(entry.split('[')[0])
        return rec['traffic_bytes'] if rec else None
    except (OSError, ValueError, KeyError):
        return None


def imagenet_config():
    """configs/imagenet_smmd.yml over the gan/main.py defaults."""
    from gan.main import default_flags
    c = default_flags()
    c.update(dict(max_iteration=150000, learning_rate=2e-4, beta1=0.5, beta2=0.9, decay_rate=.8,
                  dsteps=5, gsteps=1, start_dsteps=10, batch_size=BATCH, output_size=64,
                  c_dim=3, z_dim=128, df_dim=64, dof_dim=1, gf_dim=64, architecture='snresnet',
                  kernel='rbf', model='smmd', batch_norm=True, with_sn=True,
                  with_learnable_sn_scale=True, with_scaling=True, dataset='imagenet'))
    return argparse.Namespace(**c)


def cpu_baseline(cfg, seconds_budget=20.0):
    """Oracle mirror of the TF graph on the host CPU (bounded sample)."""
    from gan.core.architecture import get_networks
    from gan.core.snops import sn_modules
    from oracle.tf_mirror import TFMirrorStep
    threads = min(len(os.sched_getaffinity(0)), 16)
    torch.set_num_threads(threads)
    torch.manual_seed(2)
    G_cls, D_cls = get_networks(cfg.architecture)
    G = G_cls(cfg.gf_dim, 3, cfg.output_size, cfg.batch_norm, z_dim=cfg.z_dim)
    D = D_cls(cfg.df_dim, cfg.dof_dim, False, with_sn=True, with_learnable_sn_scale=True,
              input_size=cfg.output_size)
    step = TFMirrorStep(G, D, sn_modules(D), lr=cfg.learning_rate, sc=cfg.scaling_coeff)
    g = torch.Generator().manual_seed(0)
    imgs = torch.rand(BATCH, 3, cfg.output_size, cfg.output_size, generator=g)
    step.step(imgs)                                    # warm-up
    t0 = time.perf_counter()
    n = 0
    while True:
        step.step(imgs)
        n += 1
        if time.perf_counter() - t0 > seconds_budget or n >= 3:
            break
    dt = (time.perf_counter() - t0) / n
    return {'value': BATCH / dt, 'unit': 'images/s', 'cores': threads, 'kind': 'port',
            'sample': '%d critic steps (SNResNet-64 SMMD, batch %d) of the oracle torch-CPU '
                      'mirror of the TF graph (oracle/tf_mirror.py), %.2f s/step' %
                      (n, BATCH, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=60)
    ap.add_argument('--warmup', type=int, default=12)
    ap.add_argument('--dp-mode', default='global', choices=['global', 'tower'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--channels-last', type=int, default=0)
    ap.add_argument('--miopen-winograd', type=int, default=1,
                    help='0: disable MIOpen Winograd solvers (immediate mode then picks '
                         'the MFMA implicit-GEMM ones)')
    ap.add_argument('--cpu-seconds', type=float, default=20.0)
    args = ap.parse_args()

    if not args.miopen_winograd:      # read by MIOpen at its first solver query
        for k in ('MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F2X3', 'MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F3X2',
                  'MIOPEN_DEBUG_AMD_WINOGRAD_3X3', 'MIOPEN_DEBUG_AMD_WINOGRAD_RXS',
                  'MIOPEN_DEBUG_AMD_FUSED_WINOGRAD'):
            os.environ[k] = '0'
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # test hook: SMMD_DIST_BACKEND=gloo + SMMD_SAME_DEVICE=1 rehearses the N>1
    # path with every rank on one GPU (RCCL needs one GPU per rank)
    backend = os.environ.get('SMMD_DIST_BACKEND', 'nccl')
    if os.environ.get('SMMD_SAME_DEVICE') == '1':
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)
    # MIOpen immediate mode: one kernel compile per conv config on a fresh box;
    # benchmark=True would compile every candidate solver (minutes per shape).
    torch.backends.cudnn.benchmark = False

    from gan.core.smmd import SMMD
    cfg = imagenet_config()
    torch.manual_seed(2 + rank)
    model = SMMD(cfg, device=dev, process_group=dist.group.WORLD if world > 1 else None,
                 dp_mode=args.dp_mode, channels_last=bool(args.channels_last))
    gen = torch.Generator(device=dev).manual_seed(0 + rank)
    images = [torch.rand(BATCH, 3, 64, 64, device=dev, generator=gen) for _ in range(4)]
    model.step = 21          # steady-state 5D+1G schedule (model.py:474-475)

    from gan.core import _lib

    tw = time.perf_counter()
    for i in range(args.warmup):
        model.train_step(images[i % len(images)])
        if rank == 0:
            torch.cuda.synchronize()
            print('[bench] warmup step %d/%d done at %.1f s' % (i + 1, args.warmup,
                  time.perf_counter() - tw), file=sys.stderr, flush=True)
    model.check_finite()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    _lib.reset_timing()
    _lib.enable_timing(True)
    t0 = time.perf_counter()
    for i in range(args.steps):
        model.train_step(images[i % len(images)])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    _lib.enable_timing(False)
    g_loss, d_loss = model.check_finite()
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)

    # every libsmmd_hip entry point of the timed region: HIP-event time on the
    # compute stream and its algorithmic HBM bytes per call
    tm = _lib.timing_ms()
    m_all = BATCH * world
    sn_kn = sum(e.N * e.K for e in model.sn_D.entries)
    per_img = 3 * 64 * 64
    alg = {
        # sqsum pass reads g; update pass reads g, p, m, v and writes p, m, v
        'smmd_adam_flat[D]': model.d_optim.numel * 4 * 8,
        'smmd_adam_flat[G]': model.g_optim.numel * 4 * 8,
        # one read of W + one write of W_eff (2 K N 4 B per iteration)
        'smmd_sn_power_iter': sn_kn * 4 * 2,
        # one read of G and W, one write of gW
        'smmd_sn_weight_bwd': sn_kn * 4 * 3,
        # X, Y rows read, unit gradients written, sums
        'smmd_mmd2_fwd': 2 * m_all * 4 + 2 * BATCH * 4 + 8 * 4,
        'smmd_scaled_loss_fwd': BATCH * per_img * 4,
        'smmd_scaled_loss_bwd': 2 * BATCH * per_img * 4,
    }
    kernels = {}
    for name, (calls, ms) in tm.items():
        b = alg.get(name)
        row = {'calls': calls, 'avg_ms': round(ms, 5), 'ms_per_step': round(ms * calls /
                                                                           args.steps, 5)}
        if b:
            row.update(bytes=b, GB_s=round(b / (ms * 1e-3) / 1e9, 1),
                       frac=round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
        kernels[name] = row
    dom = max((k for k in kernels if 'GB_s' in kernels[k] and k != 'smmd_mmd2_fwd'),
              key=lambda k: kernels[k]['ms_per_step'])
    mk = kernels.get('smmd_mmd2_fwd', {})
    pairs = (2 * m_all) * (2 * m_all)                     # rows x columns swept per critic step

    result = {
        'metric': 'images/sec/step (64x64 SMMD, batch 64) + MMD-kernel GB/s at 1/2/4/8 GPU',
        'value': round(world * BATCH * args.steps / dt, 2),
        'unit': 'images/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': round(dt / args.steps * 1e3, 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'fp32',
        'data': 'synthetic (U[0,1] images in HBM, z~U(-1,1), random-init weights)',
        'config': {'workload': 'imagenet_smmd 64x64 SNResNet G/D, rbf kernel, scaling, SN, '
                               'batch 64/GPU, 5D+1G schedule',
                   'model': 'snresnet', 'global_batch': BATCH * world, 'seq_len': None,
                   'parallelism': 'dp%d' % world, 'dp_mode': args.dp_mode,
                   'memory_format': 'channels_last' if args.channels_last else 'nchw',
                   'miopen_winograd': bool(args.miopen_winograd)},
        'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': kernels[dom]['GB_s'],
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': kernels[dom]['frac'],
                     'traffic': pmc_traffic(dom), 'avg_ms': kernels[dom]['avg_ms'],
                     'algorithmic_bytes': kernels[dom]['bytes']},
        'mmd_kernel': {'kernel': 'smmd_mmd2_fwd (mmd2_fused_kernel<1,RBF>)',
                       'avg_ms': mk.get('avg_ms'), 'GB_s': mk.get('GB_s'),
                       'pair_evals_per_s': round(pairs / (mk['avg_ms'] * 1e-3), 1) if mk else None,
                       'bound': 'latency (D=1: %s B algorithmic per call)' % mk.get('bytes')},
        'hip_kernels': kernels,
        'losses': {'g_loss': g_loss, 'd_loss': d_loss},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result['cpu_baseline'] = cpu_baseline(cfg, args.cpu_seconds)
        except Exception as e:   # report, never hide the GPU number
            result['cpu_baseline'] = {'error': repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
