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


PMC_TRAFFIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'profiles', 'r03',
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


MFMA_F32_PEAK_TFS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense


def mmd_path(rows, d):
    """The implementation smmd_mmd2_fwd picks (csrc/smmd_mmd.hip use_gram)."""
    gram = d > 32 or (d >= 16 and rows >= 1024) or (d >= 32 and rows >= 512)
    return 'mfma-gram' if gram else 'row-sweep'


def mmd_sweep(world, rank, dev, group, quick=False):
    """SURVEY 8d MMD microbench: X, Y ~ N(0,1) [N, D] per side (global N,
    numpy default_rng(1234)), rank r owning rows [r N/w, (r+1) N/w) of each, run
    through the product path mmd.mmd2_fused (all-gather mode when w > 1) with
    its backward; HIP-event time per fwd+bwd, max over ranks.  Algorithmic
    bytes: fwd (m+n) D 4 + 16, bwd (m+n) D 4 read + (m+n) D 4 written; pairs
    P = m^2 + mn + n^2 (the reference's three matrices); for D >= 128 the Gram
    flops 4 D P (forward Gram + backward C Z) against the f32 MFMA peak."""
    import numpy as np
    from gan.core import _lib, mmd
    grid = [(32, 1), (64, 1), (256, 1), (512, 1), (2048, 1), (512, 16), (2048, 16),
            (256, 128), (512, 128), (2048, 128), (512, 1024), (2048, 1024)]
    if quick:
        grid = [(64, 1), (512, 128)]
    extra = [('mix_rq', 512, 1), ('mix_rbf', 512, 1), ('mix_rq', 512, 128),
             ('mix_rbf', 512, 128)]
    rows = []
    for kern, N, D in [('rbf', N, D) for N, D in grid] + ([] if quick else extra):
        if N % world:
            continue
        rng = np.random.default_rng(1234)
        X = (rng.standard_normal((N, D)) / np.sqrt(D)).astype(np.float32)
        Y = (rng.standard_normal((N, D)) / np.sqrt(D)).astype(np.float32)
        sl = slice(rank * N // world, (rank + 1) * N // world)
        Xl = torch.tensor(X[sl], device=dev, requires_grad=True)
        Yl = torch.tensor(Y[sl], device=dev, requires_grad=True)

        def once():
            v = mmd.mmd2_fused(Xl, Yl, kern, process_group=group)
            gx, gy = torch.autograd.grad(v, (Xl, Yl))
            return v

        for _ in range(3):
            once()
        iters = 20 if D < 1024 else 8
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        _lib.reset_timing()
        _lib.enable_timing(True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            val = once()
        e1.record()
        torch.cuda.synchronize()
        _lib.enable_timing(False)
        # op_ms: the whole mmd2_fused call + its backward as the training step
        # issues it (host overhead, collectives); kernel_ms: HIP-event time of
        # the library call alone (every launch of smmd_mmd2_fwd)
        t = torch.tensor([e0.elapsed_time(e1) / iters,
                          _lib.timing_ms().get('smmd_mmd2_fwd', (1, 0.0))[1]], device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        op_ms, ms = float(t[0]), float(t[1])
        m = n = N
        P = m * m + m * n + n * n
        b = 3 * (m + n) * D * 4 + 16
        row = {'kernel': kern, 'N': N, 'D': D, 'op_ms': round(op_ms, 5),
               'kernel_ms': round(ms, 5), 'GB_s': round(b / (ms * 1e-3) / 1e9, 2),
               'pair_evals_per_s': round(P / (ms * 1e-3), 1),
               'path': mmd_path(2 * N, D), 'mmd2': float(val.detach())}
        if D >= 128:
            tf = 4.0 * D * P / (ms * 1e-3) / 1e12
            row.update(tflops=round(tf, 2), mfma_frac=round(tf / MFMA_F32_PEAK_TFS, 4))
        rows.append(row)
    return rows


def cpu_components(cfg, threads):
    """SURVEY 8d CPU baseline rows (i) and (ii): the torch-CPU mirror of the TF
    graph for MMD fwd+bwd per N (materialised N x N matrices, D = 1) and the
    SN power iteration of the SNResNet-64 critic (all layers)."""
    import numpy as np
    from gan.core.architecture import SNResNetDiscriminator
    from gan.core.snops import sn_modules
    from oracle.tf_mirror import rbf_mmd2_tf, sn_weight_tf
    torch.set_num_threads(threads)
    out = {'mmd_fwd_bwd': []}
    for N in (64, 256, 512, 2048):
        rng = np.random.default_rng(1234)
        X = torch.tensor(rng.standard_normal((N, 1)), dtype=torch.float32, requires_grad=True)
        Y = torch.tensor(rng.standard_normal((N, 1)), dtype=torch.float32, requires_grad=True)
        rbf_mmd2_tf(X, Y).backward()
        reps, t0 = 0, time.perf_counter()
        while reps < 20 and time.perf_counter() - t0 < 2.0:
            X.grad = Y.grad = None
            rbf_mmd2_tf(X, Y).backward()
            reps += 1
        out['mmd_fwd_bwd'].append({'N': N, 'D': 1, 'kernel': 'rbf',
                                   'ms': round((time.perf_counter() - t0) / reps * 1e3, 3)})
    D = SNResNetDiscriminator(64, 1, False, with_sn=True, with_learnable_sn_scale=True)
    layers = []
    for mod in sn_modules(D):
        W = mod.weight.detach()
        perm = (2, 3, 1, 0) if W.dim() == 4 else (1, 0)
        layers.append((W, torch.randn(1, W.shape[0]), mod.sn_scale.detach(), perm))
    for W, u, sc, perm in layers:
        sn_weight_tf(W, u, sc, perm)
    reps, t0 = 0, time.perf_counter()
    while reps < 10 and time.perf_counter() - t0 < 3.0:
        for W, u, sc, perm in layers:
            sn_weight_tf(W, u, sc, perm)
        reps += 1
    out['sn_power_iter'] = {'architecture': 'snresnet-64 critic', 'layers': len(layers),
                            'weights': sum(W.numel() for W, *_ in layers),
                            'ms': round((time.perf_counter() - t0) / reps * 1e3, 3)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--batch', type=int, default=64,
                    help='images per GPU: 64 is the headline (imagenet_smmd.yml); 256 is '
                         'BASELINE configs[4] (the 256 x 256 pairwise tile per GPU)')
    ap.add_argument('--steps', type=int, default=60)
    ap.add_argument('--warmup', type=int, default=12)
    ap.add_argument('--dp-mode', default='global', choices=['global', 'tower'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--channels-last', type=int, default=0)
    ap.add_argument('--miopen-winograd', type=int, default=1,
                    help='0: disable MIOpen Winograd solvers (immediate mode then picks '
                         'the MFMA implicit-GEMM ones)')
    ap.add_argument('--miopen-find', type=int, default=0,
                    help='1: torch.backends.cudnn.benchmark (MIOpen Find: times every '
                         'applicable solver per conv problem during warmup); the find '
                         'results persist in MIOPEN_USER_DB_PATH when set')
    ap.add_argument('--cpu-seconds', type=float, default=20.0)
    ap.add_argument('--ref-schedule-steps', type=int, default=30,
                    help='steps timed with the reference schedule (both gradient sets '
                         'every step, model.py:514) after the main run; 0: skip')
    ap.add_argument('--mmd-sweep', type=int, default=1,
                    help='1: SURVEY 8d MMD microbench grid; 2: two configs; 0: skip')
    args = ap.parse_args()
    global BATCH
    BATCH = args.batch

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
    # MIOpen solver choice: the committed find db (gan/core/miopen_db.py),
    # installed before the first convolution
    from gan.core import architecture, miopen_db
    miopen_db.install()
    # MIOpen immediate mode: one kernel compile per conv config on a fresh box;
    # benchmark=True would compile every candidate solver (minutes per shape).
    torch.backends.cudnn.benchmark = bool(args.miopen_find)

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
    tm = _lib.timing_ms()            # before the extra runs below reset the records
    tb = _lib.timing_bytes()
    g_loss, d_loss = model.check_finite()
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)

    # the reference-schedule variant (both gradient sets every step)
    ref_sched = None
    if args.ref_schedule_steps > 0:
        model.schedule = 'reference'
        for i in range(6):                        # covers one generator step
            model.train_step(images[i % len(images)])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.ref_schedule_steps):
            model.train_step(images[i % len(images)])
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dtr = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dtr], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dtr = float(t)
        model.schedule = 'lean'
        ref_sched = {'value': round(world * BATCH * args.ref_schedule_steps / dtr, 2),
                     'unit': 'images/s', 'steps': args.ref_schedule_steps, 'warmup': 6,
                     'ms_per_step': round(dtr / args.ref_schedule_steps * 1e3, 3),
                     'note': 'every step also computes the other network\'s gradient set '
                             'and discards it, as each sess.run of the reference does '
                             '(model.py:514); value above is the lean schedule'}
    sweep = None
    if args.mmd_sweep:
        sweep = mmd_sweep(world, rank, dev, dist.group.WORLD if world > 1 else None,
                          quick=args.mmd_sweep == 2)

    # every libsmmd_hip entry point of the timed region: HIP-event time on the
    # compute stream and its algorithmic HBM bytes per call
    m_all = BATCH * world
    sn_kn = sum(e.N * e.K for e in model.sn_D.entries)
    per_img = 3 * 64 * 64
    alg = {
        # sqsum pass reads g; update pass reads g, p, m, v and writes p, m, v
        'smmd_adam_flat[D]': model.d_optim.numel * 4 * 8,
        'smmd_adam_flat[G]': model.g_optim.numel * 4 * 8,
        # the same update with the SN weights' first power-iteration pass folded
        # in (its column-partial writes are < 0.1 % of these bytes)
        'smmd_adam_flat_sn[D]': model.d_optim.numel * 4 * 8,
        'smmd_adam_flat_sn[G]': model.g_optim.numel * 4 * 8,
        # one read of W + one write of W_eff (2 K N 4 B per iteration)
        'smmd_sn_power_iter': sn_kn * 4 * 2,
        # one read of G and W, one write of gW
        'smmd_sn_weight_bwd': sn_kn * 4 * 3,
        # X, Y rows read, unit gradients written, sums
        'smmd_mmd2_fwd': 2 * m_all * 4 + 2 * BATCH * 4 + 8 * 4,
        'smmd_scaled_loss_fwd': BATCH * per_img * 4,
        # ConvMeanPool filter fold / adjoint: 9 floats read + 16 written (or
        # back) per filter, every ConvMeanPool layer of the critic per call
        'smmd_fold_pool_weights': sum(m.conv.weight.shape[0] * m.conv.weight.shape[1]
                                      for m in model.discriminator.modules()
                                      if isinstance(m, architecture._ConvMeanPool)) * 25 * 4,
        'smmd_scaled_loss_bwd': 2 * BATCH * per_img * 4,
    }
    # entry points whose size varies per call: mean algorithmic bytes per call
    # (the conv bias gradient: 4 B per element of gy + 4 B per channel)
    alg.update({k: int(v) for k, v in tb.items()})
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
                               'batch %d/GPU, 5D+1G schedule' % BATCH,
                   'model': 'snresnet', 'global_batch': BATCH * world, 'seq_len': None,
                   'parallelism': 'dp%d' % world, 'dp_mode': args.dp_mode,
                   'memory_format': 'channels_last' if args.channels_last else 'nchw',
                   'miopen_winograd': bool(args.miopen_winograd),
                   'miopen_find': bool(args.miopen_find),
                   'conv_mean_pool': ('folded 4x4 stride-2 conv' if architecture.FOLD_POOL
                                      else 'conv3x3 + mean pool'),
                   'miopen_db': os.environ.get('MIOPEN_USER_DB_PATH')},
        'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': kernels[dom]['GB_s'],
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': kernels[dom]['frac'],
                     'traffic': pmc_traffic(dom), 'avg_ms': kernels[dom]['avg_ms'],
                     'algorithmic_bytes': kernels[dom]['bytes']},
        'mmd_kernel': {'kernel': 'smmd_mmd2_fwd (mmd2_fused_kernel<1,RBF>)',
                       'avg_ms': mk.get('avg_ms'), 'GB_s': mk.get('GB_s'),
                       'pair_evals_per_s': round(pairs / (mk['avg_ms'] * 1e-3), 1) if mk else None,
                       'bound': 'latency (D=1: %s B algorithmic per call)' % mk.get('bytes')},
        'hip_kernels': kernels,
        'schedule_reference': ref_sched,
        'mmd_sweep': sweep,
        'losses': {'g_loss': g_loss, 'd_loss': d_loss},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result['cpu_baseline'] = cpu_baseline(cfg, args.cpu_seconds)
            result['cpu_baseline']['components'] = cpu_components(
                cfg, result['cpu_baseline']['cores'])
        except Exception as e:   # report, never hide the GPU number
            result['cpu_baseline'] = {'error': repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
