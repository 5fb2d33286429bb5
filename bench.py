"""Training-step benchmark: 64x64 ImageNet SMMD (SNResNet G/D), batch 64 per GPU.

    python bench.py --gpus N --steps K --warmup W
    (N > 1: one rank per GPU over RCCL.  Started without a launcher, the
    process starts `torch.distributed.run --nproc-per-node N bench.py ...` as
    a child before touching the GPU and exits with its code; started by a
    launcher, --gpus must equal WORLD_SIZE)

A step is one optimizer update of the reference schedule (5 critic updates,
then 1 generator update; gan/core/model.py:470-478) on a synthetic batch of
images resident in HBM (U[0,1], seed 0; z ~ U(-1,1)); random-init weights.
value = images/s of the whole job = N * batch * K / (max over ranks of the
timed region).  Multi-GPU uses the all-gather ('global') MMD mode: every rank
sees the full (N*64) x (N*64) pairwise kernel (weak scaling).

Order of the run:
  1. prime (untimed): one critic and one generator update in each schedule
     (lean and reference), so every distinct autograd graph -- and every
     MIOpen kernel it needs -- is built before anything is timed;
  2. W warmup steps, then the schedule is re-aligned to the start of a
     5D + 1G cycle;
  3. EXACTLY K timed steps (no events, no per-call instrumentation inside);
     the line reports how many were critic / generator updates;
  4. the reference schedule (both gradient sets every step, model.py:514);
  5. a separate instrumented pass over whole cycles: HIP-event time of every
     libsmmd_hip entry point and of each D / G step (the `roofline`,
     `hip_kernels` and `roofline_hot_path` blocks come from here);
  6. the MMD microbench and the CPU baseline (rank 0, N = 1).
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
FP32_PEAK_TFS = 157.3          # MI355X_MICROARCH.md: FP32 vector = f32 MFMA peak (dense)
MFMA_F32_PEAK_TFS = 157.3      # v_mfma_f32_32x32x2_f32 dense
# FP32 VALU lane-operations per second: 157.3 TFLOP/s counts an FMA as two
# flops, so one lane-op (add, mul, fma, cmp, ...) issues at half that rate
VALU_LANE_OPS = FP32_PEAK_TFS / 2 * 1e12
TRANS_SLOTS = 4                # v_exp_f32 / v_log_f32: quarter rate (MI355X_MICROARCH.md)
BATCH = 64
_JSON_OUT = sys.stdout           # the result line's stream (main: the real fd 1)

# committed counter evidence of this workload, each file stamped with the
# smmd_source_hash of the library build it was measured on (tools/stamp.py);
# embedded only when that stamp equals the running library's
PMC_TRAFFIC = os.path.join(ROOT, 'profiles', 'r15', 'pmc_traffic.json')
# executed FLOPs per kernel class over whole 5D+1G cycles of this workload
# (tools/gpu_step_pmc.sh -> tools/step_flops_pmc.py: rocprofv3 SQ_INSTS_VALU_*
# and SQ_INSTS_VALU_MFMA_MOPS_F32 counters + a kernel trace)
STEP_PMC = os.path.join(ROOT, 'profiles', 'r15', 'step_flops_pmc.json')


def load_stamped(path, stamp):
    """A committed profile file, only when it was measured with the library
    build running now: (data, None), else (None, reason).  A file without a
    stamp, or with another build's, is stale evidence and is not embedded."""
    rel = os.path.relpath(path, ROOT)
    try:
        with open(path) as f:
            d = json.load(f)
    except OSError:
        return None, 'no %s' % rel
    except ValueError:
        return None, '%s is not JSON' % rel
    got = d.get('smmd_source_hash') if isinstance(d, dict) else None
    if not got:
        return None, '%s carries no smmd_source_hash stamp' % rel
    if got != stamp:
        return None, ('%s was measured on library %s, the running library is %s'
                      % (rel, got, stamp))
    return d, None


def step_counters(ms_step, stamp):
    """The counter-based step roofline: executed TFLOP per step
    from the committed PMC file (when its stamp is the running library's), its
    rate over the GPU-busy time it was measured with and over this run's step
    time, and per kernel class (Winograd, implicit-GEMM fwd / bwd-data / wrw,
    transposes, elementwise, the library) the time share, executed TFLOP/s and
    fraction of the fp32 peak."""
    d, why = load_stamped(STEP_PMC, stamp)
    if d is None:
        return {'source': None, 'null_reason': why}
    tf_step = d['executed_tflop_per_step']
    out = {'source': os.path.relpath(STEP_PMC, ROOT),
           'smmd_source_hash': d['smmd_source_hash'],
           'executed_tflop_per_step': tf_step,
           'executed_tflops_over_gpu_busy': d['executed_tflops_over_busy'],
           'frac_of_fp32_peak_over_gpu_busy': d['frac_of_fp32_peak_over_busy'],
           'gpu_busy_ms_per_step_measured': d['gpu_busy_ms_per_step'],
           'executed_tflops_this_run': round(tf_step / (ms_step * 1e-3), 2),
           'frac_of_fp32_peak_this_run': round(tf_step / (ms_step * 1e-3) / FP32_PEAK_TFS, 4),
           'classes': {k: {q: v.get(q) for q in ('ms_per_step', 'time_frac',
                                                   'executed_gflop_per_step', 'tflops',
                                                   'frac_of_fp32_peak')}
                       for k, v in d['classes'].items()}}
    return out


# the hot-path rows a1-a9 and the library entry points that
# implement them (the roofline kernel is chosen among these)
HOT_PATH = ('smmd_mmd2_fwd', 'smmd_scaled_loss_fwd', 'smmd_scaled_loss_bwd',
            'smmd_smmd_loss_fwd', 'smmd_smmd_loss_bwd', 'smmd_sn_grad_stats',
            'smmd_sn_power_iter', 'smmd_sn_weight_bwd', 'smmd_adam_flat[D]',
            'smmd_adam_flat[G]', 'smmd_adam_flat_sn[D]', 'smmd_adam_flat_sn[G]')


def pmc_traffic(entry, stamp):
    """HBM bytes per call of a library entry point from the committed rocprofv3
    PMC passes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, tools/pmc_traffic.py
    over tools/step_cycle.py), measured on the running library build.
    Returns (bytes, source file, None) or (None, None, reason)."""
    d, why = load_stamped(PMC_TRAFFIC, stamp)
    if d is None:
        return None, None, why
    rec = d.get(entry.split('[')[0])
    if not rec:
        return None, None, 'no %s group in %s' % (entry, os.path.relpath(PMC_TRAFFIC, ROOT))
    return rec['traffic_bytes'], os.path.relpath(PMC_TRAFFIC, ROOT), None


def imagenet_config(batch=BATCH):
    """configs/imagenet_smmd.yml over the gan/main.py defaults."""
    from gan.main import make_flags
    f = make_flags(argv=['-config_file', os.path.join(PKG, 'configs', 'imagenet_smmd.yml'),
                         '-dataset', 'imagenet'])
    f.batch_size = batch
    return f


def celeba64_config(batch):
    """configs/celebA_smmd.yml (g-resnet5: ResNet G + DCGAN5 critic, SN, no BN)
    at 64 x 64, BASELINE configs[2] (the yml's own output_size is 160)."""
    from gan.main import make_flags
    f = make_flags(argv=['-config_file', os.path.join(PKG, 'configs', 'celebA_smmd.yml')])
    f.batch_size = batch
    f.output_size = 64
    return f


CONFIGS = {
    'imagenet': (lambda b: imagenet_config(b),
                 'imagenet_smmd 64x64 SNResNet G/D, rbf kernel, scaling, SN'),
    'cifar10': (lambda b: cifar_config(b),
                'cifar10_smmd 32x32 SNGAN G/D, rbf kernel, scaling, SN (BASELINE configs[1])'),
    'celebA64': (lambda b: celeba64_config(b),
                 'celebA_smmd g-resnet5 (ResNet G, DCGAN5 critic) at 64x64, rbf kernel, scaling, '
                 'SN (BASELINE configs[2])'),
}


def cifar_config(batch):
    """configs/cifar10_smmd.yml (BASELINE configs[0]: batch 32, CPU)."""
    from gan.main import make_flags
    f = make_flags(argv=['-config_file', os.path.join(PKG, 'configs', 'cifar10_smmd.yml')])
    f.batch_size = batch
    return f


def _pct(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def _mirror_trainer(cfg, batch, seed=2):
    from gan.core.architecture import get_networks
    from oracle.tf_mirror import TFMirrorTrainer
    torch.manual_seed(seed)
    G_cls, D_cls = get_networks(cfg.architecture)
    G = G_cls(cfg.gf_dim, 3, cfg.output_size, cfg.batch_norm, z_dim=cfg.z_dim)
    dbn = bool(cfg.batch_norm) and cfg.gradient_penalty <= 0
    D = D_cls(cfg.df_dim, cfg.dof_dim, dbn, with_sn=cfg.with_sn,
              with_learnable_sn_scale=cfg.with_learnable_sn_scale, input_size=cfg.output_size)
    tr = TFMirrorTrainer(cfg, G, D)     # the mirror's own nets (oracle/ref_nets.py), these weights
    tr.step_no = 21              # steady-state 5 D + 1 G (model.py:474-475)
    g = torch.Generator().manual_seed(0)
    imgs = torch.rand(batch, 3, cfg.output_size, cfg.output_size, generator=g)
    return tr, imgs


def _time_steps(tr, imgs, steps, warm=3):
    """Per-step wall times of ``steps`` reference-loop steps (>= 20
    after 3 warm-ups), started at a 5 D + 1 G cycle boundary."""
    for _ in range(warm):
        tr.train_step(imgs)                   # allocator, threads, first-touch
    tr.d_counter = tr.g_counter = 0           # cycle start
    times, kinds = [], []
    for i in range(steps):
        t0 = time.perf_counter()
        kinds.append(tr.train_step(imgs))
        times.append(time.perf_counter() - t0)
        print('[bench] cpu baseline step %d/%d: %.2f s' % (i + 1, steps, times[-1]),
              file=sys.stderr, flush=True)
    return times, kinds


def _stats(times):
    return {'median': round(_pct(times, .5), 4), 'p10': round(_pct(times, .1), 4),
            'p90': round(_pct(times, .9), 4), 'mean': round(sum(times) / len(times), 4)}


def cpu_threads():
    """Threads for the CPU baseline: the process's CPU affinity, capped at the
    GPU box's CPU share for one GPU (the harness sets OMP_NUM_THREADS to that
    share, 16, and asks worker pools to stay within it; the box's affinity
    mask lists the whole host, whose other CPUs belong to other jobs)."""
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get('OMP_NUM_THREADS', affinity) or affinity)
    return affinity, max(1, min(affinity, share))


def cpu_thread_scan(threads, steps=3):
    """The mirror's ImageNet step at half the thread count beside the
    headline's: whether more threads still pay.  The full
    affinity (256 host CPUs on the GPU box) is outside the job's CPU share and
    is not timed.  Returns {threads: median step s}."""
    out = {}
    for n in sorted({max(1, threads // 2), threads}):
        torch.set_num_threads(n)
        tr, imgs = _mirror_trainer(imagenet_config(BATCH), BATCH)
        times, _ = _time_steps(tr, imgs, steps, warm=1)
        out[n] = round(_pct(times, .5), 4)
    torch.set_num_threads(threads)
    return out


def cpu_baseline(steps=24, cifar_steps=24):
    """The oracle's CPU mirror of the TF graph (oracle/tf_mirror.py), the
    reference's training loop: both gradient sets every step, 5 D + 1 G.
    Headline: the bench's own workload (ImageNet SNResNet-64, batch 64),
    ``steps`` timed steps (4 whole cycles) after 3 warm-ups; beside it BASELINE
    configs[0] (CIFAR-10 SNGAN 32x32, batch 32, the reference's CPU case)."""
    affinity, threads = cpu_threads()
    torch.set_num_threads(threads)
    out = {'unit': 'images/s', 'cores': threads, 'cores_meaning': 'host threads used',
           'kind': 'port', 'host_cpus': os.cpu_count(), 'affinity_cpus': affinity,
           'threads_used': threads, 'omp_num_threads_env': os.environ.get('OMP_NUM_THREADS')}
    tr, imgs = _mirror_trainer(imagenet_config(BATCH), BATCH)
    times, kinds = _time_steps(tr, imgs, steps)
    mean = sum(times) / len(times)
    out.update(value=round(BATCH / mean, 3),
               sample='%d steps (%s) after 3 warm-ups of the reference loop on the torch-CPU '
                      'mirror of the TF graph (oracle/tf_mirror.py TFMirrorTrainer; both gradient '
                      'sets per step as model.py:514), ImageNet SNResNet-64 SMMD, batch %d; '
                      'value = batch / mean step time' % (len(times), ''.join(kinds), BATCH),
               steps=len(times), warmup=3, step_s=_stats(times))
    tr, imgs = _mirror_trainer(cifar_config(32), 32)
    times, kinds = _time_steps(tr, imgs, cifar_steps)
    mean = sum(times) / len(times)
    out['configs0_cifar10_sngan_b32'] = {
        'value': round(32 / mean, 3), 'unit': 'images/s', 'steps': len(times), 'warmup': 3,
        'schedule': ''.join(kinds), 'step_s': _stats(times)}
    out['components'] = cpu_components()
    scan = cpu_thread_scan(threads)
    out['thread_scan_median_step_s'] = scan
    best = min(scan, key=scan.get)
    out['thread_scan_note'] = ('median ImageNet mirror step over 3 steps per thread count; the '
                               'headline uses %d threads (the fastest of the scan is %d); the '
                               'host affinity of %d CPUs exceeds the job\'s CPU share (%s) and '
                               'is not used' % (threads, best, affinity,
                                                os.environ.get('OMP_NUM_THREADS')))
    return out


def _reps(fn, n=20, warm=3):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return {'median_ms': round(_pct(ts, .5) * 1e3, 3), 'p10_ms': round(_pct(ts, .1) * 1e3, 3),
            'p90_ms': round(_pct(ts, .9) * 1e3, 3), 'reps': n}


def cpu_components():
    """SURVEY 8d CPU components on the mirror (median of 20 after 3 warm-ups):
    (i) MMD^2 fwd + bwd per N (the three N x N matrices materialised, d = 1),
    (ii) the SN power iteration of every SN layer of each BASELINE critic
    (oracle/ref_nets.py variable shapes, reference layout)."""
    from oracle import ref_nets as R
    from oracle.tf_mirror import rbf_mmd2_tf, sn_weight_tf
    g = torch.Generator().manual_seed(0)
    out = {}
    for N in (64, 512, 2048):
        X = torch.randn(N, 1, generator=g).requires_grad_(True)
        Y = torch.randn(N, 1, generator=g).requires_grad_(True)

        def mmd_once():
            torch.autograd.grad(rbf_mmd2_tf(X, Y), (X, Y))
        out['mmd_fwd_bwd_N%d' % N] = dict(_reps(mmd_once), pairs=3 * N * N)
    for arch, size in (('snresnet', 64), ('sngan', 32), ('g-resnet5', 160)):
        vs = [v for v in R.critic_vars(arch, 64, 1, size, True, True) if v.sn]
        Ws = [torch.randn(*v.shape, generator=g) * 0.02 for v in vs]
        us = [torch.randn(1, v.shape[-1], generator=g) for v in vs]
        s1 = torch.ones(1)

        def sn_once():
            with torch.no_grad():
                for W, u in zip(Ws, us):
                    sn_weight_tf(W, u, s1)
        out['sn_power_iter_%s%d' % (arch, size)] = dict(
            _reps(sn_once), layers=len(vs), weights=sum(int(W.numel()) for W in Ws))
    return out


def mmd_path(rows, d):
    """The implementation smmd_mmd2_fwd picks (csrc/smmd_mmd.hip use_gram /
    use_tile; env overrides aside): MFMA Gram for wide features, the 2-D
    tiled sweep for d <= 8 (up to TILE_MAX_RT row tiles), else the row sweep."""
    gram = d > 32 or (d >= 16 and rows >= 1024) or (d >= 32 and rows >= 512)
    if gram:
        return 'mfma-gram'
    if d <= 8 and rows <= (16384 // 4 - 64) * 64:
        return 'tile-2d'
    return 'row-sweep'


def mmd_valu_ops_per_pair(kernel, D):
    """Algorithmic VALU lane-ops per pair of the reference's three matrices
    (SURVEY 8d): forward P (2D + 6) flops + one exp, backward P (3D + 4) flops
    reusing K; mix_rq adds 3 (4 flops + log + exp), mix_rbf 5 more (2 flops +
    exp).  A transcendental costs TRANS_SLOTS lane-op slots."""
    base = (2 * D + 6) + (3 * D + 4)
    if kernel == 'rbf':
        return base + TRANS_SLOTS
    if kernel == 'mix_rbf':
        return base + 6 * TRANS_SLOTS + 5 * 2
    if kernel == 'mix_rq':
        return base + 3 * (4 + 2 * TRANS_SLOTS)
    return base


def mmd_sweep(world, rank, dev, group, quick=False):
    """SURVEY 8d MMD microbench: X, Y ~ N(0,1) [N, D] per side (global N,
    numpy default_rng(1234)), rank r owning rows [r N/w, (r+1) N/w) of each, run
    through the product path mmd.mmd2_fused (all-gather mode when w > 1) with
    its backward; HIP-event time per fwd+bwd, max over ranks.  Algorithmic
    bytes: fwd (m+n) D 4 + 16, bwd (m+n) D 4 read + (m+n) D 4 written; pairs
    P = m^2 + mn + n^2 (the reference's three matrices).  D <= 32: VALU
    fraction (mmd_valu_ops_per_pair); D >= 128: the Gram flops 4 D P
    (forward Gram + backward C Z) against the f32 MFMA peak."""
    import numpy as np
    from gan.core import _lib, mmd
    grid = [(32, 1), (64, 1), (256, 1), (512, 1), (2048, 1), (512, 16), (2048, 16),
            (256, 128), (512, 128), (2048, 128), (512, 1024), (2048, 1024)]
    if quick:
        grid = [(64, 1), (512, 1), (2048, 1), (512, 128)]
    extra = [('mix_rq', 512, 1), ('mix_rbf', 512, 1), ('mix_rq', 2048, 1),
             ('mix_rq', 512, 128), ('mix_rbf', 512, 128)]
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
            torch.autograd.grad(v, (Xl, Yl))
            return v

        if rank == 0:
            print('[bench] mmd sweep %s N=%d D=%d' % (kern, N, D), file=sys.stderr, flush=True)
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
        else:
            ops = mmd_valu_ops_per_pair(kern, D) * P
            row.update(valu_ops_per_pair=mmd_valu_ops_per_pair(kern, D),
                       valu_frac=round(ops / (ms * 1e-3) / VALU_LANE_OPS, 4))
        rows.append(row)
    return rows


def literal_macs(net, x):
    """Forward multiply-accumulates per image of `net` on input x in the
    REFERENCE's literal layer order (gan/core/resnet/block.py:53-73,
    architecture.py:178-230, :334-343, :395-434): ConvMeanPool as a full
    resolution 3x3 conv then the pool, UpsampleConv as nearest-upsample then
    the 3x3 conv -- not the product's folded stride-2 forms, which do 4/9 of
    that work.  Counted from the layer shapes met by one forward."""
    from gan.core import architecture as A
    from gan.core import snops
    macs = [0]
    inner = set()
    for m in net.modules():
        if isinstance(m, (A._ConvMeanPool, A._Up, A._MeanPoolConv)):
            inner.add(id(m.conv))

    def conv_hook(mod, inp, out):
        if id(mod) in inner:
            return
        h, w = out.shape[2], out.shape[3]
        macs[0] += h * w * mod.cout * mod.cin * mod.k * mod.k

    def cmp_hook(mod, inp, out):          # conv at the input's resolution, then pool
        c = mod.conv
        h, w = inp[0].shape[2], inp[0].shape[3]
        macs[0] += h * w * c.cout * c.cin * c.k * c.k

    def mpc_hook(mod, inp, out):          # pool, then conv at half resolution
        c = mod.conv
        macs[0] += out.shape[2] * out.shape[3] * c.cout * c.cin * c.k * c.k

    def up_hook(mod, inp, out):           # upsample, then conv at 2x resolution
        c = mod.conv
        macs[0] += out.shape[2] * out.shape[3] * c.cout * c.cin * c.k * c.k

    def deconv_hook(mod, inp, out):
        macs[0] += inp[0].shape[2] * inp[0].shape[3] * mod.cin * mod.cout * mod.k * mod.k

    def lin_hook(mod, inp, out):
        macs[0] += mod.weight.shape[0] * mod.weight.shape[1]

    hooks = []
    for m in net.modules():
        if isinstance(m, snops.Conv2d):
            hooks.append(m.register_forward_hook(conv_hook))
        elif isinstance(m, A._ConvMeanPool):
            hooks.append(m.register_forward_hook(cmp_hook))
        elif isinstance(m, A._MeanPoolConv):
            hooks.append(m.register_forward_hook(mpc_hook))
        elif isinstance(m, A._Up):
            hooks.append(m.register_forward_hook(up_hook))
        elif isinstance(m, snops.Deconv2d):
            hooks.append(m.register_forward_hook(deconv_hook))
        elif isinstance(m, snops.Linear):
            hooks.append(m.register_forward_hook(lin_hook))
    try:
        with torch.no_grad():
            net(x[:1])
    finally:
        for h in hooks:
            h.remove()
    return macs[0]


def step_flops(model, images):
    """Algorithmic FLOPs of the lean schedule per averaged step:
    per image, D step = G_f + 9 D_f (G forward; critic forward on real and
    fake; the Jacobian pass Dx; first-order Dx + Dw through both critic calls;
    the double backward's conv + Dw through the Jacobian pass), G step =
    3 G_f + 4 D_f (G forward + Dx + Dw; critic forward x2, its Jacobian pass
    for the scale, Dx through the fake call); a cycle is 5 D + 1 G."""
    model.sn_D.refresh(update_u=False)
    if model.sn_G.entries:
        model.sn_G.refresh(update_u=False)
    z = model.sample_z(2)
    d_f = literal_macs(model.discriminator, images)
    g_f = literal_macs(model.generator, z)
    per_img_d = 2 * (g_f + 9 * d_f)
    per_img_g = 2 * (3 * g_f + 4 * d_f)
    return {'D_fwd_macs_per_image': d_f, 'G_fwd_macs_per_image': g_f,
            'flops_per_D_step': per_img_d * BATCH, 'flops_per_G_step': per_img_g * BATCH,
            'flops_per_avg_step': (5 * per_img_d + per_img_g) * BATCH / 6}


def run_steps(model, images, k, counts=None):
    for i in range(k):
        before = model.step
        model.train_step(images[i % len(images)])
        if counts is not None:
            counts['G' if model.step != before else 'D'] += 1


def sync(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def instrumented_pass(model, images, cycles, world, dev):
    """Whole 5 D + 1 G cycles with HIP events around every libsmmd_hip call
    (on the compute stream) and around each step: per entry point calls, mean
    time and algorithmic bytes; D and G step times."""
    from gan.core import _lib
    model.d_counter = model.g_counter = 0
    sync(world)
    _lib.reset_timing()
    _lib.enable_timing(True)
    ev = {'D': [], 'G': []}
    for i in range(6 * cycles):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        before = model.step
        s.record()
        model.train_step(images[i % len(images)])
        e.record()
        ev['G' if model.step != before else 'D'].append((s, e))
    sync(world)
    _lib.enable_timing(False)
    tm = _lib.timing_ms()
    tb = _lib.timing_bytes()
    tb.update({k + '#flops': v for k, v in _lib.timing_flops().items()})
    step_ms = {k: sum(a.elapsed_time(b) for a, b in v) / len(v) for k, v in ev.items() if v}
    return tm, tb, step_ms, 6 * cycles


def launch_plan(gpus, env):
    """How `bench.py --gpus N` runs (before anything touches the GPU):
    ('run', world) when this process is a rank (WORLD_SIZE set and equal to
    N) or N == 1; ('spawn', N) when N > 1 and no launcher started us -- the
    parent then starts torch.distributed.run with N ranks as a child (the
    reference's towers over num_gpus, /root/reference/gan/core/model.py:187-216,
    num_gpus from the environment, gan/main.py:126).  A launcher that started
    a different number of ranks than --gpus is an error."""
    if gpus < 1:
        raise SystemExit('bench.py: --gpus must be >= 1 (got %d)' % gpus)
    ws = env.get('WORLD_SIZE')
    if ws is None:
        return ('spawn', gpus) if gpus > 1 else ('run', 1)
    if int(ws) != gpus:
        raise SystemExit('bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks'
                         % (gpus, ws))
    return ('run', gpus)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """Start N ranks of this script under torch.distributed.run as a child
    process (this parent never initialises the GPU); rank 0's JSON line goes
    to the inherited stdout.  Returns the launcher's exit code."""
    import subprocess
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(n), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.abspath(__file__)] + list(argv)
    print('[bench] launching %d ranks: %s' % (n, ' '.join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--batch', type=int, default=64,
                    help='images per GPU: 64 is the headline (imagenet_smmd.yml); 256 is '
                         'BASELINE configs[4] (the 256 x 256 pairwise tile per GPU)')
    ap.add_argument('--config', default='imagenet', choices=sorted(CONFIGS),
                    help='imagenet: the headline (BASELINE metric); cifar10 / celebA64: '
                         'BASELINE configs[1] / [2] measured the same way')
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
    ap.add_argument('--graphs', type=int, default=-1,
                    help='1: the timed steps replay HIP graphs of the captured step kinds '
                         '(model.enable_graphs; one GPU); 0: eager; -1 (default): auto -- '
                         'on one GPU, two untimed 5D+1G cycles each way during the warmup, '
                         'graphs kept only when >= 5 %% faster (host-bound configs: CIFAR-10 '
                         'SNGAN 1.37x; the GPU-bound ImageNet step stays eager, graphs 1.3 %% '
                         'slower there)')
    ap.add_argument('--cpu-steps', type=int, default=24,
                    help='timed CPU-baseline steps of the ImageNet config (after 3 warm-ups; '
                         'SURVEY 8d asks >= 20; 24 = 4 whole 5D+1G cycles)')
    ap.add_argument('--ref-schedule-steps', type=int, default=30,
                    help='steps timed with the reference schedule (both gradient sets '
                         'every step, model.py:514) after the main run; 0: skip')
    ap.add_argument('--instrument-cycles', type=int, default=3,
                    help='5 D + 1 G cycles of the instrumented pass (per-call HIP events); '
                         '0: skip')
    ap.add_argument('--mmd-sweep', type=int, default=1,
                    help='1: SURVEY 8d MMD microbench grid; 2: four configs; 0: skip')
    args = ap.parse_args()
    global BATCH
    BATCH = args.batch

    mode, n = launch_plan(args.gpus, os.environ)
    if mode == 'spawn':
        sys.exit(spawn_ranks(n, sys.argv[1:]))
    probe = os.environ.get('SMMD_BENCH_PROBE')
    if probe == 'fail':        # launch check: a rank failing must fail the job
        sys.exit(3)
    if probe == '1':
        # launch check without a GPU (tests/test_bench_launch.py): the rank layout
        print(json.dumps({'probe': True, 'world': int(os.environ.get('WORLD_SIZE', '1')),
                          'rank': int(os.environ.get('RANK', '0')), 'gpus': args.gpus}),
              flush=True)
        return
    # ONE JSON line on stdout: whatever native code prints there (RCCL's init
    # banner goes to fd 1) is sent to stderr, and the line goes to the saved fd
    sys.stdout.flush()
    global _JSON_OUT
    _JSON_OUT = os.fdopen(os.dup(1), 'w')
    os.dup2(2, 1)

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
    # SMMD_DP_FORCE=1 at N = 1: a world-size-1 group whose rank takes the
    # data-parallel path (collectives.force_dp), so the RCCL device branches
    # run on one GPU; the line says so in config.dp_forced
    dp_forced = world == 1 and os.environ.get('SMMD_DP_FORCE', '0') != '0'
    if dp_forced:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', str(_free_port()))
        os.environ.setdefault('RANK', '0')
        os.environ.setdefault('WORLD_SIZE', '1')
    if world > 1 or dp_forced:
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
    cfg = CONFIGS[args.config][0](BATCH)
    size = int(cfg.output_size)
    torch.manual_seed(2 + rank)
    model = SMMD(cfg, device=dev,
                 process_group=dist.group.WORLD if (world > 1 or dp_forced) else None,
                 dp_mode=args.dp_mode, channels_last=bool(args.channels_last))
    gen = torch.Generator(device=dev).manual_seed(0 + rank)
    images = [torch.rand(BATCH, 3, size, size, device=dev, generator=gen) for _ in range(4)]
    log = (lambda *a: print('[bench]', *a, file=sys.stderr, flush=True)) if rank == 0 else \
        (lambda *a: None)

    # 1. prime every autograd graph (and its MIOpen kernels) once, untimed
    tw = time.perf_counter()
    for sched in ('lean', 'reference'):
        model.schedule = sched
        model.d_step(images[0])
        model.g_step(images[1])
    model.schedule = 'lean'
    graphs_probe = None
    use_graphs = args.graphs
    if use_graphs < 0:
        use_graphs = 0
        if world == 1 and not dp_forced:
            # auto: time two 5 D + 1 G cycles eagerly and with graphs (all of
            # it untimed warmup), keep graphs only when clearly faster
            def cycle_ms():
                model.step = 21
                model.d_counter = model.g_counter = 0
                torch.cuda.synchronize()
                t = time.perf_counter()
                run_steps(model, images, 12)
                torch.cuda.synchronize()
                return (time.perf_counter() - t) / 12 * 1e3
            model.step = 21
            run_steps(model, images, 6)
            eager_ms = cycle_ms()
            model.enable_graphs()
            model.step = 21
            run_steps(model, images, 6)               # captures every step kind
            graph_ms = cycle_ms()
            use_graphs = 1 if graph_ms < 0.95 * eager_ms else 0
            if not use_graphs:
                model.enable_graphs(False)
            graphs_probe = {'eager_ms_per_step': round(eager_ms, 3),
                            'graphs_ms_per_step': round(graph_ms, 3),
                            'chosen': 'graphs' if use_graphs else 'eager'}
            log('graphs probe: eager %.3f ms/step, graphs %.3f -> %s'
                % (eager_ms, graph_ms, graphs_probe['chosen']))
    elif use_graphs:
        model.enable_graphs()       # capture every step kind before the warmup
        model.step = 21
        run_steps(model, images, 6)
    args.graphs = use_graphs
    sync(world)
    log('primed D and G steps of both schedules in %.1f s' % (time.perf_counter() - tw))

    # 2. warmup, then align to the start of a 5 D + 1 G cycle
    model.step = 21          # steady state: 5 critic updates per generator update
    for i in range(args.warmup):
        model.train_step(images[i % len(images)])
        if rank == 0:
            torch.cuda.synchronize()
            log('warmup step %d/%d done at %.1f s' % (i + 1, args.warmup,
                                                     time.perf_counter() - tw))
    model.check_finite()
    model.d_counter = model.g_counter = 0
    sync(world)

    # 3. the timed region: exactly K steps, nothing instrumented
    counts = {'D': 0, 'G': 0}
    t0 = time.perf_counter()
    run_steps(model, images, args.steps, counts)
    sync(world)
    dt = max_over_ranks(time.perf_counter() - t0, world, dev)
    g_loss, d_loss = model.check_finite()
    log('timed %d steps: %.2f ms/step' % (args.steps, dt / args.steps * 1e3))

    # 4. the reference schedule (both gradient sets every step, model.py:514)
    model.enable_graphs(False)      # the rest runs eagerly
    ref_sched = None
    if args.ref_schedule_steps > 0:
        model.schedule = 'reference'
        model.d_counter = model.g_counter = 0
        run_steps(model, images, 6)                       # one cycle
        sync(world)
        model.d_counter = model.g_counter = 0
        rc = {'D': 0, 'G': 0}
        t0 = time.perf_counter()
        run_steps(model, images, args.ref_schedule_steps, rc)
        sync(world)
        dtr = max_over_ranks(time.perf_counter() - t0, world, dev)
        model.schedule = 'lean'
        ref_sched = {'value': round(world * BATCH * args.ref_schedule_steps / dtr, 2),
                     'unit': 'images/s', 'steps': args.ref_schedule_steps, 'warmup': 6,
                     'd_steps': rc['D'], 'g_steps': rc['G'],
                     'ms_per_step': round(dtr / args.ref_schedule_steps * 1e3, 3),
                     'note': 'every step also computes the other network\'s gradient set '
                             'and discards it, as each sess.run of the reference does '
                             '(model.py:514); value above is the lean schedule'}
        log('reference schedule: %.2f ms/step' % (dtr / args.ref_schedule_steps * 1e3))

    # 5. instrumented pass (separate from the headline)
    from gan.core import _lib
    stamp = _lib.lib().smmd_source_hash().decode()     # the running library build
    kernels, step_ms, roofline, hot = {}, {}, None, {}
    if args.instrument_cycles > 0:
        tm, tb, step_ms, n_inst = instrumented_pass(model, images, args.instrument_cycles,
                                                    world, dev)
        m_all = BATCH * world
        sn_kn = sum(e.N * e.K for e in model.sn_D.entries)
        # the SN output per layer: W_eff [N, K], or for a ConvMeanPool conv the
        # pool-folded 4 x 4 filter the bank writes directly (16 floats per 9)
        sn_out = sum(e.N * e.K * 16 // 9 if e.fold else e.N * e.K for e in model.sn_D.entries)
        # the refresh writes W_eff / W' only for the layers that are not lazy
        # (the Winograd-fed ones' filters are formed from W, sigma, s: sn.set_lazy)
        lazy = getattr(model.sn_D, 'lazy', set())
        sn_out_written = sum(e.N * e.K * 16 // 9 if e.fold else e.N * e.K
                             for i, e in enumerate(model.sn_D.entries) if i not in lazy)
        per_img = 3 * size * size
        gdirect = model._gdirect()
        adam_sn_d = model.d_optim.numel * 4 * 8
        if gdirect:
            # G-direct: the SN weights' gradient is never formed: no norm-pass
            # read of it; the update reads G (W_eff's or W''s size) + p, m, v
            # and writes p, m, v; every other tensor as the plain update
            adam_sn_d = (model.d_optim.numel - sn_kn) * 4 * 8 + sn_kn * 4 * 6 + sn_out * 4
        alg = {
            # sqsum pass reads g; update pass reads g, p, m, v and writes p, m, v
            'smmd_adam_flat[D]': model.d_optim.numel * 4 * 8,
            'smmd_adam_flat[G]': model.g_optim.numel * 4 * 8,
            # the same update with the SN weights' first power-iteration pass
            # folded in (its column-partial writes are < 0.1 % of these bytes)
            'smmd_adam_flat_sn[D]': adam_sn_d,
            'smmd_adam_flat_sn[G]': model.g_optim.numel * 4 * 8,
            # the G-direct backward: one read of G and of W
            'smmd_sn_grad_stats': (sn_out + sn_kn) * 4,
            # one read of W + one write of W_eff (2 K N 4 B per
            # iteration; the folded filters' 16 / 9 larger output for
            # ConvMeanPool), the write only for the layers that are not lazy
            'smmd_sn_power_iter': (sn_kn + sn_out_written) * 4,
            # one read of G (W_eff's shape) and W, one write of gW
            'smmd_sn_weight_bwd': (sn_out + 2 * sn_kn) * 4,
            # X, Y rows read, unit gradients written, sums
            'smmd_mmd2_fwd': 2 * m_all * 4 + 2 * BATCH * 4 + 8 * 4,
            'smmd_scaled_loss_fwd': BATCH * per_img * 4,
            # ConvMeanPool filter fold / adjoint: 9 floats read + 16 written (or
            # back) per filter, every ConvMeanPool layer of the critic per call
            'smmd_fold_pool_weights': sum(m.conv.weight.shape[0] * m.conv.weight.shape[1]
                                          for m in model.discriminator.modules()
                                          if isinstance(m, architecture._ConvMeanPool)) * 25 * 4,
            'smmd_scaled_loss_bwd': 2 * BATCH * per_img * 4,
            # the fused loss (one process): the Jacobian read once + the
            # features and their unit gradients; its backward as the
            # scaled loss's (the generator step writes no Jacobian gradient:
            # its mean bytes come from the D / G mix of the pass)
            'smmd_smmd_loss_fwd': BATCH * per_img * 4 + 4 * BATCH * 4 + 8 * 4,
            'smmd_smmd_loss_bwd': 2 * BATCH * per_img * 4 + 4 * BATCH * 4,
        }
        alg.update({k: int(v) for k, v in tb.items() if not k.endswith('#flops')})
        mfma_flops = {k[:-6]: v for k, v in tb.items() if k.endswith('#flops')}
        for name, (calls, ms) in tm.items():
            b = alg.get(name)
            row = {'calls': calls, 'avg_ms': round(ms, 5),
                   'ms_per_step': round(ms * calls / n_inst, 5), 'hot_path': name in HOT_PATH}
            if b:
                row.update(bytes=b, GB_s=round(b / (ms * 1e-3) / 1e9, 1),
                           frac=round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
            kernels[name] = row
        # the roofline kernel: the SURVEY 8(a) entry point with the most time
        # per step among the HBM-bound ones (the MMD launch is latency / VALU
        # bound at D = 1 and is reported in roofline_hot_path)
        cands = [k for k in kernels if k in HOT_PATH and 'GB_s' in kernels[k]
                 and k != 'smmd_mmd2_fwd']
        for name, fl in mfma_flops.items():
            if name in kernels:
                tf = fl / (kernels[name]['avg_ms'] * 1e-3) / 1e12
                kernels[name].update(mfma_flops=int(fl), tflops=round(tf, 2),
                                     mfma_frac=round(tf / MFMA_F32_PEAK_TFS, 4))
        if cands:
            dom = max(cands, key=lambda k: kernels[k]['ms_per_step'])
            traffic, src, why = pmc_traffic(dom, stamp)
            roofline = {'bound': 'hbm', 'kernel': dom, 'achieved': kernels[dom]['GB_s'],
                        'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': kernels[dom]['frac'],
                        'traffic': traffic, 'traffic_source': src, 'traffic_null_reason': why,
                        'avg_ms': kernels[dom]['avg_ms'],
                        'algorithmic_bytes': kernels[dom]['bytes']}
        # the library's dominant kernel by time per step: a Winograd
        # convolution (matrix-core bound) once they serve the conv layers
        mf = [k for k in kernels if 'tflops' in kernels[k]]
        for k in mf:
            hot[k] = {q: kernels[k][q] for q in ('avg_ms', 'ms_per_step', 'calls', 'mfma_flops',
                                                 'tflops', 'mfma_frac')}
        wk = max(mf, key=lambda k: kernels[k]['ms_per_step']) if mf else None
        if wk and (roofline is None
                   or kernels[wk]['ms_per_step'] > kernels[roofline['kernel']]['ms_per_step']):
            hot['hbm_roofline_kernel'] = roofline
            traffic, src, why = pmc_traffic(wk, stamp)
            roofline = {'bound': 'mfma', 'kernel': wk, 'achieved': kernels[wk]['tflops'],
                        'peak': MFMA_F32_PEAK_TFS, 'unit': 'TFLOP/s',
                        'frac': kernels[wk]['mfma_frac'], 'traffic': traffic,
                        'traffic_source': src, 'traffic_null_reason': why,
                        'traffic_over_algorithmic': (
                            round(traffic / kernels[wk]['bytes'], 3)
                            if traffic and kernels[wk].get('bytes') else None),
                        'avg_ms': kernels[wk]['avg_ms'],
                        'calls_per_step': round(kernels[wk]['calls'] / n_inst, 2),
                        'ms_per_step': kernels[wk]['ms_per_step'],
                        'executed_flops_per_call': kernels[wk]['mfma_flops'],
                        'algorithmic_bytes': kernels[wk].get('bytes'),
                        'note': 'executed flops = the Winograd point products on the f32 '
                                'MFMA (F(2x2,3x3): 16 per 2x2 tile and channel pair, 2.25x '
                                'fewer than the direct conv; F(2x2,2x2) polyphase: 9 per tile '
                                'and phase channel, 1.78x fewer)'}
        for k in ('smmd_sn_power_iter', 'smmd_sn_weight_bwd', 'smmd_sn_grad_stats',
                  'smmd_adam_flat_sn[D]',
                  'smmd_scaled_loss_fwd', 'smmd_scaled_loss_bwd', 'smmd_smmd_loss_fwd',
                  'smmd_smmd_loss_bwd', 'smmd_fold_pool_weights', 'smmd_wino3x3_conv',
                  'smmd_wino3x3_wgrad', 'smmd_wino4x4s2_conv', 'smmd_wino4x4s2t_conv',
                  'smmd_wino4x4s2_wgrad'):
            if k in kernels and 'bytes' in kernels[k]:
                traffic, src, why = pmc_traffic(k, stamp)
                row = hot.setdefault(k, {})
                row.update({'avg_ms': kernels[k]['avg_ms'],
                            'algorithmic_bytes': kernels[k]['bytes'],
                            'GB_s': kernels[k]['GB_s'], 'hbm_frac': kernels[k]['frac'],
                            'pmc_traffic': traffic,
                            'pmc_over_algorithmic': (round(traffic / kernels[k]['bytes'], 3)
                                                     if traffic else None),
                            'pmc_source': src, 'pmc_null_reason': why})
        # the loss side of a step: the fused launch and its backward (or,
        # unfused, mmd2 + scaled loss fwd + bwd), each once per step: the sum
        # of their mean HIP-event times per call
        loss_keys = ('smmd_smmd_loss_fwd', 'smmd_smmd_loss_bwd', 'smmd_mmd2_fwd',
                     'smmd_scaled_loss_fwd', 'smmd_scaled_loss_bwd')
        hot['loss_side_us_per_step'] = {
            'total': round(sum(kernels[k]['avg_ms'] for k in loss_keys if k in kernels) * 1e3, 2),
            'calls': {k: round(kernels[k]['avg_ms'] * 1e3, 2) for k in loss_keys if k in kernels}}
        mk_name = 'smmd_mmd2_fwd' if 'smmd_mmd2_fwd' in kernels else (
            'smmd_smmd_loss_fwd' if 'smmd_smmd_loss_fwd' in kernels else None)
        if mk_name:
            mk = kernels[mk_name]
            P = 3 * m_all * m_all
            ops = mmd_valu_ops_per_pair('rbf', 1) * P
            hot[mk_name] = {
                'avg_ms': mk['avg_ms'], 'N_per_side': m_all, 'pairs': P,
                'valu_frac': round(ops / (mk['avg_ms'] * 1e-3) / VALU_LANE_OPS, 5),
                'bound': 'latency at D = 1 (one launch per critic step)'}
        log('instrumented pass: %d steps' % n_inst)

    fl = step_flops(model, images[0])
    ms_step = dt / args.steps * 1e3
    # the timed region's own mix of D and G steps
    fl_timed = (counts['D'] * fl['flops_per_D_step'] + counts['G'] * fl['flops_per_G_step']) \
        / max(counts['D'] + counts['G'], 1)
    tfs = fl_timed / (ms_step * 1e-3) / 1e12
    hot['step'] = dict(fl, flops_per_timed_step=fl_timed,
                       literal_work_rate_tflops=round(tfs, 2),
                       literal_work_rate_over_fp32_peak=round(tfs / FP32_PEAK_TFS, 4),
                       fp32_peak_tflops=FP32_PEAK_TFS,
                       note='literal work rate = the reference\'s literal conv layers (no '
                            'fold, direct-conv MAC count) per second of this run; the '
                            'product runs Winograd and folded stride-2 convs, which execute '
                            'fewer MACs, so this rate can exceed the peak and is not a '
                            'utilisation; `counters` holds the executed-FLOP figures '
                            '(rocprofv3, stamped with the library build they were measured on)',
                       counters=step_counters(ms_step, stamp))

    sweep = None
    if args.mmd_sweep:
        sweep = mmd_sweep(world, rank, dev, dist.group.WORLD if world > 1 else None,
                          quick=args.mmd_sweep == 2)
        hot['mmd_sweep_valu'] = [{'kernel': r['kernel'], 'N': r['N'], 'kernel_ms': r['kernel_ms'],
                                  'valu_frac': r['valu_frac']}
                                 for r in sweep if r['D'] == 1 and r['N'] in (64, 512, 2048)]

    result = {
        'metric': 'images/sec/step (64x64 SMMD, batch 64) + MMD-kernel GB/s at 1/2/4/8 GPU',
        'value': round(world * BATCH * args.steps / dt, 2),
        'unit': 'images/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'prime_steps': 4 + (36 if graphs_probe else (6 if args.graphs else 0)),
        'd_steps': counts['D'],
        'g_steps': counts['G'],
        'ms_per_step': round(ms_step, 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'fp32',
        'data': 'synthetic (U[0,1] images in HBM, z~U(-1,1), random-init weights)',
        'config': {'workload': '%s, batch %d/GPU, 5D+1G schedule' % (CONFIGS[args.config][1],
                                                                       BATCH),
                   'model': cfg.architecture, 'global_batch': BATCH * world, 'seq_len': None,
                   'parallelism': 'dp%d' % world, 'dp_mode': args.dp_mode,
                   'dp_forced': dp_forced,
                   'memory_format': 'channels_last' if args.channels_last else 'nchw',
                   'miopen_winograd': bool(args.miopen_winograd),
                   'miopen_find': bool(args.miopen_find),
                   'step_graphs': bool(args.graphs),
                   'step_graphs_probe': graphs_probe,
                   'conv_mean_pool': ('folded 4x4 stride-2 conv' if architecture.FOLD_POOL
                                      else 'conv3x3 + mean pool'),
                   'miopen_db': os.environ.get('MIOPEN_USER_DB_PATH')},
        'roofline': roofline,
        'roofline_hot_path': hot,
        'smmd_source_hash': stamp,
        'step_ms_by_kind': {k: round(v, 3) for k, v in step_ms.items()},
        'hip_kernels': kernels,
        'schedule_reference': ref_sched,
        'mmd_sweep': sweep,
        'losses': {'g_loss': g_loss, 'd_loss': d_loss},
    }
    if step_ms.get('D') and step_ms.get('G'):
        # from the instrumented pass (HIP events around every library call and
        # every step: ~10 % slower than the timed region), so not a clean
        # timing; the timed region itself covers whole 5D+1G cycles when
        # `steps` is a multiple of 6 (whole_cycles_timed)
        result['instrumented_cycle_value'] = round(
            world * BATCH * 6 / ((5 * step_ms['D'] + step_ms['G']) * 1e-3), 2)
    result['whole_cycles_timed'] = (counts['G'] if counts['D'] == 5 * counts['G'] else None)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result['cpu_baseline'] = cpu_baseline(args.cpu_steps)
        except Exception as e:   # report, never hide the GPU number
            result['cpu_baseline'] = {'error': repr(e)}
    if rank == 0:
        print(json.dumps(result), file=_JSON_OUT, flush=True)
    if world > 1 or dp_forced:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
