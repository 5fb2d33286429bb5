"""world_size-2 gloo tests (CPU) of the data-parallel paths:

* all-gather ('global') MMD^2: each rank holds half of X and Y, sees the full
  pairwise kernel, gets the same estimator as one process on the
  concatenated batch, and row-local gradients equal that process's rows;
* the scaled loss over the global batch (J all-reduced);
* gradient exchange: 'tower' = per-rank clip, SUM/world, Adam (reference
  model.py:233-266, :444-456); 'global' = SUM, clip, Adam.

The HIP library is replaced by tests/fake_lib.py (oracle on CPU memory) so
only the plumbing is under test here; the kernels' parity is tested on the GPU.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip('torch')
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from oracle import smmd_oracle as O  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (root, os.path.join(root, 'scaled-mmd-gan_amd'), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import fake_lib
    fake_lib.install()


def _data(seed=0, n=8, d=2):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((2 * n, d)).astype(np.float32)
    Y = (rng.standard_normal((2 * n, d)) + 0.5).astype(np.float32)
    return X, Y


def _worker_mmd(rank, world, port, kernel, q):
    _init(rank, world, port)
    from gan.core import mmd
    X, Y = _data()
    n = X.shape[0] // world
    Xl = torch.tensor(X[rank * n:(rank + 1) * n], requires_grad=True)
    Yl = torch.tensor(Y[rank * n:(rank + 1) * n], requires_grad=True)
    val = mmd.mmd2_fused(Xl, Yl, kernel, process_group=dist.group.WORLD)
    val.backward()
    q.put((rank, float(val), Xl.grad.numpy().copy(), Yl.grad.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def _run(target, *args, world=2):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


@pytest.mark.parametrize('kernel', ['rbf', 'mix_rq_dot', 'distance'])
def test_global_mmd2_matches_single_process(kernel):
    X, Y = _data()
    spec = O.kernel_spec(kernel)
    ref = O.mmd2(spec, X, Y)
    dX, dY = O.mmd2_grad(spec, X, Y)
    res = _run(_worker_mmd, kernel)
    n = X.shape[0] // 2
    for rank, val, gx, gy in res:
        assert val == pytest.approx(ref, rel=1e-5, abs=1e-7)
        np.testing.assert_allclose(gx, dX[rank * n:(rank + 1) * n], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(gy, dY[rank * n:(rank + 1) * n], rtol=1e-5, atol=1e-7)


def _worker_scaled(rank, world, port, q):
    _init(rank, world, port)
    from gan.core import ops
    rng = np.random.default_rng(3)
    jac = rng.standard_normal((1, 2 * 4, 3, 2, 2)).astype(np.float32)
    jl = torch.tensor(jac[:, rank * 4:(rank + 1) * 4], requires_grad=True)
    base = torch.tensor(0.5, requires_grad=True)
    g, aux = ops.scaled_loss(base, jl, None, sc=10.0, process_group=dist.group.WORLD)
    g.backward()
    q.put((rank, float(g), float(aux[3]), jl.grad.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def test_global_scaled_loss_uses_global_batch():
    rng = np.random.default_rng(3)
    jac = rng.standard_normal((1, 8, 3, 2, 2)).astype(np.float64)
    J = np.mean(O.squared_norm_per_sample(jac[0]))
    scale = O.scale_factor(J, 10.0)
    res = _run(_worker_scaled)
    cq = 0.5 * (-10.0 * scale ** 2)
    for rank, g, Jg, gj in res:
        assert Jg == pytest.approx(J, rel=1e-6)
        assert g == pytest.approx(0.5 * scale, rel=1e-6)
        np.testing.assert_allclose(gj, cq * 2.0 / 8 * jac[:, rank * 4:(rank + 1) * 4], rtol=1e-5)


def _worker_exchange(rank, world, port, mode, q):
    _init(rank, world, port)
    from gan.core.model import MMD_GAN
    from gan.core.optim import FlatAdam
    rng = np.random.default_rng(10)
    p0 = rng.standard_normal(5).astype(np.float32)
    p1 = rng.standard_normal(3).astype(np.float32)
    params = [torch.nn.Parameter(torch.tensor(p0)), torch.nn.Parameter(torch.tensor(p1))]
    opt = FlatAdam(params, lr=1e-3, clip_norm=1.0)
    g = np.random.default_rng(100 + rank).standard_normal(8).astype(np.float32) * 2
    params[0].grad.copy_(torch.tensor(g[:5]))
    params[1].grad.copy_(torch.tensor(g[5:]))
    m = MMD_GAN.__new__(MMD_GAN)
    m.world, m.group, m.dp_mode = world, dist.group.WORLD, mode
    m._exchange(opt)
    q.put((rank, np.concatenate([p.detach().numpy().ravel() for p in params])))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('mode', ['tower', 'global'])
def test_gradient_exchange_semantics(mode):
    rng = np.random.default_rng(10)
    p = [rng.standard_normal(5), rng.standard_normal(3)]
    grads = [np.random.default_rng(100 + r).standard_normal(8).astype(np.float32).astype(
        np.float64) * 2 for r in range(2)]
    sl = [slice(0, 5), slice(5, 8)]
    expect = []
    for i in range(2):
        if mode == 'tower':      # clip per tower, then mean (model.py:449-455, :257-258)
            g = np.mean([O.clip_by_norm(gr[sl[i]], 1.0) for gr in grads], axis=0)
        else:                    # global loss: sum, then clip
            g = O.clip_by_norm(sum(gr[sl[i]] for gr in grads), 1.0)
        expect.append(O.adam_step(p[i].astype(np.float32).astype(np.float64), 0, 0, g, 1,
                                  1e-3)[0])
    res = _run(_worker_exchange, mode)
    for rank, flat in res:
        np.testing.assert_allclose(flat, np.concatenate(expect), rtol=1e-5, atol=1e-7)
