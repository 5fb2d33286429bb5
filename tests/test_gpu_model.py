"""End-to-end training-step checks on the GPU.

The critic update of SMMD (SN bank -> critic -> fused MMD^2 -> Jacobian ->
scaled loss -> double backward -> HIP SN backward) is compared with the
oracle's CPU op-by-op mirror of the TF graph (oracle/tf_mirror.py) from the
same weights, u vectors, images and z.  Tolerances (MIOpen fp32 convs vs CPU
fp32 convs, same graph): d_loss rtol 1e-3; per-tensor gradients
|d| <= max(t max|ref|, 5e-5 max over all tensors) + t |ref| with t = 2e-3, and
t = 5e-3 at the configs' full widths and batch >= 64 (64x longer fp32
reductions over the batch in a different order: MIOpen's vs the CPU's); and
per tensor a relative Frobenius error <= 1e-3 (2e-3 at batch >= 64), so a
systematic error in a low-magnitude tensor cannot hide under the max bound.
"""
import argparse

import numpy as np
import pytest

torch = pytest.importorskip('torch')

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    from gan.main import default_flags
    c = default_flags()
    c.update(dict(batch_size=8, output_size=32, architecture='sngan', kernel='rbf', model='smmd',
                  batch_norm=True, with_sn=True, with_learnable_sn_scale=True, with_scaling=True,
                  dof_dim=1, learning_rate=1e-4, dataset='cifar10'))
    c.update(kw)
    return argparse.Namespace(**c)


def _mirror_from(model):
    """The oracle's TF-graph mirror on its own networks (oracle/ref_nets.py),
    started from the model's weights and u vectors."""
    from oracle.tf_mirror import TFMirrorStep
    st = TFMirrorStep(model.config, model.generator, model.discriminator, sc=model.sc)
    by_weight = {id(st.prod[k]): k.rsplit('/', 1)[0] for k in st.prod}
    for e in model.sn_D.entries:
        st.us[by_weight[id(e.module.weight)]] = e.u.detach().cpu().view(1, -1).clone()
    return st


@pytest.mark.parametrize('arch,size,dim,batch,cl', [
    ('sngan', 32, 64, 8, False), ('snresnet', 64, 16, 8, False), ('snresnet', 64, 16, 8, True),
    ('g-resnet5', 64, 16, 8, False),
    ('g-resnet5', 64, 64, 64, False),         # celebA_smmd.yml's widths and batch at 64x64 (C3)
    ('snresnet', 64, 64, 64, False),          # imagenet_smmd.yml's widths and batch, once
    ('snresnet', 64, 16, 256, False)])        # BASELINE configs[4]'s 256 images per GPU
def test_critic_step_matches_tf_mirror(dev, arch, size, dim, batch, cl):
    from gan.core.smmd import SMMD
    torch.manual_seed(0)
    cfg = _cfg(architecture=arch, output_size=size, df_dim=dim, gf_dim=dim, batch_size=batch,
               batch_norm=arch != 'g-resnet5')         # celebA_smmd.yml: batch_norm False
    model = SMMD(cfg, device=dev, channels_last=cl)
    mirror = _mirror_from(model)
    g = torch.Generator().manual_seed(1)
    images = torch.rand(batch, 3, size, size, generator=g)
    z = torch.empty(batch, 128).uniform_(-1, 1, generator=g)
    ref_loss, ref_grads = mirror.grads(images, z)

    model.sample_z = lambda n: z.to(dev)
    captured = {}
    orig = model.d_optim.step

    def cap(*a, **k):
        captured['g'] = model.d_optim.dense_grad().cpu()
        return orig(*a, **k)
    model.d_optim.step = cap
    model.step = 25
    model.d_counter, model.g_counter = 0, 0
    _, d_loss, aux = model.d_step(images.to(dev))
    assert float(d_loss.detach()) == pytest.approx(float(ref_loss), rel=1e-3, abs=1e-6)
    flat = captured['g']
    gmax = max(float(rg.abs().max()) for rg in ref_grads.values())
    index = {id(p): i for i, p in enumerate(model.d_vars)}
    assert sorted(index) == sorted(id(mirror.prod[n]) for n in ref_grads)
    for name, rg in ref_grads.items():
        p = mirror.prod[name]
        i = index[id(p)]
        got = torch.as_strided(flat, p.shape, p.stride(), model.d_optim.offsets[i]).contiguous()
        got = got.numpy().astype(np.float64)
        ref = mirror.to_product(name, rg).numpy().astype(np.float64)
        # exact zeros (e.g. the output bias: RBF-MMD is translation invariant) are
        # rounding noise in both (either sign): absolute floor 5e-5 of the
        # largest gradient
        t = 5e-3 if batch >= 64 else 2e-3
        tol = max(t * np.abs(ref).max(), 5e-5 * gmax) + t * np.abs(ref)
        assert (np.abs(got - ref) <= tol + 1e-12).all(), (name, np.abs(got - ref).max(),
                                                           np.abs(ref).max())
        # a small systematic error in one low-magnitude tensor would hide under
        # the elementwise bound: its own relative Frobenius error stays small
        # (tensors whose reference is rounding noise -- |ref| under the floor --
        # are exempt)
        nref = np.linalg.norm(ref)
        if np.abs(ref).max() > 10 * 5e-5 * gmax:
            rel = np.linalg.norm(got - ref) / nref
            assert rel <= (2e-3 if batch >= 64 else 1e-3), (name, rel)
    # u advanced exactly as the reference's u.assign(u') (sn.py:39-46)
    by_weight = {id(mirror.prod[k]): k.rsplit('/', 1)[0] for k in mirror.prod}
    for e in model.sn_D.entries:
        u = mirror.us[by_weight[id(e.module.weight)]]
        np.testing.assert_allclose(e.u.cpu().numpy(), u.numpy()[0], rtol=1e-4, atol=1e-6)


def _aten_convs(prof):
    """aten convolution ops (MIOpen) recorded by a CPU-activity profile."""
    return sorted({e.name for e in prof.events()
                   if e.name.startswith('aten::') and 'conv' in e.name})


def _headline_model(dev, batch=64):
    """SNResNet-64 at imagenet_smmd.yml's widths (every conv tiles on the
    library: no MIOpen convolution in either step), fixed images and z."""
    from gan.core.smmd import SMMD
    torch.manual_seed(0)
    model = SMMD(_cfg(architecture='snresnet', output_size=64, df_dim=64, gf_dim=64,
                      batch_size=batch), device=dev)
    images = torch.rand(batch, 3, 64, 64, generator=torch.Generator().manual_seed(1)).to(dev)
    z = torch.empty(batch, 128).uniform_(-1, 1, generator=torch.Generator().manual_seed(2)).to(dev)
    model.sample_z = lambda n, z=z: z
    model.step = 25
    model.d_counter, model.g_counter = 0, 0
    return model, images


def _capture_grads(opt):
    cap = {}
    orig = opt.step

    def c(*a, **k):
        cap['g'] = opt.dense_grad().clone()
        return orig(*a, **k)
    opt.step = c
    return cap


def _step_record(model, images, profile=False):
    """Two critic updates (the second with the SN first pass written by the
    first's fused update) and one generator update: every loss, flat
    gradient, u, sigma and the parameters after each update."""
    from torch.profiler import ProfilerActivity, profile as prof_ctx
    dcap, gcap = _capture_grads(model.d_optim), _capture_grads(model.g_optim)
    rec = []
    convs = []

    def run():
        for kind in ('d', 'd', 'g'):
            g_loss, d_loss, _ = (model.d_step if kind == 'd' else model.g_step)(images)
            cap = dcap if kind == 'd' else gcap
            rec.append((kind, g_loss.detach().clone(), d_loss.detach().clone(), cap.pop('g'),
                        [e.u.clone() for e in model.sn_D.entries], model.sn_D.sigmas().clone(),
                        model.d_optim.flat_param.clone(), model.g_optim.flat_param.clone()))
    if profile:
        with prof_ctx(activities=[ProfilerActivity.CPU]) as p:
            run()
        convs = _aten_convs(p)
    else:
        run()
    torch.cuda.synchronize()
    return rec, convs


def test_headline_step_bit_identical_run_to_run(dev):
    """Run-to-run determinism of the all-library headline step (DESIGN §3:
    every library reduction is fixed-order).  Two models built from the same
    seed take the same critic, critic, generator updates, the second under
    the profiler (other host timing, so a timing-dependent kernel race shows
    as a difference): every loss, flat gradient, u, sigma and updated
    parameter is equal bit for bit (torch.equal), and no MIOpen convolution
    ran."""
    a, _ = _headline_model(dev)
    b, images = _headline_model(dev)
    assert torch.equal(a.d_optim.flat_param, b.d_optim.flat_param)
    assert torch.equal(a.g_optim.flat_param, b.g_optim.flat_param)
    ra, _ = _step_record(a, images)
    rb, convs = _step_record(b, images, profile=True)
    assert convs == [], convs
    names = ('g_loss', 'd_loss', 'grad', 'u', 'sigma', 'd params', 'g params')
    for i, (xa, xb) in enumerate(zip(ra, rb)):
        assert xa[0] == xb[0]
        for name, ta, tb in zip(names, xa[1:], xb[1:]):
            if isinstance(ta, list):
                assert all(torch.equal(p, q) for p, q in zip(ta, tb)), (i, xa[0], name)
            else:
                assert torch.equal(ta, tb), (i, xa[0], name, float((ta - tb).abs().max()))


def _critic_grad(dev, monkeypatch, mod, flag, on, counter):
    from gan.core import convops
    monkeypatch.setattr(mod, flag, on)
    model, images = _headline_model(dev, batch=8)
    cap = _capture_grads(model.d_optim)
    n0 = counter()
    model.d_step(images)
    return cap['g'], counter() - n0


def test_late_wgrad_sums_bit_identical(dev, monkeypatch):
    """convops' late sums of the critic weights' gradient contributions (real
    pass, fake pass, double backward; added at the SN node, or computed into
    the first by the *_wgrad_acc kernels, instead of by autograd as they
    arrive: the same sums in the same order) give dL/dW bit for bit, on the
    all-library step at the ImageNet config's width."""
    from gan.core import convops
    on, q_on = _critic_grad(dev, monkeypatch, convops, 'WGRAD_LATE_SUM', True,
                            lambda: convops._late['queued'])
    off, q_off = _critic_grad(dev, monkeypatch, convops, 'WGRAD_LATE_SUM', False,
                              lambda: convops._late['queued'])
    assert q_on > 0 and q_off == 0
    assert torch.equal(on, off), float((on - off).abs().max())


def test_late_bias_sums_bit_identical(dev, monkeypatch):
    """The critic biases' later gradient contributions (the fake pass after
    the real one) added to .grad after the backward (convops late bias sums):
    dL/db -- and every other gradient -- bit for bit the accumulation's."""
    from gan.core import convops
    on, q_on = _critic_grad(dev, monkeypatch, convops, 'BIAS_LATE_SUM', True,
                            lambda: convops._lateb['queued'])
    off, q_off = _critic_grad(dev, monkeypatch, convops, 'BIAS_LATE_SUM', False,
                              lambda: convops._lateb['queued'])
    assert q_on > 0 and q_off == 0
    assert torch.equal(on, off), float((on - off).abs().max())


def test_generator_gradient_gather_bit_identical(dev, monkeypatch):
    """The generator step's gradients gathered into the flat buffer by one
    multi-tensor copy (optim.FlatAdam.gather) update the generator bit for
    bit as the per-parameter accumulation does (the all-library step at the
    ImageNet config's width)."""
    from gan.core import model as M
    out = []
    for on in (True, False):
        monkeypatch.setattr(M, 'GRAD_GATHER', on)
        model, images = _headline_model(dev, batch=8)
        before = model.g_optim.flat_param.clone()
        model.g_step(images)
        assert all(p.grad is not None and p.grad.data_ptr() ==
                   model.g_optim.flat_grad[model.g_optim.offsets[i]:].data_ptr()
                   for i, p in enumerate(model.g_optim.params) if p.numel())
        out.append((model.g_optim.flat_param - before, model.g_optim.flat_grad.clone()))
    assert torch.equal(out[0][1], out[1][1]), float((out[0][1] - out[1][1]).abs().max())
    assert torch.equal(out[0][0], out[1][0])


def test_generator_step_updates_only_G(dev):
    from gan.core.smmd import SMMD
    torch.manual_seed(0)
    model = SMMD(_cfg(), device=dev)
    d_before = model.d_optim.flat_param.clone()
    g_before = model.g_optim.flat_param.clone()
    images = torch.rand(8, 3, 32, 32, device=dev)
    g_loss, d_loss, _ = model.g_step(images)
    assert torch.isfinite(g_loss)
    assert torch.equal(d_before, model.d_optim.flat_param)
    assert not torch.equal(g_before, model.g_optim.flat_param)
    assert all(p.requires_grad for p in model.d_vars)


def test_schedule_and_losses_finite(dev):
    from gan.core.smmd import SMMD
    torch.manual_seed(0)
    model = SMMD(_cfg(), device=dev)
    images = torch.rand(8, 3, 32, 32, device=dev)
    kinds = []
    for _ in range(13):
        before = model.step
        model.train_step(images)
        kinds.append('G' if model.step != before else 'D')
    assert ''.join(kinds) == 'DDDDDDDDDDGDD'      # steps < 20: 10 critic updates per G
    g, d = model.check_finite()
    assert g == pytest.approx(-d)


@pytest.mark.parametrize('model_name,extra', [
    ('swgan', {}),
    ('mmd', {'gradient_penalty': 1.0, 'kernel': 'mix_rq', 'with_scaling': False}),
    ('smmd', {'kernel': 'mix_rbf', 'scaling_variant': 'value_and_grad'}),
    ('smmd', {'architecture': 'g-resnet5', 'output_size': 64, 'batch_norm': False}),
])
def test_other_models_step(dev, model_name, extra):
    from gan.core.smmd import get_model
    torch.manual_seed(0)
    cfg = _cfg(model=model_name, **extra)
    size = cfg.output_size
    model = get_model(model_name)(cfg, device=dev)
    images = torch.rand(8, 3, size, size, device=dev)
    for _ in range(3):
        model.train_step(images)
    g, d = model.check_finite()
    assert np.isfinite(g) and np.isfinite(d)


def test_tower_and_global_agree_on_one_gpu(dev):
    """Same critic gradient in both modes at world size 1 (compared before Adam:
    its first step maps rounding noise on zero-gradient tensors to +-lr)."""
    from gan.core.smmd import SMMD
    outs = []
    for mode in ('tower', 'global'):
        torch.manual_seed(0)
        model = SMMD(_cfg(), device=dev, dp_mode=mode)
        cap = {}
        orig = model.d_optim.step

        def step(*a, _o=orig, _c=cap, _m=model, **k):
            _c['g'] = _m.d_optim.dense_grad()
            return _o(*a, **k)
        model.d_optim.step = step
        torch.manual_seed(5)
        images = torch.rand(8, 3, 32, 32, device=dev)
        model.train_step(images)
        outs.append(cap['g'])
    # two runs of the same mode differ by up to ~1e-5 of the largest entry
    # (MIOpen's nondeterministic reductions; tools/dbg_towerglobal.py), so
    # the bound sits above that noise
    scale = float(outs[0].abs().max())
    assert torch.allclose(outs[0], outs[1], rtol=1e-4, atol=1e-4 * scale)


def test_reference_schedule_applies_the_lean_update(dev):
    """schedule='reference' (both gradient sets every step, model.py:514)
    computes the extra set and discards it: the gradients each optimizer
    applies equal the lean schedule's on the same weights, images and z."""
    from gan.core.smmd import SMMD
    torch.manual_seed(0)
    cfg = _cfg()
    lean = SMMD(cfg, device=dev)
    ref = SMMD(cfg, device=dev, schedule='reference')
    ref.generator.load_state_dict(lean.generator.state_dict())
    ref.discriminator.load_state_dict(lean.discriminator.state_dict())
    for a, b in zip(lean.sn_D.entries, ref.sn_D.entries):
        b.u.copy_(a.u)
    g = torch.Generator().manual_seed(3)
    images = torch.rand(8, 3, 32, 32, generator=g).to(dev)
    z = torch.empty(8, 128).uniform_(-1, 1, generator=g).to(dev)
    caps = []
    for mdl in (lean, ref):
        mdl.sample_z = lambda n: z
        cap = {}
        for opt in (mdl.d_optim, mdl.g_optim):      # the gradient each update applies
            def step(*a, _o=opt.step, _c=cap, _opt=opt, **k):
                _c[_opt.name] = _opt.dense_grad()
                return _o(*a, **k)
            opt.step = step
        caps.append(cap)
    for step, name in (('d_step', 'D'), ('g_step', 'G')):
        outs = [getattr(mdl, step)(images) for mdl in (lean, ref)]
        # the loss value too goes through solver-dependent convs (see below)
        np.testing.assert_allclose(outs[1][1].item(), outs[0][1].item(), rtol=1e-3, atol=1e-7)
        ga, gb = caps[0][name], caps[1][name]
        scale = float(ga.abs().max())
        # The two schedules run different autograd graphs, so MIOpen picks other
        # backward solvers (combined data+weight calls, bwd-data for the fake
        # batch): measured differences up to 9.5e-3 of max for D and 6.2e-3 for
        # G (amplified through the generator's BatchNorm backward), in some runs
        # of the same build and not in others.  A schedule bug (a leaked or
        # missing gradient set) is O(1).
        rtol, atol = 1e-3, 2e-2 * scale
        assert torch.allclose(gb, ga, rtol=rtol, atol=atol), (
            name, scale, float((gb - ga).abs().max()))


def test_checkpoint_resume(dev, tmp_path):
    """save_checkpoint / load_checkpoint (model.py:585-606): a fresh model
    resumed from the latest save holds the same weights, SN u vectors, Adam
    moments, step, schedule counters and learning rate, and trains on."""
    from gan.core.smmd import SMMD
    torch.manual_seed(0)
    a = SMMD(_cfg(), device=dev)
    images = torch.rand(8, 3, 32, 32, device=dev)
    for _ in range(7):                                 # D steps and one G step
        a.train_step(images)
    a.decay_ops()
    path = a.save_checkpoint(str(tmp_path), a.step)
    assert open(tmp_path / 'checkpoint').read().strip() == 'MMDGAN.model-%d' % a.step
    assert path.endswith('.pt')
    torch.manual_seed(1)
    b = SMMD(_cfg(), device=dev)
    assert b.load_checkpoint(str(tmp_path))
    assert (b.step, b.d_counter, b.g_counter) == (a.step, a.d_counter, a.g_counter)
    assert b.lr == a.lr and b.g_optim.lr == a.g_optim.lr and b.d_optim.lr == a.d_optim.lr
    for x, y in ((a.d_optim.flat_param, b.d_optim.flat_param), (a.g_optim.m, b.g_optim.m),
                 (a.d_optim.v, b.d_optim.v)):
        assert torch.equal(x, y)
    assert a.d_optim.step_count == b.d_optim.step_count
    for ea, eb in zip(a.sn_D.entries, b.sn_D.entries):
        assert torch.equal(ea.u, eb.u)
    for pa, pb in zip(a.generator.state_dict().values(), b.generator.state_dict().values()):
        assert torch.equal(pa, pb)
    b.train_step(images)
    b.check_finite()
    assert not b.load_checkpoint(str(tmp_path / 'nothing-here'))


def test_main_cli_trains_on_cifar_files_and_checkpoints(dev, tmp_path):
    """gan/main.py end to end: CIFAR-10 binary batches (synthetic bytes) ->
    HBM-resident pipeline -> training loop -> checkpoint at step 0 -> a second
    run resumes from it."""
    from gan import main as M
    rng = np.random.default_rng(3)
    for name in ['data_batch_%d' % b for b in range(1, 6)] + ['test_batch']:
        x = rng.integers(0, 256, (20, 3073), dtype=np.uint8)
        x[:, 0] %= 10
        x.tofile(str(tmp_path / (name + '.bin')))
    ck = tmp_path / 'ck'
    argv = ['-dataset', 'cifar10', '-data_dir', str(tmp_path), '-architecture', 'sngan',
            '-model', 'smmd', '-kernel', 'rbf', '-batch_size', '8', '-with_sn', 'true',
            '-with_learnable_sn_scale', 'true', '-with_scaling', 'true', '-batch_norm', 'true',
            '-max_iteration', '1', '-checkpoint_dir', str(ck), '-name', 'run',
            '-out_dir', str(tmp_path / 'out')]
    M.main(argv)
    assert (ck / 'run' / 'MMDGAN.model-0.pt').exists()
    M.main(argv)                                       # resumes at step 1 from the save
    assert open(ck / 'run' / 'checkpoint').read().strip() == 'MMDGAN.model-0'
    # -log (default on): the run's output in <sample_dir>/log.txt (model.py:85-94)
    logs = list((tmp_path / 'out' / 'sample' / 'run').glob('*/log.txt'))
    assert len(logs) == 1
    text = logs[0].read_text()
    assert 'Execution start time' in text and 'Load SUCCESS' in text and 'G: ' in text


def test_main_cli_scorer_drives_lr_schedule(dev, tmp_path, monkeypatch):
    """-compute_scores with -featurizer random: the scorer runs after
    generator updates every MMD_sdlr_freq steps (model.py:544-545), featurizes
    the training images once (codes cached in -data_dir, scorer.py:37-64) and
    keeps KID / 3-sample state; with the reference's default 'inception'
    featurizer (unavailable offline) it warns and stays off."""
    import warnings
    from gan import main as M
    monkeypatch.setattr(M, 'SCORE_SIZE', 2048)
    rng = np.random.default_rng(4)
    for name in ['data_batch_%d' % b for b in range(1, 6)] + ['test_batch']:
        x = rng.integers(0, 256, (20, 3073), dtype=np.uint8)
        x[:, 0] %= 10
        x.tofile(str(tmp_path / (name + '.bin')))
    base = ['-dataset', 'cifar10', '-data_dir', str(tmp_path), '-architecture', 'sngan',
            '-model', 'smmd', '-kernel', 'rbf', '-batch_size', '64', '-with_sn', 'true',
            '-with_learnable_sn_scale', 'true', '-with_scaling', 'true', '-batch_norm', 'true',
            '-max_iteration', '1', '-checkpoint_dir', str(tmp_path / 'ck'), '-name', 'run',
            '-MMD_sdlr_freq', '1', '-MMD_sdlr_past_sample', '1', '-MMD_sdlr_num_test', '1',
            '-out_dir', str(tmp_path / 'out')]
    gan = M.main(base + ['-featurizer', 'random'])
    assert (tmp_path / 'cifar10-codes-random.npy').exists()
    codes = np.load(tmp_path / 'cifar10-codes-random.npy')
    assert codes.shape == (2048, 2048) and np.isfinite(codes).all()
    assert gan.step >= 1
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        M.main(base + ['-name', 'run2'])
    assert any('Inception featurizer' in str(x.message) for x in w)


def test_step_graphs_match_eager(dev):
    """model.enable_graphs(): the lean step replayed from HIP graphs (one per
    step kind) trains as the eager step does, from the same state through
    every kind (critic after critic, critic after generator, generator).
    MIOpen's weight gradients are not bitwise deterministic and the GAN
    dynamics amplify that noise over steps, so the run uses a tiny learning
    rate (the states stay equal to far below the gradients' rounding, so the
    moments compare tightly) and a second eager copy calibrates the rest:
    parameters within 5 % of the update they made (+3x the eager-vs-eager
    spread), moments within 3e-3 (+3x: graph replays have come out up to
    1.4e-3 from eager on MI355X while two eager copies agree to 1e-9, MIOpen
    picking its kernels per capture); a stale tensor or a wrong step size in a
    replay is O(1) there."""
    from gan.core.smmd import SMMD
    torch.manual_seed(0)
    cfg = _cfg(learning_rate=1e-8)
    a = SMMD(cfg, device=dev)
    g = torch.Generator().manual_seed(3)
    imgs = [torch.rand(8, 3, 32, 32, generator=g).to(dev) for _ in range(3)]
    z = torch.empty(8, 128).uniform_(-1, 1, generator=g).to(dev)
    a.sample_z = lambda n: z
    a.step = 25
    for i in range(12):                        # eager: every step kind runs once first
        a.train_step(imgs[i % 3])
    copies = []
    for _ in range(2):
        m = SMMD(cfg, device=dev)
        m.load_state_dict(a.state_dict())
        m.sample_z = lambda n: z
        copies.append(m)
    b, c = copies
    start = [t.clone() for t in (a.d_optim.flat_param, a.g_optim.flat_param)]
    b.enable_graphs()
    for i in range(14):
        for m in (a, b, c):
            m.train_step(imgs[i % 3])
    torch.cuda.synchronize()
    assert {k[0] for k in b._graphs.graphs} == {True, False}
    assert len(b._graphs.graphs) == 3
    assert (a.step, a.d_counter, a.g_counter) == (b.step, b.d_counter, b.g_counter)
    assert (a.d_optim.step_count, a.g_optim.step_count) == \
        (b.d_optim.step_count, b.g_optim.step_count)

    def dist(x, y):
        return float((x - y).norm())
    for name in ('d_optim', 'g_optim'):
        oa, ob, oc = (getattr(m, name) for m in (a, b, c))
        p0 = start[0] if name == 'd_optim' else start[1]
        moved = dist(oa.flat_param, p0)
        assert moved > 0
        for t in ('flat_param', 'm', 'v'):
            ta, tb, tc = (getattr(o, t) for o in (oa, ob, oc))
            noise = dist(ta, tc)
            lim = 0.05 * moved if t == 'flat_param' else 3e-3 * float(ta.norm())
            assert dist(ta, tb) <= 3 * noise + lim, (name, t, dist(ta, tb), noise, lim)
    b.enable_graphs(False)
    b.train_step(imgs[0])                      # back to eager


def test_step_graphs_bit_identical_to_eager_all_library(dev):
    """On the all-library step (SNResNet-64 at the ImageNet config's width: no
    MIOpen convolution) the graph replays are the eager step bit for bit:
    through every step kind (critic with and without the SN first pass
    written, generator), parameters, Adam moments and u are torch.equal.
    The capture's filter cache (one transform per weight and step) and the
    lazy W_eff in the capture are covered by this."""
    from gan.core.smmd import SMMD
    a, images = _headline_model(dev, batch=8)
    g = torch.Generator().manual_seed(3)
    imgs = [torch.rand(8, 3, 64, 64, generator=g).to(dev) for _ in range(3)]
    for i in range(7):                         # eager: every step kind once first
        a.train_step(imgs[i % 3])
    b = SMMD(a.config, device=dev)
    b.load_state_dict(a.state_dict())
    b.sample_z = a.sample_z
    b.enable_graphs()
    for i in range(13):
        for m in (a, b):
            m.train_step(imgs[i % 3])
    torch.cuda.synchronize()
    assert len(b._graphs.graphs) == 3
    for name in ('d_optim', 'g_optim'):
        for t in ('flat_param', 'm', 'v'):
            ta, tb = getattr(getattr(a, name), t), getattr(getattr(b, name), t)
            assert torch.equal(ta, tb), (name, t, float((ta - tb).abs().max()))
    for ea, eb in zip(a.sn_D.entries, b.sn_D.entries):
        assert torch.equal(ea.u, eb.u)
    b.enable_graphs(False)


@pytest.mark.parametrize('order', [1, 2])
def test_linear_out_node_vs_float64(dev, order):
    """snops._LinOut (the critic's single-output linear layer with its own
    first- and second-order backward) against torch's addmv in float64: the
    output, and the gradients of x, w, b -- through the scaling regulariser's
    pattern (the input gradient with create_graph, a loss of it) at order 2."""
    from gan.core import snops
    g = torch.Generator(device=dev).manual_seed(4 + order)
    x0 = torch.randn(64, 1024, device=dev, generator=g)
    w0 = torch.randn(1, 1024, device=dev, generator=g) / 32
    b0 = torch.randn(1, device=dev, generator=g)
    t = torch.randn(64, device=dev, generator=g)

    def run(fn, dt):
        x = x0.to(dt).requires_grad_(True)
        w = w0.to(dt).requires_grad_(True)
        b = b0.to(dt).requires_grad_(True)
        y = fn(x, w, b)
        if order == 1:
            return (y,) + torch.autograd.grad((y * t.to(dt)).sum(), (x, w, b))
        jx, = torch.autograd.grad(y.sum(), x, create_graph=True)
        loss = jx.square().sum() + (y * t.to(dt)).sum()
        return (y,) + torch.autograd.grad(loss, (x, w, b))

    got = run(lambda x, w, b: snops._LinOut.apply(x, w, b), torch.float32)
    ref = run(lambda x, w, b: torch.addmv(b, x, w.view(-1)), torch.float64)
    for a, r, what in zip(got, ref, ('y', 'dx', 'dw', 'db')):
        err = float((a.double() - r).abs().max())
        assert err <= 2e-5 * (float(r.abs().max()) + 1e-30), (what, err)
