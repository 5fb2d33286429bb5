"""Drop-in CLI of gan/main.py: same single-dash flags, same defaults, and the
same YAML-overrides-CLI rule (gan/main.py:18-25), dispatching to the MI355X
trainer.

    python scaled-mmd-gan_amd/gan/main.py -config_file configs/imagenet_smmd.yml
    torchrun --nproc-per-node 8 scaled-mmd-gan_amd/gan/main.py -config_file ... -dp_mode global

Data (gan/core/pipeline.py): cifar10 (python or binary batches under
-data_dir), imagenet / celebA (TFRecord shards tf_records_train/train-*).
Datasets are not shipped (no network); ``-dataset synthetic`` feeds U[0,1]
images of the configured size, matching the reference pipeline's value range
(pipeline.py:201, :403).  Any other dataset whose files are absent or
malformed is an error, as in the reference.

Checkpoints (model.py:559-566, :585-617): resumed from -checkpoint_dir/-name
(-ckpt_name or the latest save) at start; saved every 2000 steps after a
generator update.
"""
from __future__ import annotations

import argparse
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)


def str2bool(v):
    """gan/main.py:9-15."""
    if isinstance(v, bool):
        return v
    if v.lower() in ('yes', 'true', 't', 'y', '1'):
        return True
    if v.lower() in ('no', 'false', 'f', 'n', '0'):
        return False
    raise argparse.ArgumentTypeError('Boolean value expected.')


# (flag, default, type) -- gan/main.py:32-121
_FLAGS = [
    ('max_iteration', 150000, int), ('beta1', 0.5, float), ('beta2', 0.9, float),
    ('learning_rate', 0.0001, float), ('learning_rate_D', -1, float), ('dsteps', 5, int),
    ('gsteps', 1, int), ('start_dsteps', 10, int), ('clip_grad', True, str2bool),
    ('batch_norm', False, str2bool), ('init', 0.02, float), ('batch_size', 64, int),
    ('real_batch_size', -1, int), ('output_size', 128, int), ('c_dim', 3, int),
    ('z_dim', 128, int), ('df_dim', 64, int), ('dof_dim', 1, int), ('gf_dim', 64, int),
    ('dataset', 'cifar10', str), ('name', '', str), ('checkpoint_dir', 'checkpoint', str),
    ('sample_dir', 'sample', str), ('log_dir', 'log', str), ('data_dir', './data', str),
    ('out_dir', './out', str), ('config_file', '', str), ('architecture', 'dcgan', str),
    ('kernel', '', str), ('model', 'smmd', str), ('is_train', True, str2bool),
    ('visualize', False, str2bool), ('is_demo', False, str2bool), ('log', True, str2bool),
    ('compute_scores', True, str2bool), ('print_pca', False, str2bool), ('suffix', '', str),
    ('gpu_mem', .9, float), ('no_of_samples', 100000, int), ('save_layer_outputs', 0, int),
    ('ckpt_name', '', str), ('decay_rate', .8, float), ('gp_decay_rate', .8, float),
    ('sc_decay_rate', 1., float), ('restart_lr', False, str2bool),
    ('restart_sc', False, str2bool), ('MMD_lr_scheduler', True, str2bool),
    ('MMD_sdlr_past_sample', 10, int), ('MMD_sdlr_num_test', 3, int),
    ('MMD_sdlr_freq', 2000, int), ('gradient_penalty', 0.0, float),
    ('L2_discriminator_penalty', 0.0, float), ('with_scaling', False, str2bool),
    ('scaling_coeff', 10., float), ('scaling_variant', 'grad', str),
    ('with_sn', False, str2bool), ('with_learnable_sn_scale', False, str2bool),
    ('multi_gpu', False, str2bool), ('num_gpus', 1, int), ('with_labels', False, str2bool),
    ('use_gaussian_noise', False, str2bool),
    # this build: data-parallel mode of the all-gather extension
    ('dp_mode', 'tower', str),
    # this build: scorer features ('inception' is the reference's and is
    # unavailable offline; 'random' = seeded random features, gan/utils/featurizer.py)
    ('featurizer', 'inception', str),
]
_DOUBLE_DASH = [('use-incomplete-cho', True, str2bool), ('incho-eta', 1e-3, float),
                ('incho-max-steps', 1000, int)]


def build_parser():
    p = argparse.ArgumentParser()
    for name, default, typ in _FLAGS:
        p.add_argument('-' + name, default=default, type=typ)
    for name, default, typ in _DOUBLE_DASH:
        p.add_argument('--' + name, default=default, type=typ)
    return p


def default_flags():
    return vars(build_parser().parse_args([]))


def load_yaml(path):
    import yaml
    with open(path) as f:
        return yaml.safe_load(f) or {}


def make_flags(parser=None, argv=None):
    """YAML keys REPLACE parsed values (gan/main.py:18-25)."""
    parser = parser or build_parser()
    flags = parser.parse_args(argv)
    if flags.config_file:
        config = load_yaml(flags.config_file)
        dic = vars(flags)
        for k in config:
            dic.pop(k, None)
        dic.update(config)
    return flags


def num_gpus_from_env():
    """gan/main.py:126 reads CUDA_VISIBLE_DEVICES (KeyError when unset); here
    the process-group world size or the visible HIP devices."""
    ws = os.environ.get('WORLD_SIZE')
    if ws:
        return int(ws)
    vis = os.environ.get('HIP_VISIBLE_DEVICES') or os.environ.get('CUDA_VISIBLE_DEVICES')
    return len(vis.split(',')) if vis else 1


def output_size_for(flags):
    """gan/main.py:159-167 (cifar10 forces 32, mnist 28)."""
    if flags.dataset == 'cifar10':
        return 32, 3
    if flags.dataset == 'mnist':
        return 28, 1
    return flags.output_size, flags.c_dim


CHECKPOINT_FREQ = 2000                   # model.py:609


def description(flags, size):
    """The run's directory name (model.py:62-77)."""
    c = flags
    lr_d = c.learning_rate_D if c.learning_rate_D >= 0 else c.learning_rate
    lr = ('lr%.8f' % c.learning_rate if lr_d == c.learning_rate
          else 'lr%.8fG%fD' % (c.learning_rate, lr_d))
    d = '%s%s_%s%s_%sd%d-%d-%d_%s_%s_%s' % (
        c.dataset, '%dx%d' % (c.gf_dim, c.df_dim), c.architecture, '_dc', c.kernel, c.dsteps,
        c.start_dsteps, c.gsteps, c.batch_size, size, lr)
    return d + ('_bn' if c.batch_norm else '')


def run_dirs(flags, size, create=True):
    """{'sample', 'log', 'checkpoint'} -> out_dir/<x>_dir/name/suffix+description
    (model.py:105-120, _ensure_dirs).  The checkpoints themselves stay under
    -checkpoint_dir/-name (this build's layout, see main())."""
    desc = flags.suffix + description(flags, size)
    out = {}
    for folder in ('sample', 'log', 'checkpoint'):
        sub = getattr(flags, folder + '_dir')
        path = os.path.join(flags.out_dir, sub, flags.name, desc)
        if sub and create:
            os.makedirs(path, exist_ok=True)
        out[folder] = path
    return out


class LogRedirect:
    """-log (default True): stdout and stderr of the run go to
    <sample_dir>/log.txt, line-buffered (model.py:85-94).  Restored on exit
    (the reference never restores; a library caller keeps its streams)."""

    def __init__(self, sample_dir, on=True):
        self.path = os.path.join(sample_dir, 'log.txt')
        self.on = on
        self.f = None

    def __enter__(self):
        if self.on:
            import time
            self.old = sys.stdout, sys.stderr
            self.f = open(self.path, 'w', buffering=1)
            print('Execution start time: %s' % time.ctime())
            print('Log file: %s' % self.path)
            sys.stdout = sys.stderr = self.f
            print('Execution start time: %s' % time.ctime())
        return self

    def __exit__(self, *exc):
        if self.f is not None:
            if exc[0] is not None:
                import traceback
                traceback.print_exception(*exc, file=self.f)
            sys.stdout, sys.stderr = self.old
            self.f.close()
            self.f = None
        return False
SCORE_SIZE = 25000                       # gan/utils/scorer.py:27


def make_scorer(flags, pipe, dev, size):
    """Scorer + featurizer when -compute_scores (model.py:95-96), or
    (None, None) when scoring is off or no featurizer is available (the
    Inception graph: a warning says so).  Train codes: loaded from
    <data_dir>/<dataset>-codes[-size]-<featurizer>.npy when present, else
    featurized from SCORE_SIZE pipeline images and saved there
    (gan/utils/scorer.py:37-64)."""
    if not flags.compute_scores:
        return None, None
    import numpy as np
    import torch
    from gan.utils.featurizer import get_featurizer
    from gan.utils.scorer import Scorer
    feat = get_featurizer(flags.featurizer, dev)
    if feat is None:
        return None, None
    suffix = '' if size <= 32 else '-%d' % size
    path = os.path.join(flags.data_dir, '%s-codes%s-%s.npy' % (flags.dataset, suffix, feat.name))
    if os.path.exists(path):
        codes = np.load(path)                                   # allow_pickle=False
    else:
        ims, n = [], 0
        while n < SCORE_SIZE:
            b = pipe.next()
            ims.append(feat(b))
            n += b.shape[0]
        codes = torch.cat(ims)[:SCORE_SIZE].cpu().numpy()
        try:
            np.save(path, codes)
        except OSError:
            pass
    return Scorer(codes, lr_scheduler=flags.MMD_lr_scheduler), feat


def make_pipeline(flags, size, c_dim, dev, rank=0, world=1):
    """The dataset's pipeline (gan/core/pipeline.py:458-476).  U[0,1] images
    only for ``-dataset synthetic``: an unknown dataset name, absent files or
    malformed records raise, as the reference's pipelines do -- a run never
    trains on noise it did not ask for."""
    from gan.core import pipeline as P
    args = (size, c_dim, flags.real_batch_size, flags.data_dir)
    kw = dict(device=dev, rank=rank, world=world)
    return P.get_pipeline(flags.dataset)(*args, **kw)


def main(argv=None):
    import torch
    import torch.distributed as dist

    flags = make_flags(argv=argv)
    flags.num_gpus = num_gpus_from_env()
    from gan.core import miopen_db
    miopen_db.install()                    # before the first convolution
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)
    rank = dist.get_rank() if world > 1 else 0
    size, c_dim = output_size_for(flags)
    dirs = run_dirs(flags, size, create=(rank == 0))
    try:
        with LogRedirect(dirs['sample'], on=bool(flags.log) and rank == 0):
            if rank == 0:
                import pprint
                pprint.PrettyPrinter().pprint(vars(flags))
            return _train(flags, dev, world, rank, size, c_dim)
    finally:
        if world > 1:
            dist.destroy_process_group()


def _train(flags, dev, world, rank, size, c_dim):
    import torch
    import torch.distributed as dist
    from gan.core.smmd import get_model
    Model = get_model(flags.model)
    torch.manual_seed(rank)
    gan = Model(flags, device=dev, process_group=dist.group.WORLD if world > 1 else None,
                dp_mode=flags.dp_mode, output_size=size, c_dim=c_dim)
    if flags.is_train:
        pipe = make_pipeline(flags, size, c_dim, dev, rank, world)
        ckpt_dir = os.path.join(flags.checkpoint_dir, flags.name)
        if gan.load_checkpoint(ckpt_dir, flags.ckpt_name):
            print(' [*] Load SUCCESS, re-starting at step %d with learning rate %.7f'
                  % (gan.step, gan.lr))
        else:
            print(' [!] Load failed...')
        step = gan.step
        scorer, feat = make_scorer(flags, pipe, dev, size) if rank == 0 else (None, None)
        if world > 1:       # every rank must apply the same learning-rate decays
            flag = torch.tensor([1.0 if scorer is not None else 0.0], device=dev)
            dist.broadcast(flag, 0)
            scoring = bool(flag.item())
        else:
            scoring = scorer is not None
        try:
            while step <= flags.max_iteration:
                _, _, step = gan.train_step(pipe.next())
                if gan.d_counter == 0 and (step % 100 == 0 or step <= 10):
                    g, d = gan.check_finite()
                    if rank == 0:
                        gan.timer(step, '%s, G: %.8f, D: %.8f' % (gan.optim_name, g, d))
                if gan.d_counter == 0 and step % CHECKPOINT_FREQ == 0 and rank == 0:
                    gan.save_checkpoint(ckpt_dir, step)          # model.py:608-612
                if scoring and gan.d_counter == 0 and step % flags.MMD_sdlr_freq == 0:
                    # model.py:544-545 -> scorer.py:66-175 (rank 0), the decayed
                    # lr / sc then broadcast so every replica applies them
                    if rank == 0:
                        scorer.compute(gan, step, feat(gan.get_samples(SCORE_SIZE)),
                                       save_checkpoint=lambda: gan.save_checkpoint(ckpt_dir))
                    if world > 1:
                        ls = torch.tensor([gan.lr, gan.sc if gan.sc is not None else 0.0],
                                          device=dev, dtype=torch.float64)
                        dist.broadcast(ls, 0)
                        gan.set_lr_sc(float(ls[0]), float(ls[1]) if gan.sc is not None else None)
        finally:
            pipe.stop()
    return gan


if __name__ == '__main__':
    main()
