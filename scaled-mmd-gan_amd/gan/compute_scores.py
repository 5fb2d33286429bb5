"""KID (polynomial-kernel MMD) scoring of gan/compute_scores.py on the MI355X.

Mirrors the reference's ``polynomial_mmd_averages`` (:211-229),
``polynomial_mmd`` (:232-243) and ``_mmd2_and_variance`` (:246-335): same
arguments, same numpy return values.  The three m x m kernel matrices are
never formed: ``smmd_poly_kernel_sums`` evaluates them tile by tile on the
f32 matrix cores and keeps only their row/column sums, diagonals and squared
sums; the estimator and its variance run in double on the device.

The Inception featurizer, inception_score and fid_score need the Inception
graph, which the reference downloads (:22-39) and which is unavailable
offline: callers pass codes (e.g. synthetic [n, 2048] pool3 features).
"""
from __future__ import annotations

import sys

import numpy as np
import torch

from .core import _lib
from .core.mmd import PolySums, _codes, poly_mmd2_and_variance, polynomial_kernel_sums


def polynomial_mmd_averages(codes_g, codes_r, n_subsets=50, subset_size=1000, ret_var=True,
                            output=sys.stdout, **kernel_args):
    """KID over random subsets, drawn as the reference does (np.random.choice
    without replacement, :220-222); codes stay on the GPU between subsets."""
    m = min(codes_g.shape[0], codes_r.shape[0])
    mmds = np.zeros(n_subsets)
    if ret_var:
        vars_ = np.zeros(n_subsets)
    choice = np.random.choice
    G = _codes(codes_g)
    R = _codes(codes_r, G.device)
    for i in range(n_subsets):
        gi = torch.from_numpy(choice(len(codes_g), subset_size, replace=False)).to(G.device)
        ri = torch.from_numpy(choice(len(codes_r), subset_size, replace=False)).to(G.device)
        o = polynomial_mmd(G.index_select(0, gi), R.index_select(0, ri), var_at_m=m,
                           ret_var=ret_var, **kernel_args)
        if ret_var:
            mmds[i], vars_[i] = o
        else:
            mmds[i] = o
    return (mmds, vars_) if ret_var else mmds


def polynomial_mmd(codes_g, codes_r, degree=3, gamma=None, coef0=1, var_at_m=None,
                   ret_var=True):
    """k(x, y) = (gamma <x, y> + coef0)^degree, gamma = 1/dim by default."""
    X = _codes(codes_g)
    Y = _codes(codes_r, X.device)
    kw = dict(degree=degree, gamma=gamma, coef0=coef0)
    xx = polynomial_kernel_sums(X, X, **kw)
    yy = polynomial_kernel_sums(Y, Y, **kw)
    xy = polynomial_kernel_sums(X, Y, **kw)
    mmd2, var = poly_mmd2_and_variance(xx, yy, xy, var_at_m=var_at_m).tolist()
    return (mmd2, var) if ret_var else mmd2


def _sums_of_matrix(K):
    K = K.to(dtype=torch.float64)
    d = torch.diagonal(K)
    stats = torch.stack([K.sum(), (K * K).sum(), d.sum(), (d * d).sum()])
    return PolySums(K.sum(1).contiguous(), K.sum(0).contiguous(), d.contiguous(),
                    stats.contiguous(), tuple(K.shape))


def _mmd2_and_variance(K_XX, K_XY, K_YY, unit_diagonal=False, mmd_est='unbiased',
                       block_size=1024, var_at_m=None, ret_var=True):
    """The reference's estimator on already-formed kernel matrices (:246-335),
    reduced on the device.  unit_diagonal: the diagonals are taken as 1."""
    mats = [torch.as_tensor(np.asarray(k) if not torch.is_tensor(k) else k) for k in
            (K_XX, K_XY, K_YY)]
    dev = torch.device('cuda', torch.cuda.current_device())
    mats = [k.to(dev) for k in mats]
    m = mats[0].shape[0]
    assert all(k.shape == (m, m) for k in mats)
    if unit_diagonal:
        for k in (0, 2):
            mats[k] = mats[k].clone()
            mats[k].fill_diagonal_(1.0)
    xx, xy, yy = (_sums_of_matrix(k) for k in mats)
    mmd2, var = poly_mmd2_and_variance(xx, yy, xy, var_at_m=var_at_m, mmd_est=mmd_est).tolist()
    return (mmd2, var) if ret_var else mmd2


__all__ = ['polynomial_mmd_averages', 'polynomial_mmd', '_mmd2_and_variance', '_lib']
