"""KID scoring and the 3-sample learning-rate scheduler of gan/utils/scorer.py.

``Scorer.compute`` follows the reference (:65-170) from the point where the
Inception codes exist: KID over 10 subsets of 1000 (:103-111, best-model
callback :113-117), then the 3-sample test between the training codes X, the
current samples Y and a sample Z from ``MMD_sdlr_past_sample`` scorings ago
(:119-162): if p = Phi(test statistic) > 0.1 ``MMD_sdlr_num_test`` times in a
row, the learning rate (and scaling amplitude) decays via ``gan.decay_ops()``.
The statistics run on the GPU (gan/core/mmd.py polynomial section).

Featurizing images needs the Inception graph, unavailable offline: callers
hand over codes (``codes`` argument, e.g. synthetic pool3 features).
"""
from __future__ import annotations

import math

import numpy as np

from .. import compute_scores as cs
from ..core import mmd


def _norm_cdf(x):
    return 0.5 * (1.0 + math.erf(x / math.sqrt(2.0)))


class Scorer:
    def __init__(self, train_codes, lr_scheduler=True, n_subsets=10, subset_size=1000,
                 three_sample_size=2048):
        self.train_codes = np.asarray(train_codes, dtype=np.float32)
        self.lr_scheduler = lr_scheduler
        self.n_subsets = n_subsets
        self.subset_size = subset_size
        self.bs = three_sample_size
        self.output = []
        self.three_sample = []
        self.three_sample_chances = 0

    def compute(self, gan, step, codes, save_checkpoint=None):
        """One scoring round (gan/utils/scorer.py:65-170) on ``codes``."""
        if step % gan.config.MMD_sdlr_freq != 0:
            return None
        output = {}
        output['mmd2'] = mmd2s = cs.polynomial_mmd_averages(
            codes, self.train_codes, n_subsets=self.n_subsets, subset_size=self.subset_size,
            ret_var=False)
        if self.output and min(o['mmd2'].mean() for o in self.output) > mmd2s.mean():
            if save_checkpoint is not None:                  # 'Saving BEST model'
                save_checkpoint()
        self.output.append(output)
        if self.lr_scheduler:
            n = gan.config.MMD_sdlr_past_sample
            nc = gan.config.MMD_sdlr_num_test
            new_Y = codes[:self.bs]
            X = self.train_codes[:self.bs]
            if len(self.three_sample) >= n:
                saved_Z = self.three_sample[0]
                diff, stat, y_sums = mmd.np_diff_polynomial_mmd2_and_ratio_with_saving(
                    X, new_Y, saved_Z)
                p_val = _norm_cdf(stat)
                output.update(three_sample_stat=stat, p_value=p_val, mmd2_diff=diff)
                if p_val > .1:
                    self.three_sample_chances += 1
                    if self.three_sample_chances >= nc:
                        gan.decay_ops()
                        self.three_sample = (self.three_sample + [y_sums])[-nc:]
                        self.three_sample_chances = 0
                else:
                    self.three_sample = self.three_sample[1:] + [y_sums]
                    self.three_sample_chances = 0
            else:
                self.three_sample.append(
                    mmd.np_diff_polynomial_mmd2_and_ratio_with_saving(X, new_Y, None))
        output['lr'] = np.array([gan.lr])
        if getattr(gan.config, 'with_scaling', False):
            output['sc'] = np.array([gan.sc])
        return output
