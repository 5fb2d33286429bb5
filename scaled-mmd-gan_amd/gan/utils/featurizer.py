"""Image featurizers for the scorer (gan/compute_scores.py:20-156 analogue).

The reference featurizes with the Inception graph it downloads
(compute_scores.py:22-39) -- not available offline, so ``get_featurizer``
returns None for 'inception' and the trainer warns that scoring and the
3-sample learning-rate schedule are off.  ``-featurizer random`` selects a
seeded random-feature network instead: the KID values are then not the
Inception ones (not comparable to published numbers) but the scoring loop,
the best-model checkpoint and the 3-sample LR decay of gan/utils/scorer.py run
exactly as in the reference on those codes.
"""
from __future__ import annotations

import warnings

import torch
import torch.nn.functional as F


class RandomFeaturizer:
    """Seeded, fixed random conv features: images in [0, 1] -> [n, dim]
    codes (the reference's pool3 width, 2048, by default).  Deterministic for
    a given seed, input size and device."""

    name = 'random'

    def __init__(self, device, dim=2048, seed=1234, c_dim=3):
        g = torch.Generator().manual_seed(seed)
        self.device = device
        self.w1 = (torch.randn(64, c_dim, 3, 3, generator=g) / 3.0).to(device)
        self.w2 = (torch.randn(256, 64, 3, 3, generator=g) / 24.0).to(device)
        self.w3 = (torch.randn(dim, 256, 1, 1, generator=g) / 16.0).to(device)
        self.dim = dim

    @torch.no_grad()
    def __call__(self, images, batch=500):
        out = []
        for i in range(0, images.shape[0], batch):
            x = images[i:i + batch].to(self.device, torch.float32) * 2.0 - 1.0
            h = F.relu(F.conv2d(x, self.w1, stride=2, padding=1))
            h = F.relu(F.conv2d(h, self.w2, stride=2, padding=1))
            h = F.relu(F.conv2d(h, self.w3))
            out.append(h.mean(dim=(2, 3)))
        return torch.cat(out, 0)


def get_featurizer(name, device):
    """'inception' (the reference's; unavailable offline -> None, with a
    warning) or 'random'."""
    if name in (None, '', 'inception'):
        warnings.warn('compute_scores: the Inception featurizer of the reference is unavailable '
                      'offline; KID scoring and the 3-sample learning-rate schedule are OFF '
                      '(the learning rate and scaling coefficient stay constant). Pass '
                      '-featurizer random to run them on seeded random features.')
        return None
    if name == 'random':
        return RandomFeaturizer(device)
    raise ValueError('unknown featurizer %r (inception | random)' % name)
