"""Generate tests/golden/*.npz from the float64 oracle (TEST INFRASTRUCTURE).

The reference ships no fixtures and cannot run here (TensorFlow 1.6 absent,
SURVEY.md K7), so these vectors are produced by oracle/smmd_oracle.py, whose
own correctness is pinned by the analytic / finite-difference tests in
tests/test_oracle.py.  Inputs are fp32 (what the GPU path consumes); expected
outputs are float64.

    python oracle/gen_golden.py          # rewrites tests/golden/
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import smmd_oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests', 'golden')

MMD_SHAPES = [(4, 4, 1), (32, 32, 1), (64, 64, 1), (256, 256, 1), (64, 64, 3), (32, 32, 16)]
SN_SHAPES = [(64, 27), (128, 576), (33, 300), (1, 1024)]


def gen_mmd():
    out = {}
    for kname in O.KERNEL_NAMES:
        spec = O.kernel_spec(kname)
        for (m, n, d) in MMD_SHAPES:
            rng = np.random.default_rng(1234 + m * 7 + d)
            X = rng.standard_normal((m, d)).astype(np.float32)
            Y = (rng.standard_normal((n, d)) + 0.25).astype(np.float32)
            for biased in (0, 1):
                key = '%s__%d_%d_%d__b%d' % (kname, m, n, d, biased)
                dX, dY = O.mmd2_grad(spec, X, Y, bool(biased))
                out[key + '__X'] = X
                out[key + '__Y'] = Y
                out[key + '__mmd2'] = np.array(O.mmd2(spec, X, Y, bool(biased)))
                out[key + '__sums'] = O.mmd2_sums(spec, X, Y)
                out[key + '__dX'] = dX
                out[key + '__dY'] = dY
    return out


def gen_sn():
    out = {}
    for (N, K) in SN_SHAPES:
        rng = np.random.default_rng(2 + N + K)
        W = (rng.standard_normal((N, K)) * 0.05).astype(np.float32)
        u = rng.standard_normal(N).astype(np.float32)
        G = rng.standard_normal((N, K)).astype(np.float32)
        s = np.float32(1.25)
        sigma, u1, v1 = O.spectral_norm_rows(W, u)
        gW, gs = O.sn_weight_backward(W, float(s), sigma, u1, v1, G)
        key = 'sn__%d_%d' % (N, K)
        out[key + '__W'] = W
        out[key + '__u'] = u
        out[key + '__G'] = G
        out[key + '__s'] = np.array(s)
        out[key + '__sigma'] = np.array(sigma)
        out[key + '__u1'] = u1
        out[key + '__v1'] = v1
        out[key + '__Weff'] = W.astype(np.float64) / sigma * float(s)
        out[key + '__gW'] = gW
        out[key + '__gs'] = np.array(gs)
    return out


def main():
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, 'mmd2_cases.npz'), **gen_mmd())
    np.savez_compressed(os.path.join(OUT, 'sn_cases.npz'), **gen_sn())
    print('wrote', OUT)


if __name__ == '__main__':
    main()
