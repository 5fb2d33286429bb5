"""TEST-ONLY stand-in for libsmmd_hip.so that runs the oracle on CPU memory,
so the multi-process (gloo) tests can exercise the data-parallel plumbing of
gan.core (all_gather rows, partial sums, all_reduce, row-local gradients,
tower/global gradient exchange) without a GPU.  Never used by the product."""
import ctypes

import numpy as np

from oracle import smmd_oracle as O


def _arr(p, n, dtype=np.float32):
    if p is None:
        return None
    addr = p.value if isinstance(p, ctypes.c_void_p) else int(p)
    if not addr:
        return None
    ct = {np.float32: ctypes.c_float, np.float64: ctypes.c_double,
          np.int64: ctypes.c_int64}[dtype]
    return np.ctypeslib.as_array((ct * n).from_address(addr))


def _spec(desc):
    kinds = {0: 'rbf', 1: 'rq', 2: 'distance', 3: 'dot'}
    k = kinds[desc.kind]
    params = [desc.param[i] for i in range(desc.n_terms)]
    wts = [desc.wt[i] for i in range(desc.n_terms)]
    return O.KernelSpec(k, params, wts, add_dot=desc.add_dot, tanh=bool(desc.tanh_inputs),
                        const_diag=desc.const_diag if desc.has_const_diag else None)


class FakeLib:
    def smmd_mmd2_workspace_bytes(self, m, n, d):
        return 256

    def smmd_mmd2_fwd(self, desc, X, m, Y, n, d, biased, xb, xe, yb, ye, sums, out, gx, gy, ws,
                      wsb, stream):
        spec = _spec(desc)
        Xa = _arr(X, m * d).reshape(m, d).astype(np.float64)
        Ya = _arr(Y, n * d).reshape(n, d).astype(np.float64)
        KXX, KXY, KYY, _ = O.kernel_matrices(spec, Xa, Ya)
        S = np.zeros(8)
        S[0] = KXX[xb:xe].sum()
        S[1] = KXY[xb:xe].sum()
        S[2] = KYY[yb:ye].sum()
        S[3] = np.trace(KXX[xb:xe, xb:xe]) if xe > xb else 0.0
        S[4] = np.trace(KYY[yb:ye, yb:ye]) if ye > yb else 0.0
        S[5] = KXY[:, yb:ye].sum()
        _arr(sums, 8)[:] = S
        if out is not None and _arr(out, 1) is not None:
            _arr(out, 1)[0] = O.mmd2_from_K(KXX, KXY, KYY, spec.const_diag, bool(biased)) \
                if (xe - xb == m and ye - yb == n) else 0.0
        if _arr(gx, 1) is not None:
            dX, dY = O.mmd2_grad(spec, Xa, Ya, bool(biased))
            _arr(gx, (xe - xb) * d)[:] = dX[xb:xe].ravel()
            _arr(gy, (ye - yb) * d)[:] = dY[yb:ye].ravel()
        return 0

    def smmd_mmd2_combine(self, desc, sums, m, n, biased, out, stream):
        S = _arr(sums, 8).astype(np.float64)
        spec = _spec(desc)
        if biased:
            v = S[0] / m ** 2 + S[2] / n ** 2 - 2 * S[1] / (m * n)
        else:
            trX = m * spec.const_diag if spec.const_diag is not None else S[3]
            trY = n * spec.const_diag if spec.const_diag is not None else S[4]
            v = (S[0] - trX) / (m * (m - 1)) + (S[2] - trY) / (n * (n - 1)) - 2 * S[1] / (m * n)
        _arr(out, 1)[0] = v
        return 0

    def smmd_scaled_loss_workspace_bytes(self, rows, per):
        return 256

    def smmd_scaled_loss_fwd(self, jac, n_cols, b, b_total, per, feat, dof, base, sc, variant,
                             sqrt_scale, out, per_sample, ws, wsb, stream):
        J = _arr(jac, n_cols * b * per).reshape(n_cols, b, per).astype(np.float64)
        ps = (J ** 2).sum(axis=(0, 2))
        if _arr(per_sample, 1) is not None:
            _arr(per_sample, b)[:] = ps
        o = _arr(out, 8)
        Jm = ps.sum() / b_total
        nD = 0.0
        if variant == 1:
            f = _arr(feat, b * dof).astype(np.float64)
            nD = (f ** 2).sum() / (b_total * dof)
        bl = float(_arr(base, 1)[0]) if _arr(base, 1) is not None else 0.0
        o[3], o[4], o[5] = Jm, nD, bl
        return self.smmd_scaled_loss_finalize(out, sc, variant, sqrt_scale, stream)

    def smmd_scaled_loss_finalize(self, out, sc, variant, sqrt_scale, stream):
        o = _arr(out, 8)
        q = o[3] + o[4] if variant == 1 else o[3]
        scale = 1.0 / (sc * q + 1.0)
        g = o[5] * (np.sqrt(scale) if sqrt_scale else scale)
        o[0], o[1], o[2] = g, -g, scale
        return 0

    def smmd_scaled_loss_bwd(self, jac, n_cols, b, b_total, per, feat, dof, fwd, sc, variant,
                             sqrt_scale, go, d_base, gjac, gfeat, stream):
        o = _arr(fwd, 8).astype(np.float64)
        g = float(_arr(go, 1)[0]) if _arr(go, 1) is not None else 1.0
        scale, base = o[2], o[5]
        f = np.sqrt(scale) if sqrt_scale else scale
        fp = 0.5 / np.sqrt(scale) if sqrt_scale else 1.0
        cq = g * base * fp * (-sc * scale * scale)
        if _arr(d_base, 1) is not None:
            _arr(d_base, 1)[0] = g * f
        n = n_cols * b * per
        _arr(gjac, n)[:] = cq * 2.0 / b_total * _arr(jac, n)
        if variant == 1 and _arr(gfeat, 1) is not None:
            _arr(gfeat, b * dof)[:] = cq * 2.0 / (b_total * dof) * _arr(feat, b * dof)
        return 0

    def smmd_smmd_loss_fwd(self, desc, X, m, Y, n, d, biased, jac, n_cols, b, per, feat, dof, sc,
                           variant, sqrt_scale, sums, mm, gx, gy, out, per_sample, ws, wsb, lws,
                           lwsb, stream):
        self.smmd_mmd2_fwd(desc, X, m, Y, n, d, biased, 0, m, 0, n, sums, mm, gx, gy, ws, wsb,
                           stream)
        return self.smmd_scaled_loss_fwd(jac, n_cols, b, b, per, feat, dof, mm, sc, variant,
                                         sqrt_scale, out, per_sample, lws, lwsb, stream)

    def smmd_smmd_loss_fwd_gathered(self, desc, X, m, Y, n, d, biased, stats, world, stride, sc,
                                    variant, sqrt_scale, sums, mm, gx, gy, out, ws, wsb, lws,
                                    lwsb, stream):
        self.smmd_mmd2_fwd(desc, X, m, Y, n, d, biased, 0, m, 0, n, sums, mm, gx, gy, ws, wsb,
                           stream)
        st = _arr(stats, (world - 1) * stride + 2)
        o = _arr(out, 8)
        J, nD = np.float32(st[0]), np.float32(st[1])
        for r in range(1, world):             # rank order, fp32 as the kernel
            J = np.float32(J + st[r * stride])
            nD = np.float32(nD + st[r * stride + 1])
        o[3], o[4], o[5] = J, nD, _arr(mm, 1)[0]
        return self.smmd_scaled_loss_finalize(out, sc, variant, sqrt_scale, stream)

    def smmd_smmd_loss_bwd(self, jac, n_cols, b, per, feat, dof, fwd, sc, variant, sqrt_scale, go,
                           gm, gx, m, gy, n, d, gjac, gfeat, dX, dY, stream):
        return self.smmd_smmd_loss_bwd_ex(jac, n_cols, b, b, per, feat, dof, fwd, sc, variant,
                                          sqrt_scale, go, gm, gx, m, gy, n, d, gjac, gfeat, dX, dY,
                                          stream)

    def smmd_smmd_loss_bwd_ex(self, jac, n_cols, b, b_total, per, feat, dof, fwd, sc, variant,
                              sqrt_scale, go, gm, gx, m, gy, n, d, gjac, gfeat, dX, dY, stream):
        o = _arr(fwd, 8).astype(np.float64)
        f = np.sqrt(o[2]) if sqrt_scale else o[2]
        g = float(_arr(go, 1)[0])
        dm = (float(_arr(gm, 1)[0]) if _arr(gm, 1) is not None else 0.0) + g * f
        _arr(dX, m * d)[:] = _arr(gx, m * d) * dm
        _arr(dY, n * d)[:] = _arr(gy, n * d) * dm
        if _arr(gjac, 1) is not None:
            self.smmd_scaled_loss_bwd(jac, n_cols, b, b_total, per, feat, dof, fwd, sc, variant,
                                      sqrt_scale, go, None, gjac, gfeat, stream)
        return 0

    # spectral norm (fold = 0 layers): u' of each layer kept per workspace, as
    # the library keeps it in ws between the refresh and the backward
    _ucur = {}

    def smmd_sn_workspace_bytes(self, arr, n):
        return 256

    def _layer(self, L):
        N, K = L.N, L.K
        W = _arr(L.W, N * K).reshape(N, K).astype(np.float64)
        s = float(_arr(L.s, 1)[0]) if L.s else 1.0
        return N, K, W, s

    def smmd_sn_power_iter_ex(self, arr, n, iters, eps, update_u, flags, ws, wsb, stream):
        key = ws.value if isinstance(ws, ctypes.c_void_p) else int(ws or 0)
        for i in range(n):
            L = arr[i]
            assert not L.fold, 'fake_lib: fold layers are GPU-only'
            N, K, W, s = self._layer(L)
            sigma, u1, v1 = O.spectral_norm_rows(W, _arr(L.u, N).astype(np.float64), iters)
            _arr(L.v, K)[:] = v1
            _arr(L.sigma, 1)[0] = sigma
            if update_u:
                _arr(L.u, N)[:] = u1
            self._ucur[(key, i)] = u1
            if L.W_eff:
                _arr(L.W_eff, N * K)[:] = ((W.astype(np.float32) / np.float32(sigma))
                                           * np.float32(s)).ravel()
        return 0

    def smmd_sn_weight_bwd(self, arr, n, ws, wsb, stream):
        key = ws.value if isinstance(ws, ctypes.c_void_p) else int(ws or 0)
        for i in range(n):
            L = arr[i]
            if not L.G:
                continue
            N, K, W, s = self._layer(L)
            G = _arr(L.G, N * K).reshape(N, K)
            sigma = float(_arr(L.sigma, 1)[0])
            gW, gs = O.sn_weight_backward(W, s, sigma, self._ucur[(key, i)],
                                          _arr(L.v, K).astype(np.float64), G)
            _arr(L.gW, N * K)[:] = gW.ravel()
            if L.gs:
                _arr(L.gs, 1)[0] = gs
        return 0

    # G-direct: smmd_sn_grad_stats keeps the layer's dL/dW (the "record") per
    # workspace for the fused update, and writes dL/ds
    _gd = {}

    def smmd_sn_grad_stats(self, arr, n, ws, wsb, stream):
        key = ws.value if isinstance(ws, ctypes.c_void_p) else int(ws or 0)
        for i in range(n):
            L = arr[i]
            if not L.G:
                continue
            assert not L.fold, 'fake_lib: fold layers are GPU-only'
            N, K, W, s = self._layer(L)
            G = _arr(L.G, N * K).reshape(N, K).astype(np.float64)
            sigma = float(_arr(L.sigma, 1)[0])
            gW, gs = O.sn_weight_backward(W, s, sigma, self._ucur[(key, i)],
                                          _arr(L.v, K).astype(np.float64), G)
            self._gd[(key, i)] = gW.ravel()
            if L.gs:
                _arr(L.gs, 1)[0] = gs
        return 0

    def smmd_sn_clip_g(self, arr, n, clip, ws, wsb, stream):
        key = ws.value if isinstance(ws, ctypes.c_void_p) else int(ws or 0)
        for i in range(n):
            L = arr[i]
            if not L.G:
                continue
            N, K = L.N, L.K
            gW = self._gd[(key, i)]
            f = clip / max(float(np.sqrt((gW ** 2).sum())), clip)
            G = _arr(L.G, N * K)
            G[:] = (G.astype(np.float64) * f).astype(np.float32)
            if L.gs:
                g = float(_arr(L.gs, 1)[0])
                _arr(L.gs, 1)[0] = g * clip / max(abs(g), clip)
        return 0

    def smmd_adam_flat_sn2(self, param, grad, m, v, offs, n, gscale, clip, lr, b1, b2, eps, step,
                           lr_dev, ws, wsb, layers, idx, nl, snws, snwsb, flags, stream):
        """The fused update: with SMMD_ADAM_SN_GDIRECT the SN weights' gradient
        is the dL/dW smmd_sn_grad_stats formed from G; the P1 pass is not
        modelled (the fake refresh ignores SN_P1_READY)."""
        key = snws.value if isinstance(snws, ctypes.c_void_p) else int(snws or 0)
        tot = offs[n]
        P, G, M, V = (_arr(x, tot) for x in (param, grad, m, v))
        sn_of = {int(idx[k]): k for k in range(nl)} if flags & 1 else {}
        for i, (a, b) in enumerate(self._tensors(offs, n)):
            if b == a:
                continue
            g = G[a:b].astype(np.float64)
            if i in sn_of:                # dL/dW of the record (offsets are padded)
                d = self._gd[(key, sn_of[i])]
                g = np.zeros(b - a)
                g[:d.size] = d
            g = g * gscale
            if clip > 0:
                g = O.clip_by_norm(g, clip)
            p, mm, vv = O.adam_step(P[a:b].astype(np.float64), M[a:b].astype(np.float64),
                                    V[a:b].astype(np.float64), g, step, lr, b1, b2, eps)
            P[a:b], M[a:b], V[a:b] = p, mm, vv
        return 0

    def smmd_opt_workspace_bytes(self, offs, n):
        return 256

    def _tensors(self, offs, n):
        return [(offs[i], offs[i + 1]) for i in range(n)]

    def smmd_clip_by_norm_flat(self, grad, offs, n, clip, ws, wsb, stream):
        tot = offs[n]
        g = _arr(grad, tot)
        for a, b in self._tensors(offs, n):
            if b > a:
                g[a:b] = O.clip_by_norm(g[a:b], clip)
        return 0

    def smmd_adam_flat(self, param, grad, m, v, offs, n, gscale, clip, lr, b1, b2, eps, step, ws,
                       wsb, stream):
        tot = offs[n]
        P, G, M, V = (_arr(x, tot) for x in (param, grad, m, v))
        for a, b in self._tensors(offs, n):
            if b == a:
                continue
            g = G[a:b].astype(np.float64) * gscale
            if clip > 0:
                g = O.clip_by_norm(g, clip)
            p, mm, vv = O.adam_step(P[a:b].astype(np.float64), M[a:b].astype(np.float64),
                                    V[a:b].astype(np.float64), g, step, lr, b1, b2, eps)
            P[a:b], M[a:b], V[a:b] = p, mm, vv
        return 0

    def smmd_status_string(self, s):
        return b'fake'


def install(monkeypatch=None):
    """Route gan.core._lib to the fake (CPU tensors allowed)."""
    import torch
    from gan.core import _lib
    fake = FakeLib()
    _lib._lib = fake
    _lib.lib = lambda: fake
    _lib.require_cuda = lambda *t: None
    _lib.stream_handle = lambda device=None: None
    _lib.workspace = lambda tag, nbytes, device: torch.zeros(max(int(nbytes), 256),
                                                             dtype=torch.uint8)
    return fake
