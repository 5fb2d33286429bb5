// smmd_mmd.hip -- fused pairwise MMD^2 forward + unit gradient, and the
// witness function of the gradient penalty, for gfx950 (MI355X).
//
// Reference being replaced:
//   gan/core/mmd.py:18-188  kernel family (Gram expansion, clamp, exp/log)
//   gan/core/mmd.py:194-220 unbiased / biased estimator
//   gan/core/model.py:327-350 witness (K_XY_only row means) of the GP
// The TF graph materialises three N x N matrices and runs ~7 elementwise
// launches per matrix plus the same again for autodiff.  Here one launch
// sweeps the rows of Z = [X; Y]: each wave owns one row, its 64 lanes stride
// over all m + n columns, evaluate K and dK together (they share the exp),
// and the row's gradient d mmd2 / d z_i is complete inside the wave (no
// cross-block reduction for gradients).  Block sums go to a double-precision
// slab; the last-arriving block reduces the slab in a fixed order (agent-scope
// release/acquire, CDNA4 guide G16) and writes the estimator.
#include "smmd_common.hpp"
#include "smmd_kern.hpp"
#include "smmd_scale_dev.hpp"

#include <stdlib.h>

namespace smmd {

template <int DT>
__device__ __forceinline__ void load_feat(const float *__restrict__ p, int d, bool tanh_in,
                                          float (&z)[DT]) {
#pragma unroll
    for (int k = 0; k < DT; ++k) z[k] = (k < d) ? p[k] : 0.f;
    if (tanh_in) {
#pragma unroll
        for (int k = 0; k < DT; ++k) z[k] = tanhf(z[k]);
    }
}

// <a, b> as a k-ordered fma chain: the same routine produces the Gram entries
// and the squared norms, so raw D2 is exactly 0 on the diagonal as it is for
// the reference's diag_part(XX) (mmd.py:60-67).
template <int DT>
__device__ __forceinline__ float dotk(const float (&a)[DT], const float (&b)[DT]) {
    float s = a[0] * b[0];
#pragma unroll
    for (int k = 1; k < DT; ++k) s = fmaf(a[k], b[k], s);
    return s;
}

struct MmdArgs {
    const float *X;
    const float *Y;
    int m, n, d;
    int x_begin, x_end, y_begin, y_end;
    int tanh_in;
    int trace_mode;      // exclude j == i from the gradient (const_diag False, unbiased)
    int need_grad;
    float gw_same_x, gw_same_y, gw_cross;   // gradient weights per block
    float *grad_x;
    float *grad_y;
    double *partials;    // [gridDim.x][8]
    unsigned *counter;
    float *out_sums;
    float *out_mmd2;
    int biased;
    int has_const;
    double const_diag;
    KParams kp;
};

// NW waves per block.  A one-block launch (small batches: the configs' 64+64
// rows) reduces in LDS and writes the outputs directly; larger launches use
// the slab + last-arriver path.  STAGED: the block first copies every feature
// row of Z = [X; Y] (tanh applied) and its squared norm into LDS, so the row
// and column sweeps read LDS instead of issuing dependent global loads.
template <int DT, bool STAGED>
struct Feats {
    const float *X, *Y;
    const float *lds;      // [(m+n)][DT] features, then [(m+n)] squared norms
    int m, n, d;
    bool tanh_in;
    __device__ __forceinline__ void get(bool isx, int i, float (&z)[DT], float &sq) const {
        if (STAGED) {
            const int r = isx ? i : m + i;
#pragma unroll
            for (int k = 0; k < DT; ++k) z[k] = lds[r * DT + k];
            sq = lds[(m + n) * DT + r];
        } else {
            load_feat<DT>((isx ? X : Y) + (size_t)i * d, d, tanh_in, z);
            sq = dotk<DT>(z, z);
        }
    }
};

// Lane layout: a wave owns 8 rows; row slot = lane >> 3 and the 8 lanes of a
// slot stride over the columns (j = lane & 7, +8, ...).  The row's kernel sums
// and gradient are reduced over those 8 lanes only (3 xor-shuffle steps), so
// the per-row overhead is shared by 8 rows.
constexpr int MMD_RPW = 8;    // rows per wave
constexpr int MMD_LPR = 8;    // lanes per row

__device__ __forceinline__ float group8_sum(float x) {
    x += __shfl_xor(x, 4, SMMD_WAVE);
    x += __shfl_xor(x, 2, SMMD_WAVE);
    x += __shfl_xor(x, 1, SMMD_WAVE);
    return x;
}

template <int DT, int KIND, int NW, bool STAGED>
__global__ __launch_bounds__(NW * 64) void mmd2_fused_kernel(MmdArgs a) {
    extern __shared__ float smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int slot = lane >> 3, l8 = lane & 7;
    const int nwaves = gridDim.x * NW;
    const int nxr = a.x_end - a.x_begin;
    const int nrows = nxr + (a.y_end - a.y_begin);
    const bool tanh_in = a.tanh_in != 0;
    Feats<DT, STAGED> F{a.X, a.Y, smem, a.m, a.n, a.d, tanh_in};

    if (STAGED) {
        const int tot = a.m + a.n;
        for (int r = threadIdx.x; r < tot; r += NW * 64) {
            float z[DT];
            const bool isx = r < a.m;
            load_feat<DT>((isx ? a.X : a.Y) + (size_t)(isx ? r : r - a.m) * a.d, a.d, tanh_in, z);
#pragma unroll
            for (int k = 0; k < DT; ++k) smem[r * DT + k] = z[k];
            smem[tot * DT + r] = dotk<DT>(z, z);
        }
        __syncthreads();
    }

    float s_xx = 0.f, s_xy = 0.f, s_yy = 0.f, s_yx = 0.f, t_xx = 0.f, t_yy = 0.f;

    for (int g = blockIdx.x * NW + wid; g * MMD_RPW < nrows; g += nwaves) {
        const int r = g * MMD_RPW + slot;
        const bool active = r < nrows;
        const bool isx = r < nxr;
        const int ri = isx ? a.x_begin + r : a.y_begin + (r - nxr);
        float zi[DT], sqi = 0.f;
#pragma unroll
        for (int k = 0; k < DT; ++k) zi[k] = 0.f;
        if (active) F.get(isx, ri, zi, sqi);
        float acc[DT];
#pragma unroll
        for (int k = 0; k < DT; ++k) acc[k] = 0.f;
        float aacc = 0.f;

        // same-set block: XX for an X row, YY for a Y row
        {
            const int ns = active ? (isx ? a.m : a.n) : 0;
            const float w = isx ? a.gw_same_x : a.gw_same_y;
            float sumK = 0.f, trK = 0.f;
            for (int j = l8; j < ns; j += MMD_LPR) {
                float zc[DT], sqc;
                F.get(isx, j, zc, sqc);
                const float dot = dotk<DT>(zi, zc);
                const float raw = (-2.f * dot + sqi) + sqc;   // mmd.py:67 order
                float K, al, be;
                Kern<KIND>::eval(a.kp, raw, dot, sqi, sqc, K, al, be);
                sumK += K;
                const bool diag = (j == ri);
                if (diag) trK += K;
                if (a.need_grad && !(diag && a.trace_mode)) {
                    aacc = fmaf(w, al, aacc);
                    const float c = w * be;
#pragma unroll
                    for (int k = 0; k < DT; ++k) acc[k] = fmaf(c, zi[k] - zc[k], acc[k]);
                }
            }
            if (isx) { s_xx += sumK; t_xx += trK; } else { s_yy += sumK; t_yy += trK; }
        }
        // cross-set block: XY for an X row; YX (gradient only) for a Y row
        {
            const int ns = (active && (isx || a.need_grad)) ? (isx ? a.n : a.m) : 0;
            const float w = a.gw_cross;
            float sumK = 0.f;
            for (int j = l8; j < ns; j += MMD_LPR) {
                float zc[DT], sqc;
                F.get(!isx, j, zc, sqc);
                const float dot = dotk<DT>(zi, zc);
                const float raw = (-2.f * dot + sqi) + sqc;
                float K, al, be;
                Kern<KIND>::eval(a.kp, raw, dot, sqi, sqc, K, al, be);
                sumK += K;
                if (a.need_grad) {
                    aacc = fmaf(w, al, aacc);
                    const float c = w * be;
#pragma unroll
                    for (int k = 0; k < DT; ++k) acc[k] = fmaf(c, zi[k] - zc[k], acc[k]);
                }
            }
            if (isx) s_xy += sumK; else s_yx += sumK;
        }
        if (a.need_grad) {
            aacc = group8_sum(aacc);
#pragma unroll
            for (int k = 0; k < DT; ++k) acc[k] = group8_sum(acc[k]);
            if (active && l8 == 0) {
                float *gp = isx ? a.grad_x + (size_t)r * a.d : a.grad_y + (size_t)(r - nxr) * a.d;
#pragma unroll
                for (int k = 0; k < DT; ++k) {
                    if (k < a.d) {
                        float gk = fmaf(aacc, zi[k], acc[k]);
                        if (tanh_in) gk *= 1.f - zi[k] * zi[k];
                        gp[k] = gk;
                    }
                }
            }
        }
    }

    // ---- block partial sums (fixed order), double precision ---------------
    __shared__ double red[NW][8];
    __shared__ int is_last;
    float v[6] = {s_xx, s_xy, s_yy, t_xx, t_yy, s_yx};
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) red[wid][k] = (double)v[k];
    }
    __syncthreads();
    if (gridDim.x == 1) {                       // one block: no slab, no ticket
        if (threadIdx.x == 0) {
            double S[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                double t = 0.0;
                for (int w = 0; w < NW; ++w) t += red[w][k];
                S[k] = t;
            }
            if (a.out_sums) {
#pragma unroll
                for (int k = 0; k < 6; ++k) a.out_sums[k] = (float)S[k];
                a.out_sums[6] = 0.f;
                a.out_sums[7] = 0.f;
            }
            if (a.out_mmd2)
                a.out_mmd2[0] = (float)estimator(S, (double)a.m, (double)a.n, a.biased,
                                                 a.has_const, a.const_diag);
        }
        return;
    }
    if (threadIdx.x == 0) {
        double *slab = a.partials + (size_t)blockIdx.x * 8;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            double t = 0.0;
            for (int w = 0; w < NW; ++w) t += red[w][k];
            slab[k] = t;
        }
        // publish: release at agent scope, then the ticket (CDNA4 guide G16)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev =
            __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!is_last || wid != 0) return;

    // ---- last arriver: reduce all slabs in block order -------------------
    if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double S[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) S[k] = 0.0;
    for (int b = lane; b < (int)gridDim.x; b += 64) {
        const double *slab = a.partials + (size_t)b * 8;
#pragma unroll
        for (int k = 0; k < 6; ++k) S[k] += slab[k];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) S[k] = wave_sum(S[k]);
    if (lane == 0) {
        if (a.out_sums) {
            a.out_sums[0] = (float)S[0];
            a.out_sums[1] = (float)S[1];
            a.out_sums[2] = (float)S[2];
            a.out_sums[3] = (float)S[3];
            a.out_sums[4] = (float)S[4];
            a.out_sums[5] = (float)S[5];
            a.out_sums[6] = 0.f;
            a.out_sums[7] = 0.f;
        }
        if (a.out_mmd2)
            a.out_mmd2[0] =
                (float)estimator(S, (double)a.m, (double)a.n, a.biased, a.has_const, a.const_diag);
        __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void mmd2_combine_kernel(const float *sums, double m, double n, int biased,
                                    int has_const, double c, float *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        double S[6];
        for (int k = 0; k < 6; ++k) S[k] = (double)sums[k];
        out[0] = (float)estimator(S, m, n, biased, has_const, c);
    }
}

// ---------------------------------------------------------------------------
// witness:  w_i = mean_j K(h_i, r_j) - mean_j K(h_i, f_j)   (model.py:336-338)
// dH_i = d(sum w)/dh_i.  One wave per row of H, lanes stride over R then F.
// ---------------------------------------------------------------------------
struct WitArgs {
    const float *H;
    const float *R;
    const float *F;
    int b, nr, nf, d;
    int tanh_in;
    float *out_w;
    float *out_dH;
    KParams kp;
};

template <int DT, int KIND>
__global__ __launch_bounds__(256) void witness_fwd_kernel(WitArgs a) {
    const int lane = threadIdx.x & 63;
    const int nwaves = gridDim.x * 4;
    const bool tanh_in = a.tanh_in != 0;
    for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < a.b; i += nwaves) {
        float hi[DT];
        load_feat<DT>(a.H + (size_t)i * a.d, a.d, tanh_in, hi);
        const float sqi = dotk<DT>(hi, hi);
        float acc[DT];
#pragma unroll
        for (int k = 0; k < DT; ++k) acc[k] = 0.f;
        float aacc = 0.f, wsum[2] = {0.f, 0.f};
#pragma unroll
        for (int set = 0; set < 2; ++set) {
            const float *S = set == 0 ? a.R : a.F;
            const int ns = set == 0 ? a.nr : a.nf;
            const float w = (set == 0 ? 1.f : -1.f) / (float)ns;
            for (int j = lane; j < ns; j += 64) {
                float zc[DT];
                load_feat<DT>(S + (size_t)j * a.d, a.d, tanh_in, zc);
                const float dot = dotk<DT>(hi, zc);
                const float sqc = dotk<DT>(zc, zc);
                const float raw = (-2.f * dot + sqi) + sqc;
                float K, al, be;
                Kern<KIND>::eval(a.kp, raw, dot, sqi, sqc, K, al, be);
                wsum[set] += K;
                aacc = fmaf(w, al, aacc);
                const float c = w * be;
#pragma unroll
                for (int k = 0; k < DT; ++k) acc[k] = fmaf(c, hi[k] - zc[k], acc[k]);
            }
        }
        const float sr = wave_sum(wsum[0]), sf = wave_sum(wsum[1]);
        aacc = wave_sum(aacc);
#pragma unroll
        for (int k = 0; k < DT; ++k) acc[k] = wave_sum(acc[k]);
        if (lane == 0) {
            // reduce_mean over axis 1 of each K_XY block (model.py:336)
            if (a.out_w) a.out_w[i] = sr / (float)a.nr - sf / (float)a.nf;
            if (a.out_dH) {
#pragma unroll
                for (int k = 0; k < DT; ++k)
                    if (k < a.d) {
                        float g = fmaf(aacc, hi[k], acc[k]);
                        if (tanh_in) g *= 1.f - hi[k] * hi[k];
                        a.out_dH[(size_t)i * a.d + k] = g;
                    }
            }
        }
    }
}

// Second order of the witness gradient, for every kernel of the family.
// With h = tanh(x) for the tanh kernels (else h = x), the forward gives
//   dX_i = T_i * G_i,  G_i = sum_j c_j [al_i h_i + be_ij (h_i - z_j)],
//   T_i = 1 - h_i^2 (tanh) or 1,
// where al depends on |h_i|^2 only (grad_h al = a1 h_i) and be on the pair
// distance raw_ij only (grad_h be = b1 (h_i - z_j) = -grad_z be).  For
// L = sum_i <g_i, dX_i> and gt_i = g_i * T_i:
//   dL/dh_i = (sum_j c_j (al + be_ij)) gt_i + a1 <gt_i, h_i> (sum_j c_j) h_i
//             + sum_j c_j b1_ij <gt_i, d_ij> d_ij  [- 2 h_i g_i G_i  (tanh)]
//   dL/dz_j = sum_i -c_j be_ij gt_i - c_j b1_ij <gt_i, d_ij> d_ij,
// d_ij = h_i - z_j, each then times (1 - h^2) / (1 - z^2) for tanh inputs.
//   rbf / rq:  be = 2 f'(R) [raw >= 0] - add_dot, b1 = 4 f''(R) [raw >= 0],
//              al = add_dot, a1 = 0                      (mmd.py:55-188)
//   distance:  be = -2 s'(raw), b1 = -4 s''(raw), al = 2 s'(|h|^2),
//              a1 = 4 s''(|h|^2), s(x) = sqrt(max(x + 1e-5, 0))  (mmd.py:12-37)
//   dot:       al = 1, be = -1, a1 = b1 = 0              (mmd.py:44-52)
__device__ __forceinline__ void mysqrt_d12(float x, float &d1, float &d2) {
    const float xe = x + 1.0e-5f;
    if (xe >= 0.f) {            // tf.maximum: ties pass the gradient
        const float r = 1.f / sqrtf(xe);
        d1 = 0.5f * r;
        d2 = -0.25f * r * r * r;
    } else {
        d1 = 0.f;
        d2 = 0.f;
    }
}

template <int KIND>
__device__ __forceinline__ void pair_d2(const KParams &p, float raw, float &be, float &b1) {
    if (KIND == SMMD_KIND_DISTANCE) {
        float d1, d2;
        mysqrt_d12(raw, d1, d2);
        be = -2.f * d1;
        b1 = -4.f * d2;
    } else if (KIND == SMMD_KIND_DOT) {
        be = -1.f;
        b1 = 0.f;
    } else {
        const float R = fmaxf(raw, 0.f);
        float d1 = 0.f, d2 = 0.f;
        if (KIND == SMMD_KIND_RBF) {
            for (int t = 0; t < p.n_terms; ++t) {
                const float e = p.wt[t] * expf(p.c1[t] * R);
                d1 += p.c1[t] * e;
                d2 += p.c1[t] * p.c1[t] * e;
            }
        } else {
            for (int t = 0; t < p.n_terms; ++t) {
                const float q = 1.f + R / p.c1[t];
                const float e = p.wt[t] * expf(p.c2[t] * logf(q));
                const float dq = 1.f / p.c1[t];
                const float g1 = e * p.c2[t] / q * dq;                     // de/dR
                d1 += g1;
                d2 += g1 * (p.c2[t] - 1.f) / q * dq;                       // d2e/dR2
            }
        }
        const bool pass = raw >= 0.f;
        be = (pass ? 2.f * d1 : 0.f) - (KIND == SMMD_KIND_RQ ? p.add_dot : 0.f);
        b1 = pass ? 4.f * d2 : 0.f;
    }
}

template <int KIND>
__device__ __forceinline__ void row_d2(const KParams &p, float sqi, float &al, float &a1) {
    if (KIND == SMMD_KIND_DISTANCE) {
        float d1, d2;
        mysqrt_d12(sqi, d1, d2);
        al = 2.f * d1;
        a1 = 4.f * d2;
    } else {
        al = KIND == SMMD_KIND_DOT ? 1.f : (KIND == SMMD_KIND_RQ ? p.add_dot : 0.f);
        a1 = 0.f;
    }
}

struct WitBwdArgs {
    const float *H;
    const float *R;
    const float *F;
    const float *gdH;
    int b, nr, nf, d;
    int tanh_in;
    float *gH;
    float *gR;
    float *gF;
    KParams kp;
};

// rows of H: dL/dh_i
template <int DT, int KIND>
__global__ __launch_bounds__(256) void witness_bwd_h_kernel(WitBwdArgs a) {
    const int lane = threadIdx.x & 63;
    const int nwaves = gridDim.x * 4;
    const bool tanh_in = a.tanh_in != 0;
    for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < a.b; i += nwaves) {
        float hi[DT], gi[DT], gt[DT], acc[DT], gb[DT];
        load_feat<DT>(a.H + (size_t)i * a.d, a.d, tanh_in, hi);
        load_feat<DT>(a.gdH + (size_t)i * a.d, a.d, false, gi);
#pragma unroll
        for (int k = 0; k < DT; ++k) {
            gt[k] = tanh_in ? gi[k] * (1.f - hi[k] * hi[k]) : gi[k];
            acc[k] = 0.f;
            gb[k] = 0.f;
        }
        const float sqi = dotk<DT>(hi, hi);
        float al, a1;
        row_d2<KIND>(a.kp, sqi, al, a1);
        float cbe = 0.f, csum = 0.f;
#pragma unroll
        for (int set = 0; set < 2; ++set) {
            const float *S = set == 0 ? a.R : a.F;
            const int ns = set == 0 ? a.nr : a.nf;
            const float c = (set == 0 ? 1.f : -1.f) / (float)ns;
            for (int j = lane; j < ns; j += 64) {
                float zc[DT], df[DT];
                load_feat<DT>(S + (size_t)j * a.d, a.d, tanh_in, zc);
                const float raw = (-2.f * dotk<DT>(hi, zc) + sqi) + dotk<DT>(zc, zc);
                float be, b1;
                pair_d2<KIND>(a.kp, raw, be, b1);
#pragma unroll
                for (int k = 0; k < DT; ++k) df[k] = hi[k] - zc[k];
                const float e = c * b1 * dotk<DT>(gt, df);
                csum += c;
                cbe = fmaf(c, be, cbe);
#pragma unroll
                for (int k = 0; k < DT; ++k) {
                    acc[k] = fmaf(e, df[k], acc[k]);
                    if (tanh_in) gb[k] = fmaf(c * be, df[k], gb[k]);
                }
            }
        }
        cbe = wave_sum(cbe);
        csum = wave_sum(csum);
#pragma unroll
        for (int k = 0; k < DT; ++k) {
            acc[k] = wave_sum(acc[k]);
            if (tanh_in) gb[k] = wave_sum(gb[k]);
        }
        if (lane == 0) {
            const float gcoef = fmaf(al, csum, cbe);
            const float hcoef = a1 * csum * dotk<DT>(gt, hi);
#pragma unroll
            for (int k = 0; k < DT; ++k)
                if (k < a.d) {
                    float v = fmaf(gcoef, gt[k], fmaf(hcoef, hi[k], acc[k]));
                    if (tanh_in) {
                        const float G = fmaf(al * csum, hi[k], gb[k]);
                        v = fmaf(-2.f * hi[k] * gi[k], G, v);
                        v *= 1.f - hi[k] * hi[k];
                    }
                    a.gH[(size_t)i * a.d + k] = v;
                }
        }
    }
}

// rows of R then F: dL/dz_j (a sweep over H per column point)
template <int DT, int KIND>
__global__ __launch_bounds__(256) void witness_bwd_z_kernel(WitBwdArgs a) {
    const int lane = threadIdx.x & 63;
    const int nwaves = gridDim.x * 4;
    const int nz = a.nr + a.nf;
    const bool tanh_in = a.tanh_in != 0;
    for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < nz; r += nwaves) {
        const bool isr = r < a.nr;
        const int j = isr ? r : r - a.nr;
        const float c = (isr ? 1.f : -1.f) / (float)(isr ? a.nr : a.nf);
        float zj[DT], acc[DT];
        load_feat<DT>((isr ? a.R : a.F) + (size_t)j * a.d, a.d, tanh_in, zj);
        const float sqj = dotk<DT>(zj, zj);
#pragma unroll
        for (int k = 0; k < DT; ++k) acc[k] = 0.f;
        for (int i = lane; i < a.b; i += 64) {
            float hi[DT], gt[DT], df[DT];
            load_feat<DT>(a.H + (size_t)i * a.d, a.d, tanh_in, hi);
            load_feat<DT>(a.gdH + (size_t)i * a.d, a.d, false, gt);
            if (tanh_in) {
#pragma unroll
                for (int k = 0; k < DT; ++k) gt[k] *= 1.f - hi[k] * hi[k];
            }
            // raw in the forward's order: row = h_i, column = z_j
            const float raw = (-2.f * dotk<DT>(hi, zj) + dotk<DT>(hi, hi)) + sqj;
            float be, b1;
            pair_d2<KIND>(a.kp, raw, be, b1);
#pragma unroll
            for (int k = 0; k < DT; ++k) df[k] = hi[k] - zj[k];
            const float e = c * b1 * dotk<DT>(gt, df);
#pragma unroll
            for (int k = 0; k < DT; ++k) acc[k] = acc[k] - c * be * gt[k] - e * df[k];
        }
#pragma unroll
        for (int k = 0; k < DT; ++k) acc[k] = wave_sum(acc[k]);
        if (lane == 0) {
            float *out = isr ? a.gR : a.gF;
#pragma unroll
            for (int k = 0; k < DT; ++k)
                if (k < a.d) out[(size_t)j * a.d + k] = tanh_in ? acc[k] * (1.f - zj[k] * zj[k])
                                                                 : acc[k];
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static bool make_kparams(const smmd_kernel_desc *desc, KParams &kp) {
    memset(&kp, 0, sizeof(kp));
    if (desc->kind == SMMD_KIND_RBF || desc->kind == SMMD_KIND_RQ) {
        if (desc->n_terms < 1 || desc->n_terms > SMMD_MAX_TERMS) return false;
        kp.n_terms = desc->n_terms;
        for (int t = 0; t < desc->n_terms; ++t) {
            const double s = desc->param[t];
            if (desc->kind == SMMD_KIND_RBF) {
                if (!(s > 0)) return false;
                kp.c1[t] = (float)(-(1.0 / (2.0 * s * s)));   // -gamma, mmd.py:69-70
            } else {
                if (!(s > 0)) return false;
                kp.c1[t] = (float)(2.0 * s);                   // 2.*alpha, mmd.py:166
                kp.c2[t] = (float)(-s);                        // -alpha, mmd.py:167
            }
            kp.wt[t] = (float)desc->wt[t];
        }
        kp.add_dot = (desc->kind == SMMD_KIND_RQ) ? (float)desc->add_dot : 0.f;
        return true;
    }
    return desc->kind == SMMD_KIND_DISTANCE || desc->kind == SMMD_KIND_DOT;
}

static int pick_dt(int d) {
    if (d <= 1) return 1;
    if (d <= 2) return 2;
    if (d <= 4) return 4;
    if (d <= 8) return 8;
    if (d <= 16) return 16;
    if (d <= 32) return 32;
    return 0;
}

// one wave per row, 4 waves per 256-thread block (witness / kernel-matrix sweeps)
static int wave_grid(int rows) {
    int g = (rows + 3) / 4;
    if (g > 2048) g = 2048;
    return g < 1 ? 1 : g;
}

// rows are handed out 8 per wave.  One block (16 waves for DT <= 8, else 4:
// register budget) covers small problems without any cross-block reduction;
// beyond that one-wave blocks, ceil(rows / 8) of them (capped, grid-stride)
static int single_waves(int dt) { return dt <= 8 ? 16 : 4; }

static int mmd2_grid(int rows, int dt) {
    if (rows <= 8 * single_waves(dt)) return 1;
    int g = (rows + 7) / 8;
    if (g > 4096) g = 4096;
    return g < 1 ? 1 : g;
}

constexpr size_t MMD_STAGE_MAX_LDS = 64 * 1024;

template <int DT, int KIND>
static void launch_mmd2(const MmdArgs &a, int grid, hipStream_t s) {
    const size_t lds = (size_t)(a.m + a.n) * (DT + 1) * sizeof(float);
    const bool staged = lds <= MMD_STAGE_MAX_LDS;
    if (grid == 1) {           // one block, 8 rows per wave
        constexpr int NW1 = DT <= 8 ? 16 : 4;
        if (staged)
            hipLaunchKernelGGL((mmd2_fused_kernel<DT, KIND, NW1, true>), dim3(1), dim3(NW1 * 64), lds,
                               s, a);
        else
            hipLaunchKernelGGL((mmd2_fused_kernel<DT, KIND, NW1, false>), dim3(1), dim3(NW1 * 64), 0,
                               s, a);
    } else {                   // one wave (8 rows) per block
        if (staged)
            hipLaunchKernelGGL((mmd2_fused_kernel<DT, KIND, 1, true>), dim3(grid), dim3(64), lds, s, a);
        else
            hipLaunchKernelGGL((mmd2_fused_kernel<DT, KIND, 1, false>), dim3(grid), dim3(64), 0, s, a);
    }
}

template <int KIND>
static bool dispatch_mmd2_dt(int dt, const MmdArgs &a, int grid, hipStream_t s) {
    switch (dt) {
        case 1: launch_mmd2<1, KIND>(a, grid, s); return true;
        case 2: launch_mmd2<2, KIND>(a, grid, s); return true;
        case 4: launch_mmd2<4, KIND>(a, grid, s); return true;
        case 8: launch_mmd2<8, KIND>(a, grid, s); return true;
        case 16: launch_mmd2<16, KIND>(a, grid, s); return true;
        case 32: launch_mmd2<32, KIND>(a, grid, s); return true;
    }
    return false;
}

// ---------------------------------------------------------------------------
// materialised kernel matrix K(A, B) [na, nb] and its backward -- the tuple API
// of mmd._<kind>_kernel (mmd.py:18-188) for callers that index the matrices.
// ---------------------------------------------------------------------------
struct KmArgs {
    const float *A;
    const float *B;
    const float *G;
    int na, nb, d;
    int tanh_in;
    float *out;
    float *gA;
    float *gB;
    KParams kp;
};

template <int DT, int KIND>
__global__ __launch_bounds__(256) void kmat_fwd_kernel(KmArgs a) {
    const int j = blockIdx.x * 64 + (threadIdx.x & 63);
    const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (i >= a.na || j >= a.nb) return;
    const bool t = a.tanh_in != 0;
    float zi[DT], zc[DT];
    load_feat<DT>(a.A + (size_t)i * a.d, a.d, t, zi);
    load_feat<DT>(a.B + (size_t)j * a.d, a.d, t, zc);
    const float dot = dotk<DT>(zi, zc);
    const float sqi = dotk<DT>(zi, zi), sqc = dotk<DT>(zc, zc);
    const float raw = (-2.f * dot + sqi) + sqc;
    float K, al, be;
    Kern<KIND>::eval(a.kp, raw, dot, sqi, sqc, K, al, be);
    a.out[(size_t)i * a.nb + j] = K;
}

// one wave per output row; SIDE 0: rows of A (lanes over j), SIDE 1: rows of B
template <int DT, int KIND, int SIDE>
__global__ __launch_bounds__(256) void kmat_bwd_kernel(KmArgs a) {
    const int lane = threadIdx.x & 63;
    const int nwaves = gridDim.x * 4;
    const int nrows = SIDE == 0 ? a.na : a.nb;
    const int ncols = SIDE == 0 ? a.nb : a.na;
    const bool t = a.tanh_in != 0;
    for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < nrows; r += nwaves) {
        float zr[DT], acc[DT];
        load_feat<DT>((SIDE == 0 ? a.A : a.B) + (size_t)r * a.d, a.d, t, zr);
        const float sqr = dotk<DT>(zr, zr);
#pragma unroll
        for (int k = 0; k < DT; ++k) acc[k] = 0.f;
        float aacc = 0.f;
        for (int c = lane; c < ncols; c += 64) {
            float zc[DT];
            load_feat<DT>((SIDE == 0 ? a.B : a.A) + (size_t)c * a.d, a.d, t, zc);
            const float dot = dotk<DT>(zr, zc);
            const float sqc = dotk<DT>(zc, zc);
            // raw in the forward's orientation (row of A first)
            const float raw = SIDE == 0 ? (-2.f * dot + sqr) + sqc : (-2.f * dot + sqc) + sqr;
            float K, al, be;
            Kern<KIND>::eval(a.kp, raw, dot, sqr, sqc, K, al, be);
            const float g = SIDE == 0 ? a.G[(size_t)r * a.nb + c] : a.G[(size_t)c * a.nb + r];
            aacc = fmaf(g, al, aacc);
            const float cb = g * be;
#pragma unroll
            for (int k = 0; k < DT; ++k) acc[k] = fmaf(cb, zr[k] - zc[k], acc[k]);
        }
        aacc = wave_sum(aacc);
#pragma unroll
        for (int k = 0; k < DT; ++k) acc[k] = wave_sum(acc[k]);
        if (lane == 0) {
            float *o = (SIDE == 0 ? a.gA : a.gB) + (size_t)r * a.d;
#pragma unroll
            for (int k = 0; k < DT; ++k)
                if (k < a.d) {
                    float gk = fmaf(aacc, zr[k], acc[k]);
                    if (t) gk *= 1.f - zr[k] * zr[k];
                    o[k] = gk;
                }
        }
    }
}

}  // namespace smmd

using namespace smmd;

extern "C" {

const char *smmd_status_string(smmd_status s) {
    switch (s) {
        case SMMD_OK: return "SMMD_OK";
        case SMMD_EINVAL: return "SMMD_EINVAL: invalid argument";
        case SMMD_EHIP: return "SMMD_EHIP: HIP runtime/launch error";
        case SMMD_EWORKSPACE: return "SMMD_EWORKSPACE: workspace missing or too small";
        case SMMD_EUNSUPPORTED: return "SMMD_EUNSUPPORTED: not implemented in this build";
    }
    return "SMMD_?: unknown status";
}

int smmd_abi_version(void) { return 17; }

// Path choice.  d > 32: the MFMA Gram path (the row sweep holds a row in
// registers up to 32 features).  d <= 32: the row sweep, except where the
// Gram path measured faster on MI355X (tools/gram_bench.py --paths, rbf fwd +
// grad): d >= 16 from 2 x 512 rows (0.115 vs 0.158 ms at 2 x 1024, d = 16;
// 0.303 vs 0.408 ms at 2 x 2048) and d = 32 from 2 x 256 rows (0.040 vs
// 0.068 ms); d <= 8 stays on the row sweep at every size (0.114 vs 0.303 ms at
// 2 x 2048, d = 1).  SMMD_MMD_GRAM=1 / 0 forces either path (d <= 32).
static bool use_gram(int m, int n, int d) {
    if (pick_dt(d) == 0) return true;
    const char *e = getenv("SMMD_MMD_GRAM");
    if (e && e[0] == '1') return true;
    if (e && e[0] == '0') return false;
    const long rows = (long)(m > 0 ? m : 0) + (n > 0 ? n : 0);
    return (d >= 16 && rows >= 1024) || (d >= 32 && rows >= 512);
}

// d <= 8 (every config: d = 1): the 2-D tiled kernel (smmd_mmd_tile.hip)
// unless SMMD_MMD_TILE=0 selects the row sweep below (A/B, parity tests)
static bool use_tile(int m, int n, int d) {
    if (!tile_supported(d) || use_gram(m, n, d)) return false;
    const char *e = getenv("SMMD_MMD_TILE");
    if (e && e[0] == '0') return false;
    const long rows = (long)(m > 0 ? m : 0) + (n > 0 ? n : 0);
    return rows <= (long)TILE_MAX_RT * 64;
}

size_t smmd_mmd2_workspace_bytes(int m, int n, int d) {
    const int rows = (m > 0 ? m : 0) + (n > 0 ? n : 0);
    if (use_gram(m, n, d)) return MMD_WS_HEADER + gram_ws_bytes(m, n, d);
    size_t b = align_up((size_t)mmd2_grid(rows, pick_dt(d)) * 8 * sizeof(double), 256);
    // the tile path at any row split of this (m, n): at most m + n local rows
    if (tile_supported(d)) {
        const size_t t = tile_ws_bytes(rows, rows, d);
        if (t > b) b = t;
    }
    return MMD_WS_HEADER + b;
}

smmd_status smmd_mmd2_fwd(const smmd_kernel_desc *desc, const float *X, int m, const float *Y,
                          int n, int d, int biased, int x_begin, int x_end, int y_begin,
                          int y_end, float *out_sums, float *out_mmd2, float *grad_x,
                          float *grad_y, void *ws, size_t ws_bytes, smmd_stream_t stream) {
    if (!desc || !X || !Y || m < 1 || n < 1 || d < 1) return SMMD_EINVAL;
    if (x_begin < 0 || x_end < x_begin || x_end > m) return SMMD_EINVAL;
    if (y_begin < 0 || y_end < y_begin || y_end > n) return SMMD_EINVAL;
    const int need_grad = (grad_x != nullptr) || (grad_y != nullptr);
    if (need_grad && (!grad_x || !grad_y)) return SMMD_EINVAL;
    KParams kp;
    if (!make_kparams(desc, kp)) return SMMD_EINVAL;
    const int dt = pick_dt(d);
    const bool gram = use_gram(m, n, d);
    const int rows = (x_end - x_begin) + (y_end - y_begin);
    if (!ws || ws_bytes < smmd_mmd2_workspace_bytes(m, n, d)) return SMMD_EWORKSPACE;
    if (rows == 0) return SMMD_EINVAL;
    const double md = m, nd = n;
    const int is_biased = biased ? 1 : 0;
    const double wxx = is_biased ? 1.0 / (md * md) : 1.0 / (md * (md - 1.0));
    const double wyy = is_biased ? 1.0 / (nd * nd) : 1.0 / (nd * (nd - 1.0));
    if (gram) {
        GramArgs g;
        memset(&g, 0, sizeof(g));
        g.X = X; g.Y = Y; g.m = m; g.n = n; g.d = d;
        g.nrows = rows; g.nxr = x_end - x_begin; g.x_begin = x_begin; g.y_begin = y_begin;
        g.tanh_in = desc->tanh_inputs ? 1 : 0;
        g.biased = is_biased;
        g.has_const = desc->has_const_diag ? 1 : 0;
        g.const_diag = desc->const_diag;
        g.trace_mode = (!is_biased && !g.has_const) ? 1 : 0;
        g.need_grad = need_grad;
        g.kind = desc->kind;
        g.gw_same_x = (float)(2.0 * wxx);
        g.gw_same_y = (float)(2.0 * wyy);
        g.gw_cross = (float)(-2.0 / (md * nd));
        g.counter = (unsigned *)ws;
        g.out_sums = out_sums; g.out_mmd2 = out_mmd2;
        g.grad_x = grad_x; g.grad_y = grad_y;
        g.kp = kp;
        return gram_mmd2_launch(g, (char *)ws + MMD_WS_HEADER, (hipStream_t)stream);
    }
    if (use_tile(m, n, d)) {
        TileArgs t;
        memset(&t, 0, sizeof(t));
        t.X = X; t.Y = Y; t.m = m; t.n = n; t.d = d;
        t.nrows = rows; t.nxr = x_end - x_begin; t.x_begin = x_begin; t.y_begin = y_begin;
        t.tanh_in = desc->tanh_inputs ? 1 : 0;
        t.biased = is_biased;
        t.has_const = desc->has_const_diag ? 1 : 0;
        t.const_diag = desc->const_diag;
        t.trace_mode = (!is_biased && !t.has_const) ? 1 : 0;
        t.need_grad = need_grad;
        t.gw_same_x = (float)(2.0 * wxx);
        t.gw_same_y = (float)(2.0 * wyy);
        t.gw_cross = (float)(-2.0 / (md * nd));
        t.grad_x = grad_x; t.grad_y = grad_y;
        t.out_sums = out_sums; t.out_mmd2 = out_mmd2;
        t.kp = kp;
        return tile_mmd2_launch(t, desc->kind, ws, (hipStream_t)stream);
    }
    const int grid = mmd2_grid(rows, dt);

    MmdArgs a;
    memset(&a, 0, sizeof(a));
    a.X = X;
    a.Y = Y;
    a.m = m;
    a.n = n;
    a.d = d;
    a.x_begin = x_begin;
    a.x_end = x_end;
    a.y_begin = y_begin;
    a.y_end = y_end;
    a.tanh_in = desc->tanh_inputs ? 1 : 0;
    a.biased = biased ? 1 : 0;
    a.has_const = desc->has_const_diag ? 1 : 0;
    a.const_diag = desc->const_diag;
    a.trace_mode = (!a.biased && !a.has_const) ? 1 : 0;
    a.need_grad = need_grad;
    a.gw_same_x = (float)(2.0 * wxx);
    a.gw_same_y = (float)(2.0 * wyy);
    a.gw_cross = (float)(-2.0 / (md * nd));
    a.grad_x = grad_x;
    a.grad_y = grad_y;
    a.counter = (unsigned *)ws;
    a.partials = (double *)((char *)ws + MMD_WS_HEADER);
    a.out_sums = out_sums;
    a.out_mmd2 = out_mmd2;
    a.kp = kp;

    hipStream_t s = (hipStream_t)stream;
    bool ok = false;
    switch (desc->kind) {
        case SMMD_KIND_RBF: ok = dispatch_mmd2_dt<SMMD_KIND_RBF>(dt, a, grid, s); break;
        case SMMD_KIND_RQ: ok = dispatch_mmd2_dt<SMMD_KIND_RQ>(dt, a, grid, s); break;
        case SMMD_KIND_DISTANCE: ok = dispatch_mmd2_dt<SMMD_KIND_DISTANCE>(dt, a, grid, s); break;
        case SMMD_KIND_DOT: ok = dispatch_mmd2_dt<SMMD_KIND_DOT>(dt, a, grid, s); break;
    }
    if (!ok) return SMMD_EINVAL;
    return last_launch_status();
}

smmd_status smmd_smmd_loss_fwd(const smmd_kernel_desc *desc, const float *X, int m,
                               const float *Y, int n, int d, int biased, const float *jac,
                               int n_cols, int b, int64_t per_sample, const float *feat, int dof,
                               float sc, int variant, int sqrt_scale, float *out_sums,
                               float *out_mmd2, float *grad_x, float *grad_y, float *out,
                               float *per_sample_out, void *ws, size_t ws_bytes, void *loss_ws,
                               size_t loss_ws_bytes, smmd_stream_t stream) {
    if (!desc || !X || !Y || m < 1 || n < 1 || d < 1) return SMMD_EINVAL;
    if (!out_mmd2 || !grad_x || !grad_y || !jac || !out) return SMMD_EINVAL;
    if (n_cols < 1 || b < 1 || per_sample < 1) return SMMD_EINVAL;
    if (variant != 0 && variant != 1) return SMMD_EINVAL;
    if (variant == 1 && (!feat || dof < 1)) return SMMD_EINVAL;
    KParams kp;
    if (!make_kparams(desc, kp)) return SMMD_EINVAL;
    if (!use_tile(m, n, d)) return SMMD_EUNSUPPORTED;      // the caller runs two launches
    if (!ws || ws_bytes < smmd_mmd2_workspace_bytes(m, n, d)) return SMMD_EWORKSPACE;
    const int rows_j = n_cols * b;
    if (!loss_ws || loss_ws_bytes < smmd_scaled_loss_workspace_bytes(rows_j, per_sample))
        return SMMD_EWORKSPACE;
    const double md = m, nd = n;
    const int is_biased = biased ? 1 : 0;
    const double wxx = is_biased ? 1.0 / (md * md) : 1.0 / (md * (md - 1.0));
    const double wyy = is_biased ? 1.0 / (nd * nd) : 1.0 / (nd * (nd - 1.0));
    TileArgs t;
    memset(&t, 0, sizeof(t));
    t.X = X; t.Y = Y; t.m = m; t.n = n; t.d = d;
    t.nrows = m + n; t.nxr = m; t.x_begin = 0; t.y_begin = 0;
    t.tanh_in = desc->tanh_inputs ? 1 : 0;
    t.biased = is_biased;
    t.has_const = desc->has_const_diag ? 1 : 0;
    t.const_diag = desc->const_diag;
    t.trace_mode = (!is_biased && !t.has_const) ? 1 : 0;
    t.need_grad = 1;
    t.gw_same_x = (float)(2.0 * wxx);
    t.gw_same_y = (float)(2.0 * wyy);
    t.gw_cross = (float)(-2.0 / (md * nd));
    t.grad_x = grad_x; t.grad_y = grad_y;
    t.out_sums = out_sums; t.out_mmd2 = out_mmd2;
    t.kp = kp;
    ScaledLossArgs q;
    memset(&q, 0, sizeof(q));
    const int nchunk = (int)((per_sample + SQ_CHUNK - 1) / SQ_CHUNK);
    if ((int64_t)rows_j * nchunk > 0x7fffffff) return SMMD_EINVAL;
    q.jac = jac;
    q.per_sample = per_sample;
    q.nchunk = nchunk;
    q.vec = (per_sample % 4 == 0) && ((uintptr_t)jac % 16 == 0);
    q.counter = (unsigned *)loss_ws;          // ticket at a fixed offset, as the fwd
    q.part = (double *)((char *)loss_ws + SQ_WS_HEADER);
    q.n_cols = n_cols;
    q.b = b;
    q.b_total = b;
    q.dof = dof;
    q.variant = variant;
    q.sqrt_scale = sqrt_scale;
    q.feat = feat;
    q.base_loss = out_mmd2;                    // the estimator, stored by the MMD grid
    q.sc = sc;
    q.out = out;
    q.per_sample_out = per_sample_out;
    q.nblocks = rows_j * nchunk;
    return tile_mmd2_launch(t, desc->kind, ws, (hipStream_t)stream, &q);
}

// The all-gather mode's fused loss: X, Y are the gathered global rows (every
// rank sweeps them whole), J / nD come from the gathered per-rank partials
// (no Jacobian pass here: each rank reduced its own rows before the gather).
smmd_status smmd_smmd_loss_fwd_gathered(const smmd_kernel_desc *desc, const float *X, int m,
                                        const float *Y, int n, int d, int biased,
                                        const float *stats, int world, int stats_stride,
                                        float sc, int variant, int sqrt_scale, float *out_sums,
                                        float *out_mmd2, float *grad_x, float *grad_y, float *out,
                                        void *ws, size_t ws_bytes, void *loss_ws,
                                        size_t loss_ws_bytes, smmd_stream_t stream) {
    if (!desc || !X || !Y || m < 1 || n < 1 || d < 1) return SMMD_EINVAL;
    if (!out_mmd2 || !grad_x || !grad_y || !stats || !out || world < 1 || stats_stride < 2)
        return SMMD_EINVAL;
    if (variant != 0 && variant != 1) return SMMD_EINVAL;
    KParams kp;
    if (!make_kparams(desc, kp)) return SMMD_EINVAL;
    if (!use_tile(m, n, d)) return SMMD_EUNSUPPORTED;      // the caller runs the separate calls
    if (!ws || ws_bytes < smmd_mmd2_workspace_bytes(m, n, d)) return SMMD_EWORKSPACE;
    if (!loss_ws || loss_ws_bytes < SQ_WS_HEADER) return SMMD_EWORKSPACE;
    const double md = m, nd = n;
    const int is_biased = biased ? 1 : 0;
    const double wxx = is_biased ? 1.0 / (md * md) : 1.0 / (md * (md - 1.0));
    const double wyy = is_biased ? 1.0 / (nd * nd) : 1.0 / (nd * (nd - 1.0));
    TileArgs t;
    memset(&t, 0, sizeof(t));
    t.X = X; t.Y = Y; t.m = m; t.n = n; t.d = d;
    t.nrows = m + n; t.nxr = m; t.x_begin = 0; t.y_begin = 0;
    t.tanh_in = desc->tanh_inputs ? 1 : 0;
    t.biased = is_biased;
    t.has_const = desc->has_const_diag ? 1 : 0;
    t.const_diag = desc->const_diag;
    t.trace_mode = (!is_biased && !t.has_const) ? 1 : 0;
    t.need_grad = 1;
    t.gw_same_x = (float)(2.0 * wxx);
    t.gw_same_y = (float)(2.0 * wyy);
    t.gw_cross = (float)(-2.0 / (md * nd));
    t.grad_x = grad_x; t.grad_y = grad_y;
    t.out_sums = out_sums; t.out_mmd2 = out_mmd2;
    t.kp = kp;
    ScaledLossArgs q;
    memset(&q, 0, sizeof(q));
    q.counter = (unsigned *)loss_ws;
    q.part = (double *)((char *)loss_ws + SQ_WS_HEADER);
    q.nchunk = 1;
    q.b_total = 1;
    q.variant = variant;
    q.sqrt_scale = sqrt_scale;
    q.base_loss = out_mmd2;
    q.sc = sc;
    q.out = out;
    q.nblocks = 0;                             // no squared-norm blocks
    q.stats = stats;
    q.stats_world = world;
    q.stats_stride = stats_stride;
    return tile_mmd2_launch(t, desc->kind, ws, (hipStream_t)stream, &q);
}

smmd_status smmd_mmd2_combine(const smmd_kernel_desc *desc, const float *sums, int m, int n,
                              int biased, float *out_mmd2, smmd_stream_t stream) {
    if (!desc || !sums || !out_mmd2 || m < 1 || n < 1) return SMMD_EINVAL;
    hipLaunchKernelGGL(mmd2_combine_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, sums,
                       (double)m, (double)n, biased ? 1 : 0, desc->has_const_diag ? 1 : 0,
                       desc->const_diag, out_mmd2);
    return last_launch_status();
}

smmd_status smmd_witness_fwd(const smmd_kernel_desc *desc, const float *H, int b, const float *R,
                             int nr, const float *F, int nf, int d, float *out_w, float *out_dH,
                             smmd_stream_t stream) {
    if (!desc || !H || !R || !F || b < 1 || nr < 1 || nf < 1 || d < 1) return SMMD_EINVAL;
    KParams kp;
    if (!make_kparams(desc, kp)) return SMMD_EINVAL;
    const int dt = pick_dt(d);
    if (dt == 0) return SMMD_EUNSUPPORTED;
    WitArgs a;
    memset(&a, 0, sizeof(a));
    a.H = H; a.R = R; a.F = F; a.b = b; a.nr = nr; a.nf = nf; a.d = d;
    a.tanh_in = desc->tanh_inputs ? 1 : 0;
    a.out_w = out_w; a.out_dH = out_dH; a.kp = kp;
    const int grid = wave_grid(b);
    hipStream_t s = (hipStream_t)stream;
#define SMMD_WIT(DT_)                                                                          \
    case DT_:                                                                                  \
        switch (desc->kind) {                                                                  \
            case SMMD_KIND_RBF: hipLaunchKernelGGL((witness_fwd_kernel<DT_, SMMD_KIND_RBF>), dim3(grid), dim3(256), 0, s, a); break; \
            case SMMD_KIND_RQ: hipLaunchKernelGGL((witness_fwd_kernel<DT_, SMMD_KIND_RQ>), dim3(grid), dim3(256), 0, s, a); break; \
            case SMMD_KIND_DISTANCE: hipLaunchKernelGGL((witness_fwd_kernel<DT_, SMMD_KIND_DISTANCE>), dim3(grid), dim3(256), 0, s, a); break; \
            case SMMD_KIND_DOT: hipLaunchKernelGGL((witness_fwd_kernel<DT_, SMMD_KIND_DOT>), dim3(grid), dim3(256), 0, s, a); break; \
            default: return SMMD_EINVAL;                                                        \
        }                                                                                      \
        break;
    switch (dt) {
        SMMD_WIT(1) SMMD_WIT(2) SMMD_WIT(4) SMMD_WIT(8) SMMD_WIT(16) SMMD_WIT(32)
        default: return SMMD_EUNSUPPORTED;
    }
#undef SMMD_WIT
    return last_launch_status();
}

smmd_status smmd_witness_bwd(const smmd_kernel_desc *desc, const float *H, int b, const float *R,
                             int nr, const float *F, int nf, int d, const float *gdH, float *gH,
                             float *gR, float *gF, smmd_stream_t stream) {
    if (!desc || !H || !R || !F || !gdH || !gH || !gR || !gF) return SMMD_EINVAL;
    if (b < 1 || nr < 1 || nf < 1 || d < 1) return SMMD_EINVAL;
    KParams kp;
    if (!make_kparams(desc, kp)) return SMMD_EINVAL;
    const int dt = pick_dt(d);
    if (dt == 0) return SMMD_EUNSUPPORTED;
    WitBwdArgs a;
    memset(&a, 0, sizeof(a));
    a.H = H; a.R = R; a.F = F; a.gdH = gdH; a.b = b; a.nr = nr; a.nf = nf; a.d = d;
    a.tanh_in = desc->tanh_inputs ? 1 : 0;
    a.gH = gH; a.gR = gR; a.gF = gF; a.kp = kp;
    hipStream_t s = (hipStream_t)stream;
    const int gh = wave_grid(b), gz = wave_grid(nr + nf);
#define SMMD_WB_K(DT_, K_)                                                                     \
    hipLaunchKernelGGL((witness_bwd_h_kernel<DT_, K_>), dim3(gh), dim3(256), 0, s, a);         \
    hipLaunchKernelGGL((witness_bwd_z_kernel<DT_, K_>), dim3(gz), dim3(256), 0, s, a);
#define SMMD_WB(DT_)                                                                           \
    case DT_:                                                                                  \
        switch (desc->kind) {                                                                  \
            case SMMD_KIND_RBF: SMMD_WB_K(DT_, SMMD_KIND_RBF) break;                           \
            case SMMD_KIND_RQ: SMMD_WB_K(DT_, SMMD_KIND_RQ) break;                             \
            case SMMD_KIND_DISTANCE: SMMD_WB_K(DT_, SMMD_KIND_DISTANCE) break;                 \
            case SMMD_KIND_DOT: SMMD_WB_K(DT_, SMMD_KIND_DOT) break;                           \
            default: return SMMD_EINVAL;                                                        \
        }                                                                                      \
        break;
    switch (dt) {
        SMMD_WB(1) SMMD_WB(2) SMMD_WB(4) SMMD_WB(8) SMMD_WB(16) SMMD_WB(32)
        default: return SMMD_EUNSUPPORTED;
    }
#undef SMMD_WB_K
#undef SMMD_WB
    return last_launch_status();
}

#define SMMD_KM_SWITCH(DT_, BODY)                                                             \
    case DT_:                                                                                  \
        switch (desc->kind) {                                                                  \
            case SMMD_KIND_RBF: { constexpr int KIND_ = SMMD_KIND_RBF; BODY; } break;          \
            case SMMD_KIND_RQ: { constexpr int KIND_ = SMMD_KIND_RQ; BODY; } break;            \
            case SMMD_KIND_DISTANCE: { constexpr int KIND_ = SMMD_KIND_DISTANCE; BODY; } break; \
            case SMMD_KIND_DOT: { constexpr int KIND_ = SMMD_KIND_DOT; BODY; } break;          \
            default: return SMMD_EINVAL;                                                        \
        }                                                                                      \
        break;

smmd_status smmd_kernel_matrix_fwd(const smmd_kernel_desc *desc, const float *A, int na,
                                   const float *B, int nb, int d, float *out,
                                   smmd_stream_t stream) {
    if (!desc || !A || !B || !out || na < 1 || nb < 1 || d < 1) return SMMD_EINVAL;
    KParams kp;
    if (!make_kparams(desc, kp)) return SMMD_EINVAL;
    const int dt = pick_dt(d);
    KmArgs a;
    memset(&a, 0, sizeof(a));
    a.A = A; a.B = B; a.na = na; a.nb = nb; a.d = d; a.tanh_in = desc->tanh_inputs ? 1 : 0;
    a.out = out; a.kp = kp;
    const dim3 grid((nb + 63) / 64, (na + 3) / 4);
    hipStream_t s = (hipStream_t)stream;
    switch (dt) {
        SMMD_KM_SWITCH(1, hipLaunchKernelGGL((kmat_fwd_kernel<1, KIND_>), grid, dim3(256), 0, s, a))
        SMMD_KM_SWITCH(2, hipLaunchKernelGGL((kmat_fwd_kernel<2, KIND_>), grid, dim3(256), 0, s, a))
        SMMD_KM_SWITCH(4, hipLaunchKernelGGL((kmat_fwd_kernel<4, KIND_>), grid, dim3(256), 0, s, a))
        SMMD_KM_SWITCH(8, hipLaunchKernelGGL((kmat_fwd_kernel<8, KIND_>), grid, dim3(256), 0, s, a))
        SMMD_KM_SWITCH(16, hipLaunchKernelGGL((kmat_fwd_kernel<16, KIND_>), grid, dim3(256), 0, s, a))
        SMMD_KM_SWITCH(32, hipLaunchKernelGGL((kmat_fwd_kernel<32, KIND_>), grid, dim3(256), 0, s, a))
        default: return SMMD_EUNSUPPORTED;
    }
    return last_launch_status();
}

smmd_status smmd_kernel_matrix_bwd(const smmd_kernel_desc *desc, const float *A, int na,
                                   const float *B, int nb, int d, const float *G, float *gA,
                                   float *gB, smmd_stream_t stream) {
    if (!desc || !A || !B || !G || na < 1 || nb < 1 || d < 1) return SMMD_EINVAL;
    KParams kp;
    if (!make_kparams(desc, kp)) return SMMD_EINVAL;
    const int dt = pick_dt(d);
    KmArgs a;
    memset(&a, 0, sizeof(a));
    a.A = A; a.B = B; a.G = G; a.na = na; a.nb = nb; a.d = d;
    a.tanh_in = desc->tanh_inputs ? 1 : 0; a.gA = gA; a.gB = gB; a.kp = kp;
    hipStream_t s = (hipStream_t)stream;
    const int ga = wave_grid(na), gb = wave_grid(nb);
#define SMMD_KMB(DT_)                                                                          \
    SMMD_KM_SWITCH(DT_, {                                                                      \
        if (gA) hipLaunchKernelGGL((kmat_bwd_kernel<DT_, KIND_, 0>), dim3(ga), dim3(256), 0, s, a); \
        if (gB) hipLaunchKernelGGL((kmat_bwd_kernel<DT_, KIND_, 1>), dim3(gb), dim3(256), 0, s, a); \
    })
    switch (dt) {
        SMMD_KMB(1) SMMD_KMB(2) SMMD_KMB(4) SMMD_KMB(8) SMMD_KMB(16) SMMD_KMB(32)
        default: return SMMD_EUNSUPPORTED;
    }
#undef SMMD_KMB
    return last_launch_status();
}

}  // extern "C"
