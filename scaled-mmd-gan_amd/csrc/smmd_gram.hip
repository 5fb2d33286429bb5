// smmd_gram.hip -- MMD^2 forward + unit gradient through the Gram matrix on the
// f32 matrix cores (gfx950 v_mfma_f32_32x32x2_f32), for any feature width d.
//
// Reference being replaced: the same as smmd_mmd.hip -- the kernel family of
// gan/core/mmd.py:18-188 (XX = X X^T, XY, YY Gram matmuls, mmd.py:57-59, then
// the elementwise kernel), the estimator mmd.py:194-220 and TF's autodiff of
// it -- at the widths where the pairwise dot products dominate (critic
// dof_dim > 32; SURVEY 8d's D in {128, 1024} sweep).  Three launches:
//
//   prep   Z = [X; Y] (tanh applied when the kernel asks) -> padded Zp [Rp, dp]
//          and ||z_r||^2 as the same k-ordered fma chain the MFMA produces, so
//          raw D2 is exactly 0 on the diagonal (mmd.py:60-67)
//   nt     S = Z_rows Z^T tile by tile (64 x 64 per block, 32 x 32 per wave,
//          K staged through LDS in chunks of 32); epilogue per pair: raw D2 in
//          the reference's order, K and dK (smmd_kern.hpp), the six block sums
//          and the gradient coefficient c_ij -> C [rows, Rp]; sums go to a
//          double slab reduced by the last-arriving block
//   nn     G = C Z (the same MFMA tiling, reduction over the Rp columns),
//          epilogue grad_i = (a_i + sum_j c_ij) z_i - G_i   (a_i: the al terms
//          of the RQ add_dot / dot / distance kernels, closed form per row)
//
// v_mfma_f32_32x32x2_f32 is bit-for-bit a k-ordered fmaf chain (CDNA4 guide,
// 'FP32-input MFMA'), i.e. the dot products equal smmd_mmd.hip's dotk().
#include "smmd_kern.hpp"

namespace smmd {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int GT = 64;       // block tile (rows x cols)
constexpr int GK = 32;       // K chunk staged in LDS
constexpr int GLD = GK + 1;  // LDS row stride of a [64][32] operand tile

__device__ __forceinline__ int gram_zrow(const GramArgs &g, int e) {
    return e < g.nxr ? g.x_begin + e : g.m + g.y_begin + (e - g.nxr);
}

// one wave per row of Zp: copy (tanh), zero padding, then lane 0 forms the
// squared norm as a k-ordered fma chain over the row it just wrote
__global__ __launch_bounds__(256) void gram_prep_kernel(GramArgs g) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r < g.Rp) {
        const float *src = nullptr;
        if (r < g.m) src = g.X + (size_t)r * g.d;
        else if (r < g.R) src = g.Y + (size_t)(r - g.m) * g.d;
        float *dst = g.Zp + (size_t)r * g.dp;
        for (int k = lane; k < g.dp; k += 64) {
            float v = 0.f;
            if (src && k < g.d) {
                v = src[k];
                if (g.tanh_in) v = tanhf(v);
            }
            dst[k] = v;
        }
    }
    __syncthreads();
    if (r < g.Rp && lane == 0) {
        const float *row = g.Zp + (size_t)r * g.dp;
        float s = row[0] * row[0];
        for (int k = 1; k < g.dp; ++k) s = fmaf(row[k], row[k], s);
        g.sq[r] = s;
    }
}

// stage a [64 rows][32 k] tile: 512 float4, two per thread (rows < 0: zero)
__device__ __forceinline__ void gram_fetch(const float *__restrict__ base, int ld, const int *rows,
                                           int k0, float4 (&v)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int idx = threadIdx.x + 256 * q;
        const int r = rows[idx >> 3];
        v[q] = (r >= 0) ? *reinterpret_cast<const float4 *>(base + (size_t)r * ld + k0 + (idx & 7) * 4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

__device__ __forceinline__ void gram_stash(float (*T)[GLD], const float4 (&v)[2]) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int idx = threadIdx.x + 256 * q;
        float *p = &T[idx >> 3][(idx & 7) * 4];
        p[0] = v[q].x; p[1] = v[q].y; p[2] = v[q].z; p[3] = v[q].w;
    }
}

template <int KIND>
__global__ __launch_bounds__(256) void gram_nt_kernel(GramArgs g) {
    __shared__ float As[GT][GLD], Bs[GT][GLD];
    __shared__ int arow[GT], brow[GT];
    __shared__ double red[4][8];
    __shared__ int is_last;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int e0 = blockIdx.y * GT, j0 = blockIdx.x * GT;
    if (threadIdx.x < GT) {
        const int e = e0 + threadIdx.x;
        arow[threadIdx.x] = (e < g.nrows) ? gram_zrow(g, e) : -1;
        brow[threadIdx.x] = j0 + threadIdx.x;          // < Rp: padded rows are zero
    }
    __syncthreads();

    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float4 va[2], vb[2];
    gram_fetch(g.Zp, g.dp, arow, 0, va);
    gram_fetch(g.Zp, g.dp, brow, 0, vb);
    for (int k0 = 0; k0 < g.dp; k0 += GK) {
        gram_stash(As, va);
        gram_stash(Bs, vb);
        __syncthreads();
        if (k0 + GK < g.dp) {                            // next chunk in flight
            gram_fetch(g.Zp, g.dp, arow, k0 + GK, va);
            gram_fetch(g.Zp, g.dp, brow, k0 + GK, vb);
        }
        const float *ar = &As[wm * 32 + (lane & 31)][lane >> 5];
        const float *br = &Bs[wn * 32 + (lane & 31)][lane >> 5];
#pragma unroll
        for (int kk = 0; kk < GK / 2; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * kk], br[2 * kk], acc, 0, 0, 0);
        __syncthreads();
    }

    // epilogue: C/D map of 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
    float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // XX XY YY trXX trYY YX
    const int j = j0 + wn * 32 + (lane & 31);
    const float sqc = g.sq[j];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rs = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int e = e0 + wm * 32 + rs;
        if (e >= g.nrows) continue;
        const int i = arow[wm * 32 + rs];
        float c = 0.f;
        if (j < g.R) {
            const float dot = acc[r];
            const float sqi = g.sq[i];
            const float raw = (-2.f * dot + sqi) + sqc;          // mmd.py:67 order
            float K, al, be;
            Kern<KIND>::eval(g.kp, raw, dot, sqi, sqc, K, al, be);
            const bool isx = e < g.nxr, colx = j < g.m;
            const bool diag = (j == i);
            if (isx) {
                if (colx) { s[0] += K; if (diag) s[3] += K; }
                else s[1] += K;
            } else {
                if (colx) s[5] += K;
                else { s[2] += K; if (diag) s[4] += K; }
            }
            if (g.need_grad && !(diag && g.trace_mode)) {
                const float wgt = (isx == colx) ? (isx ? g.gw_same_x : g.gw_same_y) : g.gw_cross;
                c = wgt * be;
            }
        }
        if (g.need_grad) g.C[(size_t)e * g.Rp + j] = c;
    }

    // block sums (fixed order, double) -> slab -> last arriver
#pragma unroll
    for (int k = 0; k < 6; ++k) s[k] = wave_sum(s[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) red[w][k] = (double)s[k];
    }
    __syncthreads();
    const int nblk = gridDim.x * gridDim.y;
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    if (threadIdx.x == 0) {
        double *slab = g.slab + (size_t)bid * 8;
#pragma unroll
        for (int k = 0; k < 6; ++k) slab[k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev =
            __hip_atomic_fetch_add(g.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (prev == (unsigned)nblk - 1);
    }
    __syncthreads();
    if (!is_last || w != 0) return;
    if (lane == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    double S[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int b = lane; b < nblk; b += 64) {
        const double *slab = g.slab + (size_t)b * 8;
#pragma unroll
        for (int k = 0; k < 6; ++k) S[k] += slab[k];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) S[k] = wave_sum(S[k]);
    if (lane == 0) {
        if (g.out_sums) {
#pragma unroll
            for (int k = 0; k < 6; ++k) g.out_sums[k] = (float)S[k];
            g.out_sums[6] = 0.f;
            g.out_sums[7] = 0.f;
        }
        if (g.out_mmd2)
            g.out_mmd2[0] = (float)estimator(S, (double)g.m, (double)g.n, g.biased, g.has_const,
                                             g.const_diag);
        __hip_atomic_store(g.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// G = C Z over the Rp columns; grad_i = (a_i + sum_j c_ij) z_i - G_i
__global__ __launch_bounds__(256) void gram_nn_kernel(GramArgs g) {
    constexpr int BLD = GT + 4;
    __shared__ float As[GT][GLD];
    __shared__ float Bs[GK][BLD];
    __shared__ int arow[GT];
    __shared__ float rsum[GT];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int e0 = blockIdx.y * GT, k0c = blockIdx.x * GT;
    if (threadIdx.x < GT) arow[threadIdx.x] = (e0 + threadIdx.x < g.nrows) ? e0 + threadIdx.x : -1;
    __syncthreads();

    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float rs = 0.f;                                   // thread t < 64: row t's sum_j c_ij
    // B tile [32 j][64 cols] of Zp: 512 float4, two per thread
    auto fetch_b = [&](int jb, float4 (&v)[2]) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int idx = threadIdx.x + 256 * q;
            const int jr = idx >> 4, c = k0c + (idx & 15) * 4;
            v[q] = (c < g.dp) ? *reinterpret_cast<const float4 *>(g.Zp + (size_t)(jb + jr) * g.dp + c)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    float4 va[2], vb[2];
    gram_fetch(g.C, g.Rp, arow, 0, va);
    fetch_b(0, vb);
    for (int jb = 0; jb < g.Rp; jb += GK) {
        gram_stash(As, va);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int idx = threadIdx.x + 256 * q;
            *reinterpret_cast<float4 *>(&Bs[idx >> 4][(idx & 15) * 4]) = vb[q];
        }
        __syncthreads();
        if (jb + GK < g.Rp) {
            gram_fetch(g.C, g.Rp, arow, jb + GK, va);
            fetch_b(jb + GK, vb);
        }
        if (threadIdx.x < GT) {
#pragma unroll
            for (int c = 0; c < GK; ++c) rs += As[threadIdx.x][c];
        }
        const float *ar = &As[wm * 32 + (lane & 31)][lane >> 5];
        const float *br = &Bs[lane >> 5][wn * 32 + (lane & 31)];
#pragma unroll
        for (int kk = 0; kk < GK / 2; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * kk], br[2 * kk * BLD], acc, 0, 0, 0);
        __syncthreads();
    }
    if (threadIdx.x < GT) rsum[threadIdx.x] = rs;
    __syncthreads();

    const int k = k0c + wn * 32 + (lane & 31);
    if (k >= g.d) return;
    const double md = g.m, nd = g.n;
    const int tm = g.trace_mode ? 1 : 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rsi = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int e = e0 + rsi;
        if (e >= g.nrows) continue;
        const int i = gram_zrow(g, e);
        const bool isx = e < g.nxr;
        // a_i = al_i * sum_j w_ij over the columns the gradient includes
        float a = 0.f;
        if (g.kind != SMMD_KIND_RBF) {
            const float W = isx ? (float)(g.gw_same_x * (md - tm) + g.gw_cross * nd)
                                : (float)(g.gw_same_y * (nd - tm) + g.gw_cross * md);
            float al = 0.f;
            if (g.kind == SMMD_KIND_RQ) al = g.kp.add_dot;
            else if (g.kind == SMMD_KIND_DOT) al = 1.f;
            else al = 2.f * mysqrt_grad(g.sq[i]);
            a = al * W;
        }
        const float zk = g.Zp[(size_t)i * g.dp + k];
        float gk = (a + rsum[rsi]) * zk - acc[r];
        if (g.tanh_in) gk *= 1.f - zk * zk;
        float *dst = isx ? g.grad_x + (size_t)e * g.d : g.grad_y + (size_t)(e - g.nxr) * g.d;
        dst[k] = gk;
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int gram_pad(int x, int q) { return (x + q - 1) / q * q; }

size_t gram_ws_bytes(int m, int n, int d) {
    const size_t R = (size_t)(m > 0 ? m : 0) + (n > 0 ? n : 0);
    const size_t Rp = gram_pad((int)R, GT), dp = gram_pad(d > 0 ? d : 1, GK);
    const size_t blocks = (Rp / GT) * (Rp / GT);
    size_t b = 0;
    b += align_up(Rp * dp * 4, 256);        // Zp
    b += align_up(Rp * 4, 256);             // sq
    b += align_up(Rp * Rp * 4, 256);        // C (rows <= R)
    b += align_up(blocks * 8 * 8, 256);     // slab
    return b;
}

smmd_status gram_mmd2_launch(const GramArgs &proto, void *ws_body, hipStream_t s) {
    GramArgs g = proto;
    g.R = g.m + g.n;
    g.Rp = gram_pad(g.R, GT);
    g.dp = gram_pad(g.d, GK);
    char *p = (char *)ws_body;
    g.Zp = (float *)p;   p += align_up((size_t)g.Rp * g.dp * 4, 256);
    g.sq = (float *)p;   p += align_up((size_t)g.Rp * 4, 256);
    g.C = (float *)p;    p += align_up((size_t)g.Rp * g.Rp * 4, 256);
    g.slab = (double *)p;
    const int nrt = (g.nrows + GT - 1) / GT;
    hipLaunchKernelGGL(gram_prep_kernel, dim3((g.Rp + 3) / 4), dim3(256), 0, s, g);
    const dim3 grid_nt(g.Rp / GT, nrt);
    switch (g.kind) {
        case SMMD_KIND_RBF: hipLaunchKernelGGL(gram_nt_kernel<SMMD_KIND_RBF>, grid_nt, dim3(256), 0, s, g); break;
        case SMMD_KIND_RQ: hipLaunchKernelGGL(gram_nt_kernel<SMMD_KIND_RQ>, grid_nt, dim3(256), 0, s, g); break;
        case SMMD_KIND_DISTANCE: hipLaunchKernelGGL(gram_nt_kernel<SMMD_KIND_DISTANCE>, grid_nt, dim3(256), 0, s, g); break;
        case SMMD_KIND_DOT: hipLaunchKernelGGL(gram_nt_kernel<SMMD_KIND_DOT>, grid_nt, dim3(256), 0, s, g); break;
        default: return SMMD_EINVAL;
    }
    if (g.need_grad)
        hipLaunchKernelGGL(gram_nn_kernel, dim3((g.dp + GT - 1) / GT, nrt), dim3(256), 0, s, g);
    return last_launch_status();
}

}  // namespace smmd
