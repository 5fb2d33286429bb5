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

#include <stdlib.h>

namespace smmd {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int GT = 64;       // block tile (rows x cols)
constexpr int GK = 32;       // K chunk staged in LDS
constexpr int GLD = GK + 1;  // LDS row stride of a [64][32] operand tile

__device__ __forceinline__ int gram_zrow(const GramArgs &g, int e) {
    return e < g.nxr ? g.x_begin + e : g.m + g.y_begin + (e - g.nxr);
}

// one wave per row of Zp: copy (tanh), zero padding, then lane 0 forms the
// squared norm as a k-ordered fma chain over the row.  The chain is inherently
// serial (it must equal the MFMA's k-ordered accumulation bit for bit, so raw
// D2 is exactly 0 on the diagonal); lane 0 reads the row back from LDS four
// values per ds_read_b128 instead of from global memory one load per step
// (that form took 140 us at 4096 x 1024, a sixth of the whole MMD call)
constexpr int GP_CHUNK = 256;   // floats of a row staged per wave per step

__global__ __launch_bounds__(256) void gram_prep_kernel(GramArgs g) {
    __shared__ float4 rowbuf[4][GP_CHUNK / 4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 4 + w;
    const bool live = r < g.Rp;
    const float *src = nullptr;
    if (live && r < g.m) src = g.X + (size_t)r * g.d;
    else if (live && r < g.R) src = g.Y + (size_t)(r - g.m) * g.d;
    float *dst = live ? g.Zp + (size_t)r * g.dp : nullptr;
    float *rb = reinterpret_cast<float *>(rowbuf[w]);
    float s = 0.f;
    for (int k0 = 0; k0 < g.dp; k0 += GP_CHUNK) {          // dp: same for every wave
        const int n = (g.dp - k0 < GP_CHUNK) ? g.dp - k0 : GP_CHUNK;   // multiple of 32
        for (int kk = lane; kk < n; kk += 64) {
            const int k = k0 + kk;
            float v = 0.f;
            if (src && k < g.d) {
                v = src[k];
                if (g.tanh_in) v = tanhf(v);
            }
            if (live) dst[k] = v;
            rb[kk] = v;
        }
        __syncthreads();
        if (live && lane == 0) {
#pragma unroll 4
            for (int q = 0; q < n / 4; ++q) {
                const float4 x = rowbuf[w][q];
                s = (k0 == 0 && q == 0) ? x.x * x.x : fmaf(x.x, x.x, s);
                s = fmaf(x.y, x.y, s);
                s = fmaf(x.z, x.z, s);
                s = fmaf(x.w, x.w, s);
            }
        }
        __syncthreads();
    }
    if (live && lane == 0) g.sq[r] = s;
}

// stage a [TM rows][KC k] tile: TM * KC / 4 float4, TM * KC / 1024 per thread
// (rows < 0: zero); LDS rows padded to KC + 1 floats (conflict-free fragment reads)
template <int TM, int KC>
__device__ __forceinline__ void gram_fetch(const float *__restrict__ base, int ld, const int *rows,
                                           int k0, float4 (&v)[TM * KC / 1024]) {
#pragma unroll
    for (int q = 0; q < TM * KC / 1024; ++q) {
        const int idx = threadIdx.x + 256 * q;
        const int r = rows[idx / (KC / 4)];
        v[q] = (r >= 0) ? *reinterpret_cast<const float4 *>(base + (size_t)r * ld + k0 +
                                                            (idx % (KC / 4)) * 4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

template <int TM, int KC>
__device__ __forceinline__ void gram_stash(float (*T)[KC + 1], const float4 (&v)[TM * KC / 1024]) {
#pragma unroll
    for (int q = 0; q < TM * KC / 1024; ++q) {
        const int idx = threadIdx.x + 256 * q;
        float *p = &T[idx / (KC / 4)][(idx % (KC / 4)) * 4];
        p[0] = v[q].x; p[1] = v[q].y; p[2] = v[q].z; p[3] = v[q].w;
    }
}

// S = Z_rows Z^T on TM x TM block tiles: 4 waves in 2 x 2, each wave TM/2 x TM/2
// = NS x NS MFMA tiles of 32 x 32 (NS accumulators per operand fragment, so a
// 128 tile reads each LDS fragment once per 2 MFMAs and fetches half the L2 /
// Infinity-Cache bytes per flop of a 64 tile)
template <int KIND, int TM, int KC>
__global__ __launch_bounds__(256) void gram_nt_kernel(GramArgs g) {
    constexpr int NS = TM / 64;
    constexpr int LD = KC + 1;
    __shared__ float As[TM][LD], Bs[TM][LD];
    __shared__ int arow[TM], brow[TM];
    __shared__ double red[4][8];
    __shared__ int is_last;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int e0 = blockIdx.y * TM, j0 = blockIdx.x * TM;
    if (threadIdx.x < TM) {
        const int e = e0 + threadIdx.x;
        arow[threadIdx.x] = (e < g.nrows) ? gram_zrow(g, e) : -1;
        brow[threadIdx.x] = j0 + threadIdx.x;          // < Rp: padded rows are zero
    }
    __syncthreads();

    floatx16 acc[NS][NS];
#pragma unroll
    for (int a = 0; a < NS; ++a)
#pragma unroll
        for (int b = 0; b < NS; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    float4 va[TM * KC / 1024], vb[TM * KC / 1024];
    gram_fetch<TM, KC>(g.Zp, g.dp, arow, 0, va);
    gram_fetch<TM, KC>(g.Zp, g.dp, brow, 0, vb);
    for (int k0 = 0; k0 < g.dp; k0 += KC) {
        gram_stash<TM, KC>(As, va);
        gram_stash<TM, KC>(Bs, vb);
        __syncthreads();
        if (k0 + KC < g.dp) {                            // next chunk in flight
            gram_fetch<TM, KC>(g.Zp, g.dp, arow, k0 + KC, va);
            gram_fetch<TM, KC>(g.Zp, g.dp, brow, k0 + KC, vb);
        }
        const float *ar = &As[wm * (TM / 2) + (lane & 31)][lane >> 5];
        const float *br = &Bs[wn * (TM / 2) + (lane & 31)][lane >> 5];
#pragma unroll
        for (int kk = 0; kk < KC / 2; ++kk) {
            float af[NS], bf[NS];
#pragma unroll
            for (int a = 0; a < NS; ++a) af[a] = ar[a * 32 * LD + 2 * kk];
#pragma unroll
            for (int b = 0; b < NS; ++b) bf[b] = br[b * 32 * LD + 2 * kk];
#pragma unroll
            for (int a = 0; a < NS; ++a)
#pragma unroll
                for (int b = 0; b < NS; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }

    // epilogue: C/D map of 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
    float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};   // XX XY YY trXX trYY YX
#pragma unroll
    for (int b = 0; b < NS; ++b) {
        const int j = j0 + wn * (TM / 2) + b * 32 + (lane & 31);
        const float sqc = g.sq[j];
#pragma unroll
        for (int a = 0; a < NS; ++a) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rl = wm * (TM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int e = e0 + rl;
                if (e >= g.nrows) continue;
                const int i = arow[rl];
                float c = 0.f;
                if (j < g.R) {
                    const float dot = acc[a][b][r];
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
                        const float wgt = (isx == colx) ? (isx ? g.gw_same_x : g.gw_same_y)
                                                        : g.gw_cross;
                        c = wgt * be;
                    }
                }
                if (g.need_grad) g.C[(size_t)e * g.Rp + j] = c;
            }
        }
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

// G = C Z over the Rp columns; grad_i = (a_i + sum_j c_ij) z_i - G_i, on TM x TM
// output tiles (rows x feature columns), the same wave layout as gram_nt
template <int TM, int KC>
__global__ __launch_bounds__(256) void gram_nn_kernel(GramArgs g) {
    constexpr int NS = TM / 64;
    constexpr int LD = KC + 1;
    constexpr int BLD = TM + 4;
    __shared__ float As[TM][LD];
    __shared__ float Bs[KC][BLD];
    __shared__ int arow[TM];
    __shared__ float rsum[TM];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int e0 = blockIdx.y * TM, k0c = blockIdx.x * TM;
    if (threadIdx.x < TM) arow[threadIdx.x] = (e0 + threadIdx.x < g.nrows) ? e0 + threadIdx.x : -1;
    __syncthreads();

    floatx16 acc[NS][NS];
#pragma unroll
    for (int a = 0; a < NS; ++a)
#pragma unroll
        for (int b = 0; b < NS; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    float rs = 0.f;                                   // thread t < TM: row t's sum_j c_ij
    // B tile [KC j][TM cols] of Zp: KC * TM / 4 float4, TM * KC / 1024 per thread
    auto fetch_b = [&](int jb, float4 (&v)[TM * KC / 1024]) {
#pragma unroll
        for (int q = 0; q < TM * KC / 1024; ++q) {
            const int idx = threadIdx.x + 256 * q;
            const int jr = idx / (TM / 4), c = k0c + (idx % (TM / 4)) * 4;
            v[q] = (c < g.dp) ? *reinterpret_cast<const float4 *>(g.Zp + (size_t)(jb + jr) * g.dp + c)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    float4 va[TM * KC / 1024], vb[TM * KC / 1024];
    gram_fetch<TM, KC>(g.C, g.Rp, arow, 0, va);
    fetch_b(0, vb);
    for (int jb = 0; jb < g.Rp; jb += KC) {
        gram_stash<TM, KC>(As, va);
#pragma unroll
        for (int q = 0; q < TM * KC / 1024; ++q) {
            const int idx = threadIdx.x + 256 * q;
            *reinterpret_cast<float4 *>(&Bs[idx / (TM / 4)][(idx % (TM / 4)) * 4]) = vb[q];
        }
        __syncthreads();
        if (jb + KC < g.Rp) {
            gram_fetch<TM, KC>(g.C, g.Rp, arow, jb + KC, va);
            fetch_b(jb + KC, vb);
        }
        if (threadIdx.x < TM) {
#pragma unroll
            for (int c = 0; c < KC; ++c) rs += As[threadIdx.x][c];
        }
        const float *ar = &As[wm * (TM / 2) + (lane & 31)][lane >> 5];
        const float *br = &Bs[lane >> 5][wn * (TM / 2) + (lane & 31)];
#pragma unroll
        for (int kk = 0; kk < KC / 2; ++kk) {
            float af[NS], bf[NS];
#pragma unroll
            for (int a = 0; a < NS; ++a) af[a] = ar[a * 32 * LD + 2 * kk];
#pragma unroll
            for (int b = 0; b < NS; ++b) bf[b] = br[2 * kk * BLD + b * 32];
#pragma unroll
            for (int a = 0; a < NS; ++a)
#pragma unroll
                for (int b = 0; b < NS; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a], bf[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    if (threadIdx.x < TM) rsum[threadIdx.x] = rs;
    __syncthreads();

    const double md = g.m, nd = g.n;
    const int tm = g.trace_mode ? 1 : 0;
#pragma unroll
    for (int b = 0; b < NS; ++b) {
        const int k = k0c + wn * (TM / 2) + b * 32 + (lane & 31);
        if (k >= g.d) continue;
#pragma unroll
        for (int a = 0; a < NS; ++a) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int rsi = wm * (TM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int e = e0 + rsi;
                if (e >= g.nrows) continue;
                const int i = gram_zrow(g, e);
                const bool isx = e < g.nxr;
                // a_i = al_i * sum_j w_ij over the columns the gradient includes
                float av = 0.f;
                if (g.kind != SMMD_KIND_RBF) {
                    const float W = isx ? (float)(g.gw_same_x * (md - tm) + g.gw_cross * nd)
                                        : (float)(g.gw_same_y * (nd - tm) + g.gw_cross * md);
                    float al = 0.f;
                    if (g.kind == SMMD_KIND_RQ) al = g.kp.add_dot;
                    else if (g.kind == SMMD_KIND_DOT) al = 1.f;
                    else al = 2.f * mysqrt_grad(g.sq[i]);
                    av = al * W;
                }
                const float zk = g.Zp[(size_t)i * g.dp + k];
                float gk = (av + rsum[rsi]) * zk - acc[a][b][r];
                if (g.tanh_in) gk *= 1.f - zk * zk;
                float *dst = isx ? g.grad_x + (size_t)e * g.d : g.grad_y + (size_t)(e - g.nxr) * g.d;
                dst[k] = gk;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int gram_pad(int x, int q) { return (x + q - 1) / q * q; }

// 128 x 128 tiles (2 x 2 MFMA tiles per wave, half the operand bytes per flop)
// only where the K loop dominates and 1024+ blocks remain: measured on MI355X
// (tools/gram_bench.py, fwd + grad, rbf) 75.5 -> 80.6 TF at 2 x 2048 rows,
// d = 1024 and 79 -> 91 TF at 2 x 4096, d = 512; but 50 -> 42 TF at 2 x 1024,
// d = 1024 and 25 -> 18 TF at 2 x 2048, d = 128, where the per-pair epilogue
// and the block count matter more
static int gram_tile(int R, int d) {
    return (R >= 4096 && d >= 512) ? 128 : 64;
}

size_t gram_ws_bytes(int m, int n, int d) {
    const size_t R = (size_t)(m > 0 ? m : 0) + (n > 0 ? n : 0);
    const size_t Rp = gram_pad((int)R, 128), dp = gram_pad(d > 0 ? d : 1, 64);   // covers both tilings
    const size_t blocks = (Rp / 64) * (Rp / 64);
    size_t b = 0;
    b += align_up(Rp * dp * 4, 256);        // Zp
    b += align_up(Rp * 4, 256);             // sq
    b += align_up(Rp * Rp * 4, 256);        // C (rows <= R)
    b += align_up(blocks * 8 * 8, 256);     // slab
    return b;
}

template <int TM, int KC>
static smmd_status gram_launch_tiles(const GramArgs &g, hipStream_t s) {
    const int nrt = (g.nrows + TM - 1) / TM;
    const dim3 grid_nt(g.Rp / TM, nrt);
    switch (g.kind) {
        case SMMD_KIND_RBF: hipLaunchKernelGGL((gram_nt_kernel<SMMD_KIND_RBF, TM, KC>), grid_nt, dim3(256), 0, s, g); break;
        case SMMD_KIND_RQ: hipLaunchKernelGGL((gram_nt_kernel<SMMD_KIND_RQ, TM, KC>), grid_nt, dim3(256), 0, s, g); break;
        case SMMD_KIND_DISTANCE: hipLaunchKernelGGL((gram_nt_kernel<SMMD_KIND_DISTANCE, TM, KC>), grid_nt, dim3(256), 0, s, g); break;
        case SMMD_KIND_DOT: hipLaunchKernelGGL((gram_nt_kernel<SMMD_KIND_DOT, TM, KC>), grid_nt, dim3(256), 0, s, g); break;
        default: return SMMD_EINVAL;
    }
    if (g.need_grad)
        hipLaunchKernelGGL((gram_nn_kernel<TM, KC>), dim3((g.dp + TM - 1) / TM, nrt), dim3(256), 0, s, g);
    return last_launch_status();
}

smmd_status gram_mmd2_launch(const GramArgs &proto, void *ws_body, hipStream_t s) {
    GramArgs g = proto;
    g.R = g.m + g.n;
    const char *force = getenv("SMMD_GRAM_TILE");          // 64 / 128: A/B and tests
    int tm = gram_tile(g.R, g.d);
    if (force && (atoi(force) == 64 || atoi(force) == 128)) tm = atoi(force);
    // K chunk staged per step: 32 for both tilings (64 for the 128 tile measured
    // 3-9 % slower: 66 KB of LDS per block halves the blocks per CU)
    const int kc = GK;
    g.Rp = gram_pad(g.R, tm);
    g.dp = gram_pad(g.d, kc);
    char *p = (char *)ws_body;
    g.Zp = (float *)p;   p += align_up((size_t)g.Rp * g.dp * 4, 256);
    g.sq = (float *)p;   p += align_up((size_t)g.Rp * 4, 256);
    g.C = (float *)p;    p += align_up((size_t)g.Rp * g.Rp * 4, 256);
    g.slab = (double *)p;
    hipLaunchKernelGGL(gram_prep_kernel, dim3((g.Rp + 3) / 4), dim3(256), 0, s, g);
    return tm == 128 ? gram_launch_tiles<128, GK>(g, s) : gram_launch_tiles<64, GK>(g, s);
}

// ---------------------------------------------------------------------------
// Polynomial-kernel statistics of the KID scorer / 3-sample test
// (gan/compute_scores.py:232-335, gan/core/mmd.py:429-539):
// K = (gamma A B^T + coef0)^degree on the same MFMA tiles, never stored.
// Per 64 x 64 tile: the K values go through LDS once for the row and column
// sums (double, fixed order); sum K, sum K^2 and the diagonal come from the
// registers.  A second launch reduces the per-tile partials in tile order.
// ---------------------------------------------------------------------------
struct PolyArgs {
    const float *Ap;       // ws [nap][dimp]
    const float *Bp;       // ws [nbp][dimp]
    int na, nb, nap, nbp, dimp;
    float gamma, coef0;
    int degree;
    double *rowpart;       // ws [nbp/64][nap]
    double *colpart;       // ws [nap/64][nbp]
    double *slab;          // ws [tiles][4]
    double *row_sums, *col_sums, *diag, *stats;
};

// one wave per destination row: copy with zero padding
__global__ __launch_bounds__(256) void pad_rows_kernel(const float *src, int n, int dim, float *dst,
                                                       int np, int dimp) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= np) return;
    for (int k = lane; k < dimp; k += 64)
        dst[(size_t)r * dimp + k] = (r < n && k < dim) ? src[(size_t)r * dim + k] : 0.f;
}

__global__ __launch_bounds__(256) void poly_tile_kernel(PolyArgs p) {
    __shared__ float As[GT][GLD], Bs[GT][GLD];
    __shared__ float T[GT][GT + 1];
    __shared__ int arow[GT], brow[GT];
    __shared__ double red[4][4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int e0 = blockIdx.y * GT, j0 = blockIdx.x * GT;
    if (threadIdx.x < GT) {
        arow[threadIdx.x] = e0 + threadIdx.x;           // padded: always a valid row
        brow[threadIdx.x] = j0 + threadIdx.x;
    }
    __syncthreads();
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float4 va[2], vb[2];
    gram_fetch<GT, GK>(p.Ap, p.dimp, arow, 0, va);
    gram_fetch<GT, GK>(p.Bp, p.dimp, brow, 0, vb);
    for (int k0 = 0; k0 < p.dimp; k0 += GK) {
        gram_stash<GT, GK>(As, va);
        gram_stash<GT, GK>(Bs, vb);
        __syncthreads();
        if (k0 + GK < p.dimp) {
            gram_fetch<GT, GK>(p.Ap, p.dimp, arow, k0 + GK, va);
            gram_fetch<GT, GK>(p.Bp, p.dimp, brow, k0 + GK, vb);
        }
        const float *ar = &As[wm * 32 + (lane & 31)][lane >> 5];
        const float *br = &Bs[wn * 32 + (lane & 31)][lane >> 5];
#pragma unroll
        for (int kk = 0; kk < GK / 2; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * kk], br[2 * kk], acc, 0, 0, 0);
        __syncthreads();
    }
    // epilogue: sklearn polynomial_kernel order -- K = X Y^T; K *= gamma;
    // K += coef0; K **= degree (float32), gan/compute_scores.py:237-239
    const int jc = wn * 32 + (lane & 31);
    const int j = j0 + jc;
    double s1 = 0.0, s2 = 0.0, d1 = 0.0, d2 = 0.0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rr = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int e = e0 + rr;
        float K = 0.f;
        if (e < p.na && j < p.nb) {
            const float v = __fadd_rn(__fmul_rn(acc[r], p.gamma), p.coef0);
            K = v;
            for (int t = 1; t < p.degree; ++t) K = __fmul_rn(K, v);
            s1 += (double)K;
            s2 += (double)K * (double)K;
            if (e == j) {
                d1 += (double)K;
                d2 += (double)K * (double)K;
                if (p.diag) p.diag[e] = (double)K;
            }
        }
        T[rr][jc] = K;
    }
    __syncthreads();
    if (threadIdx.x < GT) {                            // row sums over the tile's columns
        double t = 0.0;
        for (int c = 0; c < GT; ++c) t += (double)T[threadIdx.x][c];
        p.rowpart[(size_t)blockIdx.x * p.nap + e0 + threadIdx.x] = t;
    } else if (threadIdx.x < 2 * GT) {                 // column sums over its rows
        const int c = threadIdx.x - GT;
        double t = 0.0;
        for (int r = 0; r < GT; ++r) t += (double)T[r][c];
        p.colpart[(size_t)blockIdx.y * p.nbp + j0 + c] = t;
    }
    double v[4] = {s1, s2, d1, d2};
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) red[w][k] = v[k];
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int k = threadIdx.x;
        p.slab[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + k] =
            ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
    }
}

// reduce the per-tile partials in tile order: rows, columns, then the stats
__global__ __launch_bounds__(256) void poly_reduce_kernel(PolyArgs p, int nct, int nrt) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (p.row_sums && i < p.na) {
        double t = 0.0;
        for (int c = 0; c < nct; ++c) t += p.rowpart[(size_t)c * p.nap + i];
        p.row_sums[i] = t;
    }
    if (p.col_sums && i < p.nb) {
        double t = 0.0;
        for (int r = 0; r < nrt; ++r) t += p.colpart[(size_t)r * p.nbp + i];
        p.col_sums[i] = t;
    }
    if (blockIdx.x == 0 && p.stats) {
        __shared__ double red[4][4];
        double v[4] = {0.0, 0.0, 0.0, 0.0};
        const int tiles = nct * nrt;
        for (int b = threadIdx.x; b < tiles; b += 256) {
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] += p.slab[(size_t)b * 4 + k];
        }
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = wave_sum(v[k]);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) red[w][k] = v[k];
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            const int k = threadIdx.x;
            p.stats[k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
        }
    }
}

// ---- estimators from the sums records (one block, double) ----------------
struct PolySumsDev {
    const double *rows, *cols, *diag, *stats;
};

template <int NV>
__device__ __forceinline__ void block_sums(double (&v)[NV], double (*red)[NV]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < NV; ++k) red[w][k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
}

// gan/compute_scores.py:246-335 (_mmd2_and_variance)
__global__ __launch_bounds__(256) void poly_mmd2_var_kernel(PolySumsDev xx, PolySumsDev yy,
                                                            PolySumsDev xy, int m_, double vm,
                                                            int est, double *out) {
    __shared__ double red[4][9];
    // 0 Kt_XX_sum 1 Kt_YY_sum 2 K_XY_sum 3 sqn(Kt_XX_sums) 4 sqn(Kt_YY_sums)
    // 5 sqn(K_XY_sums_1) 6 sqn(K_XY_sums_0) 7 dot_XX_XY 8 dot_YY_YX
    double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < m_; i += 256) {
        const double kx = xx.rows[i] - xx.diag[i], ky = yy.rows[i] - yy.diag[i];
        const double s1 = xy.rows[i], s0 = xy.cols[i];
        v[0] += kx; v[1] += ky; v[2] += s0;
        v[3] += kx * kx; v[4] += ky * ky; v[5] += s1 * s1; v[6] += s0 * s0;
        v[7] += kx * s1; v[8] += ky * s0;
    }
    block_sums<9>(v, red);
    if (threadIdx.x != 0) return;
    const double m = m_;
    const double Kt_XX_sum = v[0], Kt_YY_sum = v[1], K_XY_sum = v[2];
    const double sum_diag_X = xx.stats[2], sum_diag_Y = yy.stats[2];
    double mmd2;
    if (est == 1)
        mmd2 = (Kt_XX_sum + sum_diag_X) / (m * m) + (Kt_YY_sum + sum_diag_Y) / (m * m) -
               2 * K_XY_sum / (m * m);
    else if (est == 2)
        mmd2 = (Kt_XX_sum + Kt_YY_sum) / (m * (m - 1)) -
               2 * (K_XY_sum - xy.stats[2]) / (m * (m - 1));
    else
        mmd2 = (Kt_XX_sum + Kt_YY_sum) / (m * (m - 1)) - 2 * K_XY_sum / (m * m);
    const double Kt_XX_2_sum = xx.stats[1] - xx.stats[3];
    const double Kt_YY_2_sum = yy.stats[1] - yy.stats[3];
    const double K_XY_2_sum = xy.stats[1];
    const double dot_XX_XY = v[7], dot_YY_YX = v[8];
    const double m1 = m - 1, m2 = m - 2;
    const double zeta1 =
        1 / (m * m1 * m2) * (v[3] - Kt_XX_2_sum + v[4] - Kt_YY_2_sum) -
        1 / ((m * m1) * (m * m1)) * (Kt_XX_sum * Kt_XX_sum + Kt_YY_sum * Kt_YY_sum) +
        1 / (m * m * m1) * (v[5] + v[6] - 2 * K_XY_2_sum) -
        2 / (m * m * m * m) * K_XY_sum * K_XY_sum -
        2 / (m * m * m1) * (dot_XX_XY + dot_YY_YX) +
        2 / (m * m * m * m1) * (Kt_XX_sum + Kt_YY_sum) * K_XY_sum;
    const double zeta2 =
        1 / (m * m1) * (Kt_XX_2_sum + Kt_YY_2_sum) -
        1 / ((m * m1) * (m * m1)) * (Kt_XX_sum * Kt_XX_sum + Kt_YY_sum * Kt_YY_sum) +
        2 / (m * m) * K_XY_2_sum -
        2 / (m * m * m * m) * K_XY_sum * K_XY_sum -
        4 / (m * m * m1) * (dot_XX_XY + dot_YY_YX) +
        4 / (m * m * m * m1) * (Kt_XX_sum + Kt_YY_sum) * K_XY_sum;
    out[0] = mmd2;
    out[1] = 4 * (vm - 2) / (vm * (vm - 1)) * zeta1 + 2 / (vm * (vm - 1)) * zeta2;
}

// gan/core/mmd.py:444-512 (_np_diff_mmd2_and_ratio_from_sums), X shared
__global__ __launch_bounds__(256) void poly_diff_ratio_kernel(PolySumsDev yy, PolySumsDev xy,
                                                              PolySumsDev zz, PolySumsDev xz,
                                                              int m_, double *out) {
    __shared__ double red[4][13];
    // 0 Kt_YY_sum 1 Kt_ZZ_sum 2 K_XY_sum 3 K_XZ_sum 4 <KtYY,KtYY> 5 <KtZZ,KtZZ>
    // 6 <XY1,XY1> 7 <XZ1,XZ1> 8 <XY0,XY0> 9 <XZ0,XZ0> 10 <KtYY,XY0>
    // 11 <KtZZ,XZ0> 12 <XY1,XZ1>
    double v[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < m_; i += 256) {
        const double ky = yy.rows[i] - yy.diag[i], kz = zz.rows[i] - zz.diag[i];
        const double y0 = xy.cols[i], y1 = xy.rows[i], z0 = xz.cols[i], z1 = xz.rows[i];
        v[0] += ky; v[1] += kz; v[2] += y0; v[3] += z0;
        v[4] += ky * ky; v[5] += kz * kz; v[6] += y1 * y1; v[7] += z1 * z1;
        v[8] += y0 * y0; v[9] += z0 * z0; v[10] += ky * y0; v[11] += kz * z0; v[12] += y1 * z1;
    }
    block_sums<13>(v, red);
    if (threadIdx.x != 0) return;
    const double m = m_;
    const double Kt_YY_2_sum = yy.stats[1] - yy.stats[3];
    const double Kt_ZZ_2_sum = zz.stats[1] - zz.stats[3];
    const double K_XY_2_sum = xy.stats[1], K_XZ_2_sum = xz.stats[1];
    const double muY_muY = v[0] / (m * (m - 1));
    const double muZ_muZ = v[1] / (m * (m - 1));
    const double muX_muY = v[2] / (m * m);
    const double muX_muZ = v[3] / (m * m);
    const double E_y_muY_sq = (v[4] - Kt_YY_2_sum) / (m * (m - 1) * (m - 2));
    const double E_z_muZ_sq = (v[5] - Kt_ZZ_2_sum) / (m * (m - 1) * (m - 2));
    const double E_x_muY_sq = (v[6] - K_XY_2_sum) / (m * m * (m - 1));
    const double E_x_muZ_sq = (v[7] - K_XZ_2_sum) / (m * m * (m - 1));
    const double E_y_muX_sq = (v[8] - K_XY_2_sum) / (m * m * (m - 1));
    const double E_z_muX_sq = (v[9] - K_XZ_2_sum) / (m * m * (m - 1));
    const double E_y_muY_y_muX = v[10] / (m * m * (m - 1));
    const double E_z_muZ_z_muX = v[11] / (m * m * (m - 1));
    const double E_x_muY_x_muZ = v[12] / (m * m * m);
    const double E_kyy2 = Kt_YY_2_sum / (m * (m - 1));
    const double E_kzz2 = Kt_ZZ_2_sum / (m * (m - 1));
    const double E_kxy2 = K_XY_2_sum / (m * m);
    const double E_kxz2 = K_XZ_2_sum / (m * m);
    const double mmd2_diff = muY_muY - 2 * muX_muY - muZ_muZ + 2 * muX_muZ;
    const double first_order =
        4 * (m - 2) / (m * (m - 1)) *
        (E_y_muY_sq - muY_muY * muY_muY + E_x_muY_sq - muX_muY * muX_muY + E_y_muX_sq -
         muX_muY * muX_muY + E_z_muZ_sq - muZ_muZ * muZ_muZ + E_x_muZ_sq - muX_muZ * muX_muZ +
         E_z_muX_sq - muX_muZ * muX_muZ - 2 * E_y_muY_y_muX + 2 * muY_muY * muX_muY -
         2 * E_x_muY_x_muZ + 2 * muX_muY * muX_muZ - 2 * E_z_muZ_z_muX + 2 * muZ_muZ * muX_muZ);
    const double second_order =
        2 / (m * (m - 1)) *
        (E_kyy2 - muY_muY * muY_muY + 2 * E_kxy2 - 2 * muX_muY * muX_muY + E_kzz2 -
         muZ_muZ * muZ_muZ + 2 * E_kxz2 - 2 * muX_muZ * muX_muZ - 4 * E_y_muY_y_muX +
         4 * muY_muY * muX_muY - 4 * E_x_muY_x_muZ + 4 * muX_muY * muX_muZ -
         4 * E_z_muZ_z_muX + 4 * muZ_muZ * muX_muZ);
    const double var_est = first_order + second_order;
    out[0] = mmd2_diff;
    out[1] = mmd2_diff / sqrt(fmax(var_est, 1.0e-5));            // _eps, mmd.py:6
}

size_t poly_ws_bytes(int na, int nb, int dim) {
    const size_t nap = gram_pad(na, GT), nbp = gram_pad(nb, GT), dimp = gram_pad(dim, GK);
    size_t b = 0;
    b += align_up(nap * dimp * 4, 256);
    b += align_up(nbp * dimp * 4, 256);
    b += align_up((nbp / GT) * nap * 8, 256);
    b += align_up((nap / GT) * nbp * 8, 256);
    b += align_up((nap / GT) * (nbp / GT) * 4 * 8, 256);
    return b;
}

smmd_status poly_sums_launch(const float *A, int na, const float *B, int nb, int dim, double gamma,
                             double coef0, int degree, double *row_sums, double *col_sums,
                             double *diag, double *stats, void *ws, hipStream_t s) {
    PolyArgs p;
    memset(&p, 0, sizeof(p));
    p.na = na; p.nb = nb;
    p.nap = gram_pad(na, GT); p.nbp = gram_pad(nb, GT); p.dimp = gram_pad(dim, GK);
    p.gamma = (float)gamma; p.coef0 = (float)coef0; p.degree = degree;
    char *q = (char *)ws;
    float *Ap = (float *)q; q += align_up((size_t)p.nap * p.dimp * 4, 256);
    float *Bp = (float *)q; q += align_up((size_t)p.nbp * p.dimp * 4, 256);
    p.rowpart = (double *)q; q += align_up((size_t)(p.nbp / GT) * p.nap * 8, 256);
    p.colpart = (double *)q; q += align_up((size_t)(p.nap / GT) * p.nbp * 8, 256);
    p.slab = (double *)q;
    p.Ap = Ap; p.Bp = Bp;
    p.row_sums = row_sums; p.col_sums = col_sums; p.diag = diag; p.stats = stats;
    hipLaunchKernelGGL(pad_rows_kernel, dim3((p.nap + 3) / 4), dim3(256), 0, s, A, na, dim, Ap,
                       p.nap, p.dimp);
    hipLaunchKernelGGL(pad_rows_kernel, dim3((p.nbp + 3) / 4), dim3(256), 0, s, B, nb, dim, Bp,
                       p.nbp, p.dimp);
    const int nct = p.nbp / GT, nrt = p.nap / GT;
    hipLaunchKernelGGL(poly_tile_kernel, dim3(nct, nrt), dim3(256), 0, s, p);
    const int rmax = na > nb ? na : nb;
    hipLaunchKernelGGL(poly_reduce_kernel, dim3((rmax + 255) / 256), dim3(256), 0, s, p, nct, nrt);
    return last_launch_status();
}

}  // namespace smmd

using namespace smmd;

extern "C" {

size_t smmd_poly_sums_workspace_bytes(int na, int nb, int dim) {
    if (na < 1 || nb < 1 || dim < 1) return 0;
    return poly_ws_bytes(na, nb, dim);
}

smmd_status smmd_poly_kernel_sums(const float *A, int na, const float *B, int nb, int dim,
                                  double gamma, double coef0, int degree, double *row_sums,
                                  double *col_sums, double *diag, double *stats, void *ws,
                                  size_t ws_bytes, smmd_stream_t stream) {
    if (!A || !B || na < 1 || nb < 1 || dim < 1 || degree < 1 || degree > 8) return SMMD_EINVAL;
    if (!ws || ws_bytes < poly_ws_bytes(na, nb, dim)) return SMMD_EWORKSPACE;
    return poly_sums_launch(A, na, B, nb, dim, gamma, coef0, degree, row_sums, col_sums, diag,
                            stats, ws, (hipStream_t)stream);
}

static bool poly_rec(const smmd_poly_sums *r, PolySumsDev &d) {
    if (!r || !r->rows || !r->cols || !r->diag || !r->stats) return false;
    d.rows = r->rows; d.cols = r->cols; d.diag = r->diag; d.stats = r->stats;
    return true;
}

smmd_status smmd_poly_mmd2_var(const smmd_poly_sums *xx, const smmd_poly_sums *yy,
                               const smmd_poly_sums *xy, int m, double var_at_m, int estimator,
                               double *out, smmd_stream_t stream) {
    PolySumsDev a, b, c;
    if (!poly_rec(xx, a) || !poly_rec(yy, b) || !poly_rec(xy, c) || !out || m < 3 ||
        estimator < 0 || estimator > 2)
        return SMMD_EINVAL;
    const double vm = var_at_m > 0 ? var_at_m : (double)m;
    hipLaunchKernelGGL(poly_mmd2_var_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, a, b, c, m,
                       vm, estimator, out);
    return last_launch_status();
}

smmd_status smmd_poly_diff_ratio(const smmd_poly_sums *yy, const smmd_poly_sums *xy,
                                 const smmd_poly_sums *zz, const smmd_poly_sums *xz, int m,
                                 double *out, smmd_stream_t stream) {
    PolySumsDev a, b, c, d;
    if (!poly_rec(yy, a) || !poly_rec(xy, b) || !poly_rec(zz, c) || !poly_rec(xz, d) || !out ||
        m < 3)
        return SMMD_EINVAL;
    hipLaunchKernelGGL(poly_diff_ratio_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, a, b, c,
                       d, m, out);
    return last_launch_status();
}

}  // extern "C"
