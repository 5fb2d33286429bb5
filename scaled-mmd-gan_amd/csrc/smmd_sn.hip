// smmd_sn.hip -- spectral normalisation of every SN layer of a network in one
// set of launches (gfx950 / MI355X).
//
// Reference: gan/core/sn.py:12-59 (power iteration, sigma, W_bar = W/sigma),
// gan/core/snops.py:82-84 (W_eff = s * W_bar), their TF autodiff (backward).
// The TF graph runs ~8 small ops per layer per discriminator call (2 GEMV,
// 2 norms, sigma, RealDiv, Mul, assign).  Here all layers are cut into
// 32 x 256 fp32 tiles (32 KiB) and one launch walks every tile of every layer:
//
//   P1  tile -> partial column sums  sum_rows u_n W[n, k]     (HBM pass 1)
//   P2  tile -> v_raw for its 256 columns from the P1 slab, then partial row
//       dots sum_cols v_raw_k W[n, k]                          (HBM pass 2,
//       usually served by the Infinity Cache: the net fits in 256 MiB)
//   R2  one block per layer: ||v_raw||, v, u_raw, ||u_raw||, u', sigma
//   P3  tile -> W_eff = (W / sigma) * s                        (read + write)
//       ConvMeanPool layers (fold = 1): 256 filters per block -> the 4 x 4
//       pool-folded W' of W_eff written directly (9 floats in, 16 out)
//
// Lanes own 4 consecutive columns (16-byte loads), waves own 8 rows, so a
// wave-instruction reads 1 KiB of one row.  All reductions have a fixed order.
//
// Measured alternative (not kept): P1 electing the last row tile of each column
// tile to reduce v_raw, and P2 electing the last tile of each layer to run R2
// (arrival tickets, write-through partials).  It removes the R2 launch but puts
// each reducer's serial chain of dependent L2 loads at the tail of its kernel:
// P1 11 -> 19 us, P2 + R2 20 -> 34 us on the SNResNet-64 critic.
// Also measured and not kept: P2 + R2 + P3 as ONE launch that reads W once
// (each tile keeps W in registers, row-tile and layer tickets, sigma
// broadcast behind a generation flag that every tile polls, a timeout rescue
// for non-resident grids): 57 us against 35 us for P2 + R2 + P3.  With no
// wait it took 33 us: the re-read P3 saves is served by the Infinity Cache
// (W is 40 MB), while the hand-off chain (about 8 dependent hops of ~2-3 us
// under load) costs 25 us (profiles/r08/sn_p23_experiment.txt).
#include "smmd_sn_tile.hpp"

#ifndef SN_GSTAT_DIRECT
#define SN_GSTAT_DIRECT 1   // smmd_sn_grad_stats' fold units without the LDS stage
#endif

#include <stdlib.h>

namespace smmd {

struct SnLayerDev {
    const float *W;
    float *W_eff;
    float *u;        // user u (read at iteration 0, written when update_u)
    float *v;
    float *sigma;
    const float *s;
    const float *G;
    float *gW;
    float *gs;
    float *p1;       // ws [nrt][K]
    float *vraw;     // ws [K]
    float *q2;       // ws [N][nctp] row partials, one contiguous 16-B aligned row per n
    float *ucur;     // ws [N]  u' of the last iteration
    float *dotp;     // ws [units] backward partial <G, W>
    float *ggp;      // ws [units] partial ||G||^2 (adjoint G for fold layers)
    float *ugvp;     // ws [units] partial u'^T G v
    float *stats;    // ws [16] smmd_sn_grad_stats record (SnGradStats)
    int N, K, nrt, nct;
    int nctp;        // nct rounded up to a multiple of 4
    int tile_begin;
    int vec;         // K % 4 == 0 and 16-byte aligned rows
    int fold;        // W_eff / G are the pool-folded 4 x 4 filters (K = 9 nfc)
    int nfc;         // filters per row (fold)
    int unit_begin;  // first P3 / backward work unit: tiles, or fold blocks
    int p3_begin;    // first unit in the P3 launch (layers it writes; others own 0 units)
    int m3_begin;    // first tile in R2's launch (small plain layers whose W_eff R2 writes)
};

struct SnTable {
    int n_layers;
    int total_tiles;
    int total_units;
    int total_p3;    // units of the P3 launch
    int total_m3;    // W_eff tiles of the R2 launch
    int iter;        // current power iteration (0 -> read layer.u)
    int last_iter;
    int update_u;
    float eps;
    SnLayerDev L[SN_CHUNK];
};

// Layer of a tile: static-index scan of the (monotone) tile_begin fields, then
// readfirstlane so the index is provably wave-uniform and the descriptor is
// read with scalar loads instead of a dependent chain of vector loads.
__device__ __forceinline__ int find_layer(const SnTable &t, int tile) {
    int l = 0;
#pragma unroll
    for (int i = 1; i < SN_CHUNK; ++i)
        l += (i < t.n_layers && tile >= t.L[i].tile_begin) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(l);
}

// layer of a P3 / backward unit (unit_begin is monotone like tile_begin)
__device__ __forceinline__ int find_unit_layer(const SnTable &t, int unit) {
    int l = 0;
#pragma unroll
    for (int i = 1; i < SN_CHUNK; ++i)
        l += (i < t.n_layers && unit >= t.L[i].unit_begin) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(l);
}

// layer of a unit of the P3 launch / of a W_eff tile of the R2 launch.  The
// begins are monotone and a layer with no units shares its begin with the
// next layer, so the scan (the largest i with begin <= unit) never stops at it
__device__ __forceinline__ int find_p3_layer(const SnTable &t, int unit) {
    int l = 0;
#pragma unroll
    for (int i = 1; i < SN_CHUNK; ++i)
        l += (i < t.n_layers && unit >= t.L[i].p3_begin) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(l);
}

__device__ __forceinline__ int find_m3_layer(const SnTable &t, int unit) {
    int l = 0;
#pragma unroll
    for (int i = 1; i < SN_CHUNK; ++i)
        l += (i < t.n_layers && unit >= t.L[i].m3_begin) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(l);
}

// ---- fold layers: one (n, c) filter per thread, 256 per block ---------------
// The block's filters are consecutive (q = n * nfc + c), so its 9-float side
// is the contiguous run W[9 q0, 9 (q0 + nb)) and its 16-float side
// W'[16 q0, 16 (q0 + nb)): both staged through LDS for coalesced float4 global
// accesses.  The fold / adjoint arithmetic is smmd_fold.hip's, in its order.
constexpr int SNF_T = 256;
constexpr int SNF_S16 = SNF_T + 4;      // conflict-free LDS row stride (smmd_fold.hip)

__device__ __forceinline__ void snf_load9(const float *__restrict__ src, float *s9, int n9) {
    const int n4 = n9 >> 2;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    for (int i = threadIdx.x; i < n4; i += SNF_T) {
        const float4 x = s4[i];
        s9[4 * i + 0] = x.x;
        s9[4 * i + 1] = x.y;
        s9[4 * i + 2] = x.z;
        s9[4 * i + 3] = x.w;
    }
    const int t = 4 * n4 + threadIdx.x;
    if (t < n9) s9[t] = src[t];
}

__device__ __forceinline__ void snf_store9(float *__restrict__ dst, const float *s9, int n9) {
    const int n4 = n9 >> 2;
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    for (int i = threadIdx.x; i < n4; i += SNF_T)
        d4[i] = make_float4(s9[4 * i + 0], s9[4 * i + 1], s9[4 * i + 2], s9[4 * i + 3]);
    const int t = 4 * n4 + threadIdx.x;
    if (t < n9) dst[t] = s9[t];
}

__device__ __forceinline__ void snf_load16(const float *__restrict__ src, float *s16, int nb) {
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    for (int i = threadIdx.x; i < nb * 4; i += SNF_T) {
        const int ff = i >> 2, q = i & 3;
        const float4 x = s4[i];
        s16[(q * 4 + 0) * SNF_S16 + ff] = x.x;
        s16[(q * 4 + 1) * SNF_S16 + ff] = x.y;
        s16[(q * 4 + 2) * SNF_S16 + ff] = x.z;
        s16[(q * 4 + 3) * SNF_S16 + ff] = x.w;
    }
}

__device__ __forceinline__ void snf_store16(float *__restrict__ dst, const float *s16, int nb) {
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    for (int i = threadIdx.x; i < nb * 4; i += SNF_T) {
        const int ff = i >> 2, q = i & 3;
        d4[i] = make_float4(s16[(q * 4 + 0) * SNF_S16 + ff], s16[(q * 4 + 1) * SNF_S16 + ff],
                            s16[(q * 4 + 2) * SNF_S16 + ff], s16[(q * 4 + 3) * SNF_S16 + ff]);
    }
}

// adjoint of the fold for thread f's filter: g[u][v] = 1/4 sum_{a,b} G'[u+a][v+b]
__device__ __forceinline__ void snf_adjoint(const float *s16, int f, float (&g)[9]) {
    float k[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) k[j] = s16[j * SNF_S16 + f];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
#pragma unroll
        for (int v = 0; v < 3; ++v) {
            float acc = 0.f;
#pragma unroll
            for (int a = 0; a < 2; ++a) {
#pragma unroll
                for (int b = 0; b < 2; ++b) acc += k[(u + a) * 4 + (v + b)];
            }
            g[u * 3 + v] = acc * 0.25f;
        }
    }
}

// P3 of a fold layer: W' = fold((W / sigma) * s) for the block's filters.
// No contraction: each W_bar element is rounded before the sums (an fma of
// the product into the sum would differ in the last bit), so W' is
// bit-identical to smmd_fold_pool_weights applied to the stored W_eff.
__device__ __forceinline__ void snf_p3(const SnLayerDev &L, int unit) {
#pragma clang fp contract(off)
    __shared__ float s9[SNF_T * 9];
    __shared__ float s16[16 * SNF_S16];
    const int64_t nf = (int64_t)L.N * L.nfc;
    const int64_t q0 = (int64_t)unit * SNF_T;
    const int nb = (int)min<int64_t>(SNF_T, nf - q0);
    snf_load9(L.W + q0 * 9, s9, nb * 9);
    __syncthreads();
    const float sigma = L.sigma[0];
    const float s = L.s ? L.s[0] : 1.f;
    const int f = threadIdx.x;
    if (f < nb) {
        float k[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) k[j] = (s9[f * 9 + j] / sigma) * s;   // sn.py:43, snops.py:84
#pragma unroll
        for (int si = 0; si < 4; ++si) {
#pragma unroll
            for (int ti = 0; ti < 4; ++ti) {
                float acc = 0.f;
#pragma unroll
                for (int a = 0; a < 2; ++a) {
#pragma unroll
                    for (int b = 0; b < 2; ++b) {
                        const int u = si - a, v = ti - b;
                        if (u >= 0 && u < 3 && v >= 0 && v < 3) acc += k[u * 3 + v];
                    }
                }
                s16[(si * 4 + ti) * SNF_S16 + f] = acc * 0.25f;   // block.py:65 mean
            }
        }
    }
    __syncthreads();
    snf_store16(L.W_eff + q0 * 16, s16, nb);
}

// backward A of a fold layer: partial <adj(G'), W> of the block's filters
__device__ __forceinline__ void snf_bwd_a(const SnLayerDev &L, int unit, int lu) {
    __shared__ float s9[SNF_T * 9];
    __shared__ float s16[16 * SNF_S16];
    __shared__ float red[4];
    const int64_t nf = (int64_t)L.N * L.nfc;
    const int64_t q0 = (int64_t)unit * SNF_T;
    const int nb = (int)min<int64_t>(SNF_T, nf - q0);
    snf_load16(L.G + q0 * 16, s16, nb);
    snf_load9(L.W + q0 * 9, s9, nb * 9);
    __syncthreads();
    const int f = threadIdx.x;
    float acc = 0.f;
    if (f < nb) {
        float g[9];
        snf_adjoint(s16, f, g);
#pragma unroll
        for (int j = 0; j < 9; ++j) acc = fmaf(g[j], s9[f * 9 + j], acc);
    }
    acc = block_sum<4>(acc, red);
    if (threadIdx.x == 0) L.dotp[lu] = acc;
}

// backward B of a fold layer: gW = (s adj(G')) / sigma - coef u'_n v_k
__device__ __forceinline__ float layer_dot(const SnLayerDev &L, float *sh);

__device__ __forceinline__ void snf_bwd_b(const SnLayerDev &L, int unit, float *sh_d) {
    __shared__ float s9[SNF_T * 9];
    __shared__ float s16[16 * SNF_S16];
    const int64_t nf = (int64_t)L.N * L.nfc;
    const int64_t q0 = (int64_t)unit * SNF_T;
    const int nb = (int)min<int64_t>(SNF_T, nf - q0);
    snf_load16(L.G + q0 * 16, s16, nb);
    const int f = threadIdx.x;
    float un = 0.f, vk[9];                       // in flight with G' and the dot
    {
        const int64_t q = q0 + (f < nb ? f : 0);
        const int n = (int)(q / L.nfc), c = (int)(q - (int64_t)n * L.nfc);
        un = L.ucur[n];
#pragma unroll
        for (int j = 0; j < 9; ++j) vk[j] = L.v[c * 9 + j];
    }
    const float sigma = L.sigma[0];
    const float s = L.s ? L.s[0] : 1.f;
    const float d = layer_dot(L, sh_d);          // its barrier also publishes s16
    if (unit == 0 && threadIdx.x == 0 && L.gs) L.gs[0] = d / sigma;
    const float coef = (s * d) / (sigma * sigma);
    if (f < nb) {
        const float cu = coef * un;
        float g[9];
        snf_adjoint(s16, f, g);
#pragma unroll
        for (int j = 0; j < 9; ++j) s9[f * 9 + j] = (s * g[j]) / sigma - cu * vk[j];
    }
    __syncthreads();
    snf_store9(L.gW + q0 * 9, s9, nb * 9);
}

__global__ __launch_bounds__(256) void sn_p1_kernel(SnTable t) {
    const int tile = blockIdx.x;
    const SnLayerDev L = t.L[find_layer(t, tile)];
    const int lt = tile - L.tile_begin;
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    const float *uin = (t.iter == 0) ? L.u : L.ucur;
    float4 wt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);
    p1_tile(uin, L.p1, L.N, L.K, rt, r0, c0, wt);
}

// P2 walks each layer's tiles column-major and XCD-aware: the nrt row tiles of
// a column tile run on one XCD, so the P1 slab column they all sum is fetched
// into that L2 once instead of once per row tile on whichever XCD it landed
// (the slab re-read was ~28 MB per refresh on the SNResNet-64 critic, 0.7x
// its 40 MB of W).
__global__ __launch_bounds__(256) void sn_p2_kernel(SnTable t) {
    const int tile = xcd_order(blockIdx.x, t.total_tiles);
    const SnLayerDev L = t.L[find_layer(t, tile)];
    const int lt = tile - L.tile_begin;
    const int ct = lt / L.nrt, rt = lt - ct * L.nrt;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;

    float4 wt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);   // issue the tile loads first

    // v_raw for this tile's columns: fixed-order sum over row tiles of P1.  The
    // slab was just written by other XCDs, so each batch of 16 loads is issued
    // before its adds (one memory round trip per 16 row tiles, not per 4)
    __shared__ float vr[SN_TC];
    {
        const int c = ct * SN_TC + threadIdx.x;
        float s = 0.f;
        if (c < L.K) {
            const float *col = L.p1 + c;
            for (int r0 = 0; r0 < L.nrt; r0 += 16) {
                float t[16];
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    t[j] = (r0 + j < L.nrt) ? col[(size_t)(r0 + j) * L.K] : 0.f;
#pragma unroll
                for (int j = 0; j < 16; ++j)
                    if (r0 + j < L.nrt) s += t[j];
            }
        }
        vr[threadIdx.x] = s;
        if (rt == 0 && c < L.K) L.vraw[c] = s;
    }
    __syncthreads();
    const float v0 = vr[lane * 4 + 0], v1 = vr[lane * 4 + 1];
    const float v2 = vr[lane * 4 + 2], v3 = vr[lane * 4 + 3];
    float part[SN_RPW];
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i)
        part[i] = fmaf(v3, wt[i].w, fmaf(v2, wt[i].z, fmaf(v1, wt[i].y, v0 * wt[i].x)));
    // the wave's 8 row sums by a transposed butterfly: each exchange halves
    // the values a lane carries (10 cross-lane moves instead of 8 x 6); lane
    // 8 i ends with row i's sum
    static_assert(SN_RPW == 8, "P2's row-sum butterfly is written for 8 rows per wave");
    float a4[4], b2[2];
    {
        const bool h = lane & 32;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            a4[j] = (h ? part[4 + j] : part[j]) + __shfl_xor(h ? part[j] : part[4 + j], 32);
    }
    {
        const bool h = lane & 16;
#pragma unroll
        for (int j = 0; j < 2; ++j)
            b2[j] = (h ? a4[2 + j] : a4[j]) + __shfl_xor(h ? a4[j] : a4[2 + j], 16);
    }
    const bool h3 = lane & 8;
    float rsum = (h3 ? b2[1] : b2[0]) + __shfl_xor(h3 ? b2[0] : b2[1], 8);
    rsum += __shfl_xor(rsum, 4);
    rsum += __shfl_xor(rsum, 2);
    rsum += __shfl_xor(rsum, 1);
    const int row = r0 + (lane >> 3);
    if ((lane & 7) == 0 && row < L.N) L.q2[(size_t)row * L.nctp + ct] = rsum;
}

// u_raw[n] * ||v_raw|| = sum over column tiles c < nct of q2[n][c], in order.
// The row is contiguous and 16-B aligned, so all of its loads are issued
// before the first add (the [nct][N] layout cost one L2 round trip per pair).
__device__ __forceinline__ float q2_row_sum(const SnLayerDev &L, int n) {
    const float4 *q = reinterpret_cast<const float4 *>(L.q2 + (size_t)n * L.nctp);
    const int n4 = L.nctp >> 2;
    float s = 0.f;
    for (int j0 = 0; j0 < n4; j0 += 8) {
        float4 b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            b[j] = (j0 + j < n4) ? q[j0 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = (j0 + j) * 4;
            if (c + 0 < L.nct) s += b[j].x;
            if (c + 1 < L.nct) s += b[j].y;
            if (c + 2 < L.nct) s += b[j].z;
            if (c + 3 < L.nct) s += b[j].w;
        }
    }
    return s;
}

// norms, v, u', sigma of one layer (sn.py:12-13, :38-42) by one 1024-thread
// block, from v_raw [K] and the row partials q2.  With r_n = (W v_raw)_n:
//   nv = ||v_raw|| + eps, u_raw = r / nv, nu = ||u_raw|| + eps,
//   u' = u_raw / nu, sigma = u_raw . u' = ||u_raw||^2 / nu.
// Every input is loaded up front and the two norms share ONE block
// reduction (||u_raw||^2 = sum r_n^2 / nv^2), so the block makes one round
// of dependent global loads instead of four.
constexpr int EP_KREG = 8;    // v_raw values per thread kept in registers (K <= 8192)
constexpr int EP_NREG = 2;    // rows per thread kept in registers (N <= 2048)

struct SnNorms {
    double sa, uu;   // ||v_raw||^2, ||u_raw||^2
    float nv, nu;
};

// The norms of one layer by a 1024-thread block (every thread gets them); vr
// and rs keep this thread's v_raw values and row sums.  The same code, so the
// same bits, in R2's layer block and in R2's W_eff tiles (sn_m3_tile).  Only a
// layer with N > EP_NREG * 1024 writes (raw u into ucur), and such a layer
// has no W_eff tiles in R2.
__device__ __forceinline__ SnNorms sn_layer_norms(const SnTable &t, const SnLayerDev &L,
                                                  float (&vr)[EP_KREG], float (&rs)[EP_NREG],
                                                  double *red) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
    for (int j = 0; j < EP_KREG; ++j) {
        const int k = tid + j * 1024;
        vr[j] = (k < L.K) ? L.vraw[k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < EP_NREG; ++j) {
        const int n = tid + j * 1024;
        rs[j] = (n < L.N) ? q2_row_sum(L, n) : 0.f;
    }
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int j = 0; j < EP_KREG; ++j) a += (double)vr[j] * (double)vr[j];
    for (int k = tid + EP_KREG * 1024; k < L.K; k += 1024) {
        const double x = (double)L.vraw[k];
        a += x * x;
    }
#pragma unroll
    for (int j = 0; j < EP_NREG; ++j) b += (double)rs[j] * (double)rs[j];
    for (int n = tid + EP_NREG * 1024; n < L.N; n += 1024) {      // rare: N > 2048
        const float r = q2_row_sum(L, n);
        L.ucur[n] = r;
        b += (double)r * (double)r;
    }
    a = wave_sum(a);
    b = wave_sum(b);
    __syncthreads();
    if (lane == 0) {
        red[w] = a;
        red[16 + w] = b;
    }
    __syncthreads();
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        sa += red[i];
        sb += red[16 + i];
    }
    SnNorms q;
    q.sa = sa;
    q.nv = (float)sqrt(sa) + t.eps;                             // sn.py:13
    q.uu = sb / ((double)q.nv * (double)q.nv);                  // ||u_raw||^2
    q.nu = (float)sqrt(q.uu) + t.eps;
    return q;
}

__device__ void sn_layer_epilogue(const SnTable &t, const SnLayerDev &L, int last_iter,
                                  double *red) {
    const int tid = threadIdx.x;
    float vr[EP_KREG], rs[EP_NREG];
    const SnNorms q = sn_layer_norms(t, L, vr, rs, red);
    const double sa = q.sa, uu = q.uu;
    const float nv = q.nv, nu = q.nu;
#pragma unroll
    for (int j = 0; j < EP_KREG; ++j) {
        const int k = tid + j * 1024;
        if (k < L.K) L.v[k] = vr[j] / nv;
    }
    for (int k = tid + EP_KREG * 1024; k < L.K; k += 1024) L.v[k] = L.vraw[k] / nv;
    const bool upd = t.update_u && last_iter;
#pragma unroll
    for (int j = 0; j < EP_NREG; ++j) {
        const int n = tid + j * 1024;
        if (n < L.N) {
            const float un = (rs[j] / nv) / nu;                 // u' = l2n(v W)
            L.ucur[n] = un;
            if (upd) L.u[n] = un;
        }
    }
    for (int n = tid + EP_NREG * 1024; n < L.N; n += 1024) {
        const float un = (L.ucur[n] / nv) / nu;
        L.ucur[n] = un;
        if (upd) L.u[n] = un;
    }
    if (tid == 0) {
        L.sigma[0] = (float)(uu / (double)nu);     // (v W) . u', sn.py:42
        // ||v||^2 and ||u'||^2 for the G-direct clip norm (sn_gstat_r_kernel)
        L.stats[4] = (float)(sa / ((double)nv * (double)nv));
        L.stats[5] = (float)(uu / ((double)nu * (double)nu));
    }
}

// W_eff of one 32 x 256 tile of a small plain layer inside R2's launch: the
// block forms sigma itself from v_raw and the row partials, with the layer
// block's code (so its bits), instead of a P3 launch waiting for R2.  The
// redundant reads, (nctp N + K) floats per tile, are bounded by the tile's own
// 8 K (m3_fits); 16 waves x 2 rows.
constexpr int M3_RPW = SN_TR / 16;
static_assert(SN_TR % 16 == 0, "R2's W_eff tiles: 16 waves over the tile rows");

__device__ __forceinline__ void sn_m3_tile(const SnTable &t, const SnLayerDev &L, int lt,
                                           double *red) {
    const int rt = lt / L.nct, ct = lt - (lt / L.nct) * L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * M3_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    float4 wt[M3_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);    // in flight with the norms' loads
    float vr[EP_KREG], rs[EP_NREG];
    const SnNorms q = sn_layer_norms(t, L, vr, rs, red);
    const float sigma = (float)(q.uu / (double)q.nu);           // R2's sigma, bit for bit
    const float s = L.s ? L.s[0] : 1.f;
#pragma unroll
    for (int i = 0; i < M3_RPW; ++i) {
        // W_bar = W / sigma (sn.py:43), then s * W_bar (snops.py:84)
        wt[i].x = (wt[i].x / sigma) * s;
        wt[i].y = (wt[i].y / sigma) * s;
        wt[i].z = (wt[i].z / sigma) * s;
        wt[i].w = (wt[i].w / sigma) * s;
    }
    store_tile(L.W_eff, L.N, L.K, L.vec, r0, c0, wt);
}

// R2: one 1024-thread block per layer runs the epilogue; on the last
// iteration the blocks after them write the small layers' W_eff tiles
__global__ __launch_bounds__(1024) void sn_r2_kernel(SnTable t) {
    __shared__ double red[32];
    if ((int)blockIdx.x < t.n_layers) {
        sn_layer_epilogue(t, t.L[blockIdx.x], t.last_iter, red);
        return;
    }
    const int unit = blockIdx.x - t.n_layers;
    const SnLayerDev &L = t.L[find_m3_layer(t, unit)];
    sn_m3_tile(t, L, unit - L.m3_begin, red);
}

// P3 over the units of the layers it writes (W_eff not NULL, not R2's)
__global__ __launch_bounds__(256) void sn_p3_kernel(SnTable t) {
    const int unit = blockIdx.x;
    const SnLayerDev L = t.L[find_p3_layer(t, unit)];
    const int lt = unit - L.p3_begin;
    if (L.fold) {
        snf_p3(L, lt);
        return;
    }
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    const float sigma = L.sigma[0];
    const float s = L.s ? L.s[0] : 1.f;
    float4 wt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);
    const bool full_cols = (c0 + 3 < L.K);
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) {
        const int r = r0 + i;
        if (r >= L.N) break;
        // W_bar = W / sigma (sn.py:43), then s * W_bar (snops.py:84)
        float4 o;
        o.x = (wt[i].x / sigma) * s;
        o.y = (wt[i].y / sigma) * s;
        o.z = (wt[i].z / sigma) * s;
        o.w = (wt[i].w / sigma) * s;
        float *p = L.W_eff + (size_t)r * L.K + c0;
        if (L.vec && full_cols) {
            *reinterpret_cast<float4 *>(p) = o;
        } else {
            if (c0 + 0 < L.K) p[0] = o.x;
            if (c0 + 1 < L.K) p[1] = o.y;
            if (c0 + 2 < L.K) p[2] = o.z;
            if (c0 + 3 < L.K) p[3] = o.w;
        }
    }
}

// backward A: partial <G, W> per unit (tile, or fold block)
__global__ __launch_bounds__(256) void sn_bwd_a_kernel(SnTable t) {
    const int unit = blockIdx.x;
    const SnLayerDev L = t.L[find_unit_layer(t, unit)];
    if (!L.G) return;                            // a layer of another group this call
    const int lt = unit - L.unit_begin;
    if (L.fold) {
        snf_bwd_a(L, lt, lt);
        return;
    }
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    float4 wt[SN_RPW], gt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);
    load_tile(L.G, L.N, L.K, L.vec, r0, c0, gt);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) {
        acc = fmaf(gt[i].x, wt[i].x, acc);
        acc = fmaf(gt[i].y, wt[i].y, acc);
        acc = fmaf(gt[i].z, wt[i].z, acc);
        acc = fmaf(gt[i].w, wt[i].w, acc);
    }
    __shared__ float red[4];
    acc = block_sum<4>(acc, red);
    if (threadIdx.x == 0) L.dotp[lt] = acc;
}

// units of a layer in the P3 / backward launches
__device__ __forceinline__ int layer_units(const SnLayerDev &L) {
    return L.fold ? (int)(((int64_t)L.N * L.nfc + SNF_T - 1) / SNF_T) : L.nrt * L.nct;
}

// <G, W> of the unit's layer: wave 0 sums the layer's A partials in a fixed
// order; every thread gets it.  Called after the unit's G loads are issued, so
// the two memory round trips overlap.
__device__ __forceinline__ float layer_dot(const SnLayerDev &L, float *sh) {
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < 64) {
        double d = strided_sum(L.dotp, lane, layer_units(L), 64);
        d = wave_sum(d);
        if (lane == 0) sh[0] = (float)d;
    }
    __syncthreads();
    return sh[0];
}

// backward B: gW = (s G)/sigma - (s <G,W> / sigma^2) u' v^T ; gs = <G,W>/sigma
__global__ __launch_bounds__(256) void sn_bwd_b_kernel(SnTable t) {
    const int unit = blockIdx.x;
    const SnLayerDev L = t.L[find_unit_layer(t, unit)];
    if (!L.G) return;
    const int lt = unit - L.unit_begin;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ float sh_d[1];
    if (L.fold) {
        snf_bwd_b(L, lt, sh_d);
        return;
    }
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    float4 gt[SN_RPW];
    load_tile(L.G, L.N, L.K, L.vec, r0, c0, gt);
    float vv[4], uc[SN_RPW];                       // in flight with G and the dot
#pragma unroll
    for (int k = 0; k < 4; ++k) vv[k] = (c0 + k < L.K) ? L.v[c0 + k] : 0.f;
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) uc[i] = (r0 + i < L.N) ? L.ucur[r0 + i] : 0.f;
    const float sigma = L.sigma[0];
    const float s = L.s ? L.s[0] : 1.f;
    const float d = layer_dot(L, sh_d);            // <G, W>
    if (lt == 0 && threadIdx.x == 0 && L.gs) L.gs[0] = d / sigma;
    const float coef = (s * d) / (sigma * sigma);  // -dsigma factor
    const bool full_cols = (c0 + 3 < L.K);
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) {
        const int r = r0 + i;
        if (r >= L.N) break;
        const float cu = coef * uc[i];
        float4 o;
        o.x = (s * gt[i].x) / sigma - cu * vv[0];
        o.y = (s * gt[i].y) / sigma - cu * vv[1];
        o.z = (s * gt[i].z) / sigma - cu * vv[2];
        o.w = (s * gt[i].w) / sigma - cu * vv[3];
        float *p = L.gW + (size_t)r * L.K + c0;
        if (L.vec && full_cols) {
            *reinterpret_cast<float4 *>(p) = o;
        } else {
            if (c0 + 0 < L.K) p[0] = o.x;
            if (c0 + 1 < L.K) p[1] = o.y;
            if (c0 + 2 < L.K) p[2] = o.z;
            if (c0 + 3 < L.K) p[3] = o.w;
        }
    }
}

// The layer sums of the gstat partials (4 waves, each lane strided by 256, 8
// loads per slab in flight; waves added in order), then the record {coef,
// ||dL/dW||^2, sigma, s} and gs.

__device__ __forceinline__ void gstat_finish(const SnLayerDev &L) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int units = layer_units(L);
    // the record's inputs (earlier launches' writes) in flight with the partials
    const double vv = L.stats[4], uu = L.stats[5];   // ||v||^2, ||u'||^2 (refresh R2)
    const float sigma = L.sigma[0];
    const float s = L.s ? L.s[0] : 1.f;
    double dd = 0.0, gg = 0.0, ug = 0.0;
    for (int base = threadIdx.x; base < units; base += 8 * 256) {
        float a[8], b[8], c[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = base + j * 256;
            a[j] = (i < units) ? L.dotp[i] : 0.f;
            b[j] = (i < units) ? L.ggp[i] : 0.f;
            c[j] = (i < units) ? L.ugvp[i] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            dd += (double)a[j];
            gg += (double)b[j];
            ug += (double)c[j];
        }
    }
    __shared__ double red[3][4];
    dd = wave_sum(dd);
    gg = wave_sum(gg);
    ug = wave_sum(ug);
    if (lane == 0) {
        red[0][w] = dd;
        red[1][w] = gg;
        red[2][w] = ug;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        dd = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
        gg = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
        ug = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
        const float d = (float)dd;
        if (L.gs) L.gs[0] = d / sigma;                   // dL/ds, as sn_bwd_b
        const float coef = (s * d) / (sigma * sigma);    // as sn_bwd_b
        const double a = (double)s / (double)sigma;
        double nsq = a * a * gg - 2.0 * a * (double)coef * ug +
                     (double)coef * (double)coef * uu * vv;
        if (!(nsq > 0.0)) nsq = 0.0;
        L.stats[0] = coef;
        L.stats[1] = (float)nsq;
        L.stats[2] = sigma;
        L.stats[3] = s;
    }
}

// ---- gradient statistics for the G-direct update (smmd_sn_grad_stats) ------
// Instead of writing dL/dW, the backward reduces what the optimizer needs to
// form it on the fly from G (smmd_adam_flat_sn2, SMMD_ADAM_SN_GDIRECT):
// d = <G, W> (sn_bwd_a's partials; the layer sum in a fixed order of its own),
// ||G||^2 and u'^T G v (G = the adjoint of G' on fold layers).  Then per
// layer: gs = d / sigma, coef = s d / sigma^2 and the clip norm
// ||dL/dW||^2 = a^2 ||G||^2 - 2 a coef u'^T G v + coef^2 ||u'||^2 ||v||^2
// with a = s / sigma (dL/dW = a G - coef u' v^T).
__global__ __launch_bounds__(256) void sn_gstat_a_kernel(SnTable t) {
    const int unit = blockIdx.x;
    const SnLayerDev L = t.L[find_unit_layer(t, unit)];
    if (!L.G) return;                            // this call skips the layer
    const int lt = unit - L.unit_begin;
    float ad = 0.f, ag = 0.f, au = 0.f;
#if SN_GSTAT_DIRECT
    if (L.fold) {
        // each thread its own filter straight from global memory (G' as four
        // float4, W as nine floats): no LDS stage and no barrier, the same
        // arithmetic in the same order as the staged form (snf_adjoint)
        const uint32_t nf = (uint32_t)L.N * (uint32_t)L.nfc;
        const uint32_t q = (uint32_t)lt * SNF_T + threadIdx.x;
        if (q < nf) {
            const float4 *g4 = reinterpret_cast<const float4 *>(L.G) + (size_t)q * 4;
            const float4 k0 = g4[0], k1 = g4[1], k2 = g4[2], k3 = g4[3];
            const float *wq = L.W + (size_t)q * 9;
            float wv[9], vk[9];
#pragma unroll
            for (int j = 0; j < 9; ++j) wv[j] = wq[j];
            const uint32_t n = q / (uint32_t)L.nfc, c = q - n * (uint32_t)L.nfc;
            const float un = L.ucur[n];
#pragma unroll
            for (int j = 0; j < 9; ++j) vk[j] = L.v[c * 9 + j];
            const float k[16] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w,
                                 k2.x, k2.y, k2.z, k2.w, k3.x, k3.y, k3.z, k3.w};
            float gv = 0.f;
#pragma unroll
            for (int u = 0; u < 3; ++u)
#pragma unroll
                for (int v = 0; v < 3; ++v) {
                    float acc = 0.f;
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int b = 0; b < 2; ++b) acc += k[(u + a) * 4 + (v + b)];
                    const float g = acc * 0.25f;
                    const int j = u * 3 + v;
                    ad = fmaf(g, wv[j], ad);
                    ag = fmaf(g, g, ag);
                    gv = fmaf(g, vk[j], gv);
                }
            au = un * gv;
        }
    } else
#else
    if (L.fold) {
        __shared__ float s9[SNF_T * 9];
        __shared__ float s16[16 * SNF_S16];
        const int64_t nf = (int64_t)L.N * L.nfc;
        const int64_t q0 = (int64_t)lt * SNF_T;
        const int nb = (int)min<int64_t>(SNF_T, nf - q0);
        snf_load16(L.G + q0 * 16, s16, nb);
        snf_load9(L.W + q0 * 9, s9, nb * 9);
        const int f = threadIdx.x;
        float un = 0.f, vk[9];
        {
            const int64_t q = q0 + (f < nb ? f : 0);
            const int n = (int)(q / L.nfc), c = (int)(q - (int64_t)n * L.nfc);
            un = L.ucur[n];
#pragma unroll
            for (int j = 0; j < 9; ++j) vk[j] = L.v[c * 9 + j];
        }
        __syncthreads();
        if (f < nb) {
            float g[9];
            snf_adjoint(s16, f, g);
            float gv = 0.f;
#pragma unroll
            for (int j = 0; j < 9; ++j) {
                ad = fmaf(g[j], s9[f * 9 + j], ad);
                ag = fmaf(g[j], g[j], ag);
                gv = fmaf(g[j], vk[j], gv);
            }
            au = un * gv;
        }
    } else
#endif
    {
        const int rt = lt / L.nct, ct = lt % L.nct;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        const int r0 = rt * SN_TR + w * SN_RPW;
        const int c0 = ct * SN_TC + lane * 4;
        float4 wt[SN_RPW], gt[SN_RPW];
        load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);
        load_tile(L.G, L.N, L.K, L.vec, r0, c0, gt);
        float vv[4], uc[SN_RPW];
#pragma unroll
        for (int k = 0; k < 4; ++k) vv[k] = (c0 + k < L.K) ? L.v[c0 + k] : 0.f;
#pragma unroll
        for (int i = 0; i < SN_RPW; ++i) uc[i] = (r0 + i < L.N) ? L.ucur[r0 + i] : 0.f;
#pragma unroll
        for (int i = 0; i < SN_RPW; ++i) {
            ad = fmaf(gt[i].x, wt[i].x, ad);
            ad = fmaf(gt[i].y, wt[i].y, ad);
            ad = fmaf(gt[i].z, wt[i].z, ad);
            ad = fmaf(gt[i].w, wt[i].w, ad);
            ag = fmaf(gt[i].x, gt[i].x, ag);
            ag = fmaf(gt[i].y, gt[i].y, ag);
            ag = fmaf(gt[i].z, gt[i].z, ag);
            ag = fmaf(gt[i].w, gt[i].w, ag);
            const float gv = fmaf(gt[i].w, vv[3], fmaf(gt[i].z, vv[2],
                                  fmaf(gt[i].y, vv[1], gt[i].x * vv[0])));
            au = fmaf(uc[i], gv, au);
        }
    }
    // the three block sums through one barrier (block_sum's order, so its bits)
    ad = wave_sum(ad);
    ag = wave_sum(ag);
    au = wave_sum(au);
    __shared__ float red3[3][4];
    {
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        if (lane == 0) {
            red3[0][w] = ad;
            red3[1][w] = ag;
            red3[2][w] = au;
        }
    }
    __syncthreads();
    ad = ag = au = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ad += red3[0][i];
        ag += red3[1][i];
        au += red3[2][i];
    }
    // Measured and not kept: the layer's last unit reducing the partials in
    // this launch (write-through partials, one arrival ticket per unit on a
    // per-layer counter): 30 -> 45 us per call, the 2048 units of the largest
    // layer serialising on one counter's atomics
    if (threadIdx.x == 0) {
        L.dotp[lt] = ad;
        L.ggp[lt] = ag;
        L.ugvp[lt] = au;
    }
}

// one 256-thread block per layer: the layer sums and the record
__global__ __launch_bounds__(256) void sn_gstat_r_kernel(SnTable t) {
    const SnLayerDev &L = t.L[blockIdx.x];
    if (!L.G) return;
    gstat_finish(L);
}

// ---------------------------------------------------------------------------
// host side: workspace carve and launch sets
// ---------------------------------------------------------------------------
static int ceil_div(int a, int b) { return (a + b - 1) / b; }

// backward partials of a layer: one per tile, or per fold block (K = 9 C)
static int64_t dotp_slots(int N, int K) {
    const int64_t tiles = (int64_t)ceil_div(N, SN_TR) * ceil_div(K, SN_TC);
    const int64_t fblk = (K % 9 == 0) ? ((int64_t)N * (K / 9) + SNF_T - 1) / SNF_T : 0;
    return tiles > fblk ? tiles : fblk;
}

static size_t layer_ws_bytes(int N, int K) {
    const int nrt = ceil_div(N, SN_TR), nct = ceil_div(K, SN_TC);
    size_t b = 0;
    b += align_up((size_t)nrt * K * 4, 256);   // p1
    b += align_up((size_t)K * 4, 256);         // vraw
    b += align_up((size_t)((nct + 3) & ~3) * N * 4, 256);   // q2
    b += align_up((size_t)N * 4, 256);         // ucur
    b += align_up((size_t)dotp_slots(N, K) * 4, 256);       // dotp
    b += 2 * align_up((size_t)dotp_slots(N, K) * 4, 256);   // ggp, ugvp
    b += 256;                                                // stats
    return b;
}

static bool build_table(const smmd_sn_layer *layers, int first, int count, char *ws,
                        SnTable &t) {
    memset(&t, 0, sizeof(t));
    t.n_layers = count;
    int tiles = 0;
    int64_t units = 0;
    // every chunk gets the workspace region of its layers (by global index)
    size_t off = 0;
    for (int i = 0; i < first; ++i) off += layer_ws_bytes(layers[i].N, layers[i].K);
    for (int i = 0; i < count; ++i) {
        const smmd_sn_layer &src = layers[first + i];
        if (!src.W || src.N < 1 || src.K < 1) return false;
        SnLayerDev &L = t.L[i];
        L.W = src.W;
        L.W_eff = src.W_eff;
        L.u = src.u;
        L.v = src.v;
        L.sigma = src.sigma;
        L.s = src.s;
        L.G = src.G;
        L.gW = src.gW;
        L.gs = src.gs;
        L.N = src.N;
        L.K = src.K;
        L.nrt = ceil_div(src.N, SN_TR);
        L.nct = ceil_div(src.K, SN_TC);
        L.tile_begin = tiles;
        tiles += L.nrt * L.nct;
        const uintptr_t al = (uintptr_t)src.W | (uintptr_t)(src.W_eff ? src.W_eff : src.W) |
                             (uintptr_t)(src.G ? src.G : src.W) | (uintptr_t)(src.gW ? src.gW : src.W);
        L.vec = (src.K % 4 == 0) && (al % 16 == 0);
        if (src.fold != 0 && src.fold != 1) return false;
        L.fold = src.fold;
        if (L.fold) {
            // whole filters, float4 staging of both sides
            if (src.K % 9 != 0 || (al % 16) != 0) return false;
            L.nfc = src.K / 9;
        }
        L.unit_begin = (int)units;
        const int64_t lu = L.fold ? ((int64_t)src.N * L.nfc + SNF_T - 1) / SNF_T
                                  : (int64_t)L.nrt * L.nct;
        units += lu;
        if (units > 0x7fffffff) return false;
        L.nctp = (L.nct + 3) & ~3;
        // W_eff written by R2's launch (small plain layers: the tile's redundant
        // norm reads <= its own 8 K floats) or by P3 (the rest)
        const bool m3 = src.W_eff && !L.fold && L.N <= EP_NREG * 1024 && L.K <= EP_KREG * 1024 &&
                        (int64_t)L.nctp * L.N + L.K <= (int64_t)SN_TR * SN_TC;
        L.m3_begin = t.total_m3;
        L.p3_begin = t.total_p3;
        if (m3) t.total_m3 += (int)lu;
        else if (src.W_eff) t.total_p3 += (int)lu;
        char *p = ws + off;
        L.p1 = (float *)p;   p += align_up((size_t)L.nrt * L.K * 4, 256);
        L.vraw = (float *)p; p += align_up((size_t)L.K * 4, 256);
        L.q2 = (float *)p;   p += align_up((size_t)L.nctp * L.N * 4, 256);
        L.ucur = (float *)p; p += align_up((size_t)L.N * 4, 256);
        L.dotp = (float *)p; p += align_up((size_t)dotp_slots(L.N, L.K) * 4, 256);
        L.ggp = (float *)p;  p += align_up((size_t)dotp_slots(L.N, L.K) * 4, 256);
        L.ugvp = (float *)p; p += align_up((size_t)dotp_slots(L.N, L.K) * 4, 256);
        L.stats = (float *)p; p += 256;
        off += layer_ws_bytes(L.N, L.K);
    }
    t.total_tiles = tiles;
    t.total_units = (int)units;
    return true;
}

smmd_status sn_adam_table(const smmd_sn_layer *layers, const int32_t *sn_tensor, int n_layers,
                          const SnAdamHost &a, void *sn_ws, size_t sn_ws_bytes, SnAdamTable &t) {
    if (n_layers < 1 || n_layers > SN_CHUNK) return SMMD_EUNSUPPORTED;
    if (!sn_ws || sn_ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    SnTable st;
    if (!build_table(layers, 0, n_layers, (char *)sn_ws + 256, st)) return SMMD_EINVAL;
    memset(&t, 0, sizeof(t));
    t.n_layers = n_layers;
    t.total_tiles = st.total_tiles;
    for (int i = 0; i < n_layers; ++i) {
        const smmd_sn_layer &src = layers[i];
        const int ti = sn_tensor[i];
        const int64_t off = a.offsets[ti];
        // the SN weight must be tensor ti of the flat buffer, N x K rows
        if (!src.u || src.W != a.param + off || a.offsets[ti + 1] - off < (int64_t)src.N * src.K)
            return SMMD_EINVAL;
        SnAdamLayerDev &L = t.L[i];
        L.p = const_cast<float *>(a.param) + off;
        L.m = const_cast<float *>(a.m) + off;
        L.v = const_cast<float *>(a.v) + off;
        L.g = a.grad + off;
        L.u = src.u;
        L.p1 = st.L[i].p1;
        L.N = src.N;
        L.K = src.K;
        L.nct = st.L[i].nct;
        L.tile_begin = st.L[i].tile_begin;
        const uintptr_t al = (uintptr_t)L.p | (uintptr_t)L.m | (uintptr_t)L.v | (uintptr_t)L.g;
        L.vec = (src.K % 4 == 0) && (al % 16 == 0);
        L.sb0 = a.sblk[ti];
        L.sb1 = a.sblk[ti + 1];
        L.G = nullptr;
        if (a.gdirect) {
            // dL/dW formed from G and the smmd_sn_grad_stats record
            if (!src.G || !src.v || (src.fold && (src.K % 9 != 0 || ((uintptr_t)src.G & 15))))
                return SMMD_EINVAL;
            L.G = src.G;
            L.ucur = st.L[i].ucur;
            L.vsn = src.v;
            L.stats = st.L[i].stats;
            L.fold = src.fold;
            L.nfc = src.fold ? src.K / 9 : 0;
            L.gvec = !src.fold && (src.K % 4 == 0) && ((uintptr_t)src.G % 16 == 0);
        }
    }
    return SMMD_OK;
}

}  // namespace smmd

using namespace smmd;

extern "C" {

size_t smmd_sn_workspace_bytes(const smmd_sn_layer *layers, int n_layers) {
    if (!layers || n_layers < 1) return 0;
    size_t b = 256;
    for (int i = 0; i < n_layers; ++i) b += layer_ws_bytes(layers[i].N, layers[i].K);
    return b;
}

smmd_status smmd_sn_power_iter(const smmd_sn_layer *layers, int n_layers, int num_iters,
                               float eps, int update_u, void *ws, size_t ws_bytes,
                               smmd_stream_t stream) {
    return smmd_sn_power_iter_ex(layers, n_layers, num_iters, eps, update_u, 0, ws, ws_bytes,
                                 stream);
}

smmd_status smmd_sn_power_iter_ex(const smmd_sn_layer *layers, int n_layers, int num_iters,
                                  float eps, int update_u, int flags, void *ws, size_t ws_bytes,
                                  smmd_stream_t stream) {
    if (flags & ~SMMD_SN_P1_READY) return SMMD_EINVAL;
    if (!layers || n_layers < 1 || n_layers > SMMD_SN_MAX_LAYERS || num_iters < 1)
        return SMMD_EINVAL;
    for (int i = 0; i < n_layers; ++i)
        if (!layers[i].u || !layers[i].v || !layers[i].sigma) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    for (int first = 0; first < n_layers; first += SN_CHUNK) {
        const int count = (n_layers - first < SN_CHUNK) ? n_layers - first : SN_CHUNK;
        SnTable t;
        if (!build_table(layers, first, count, (char *)ws + 256, t)) return SMMD_EINVAL;
        t.eps = eps;
        t.update_u = update_u ? 1 : 0;
        for (int it = 0; it < num_iters; ++it) {
            t.iter = it;
            t.last_iter = (it == num_iters - 1);
            if (it > 0 || !(flags & SMMD_SN_P1_READY))   // else written by smmd_adam_flat_sn
                hipLaunchKernelGGL(sn_p1_kernel, dim3(t.total_tiles), dim3(256), 0, s, t);
            hipLaunchKernelGGL(sn_p2_kernel, dim3(t.total_tiles), dim3(256), 0, s, t);
            const int m3 = t.last_iter ? t.total_m3 : 0;
            hipLaunchKernelGGL(sn_r2_kernel, dim3(t.n_layers + m3), dim3(1024), 0, s, t);
        }
        if (t.total_p3 > 0)
            hipLaunchKernelGGL(sn_p3_kernel, dim3(t.total_p3), dim3(256), 0, s, t);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

// The per-rank clip of the G-direct data-parallel tower mode
// (smmd_sn_clip_g): G *= c / max(||dL/dW||, c) with the norm of the layer's
// smmd_sn_grad_stats record (dL/dW is linear in G, so this is clip_by_norm of
// the rank's dL/dW, model.py:449-455) and gs *= c / max(|gs|, c).
// Grid (element blocks, layer); float4 over the layer's contiguous G.
__global__ __launch_bounds__(256) void sn_clip_g_kernel(SnTable t, float clip) {
    const SnLayerDev L = t.L[blockIdx.y];
    if (!L.G) return;
    const float ss = L.stats[1];
    const float inv = (ss > 0.f) ? rsqrtf(ss) : INFINITY;
    const float f = clip * fminf(inv, 1.f / clip);
    float *G = const_cast<float *>(L.G);
    const int64_t n = (int64_t)L.N * L.K;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (L.vec) {
        float4 *G4 = reinterpret_cast<float4 *>(G);
        for (; i < n / 4; i += stride) {
            float4 v = G4[i];
            v.x *= f; v.y *= f; v.z *= f; v.w *= f;
            G4[i] = v;
        }
    } else {
        for (; i < n; i += stride) G[i] *= f;
    }
    if (L.gs && blockIdx.x == 0 && threadIdx.x == 0) {
        const float g = L.gs[0], a = fabsf(g);
        L.gs[0] = g * (clip * fminf(a > 0.f ? 1.f / a : INFINITY, 1.f / clip));
    }
}

smmd_status smmd_sn_clip_g(const smmd_sn_layer *layers, int n_layers, float clip, void *ws,
                           size_t ws_bytes, smmd_stream_t stream) {
    if (!layers || n_layers < 1 || n_layers > SMMD_SN_MAX_LAYERS || !(clip > 0.f))
        return SMMD_EINVAL;
    for (int i = 0; i < n_layers; ++i)
        if (layers[i].G && layers[i].fold) return SMMD_EINVAL;    // W-shaped G only
    if (!ws || ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    for (int first = 0; first < n_layers; first += SN_CHUNK) {
        const int count = (n_layers - first < SN_CHUNK) ? n_layers - first : SN_CHUNK;
        SnTable t;
        if (!build_table(layers, first, count, (char *)ws + 256, t)) return SMMD_EINVAL;
        hipLaunchKernelGGL(sn_clip_g_kernel, dim3(64, t.n_layers), dim3(256), 0, s, t, clip);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

smmd_status smmd_sn_grad_stats(const smmd_sn_layer *layers, int n_layers, void *ws,
                               size_t ws_bytes, smmd_stream_t stream) {
    if (!layers || n_layers < 1 || n_layers > SMMD_SN_MAX_LAYERS) return SMMD_EINVAL;
    int any = 0;
    for (int i = 0; i < n_layers; ++i) {
        if (!layers[i].v || !layers[i].sigma) return SMMD_EINVAL;
        any |= layers[i].G != nullptr;       // a layer with G NULL is skipped
    }
    if (!any) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    for (int first = 0; first < n_layers; first += SN_CHUNK) {
        const int count = (n_layers - first < SN_CHUNK) ? n_layers - first : SN_CHUNK;
        SnTable t;
        if (!build_table(layers, first, count, (char *)ws + 256, t)) return SMMD_EINVAL;
        hipLaunchKernelGGL(sn_gstat_a_kernel, dim3(t.total_units), dim3(256), 0, s, t);
        hipLaunchKernelGGL(sn_gstat_r_kernel, dim3(t.n_layers), dim3(256), 0, s, t);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

smmd_status smmd_sn_weight_bwd(const smmd_sn_layer *layers, int n_layers, void *ws,
                               size_t ws_bytes, smmd_stream_t stream) {
    if (!layers || n_layers < 1 || n_layers > SMMD_SN_MAX_LAYERS) return SMMD_EINVAL;
    int any = 0;
    for (int i = 0; i < n_layers; ++i) {
        if (!layers[i].G) continue;              // skipped (its gradient comes another call)
        if (!layers[i].gW || !layers[i].v || !layers[i].sigma) return SMMD_EINVAL;
        any = 1;
    }
    if (!any) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    for (int first = 0; first < n_layers; first += SN_CHUNK) {
        const int count = (n_layers - first < SN_CHUNK) ? n_layers - first : SN_CHUNK;
        int here = 0;
        for (int i = first; i < first + count; ++i) here |= layers[i].G != nullptr;
        if (!here) continue;
        SnTable t;
        if (!build_table(layers, first, count, (char *)ws + 256, t)) return SMMD_EINVAL;
        hipLaunchKernelGGL(sn_bwd_a_kernel, dim3(t.total_units), dim3(256), 0, s, t);
        hipLaunchKernelGGL(sn_bwd_b_kernel, dim3(t.total_units), dim3(256), 0, s, t);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

}  // extern "C"
