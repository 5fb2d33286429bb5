// smmd_sn_tile.hpp -- the 32 x 256 weight tiles of the spectral-norm launch
// set (smmd_sn.hip) and the SN-fused Adam update that shares them
// (smmd_scale.hip): tile geometry, tile load / store, the P1 column partials.
#pragma once
#include "smmd_common.hpp"

namespace smmd {

#ifndef SMMD_SN_TR
#define SMMD_SN_TR 32
#endif
constexpr int SN_TR = SMMD_SN_TR;   // tile rows (multi-launch path)
constexpr int SN_TC = 256;     // tile cols (64 lanes x 4)
constexpr int SN_RPW = SN_TR / 4;   // rows per wave
constexpr int SN_CHUNK = 16;   // layers per launch set

// float4 loads / stores with the non-temporal hint (streamed once per step:
// the Adam moments), so they do not displace the weights the next power
// iteration reads from the Infinity Cache
typedef float smmd_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ld_nt(const float4 *p) {
    const smmd_f4v v = __builtin_nontemporal_load(reinterpret_cast<const smmd_f4v *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(float4 *p, float4 x) {
    const smmd_f4v v = {x.x, x.y, x.z, x.w};
    __builtin_nontemporal_store(v, reinterpret_cast<smmd_f4v *>(p));
}

// load the NR rows x 4 cols this thread owns from row r0 (zero outside the
// matrix).  Interior tiles of 16-B aligned layers take one branch-free path:
// NR independent float4 loads issued back to back.
template <int NR, bool NT = false>
__device__ __forceinline__ void load_tile(const float *__restrict__ base, int N, int K, int vec,
                                          int r0, int c0, float4 (&w)[NR]) {
    if (vec && r0 + NR <= N && c0 + 3 < K) {
        const float4 *p = reinterpret_cast<const float4 *>(base + (size_t)r0 * K + c0);
        const int stride4 = K / 4;
#pragma unroll
        for (int i = 0; i < NR; ++i) w[i] = NT ? ld_nt(p + (size_t)i * stride4) : p[(size_t)i * stride4];
        return;
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int r = r0 + i;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r < N) {
            const float *p = base + (size_t)r * K + c0;
            if (c0 + 0 < K) x.x = p[0];
            if (c0 + 1 < K) x.y = p[1];
            if (c0 + 2 < K) x.z = p[2];
            if (c0 + 3 < K) x.w = p[3];
        }
        w[i] = x;
    }
}

// masked / vector store of NR rows x 4 cols (load_tile's inverse)
template <int NR, bool NT = false>
__device__ __forceinline__ void store_tile(float *__restrict__ base, int N, int K, int vec, int r0,
                                           int c0, const float4 (&w)[NR]) {
    if (vec && r0 + NR <= N && c0 + 3 < K) {
        float4 *p = reinterpret_cast<float4 *>(base + (size_t)r0 * K + c0);
        const int stride4 = K / 4;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            if (NT) st_nt(p + (size_t)i * stride4, w[i]);
            else p[(size_t)i * stride4] = w[i];
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int r = r0 + i;
        if (r < N) {
            float *p = base + (size_t)r * K + c0;
            if (c0 + 0 < K) p[0] = w[i].x;
            if (c0 + 1 < K) p[1] = w[i].y;
            if (c0 + 2 < K) p[2] = w[i].z;
            if (c0 + 3 < K) p[3] = w[i].w;
        }
    }
}

// column partials of one tile (u^T W over its SN_TR rows) -> p1[rt][c]: each
// wave's fmaf chain over its rows in order, then the 4 waves summed in order.
// sn_p1_kernel and the fused update below both run exactly this, so they
// write the same bits.
template <int NR>
__device__ __forceinline__ void p1_accum(const float *__restrict__ uin, int N, int r0,
                                         const float4 (&wt)[NR], float4 &acc) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const float un = (r0 + i < N) ? uin[r0 + i] : 0.f;
        acc.x = fmaf(un, wt[i].x, acc.x);
        acc.y = fmaf(un, wt[i].y, acc.y);
        acc.z = fmaf(un, wt[i].z, acc.z);
        acc.w = fmaf(un, wt[i].w, acc.w);
    }
}

__device__ __forceinline__ void p1_store(float4 acc, float *p1, int K, int rt, int c0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ float4 red[4][64];
    red[w][lane] = acc;
    __syncthreads();
    if (w == 0) {
        float4 s = red[0][lane];
#pragma unroll
        for (int i = 1; i < 4; ++i) {
            s.x += red[i][lane].x; s.y += red[i][lane].y;
            s.z += red[i][lane].z; s.w += red[i][lane].w;
        }
        float *dst = p1 + (size_t)rt * K;
        const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (c0 + k < K) dst[c0 + k] = sv[k];
    }
}

__device__ __forceinline__ void p1_tile(const float *__restrict__ uin, float *p1, int N, int K,
                                        int rt, int r0, int c0, const float4 (&wt)[SN_RPW]) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    p1_accum(uin, N, r0, wt, acc);
    p1_store(acc, p1, K, rt, c0);
}

// ---- SN-fused Adam: one tile of an SN weight per block -----------------------
// The critic update streams every SN weight anyway (read p, g, m, v; write p,
// m, v); the first pass of the next power iteration (P1, one more read of W)
// is folded into it from the updated registers.  Zero padding outside the
// matrix stays zero through the update (g = m = v = 0 -> p -= 0), as P1 needs.
struct SnAdamLayerDev {
    float *p, *m, *v;
    const float *g;
    const float *u;
    float *p1;
    int N, K, nct, tile_begin, vec, sb0, sb1;
    // G-direct (smmd_adam_flat_sn2 with SMMD_ADAM_SN_GDIRECT): dL/dW formed
    // here from G = dL/dW_eff (or dL/dW' of a fold layer) and the layer's
    // smmd_sn_grad_stats record {coef, ||dL/dW||^2, sigma, s}; G == nullptr:
    // dL/dW read from the flat gradient
    const float *G;
    const float *ucur, *vsn, *stats;
    int fold, nfc, gvec;
};

struct SnAdamTable {
    int n_layers, total_tiles;
    SnAdamLayerDev L[SN_CHUNK];
};

// tile `tile` of the table: clip factor (norm-pass partials [sb0, sb1) of its
// tensor), Adam on the thread's rows x 4 cols, store, P1 of the result.  The
// 8 rows of a wave go in H groups: H = 1 keeps all 32 float4 of p, g, m, v in
// flight at once (155 VGPRs, 3 waves / SIMD), H = 2 halves the registers for
// twice the occupancy.  Same arithmetic in the same order either way.
// G-direct: the adjoint of the fold, G[n][c][u][v] = 1/4 sum_{a,b}
// G'[n][c][u+a][v+b] (smmd_sn.hip snf_adjoint's order), for this thread's 4
// columns of its NR rows.  Each wave stages its rows' span of 4 x 4 filters
// (<= 30 per 256 columns) through LDS: 16-byte loads, the whole span of the
// NR rows in flight at once.
constexpr int SNG_FMAX = 30;                     // filters touched by 256 columns

template <int NR>
__device__ __forceinline__ void sn_fold_adjoint(const SnAdamLayerDev &L, int ct, int r0, int c0,
                                                float (*lds)[SNG_FMAX * 16], float4 (&gg)[NR]) {
    const int lane = threadIdx.x & 63;
    const int fa = (ct * SN_TC) / 9;
    int fb = (ct * SN_TC + SN_TC - 1) / 9;
    if (fb > L.nfc - 1) fb = L.nfc - 1;
    const int n4 = (fb - fa + 1) * 4;            // float4 of one row's span
    float4 x[NR][2];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int r = r0 + i;
        const float4 *src = reinterpret_cast<const float4 *>(L.G + ((size_t)r * L.nfc + fa) * 16);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = lane + 64 * h;
            x[i][h] = (r < L.N && q < n4) ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __syncthreads();                             // the previous group's reads are done
#pragma unroll
    for (int i = 0; i < NR; ++i) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = lane + 64 * h;
            if (q < n4) *reinterpret_cast<float4 *>(&lds[i][4 * q]) = x[i][h];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int kk = c0 + j;
            float a = 0.f;
            if (kk < L.K) {
                const int f = kk / 9 - fa, tap = kk - (kk / 9) * 9;
                const int u = tap / 3, vq = tap - u * 3;
                const float *b = &lds[i][f * 16];
                a = (((b[u * 4 + vq] + b[u * 4 + vq + 1]) + b[(u + 1) * 4 + vq]) +
                     b[(u + 1) * 4 + vq + 1]) * 0.25f;
            }
            o[j] = a;
        }
        gg[i] = make_float4(o[0], o[1], o[2], o[3]);
    }
}

template <int H, bool GD>
__device__ __forceinline__ void sn_adam_tile(const SnAdamTable &t, int tile, AdamK k,
                                             const double *part, float clip) {
    constexpr int NR = SN_RPW / H;
    int li = 0;
#pragma unroll
    for (int i = 1; i < SN_CHUNK; ++i)
        li += (i < t.n_layers && tile >= t.L[i].tile_begin) ? 1 : 0;
    li = __builtin_amdgcn_readfirstlane(li);
    const SnAdamLayerDev L = t.L[li];
    const int lt = tile - L.tile_begin;
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c0 = ct * SN_TC + lane * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    __shared__ float sh[1];
    constexpr bool gd = GD;     // the G-direct instantiation (every SN layer of the call)
    float coef = 0.f, sigma = 1.f, s = 1.f;
    if constexpr (GD) {
        coef = L.stats[0];
        sigma = L.stats[2];
        s = L.stats[3];
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
        const int r0 = rt * SN_TR + w * SN_RPW + h * NR;
        float4 pp[NR], gg[NR], mm[NR], vv[NR];
        float uc[NR], vk[4];
        if constexpr (GD) {
            // p, m, v in flight first: the fold staging below waits on its own loads
            load_tile(L.p, L.N, L.K, L.vec, r0, c0, pp);
            load_tile<NR, true>(L.m, L.N, L.K, L.vec, r0, c0, mm);
            load_tile<NR, true>(L.v, L.N, L.K, L.vec, r0, c0, vv);
#pragma unroll
            for (int i = 0; i < NR; ++i) uc[i] = (r0 + i < L.N) ? L.ucur[r0 + i] : 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) vk[j] = (c0 + j < L.K) ? L.vsn[c0 + j] : 0.f;
            __shared__ float lds_g[4][NR][SNG_FMAX * 16];   // fold staging
            if (L.fold) sn_fold_adjoint<NR>(L, ct, r0, c0, lds_g[w], gg);
            else load_tile(L.G, L.N, L.K, L.gvec, r0, c0, gg);
        } else {
            load_tile(L.g, L.N, L.K, L.vec, r0, c0, gg);
            load_tile(L.p, L.N, L.K, L.vec, r0, c0, pp);
            load_tile<NR, true>(L.m, L.N, L.K, L.vec, r0, c0, mm);
            load_tile<NR, true>(L.v, L.N, L.K, L.vec, r0, c0, vv);
        }
        if (h == 0) {
            if (!(clip > 0.f)) {
                k.f = 1.f;
            } else if (gd) {                         // the analytic norm of the record
                const float ss = L.stats[1];
                const float inv = (ss > 0.f) ? rsqrtf(ss) : INFINITY;
                k.f = clip * fminf(inv, 1.f / clip);
            } else {
                k.f = clip_factor_slab(part, L.sb0, L.sb1, clip, sh);
            }
        }
        if constexpr (GD) {
            // dL/dW = (s G) / sigma - (coef u'_n) v_k   (sn_bwd_b's form)
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                const float cu = coef * uc[i];
                gg[i].x = (s * gg[i].x) / sigma - cu * vk[0];
                gg[i].y = (s * gg[i].y) / sigma - cu * vk[1];
                gg[i].z = (s * gg[i].z) / sigma - cu * vk[2];
                gg[i].w = (s * gg[i].w) / sigma - cu * vk[3];
            }
        }
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            k.upd(pp[i].x, gg[i].x, mm[i].x, vv[i].x);
            k.upd(pp[i].y, gg[i].y, mm[i].y, vv[i].y);
            k.upd(pp[i].z, gg[i].z, mm[i].z, vv[i].z);
            k.upd(pp[i].w, gg[i].w, mm[i].w, vv[i].w);
        }
        store_tile(L.p, L.N, L.K, L.vec, r0, c0, pp);
        store_tile<NR, true>(L.m, L.N, L.K, L.vec, r0, c0, mm);
        store_tile<NR, true>(L.v, L.N, L.K, L.vec, r0, c0, vv);
        p1_accum(L.u, L.N, r0, pp, acc);
    }
    p1_store(acc, L.p1, L.K, rt, c0);
}

// host (smmd_sn.hip): the table of the SN tensors of a flat update, P1 slabs
// carved from the power iteration's workspace exactly as it carves them
struct SnAdamHost {
    const float *param, *m, *v, *grad;
    const int64_t *offsets;       // n_tensors + 1
    const int *sblk;              // first norm-pass partial of each tensor
    int gdirect;                  // layers[].G / .fold: the G-direct update
};
smmd_status sn_adam_table(const smmd_sn_layer *layers, const int32_t *sn_tensor, int n_layers,
                          const SnAdamHost &a, void *sn_ws, size_t sn_ws_bytes, SnAdamTable &t);

}  // namespace smmd
