// smmd_fold.hip -- 3x3 -> 4x4 filter fold of ConvMeanPool and its adjoint
// (gfx950 / MI355X).
//
// Reference: gan/core/resnet/block.py:63-66 (ConvMeanPool = conv3x3 SAME, then
// the mean of the four strided slices).  The product runs it as ONE 4x4
// stride-2 conv (gan/core/architecture.py `_ConvMeanPool`) on
//   W'[s, t] = 1/4 sum_{a, b in {0, 1}} W[s - a, t - b]      (fold)
// and its gradient maps back through the adjoint
//   g[u, v]  = 1/4 sum_{a, b in {0, 1}} g'[u + a, v + b]     (adjoint).
// A filter is one (cout, cin) pair: 9 floats in, 16 out (or back).  Both are
// HBM streams: 25 floats (100 B) moved per filter.
//
// One launch folds every listed layer (a table of up to 16, like the SN bank).
// One thread per filter, 256 filters per block.  Both sides go through LDS so
// every global access is a coalesced float4 (consecutive lanes, consecutive
// 16 B: the block's 9 KiB and 16 KiB runs); the LDS layouts are bank-conflict
// free for the per-thread and the copy patterns (see FOLD_S16).  Sums run in (a, b) = (0,0), (0,1), (1,0), (1,1)
// order, then * 0.25 (exact), like a 2x2 mean pool of the zero-padded filter.
#include "smmd_common.hpp"

namespace smmd {

constexpr int FOLD_T = 256;
constexpr int FOLD_MAXL = 16;

// every layer of one call in one launch: blocks [blk_begin[l], blk_begin[l+1])
// belong to layer l (a network's ConvMeanPool filters fold in one launch)
struct FoldTable {
    const float *src[FOLD_MAXL];
    float *dst[FOLD_MAXL];
    int64_t nf[FOLD_MAXL];
    int blk_begin[FOLD_MAXL + 1];
    int n_layers;
};

__device__ __forceinline__ int fold_layer(const FoldTable &t, int blk) {
    int l = 0;
#pragma unroll
    for (int i = 1; i < FOLD_MAXL; ++i) l += (i < t.n_layers && blk >= t.blk_begin[i]) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(l);
}

// LDS image of the 16-float side: element j of the block's filter f at
// [j * FOLD_S16 + f].  Row stride 260 = 256 + 4 words makes both access
// patterns conflict-free: a thread's own 16 values (lanes = consecutive f), and
// the coalesced float4 copy (lane i <-> filter i/4, quarter i%4: bank
// 16 (i%4) + 4 e + (i/4) % 16 is distinct across 64 lanes).
constexpr int FOLD_S16 = FOLD_T + 4;

// 9-float side: block-contiguous run of nb * 9 floats <-> LDS s9 (thread f's
// values at [f * 9 + u], stride 9 is odd so per-thread access is
// conflict-free); float4 global accesses, scalar tail for a ragged block.
__device__ __forceinline__ void load9(const float *__restrict__ src, float *s9, int n9) {
    const int n4 = n9 >> 2;
    const float4 *s4 = reinterpret_cast<const float4 *>(src);
    for (int i = threadIdx.x; i < n4; i += FOLD_T) {
        const float4 x = s4[i];
        s9[4 * i + 0] = x.x;
        s9[4 * i + 1] = x.y;
        s9[4 * i + 2] = x.z;
        s9[4 * i + 3] = x.w;
    }
    const int t = 4 * n4 + threadIdx.x;
    if (t < n9) s9[t] = src[t];
}

__device__ __forceinline__ void store9(float *__restrict__ dst, const float *s9, int n9) {
    const int n4 = n9 >> 2;
    float4 *d4 = reinterpret_cast<float4 *>(dst);
    for (int i = threadIdx.x; i < n4; i += FOLD_T)
        d4[i] = make_float4(s9[4 * i + 0], s9[4 * i + 1], s9[4 * i + 2], s9[4 * i + 3]);
    const int t = 4 * n4 + threadIdx.x;
    if (t < n9) dst[t] = s9[t];
}

__global__ __launch_bounds__(FOLD_T) void fold_fwd_kernel(FoldTable t) {
    __shared__ float s9[FOLD_T * 9];
    __shared__ float s16[16 * FOLD_S16];
    const int l = fold_layer(t, blockIdx.x);
    const int64_t nf = t.nf[l];
    const int64_t f0 = (int64_t)(blockIdx.x - t.blk_begin[l]) * FOLD_T;
    const int nb = (int)min<int64_t>(FOLD_T, nf - f0);
    load9(t.src[l] + f0 * 9, s9, nb * 9);
    __syncthreads();
    const int f = threadIdx.x;
    if (f < nb) {
        float k[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) k[j] = s9[f * 9 + j];
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
                s16[(si * 4 + ti) * FOLD_S16 + f] = acc * 0.25f;
            }
        }
    }
    __syncthreads();
    float4 *d4 = reinterpret_cast<float4 *>(t.dst[l] + f0 * 16);
    for (int i = threadIdx.x; i < nb * 4; i += FOLD_T) {
        const int ff = i >> 2, q = i & 3;
        d4[i] = make_float4(s16[(q * 4 + 0) * FOLD_S16 + ff], s16[(q * 4 + 1) * FOLD_S16 + ff],
                            s16[(q * 4 + 2) * FOLD_S16 + ff], s16[(q * 4 + 3) * FOLD_S16 + ff]);
    }
}

__global__ __launch_bounds__(FOLD_T) void fold_adj_kernel(FoldTable t) {
    __shared__ float s9[FOLD_T * 9];
    __shared__ float s16[16 * FOLD_S16];
    const int l = fold_layer(t, blockIdx.x);
    const int64_t nf = t.nf[l];
    const int64_t f0 = (int64_t)(blockIdx.x - t.blk_begin[l]) * FOLD_T;
    const int nb = (int)min<int64_t>(FOLD_T, nf - f0);
    const float4 *s4 = reinterpret_cast<const float4 *>(t.src[l] + f0 * 16);
    for (int i = threadIdx.x; i < nb * 4; i += FOLD_T) {
        const int ff = i >> 2, q = i & 3;
        const float4 x = s4[i];
        s16[(q * 4 + 0) * FOLD_S16 + ff] = x.x;
        s16[(q * 4 + 1) * FOLD_S16 + ff] = x.y;
        s16[(q * 4 + 2) * FOLD_S16 + ff] = x.z;
        s16[(q * 4 + 3) * FOLD_S16 + ff] = x.w;
    }
    __syncthreads();
    const int f = threadIdx.x;
    if (f < nb) {
        float k[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) k[j] = s16[j * FOLD_S16 + f];
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
                s9[f * 9 + u * 3 + v] = acc * 0.25f;
            }
        }
    }
    __syncthreads();
    store9(t.dst[l] + f0 * 9, s9, nb * 9);
}

// ---- UpsampleConv fold (block.py:53-60) -------------------------------------
// K [cin][cout][s][t] = 4 W'[cout][cin][3-s][3-t] with W' = fold(W): the
// transposed 4x4 stride-2 conv equal to conv3x3(upsample_nearest2(x), W)
// (convops.fold_up_weight).  4 * (1/4 * sum) is the plain sum (exact), so a
// K value is the fold's sum in its (a, b) order.  Thread per source filter
// (cout, cin) of the block's 256: its 9 floats staged through LDS (coalesced
// float4), its 16 outputs one 64-byte line of K written by four float4
// stores (the line's filter is (cin, cout): lanes stride cout * 64 B, each a
// whole line).  The adjoint reads that line back and sums the 2 x 2 windows
// of the un-flipped G'[s][t] = gK[3-s][3-t]: gW[u][v] = sum_{a,b} G'[u+a][v+b].
__global__ __launch_bounds__(FOLD_T) void fold_up_kernel(const float *__restrict__ w,
                                                         float *__restrict__ k, int cout, int cin) {
    __shared__ float s9[FOLD_T * 9];
    const int64_t nf = (int64_t)cout * cin;
    const int64_t f0 = (int64_t)blockIdx.x * FOLD_T;
    const int nb = (int)min<int64_t>(FOLD_T, nf - f0);
    load9(w + f0 * 9, s9, nb * 9);
    __syncthreads();
    const int f = threadIdx.x;
    if (f >= nb) return;
    const int64_t q = f0 + f;
    const int co = (int)(q / cin), ci = (int)(q - (int64_t)co * cin);
    float kk[9], o[16];
#pragma unroll
    for (int j = 0; j < 9; ++j) kk[j] = s9[f * 9 + j];
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
                    if (u >= 0 && u < 3 && v >= 0 && v < 3) acc += kk[u * 3 + v];
                }
            }
            o[15 - (si * 4 + ti)] = acc;               // flipped in both axes
        }
    }
    float4 *d4 = reinterpret_cast<float4 *>(k + ((int64_t)ci * cout + co) * 16);
#pragma unroll
    for (int i = 0; i < 4; ++i) d4[i] = make_float4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

__global__ __launch_bounds__(FOLD_T) void fold_up_adj_kernel(const float *__restrict__ gk,
                                                             float *__restrict__ gw, int cout,
                                                             int cin) {
    __shared__ float s9[FOLD_T * 9];
    const int64_t nf = (int64_t)cout * cin;
    const int64_t f0 = (int64_t)blockIdx.x * FOLD_T;
    const int nb = (int)min<int64_t>(FOLD_T, nf - f0);
    const int f = threadIdx.x;
    if (f < nb) {
        const int64_t q = f0 + f;
        const int co = (int)(q / cin), ci = (int)(q - (int64_t)co * cin);
        const float4 *s4 = reinterpret_cast<const float4 *>(gk + ((int64_t)ci * cout + co) * 16);
        float g[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 x = s4[i];
            // G'[j] = gK[15 - j]
            g[15 - 4 * i] = x.x;
            g[14 - 4 * i] = x.y;
            g[13 - 4 * i] = x.z;
            g[12 - 4 * i] = x.w;
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
#pragma unroll
            for (int v = 0; v < 3; ++v) {
                float acc = 0.f;
#pragma unroll
                for (int a = 0; a < 2; ++a) {
#pragma unroll
                    for (int b = 0; b < 2; ++b) acc += g[(u + a) * 4 + (v + b)];
                }
                s9[f * 9 + u * 3 + v] = acc;
            }
        }
    }
    __syncthreads();
    store9(gw + f0 * 9, s9, nb * 9);
}

}  // namespace smmd

using namespace smmd;

extern "C" smmd_status smmd_fold_up_weight(const float *src, float *dst, int cout, int cin,
                                           int adjoint, smmd_stream_t stream) {
    if (cout < 0 || cin < 0) return SMMD_EINVAL;
    const int64_t nf = (int64_t)cout * cin;
    if (nf == 0) return SMMD_OK;
    if (!src || !dst) return SMMD_EINVAL;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) != 0)
        return SMMD_EINVAL;
    const int64_t blocks = (nf + FOLD_T - 1) / FOLD_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (adjoint)
        fold_up_adj_kernel<<<dim3((unsigned)blocks), dim3(FOLD_T), 0, s>>>(src, dst, cout, cin);
    else
        fold_up_kernel<<<dim3((unsigned)blocks), dim3(FOLD_T), 0, s>>>(src, dst, cout, cin);
    return last_launch_status();
}

extern "C" smmd_status smmd_fold_pool_weights(const float *const *src, float *const *dst,
                                              const int64_t *n_filters, int n_layers,
                                              int adjoint, smmd_stream_t stream) {
    if (n_layers < 0 || n_layers > FOLD_MAXL || (n_layers > 0 && (!src || !dst || !n_filters)))
        return SMMD_EINVAL;
    FoldTable t;
    memset(&t, 0, sizeof(t));
    int64_t blocks = 0;
    int nl = 0;
    for (int i = 0; i < n_layers; ++i) {
        const int64_t nf = n_filters[i];
        if (nf < 0) return SMMD_EINVAL;
        if (nf == 0) continue;
        if (!src[i] || !dst[i]) return SMMD_EINVAL;
        if (((reinterpret_cast<uintptr_t>(src[i]) | reinterpret_cast<uintptr_t>(dst[i])) & 15) != 0)
            return SMMD_EINVAL;
        t.src[nl] = src[i];
        t.dst[nl] = dst[i];
        t.nf[nl] = nf;
        t.blk_begin[nl] = (int)blocks;
        blocks += (nf + FOLD_T - 1) / FOLD_T;
        if (blocks > 0x7fffffff) return SMMD_EINVAL;
        ++nl;
    }
    if (nl == 0) return SMMD_OK;
    t.blk_begin[nl] = (int)blocks;
    t.n_layers = nl;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (adjoint)
        fold_adj_kernel<<<dim3((unsigned)blocks), dim3(FOLD_T), 0, s>>>(t);
    else
        fold_fwd_kernel<<<dim3((unsigned)blocks), dim3(FOLD_T), 0, s>>>(t);
    return last_launch_status();
}
