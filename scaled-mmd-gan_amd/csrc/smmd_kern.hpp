// smmd_kern.hpp -- the kernel family of gan/core/mmd.py:18-188 evaluated per
// pair, and the estimator of mmd.py:199-220, shared by the row-sweep path
// (smmd_mmd.hip, d <= 32) and the MFMA Gram path (smmd_gram.hip, any d).
#pragma once
#include "smmd_common.hpp"

namespace smmd {

struct KParams {
    int n_terms;
    float c1[SMMD_MAX_TERMS];   // RBF: -gamma_k ; RQ: 2*alpha_k
    float c2[SMMD_MAX_TERMS];   // RQ: -alpha_k
    float wt[SMMD_MAX_TERMS];
    float add_dot;
};

// d/dz_i K(z_i, z_j) = alpha * z_i + beta * (z_i - z_j)
template <int KIND>
struct Kern;

template <>
struct Kern<SMMD_KIND_RBF> {   // mmd.py:55-116: K = sum wt exp(-gamma max(raw,0))
    static __device__ __forceinline__ void eval(const KParams &p, float raw, float, float,
                                                float, float &K, float &al, float &be) {
        const float R = fmaxf(raw, 0.f);
        float k = 0.f, dk = 0.f;
        for (int t = 0; t < p.n_terms; ++t) {
            const float e = p.wt[t] * expf(p.c1[t] * R);
            k += e;
            dk += p.c1[t] * e;
        }
        K = k;
        al = 0.f;
        be = (raw >= 0.f) ? 2.f * dk : 0.f;   // tf.maximum: ties pass the gradient
    }
};

template <>
struct Kern<SMMD_KIND_RQ> {    // mmd.py:143-188
    static __device__ __forceinline__ void eval(const KParams &p, float raw, float dot, float,
                                                float, float &K, float &al, float &be) {
        const float R = fmaxf(raw, 0.f);
        float k = 0.f, dk = 0.f;
        for (int t = 0; t < p.n_terms; ++t) {
            const float q = 1.f + R / p.c1[t];
            const float e = p.wt[t] * expf(p.c2[t] * logf(q));
            k += e;
            dk += e * p.c2[t] / (q * p.c1[t]);
        }
        if (p.add_dot > 0.f) k += p.add_dot * dot;
        K = k;
        al = p.add_dot;
        be = ((raw >= 0.f) ? 2.f * dk : 0.f) - p.add_dot;
    }
};

__device__ __forceinline__ float mysqrt(float x) {      // mmd.py:12
    return sqrtf(fmaxf(x + 1.0e-5f, 0.f));
}
__device__ __forceinline__ float mysqrt_grad(float x) {
    const float xe = x + 1.0e-5f;
    return (xe >= 0.f) ? 0.5f / sqrtf(xe) : 0.f;
}

template <>
struct Kern<SMMD_KIND_DISTANCE> {   // mmd.py:18-37 (no clamp; eps inside sqrt)
    static __device__ __forceinline__ void eval(const KParams &, float raw, float, float sqr,
                                                float sqc, float &K, float &al, float &be) {
        K = (mysqrt(sqr) + mysqrt(sqc)) - mysqrt(raw);
        al = 2.f * mysqrt_grad(sqr);
        be = -2.f * mysqrt_grad(raw);
    }
};

template <>
struct Kern<SMMD_KIND_DOT> {   // mmd.py:44-52
    static __device__ __forceinline__ void eval(const KParams &, float, float dot, float,
                                                float, float &K, float &al, float &be) {
        K = dot;
        al = 1.f;
        be = -1.f;
    }
};

__device__ __forceinline__ double estimator(const double *S, double m, double n, int biased,
                                            int has_const, double c) {
    // gan/core/mmd.py:199-220
    if (biased) return S[0] / (m * m) + S[2] / (n * n) - 2.0 * S[1] / (m * n);
    const double trX = has_const ? m * c : S[3];
    const double trY = has_const ? n * c : S[4];
    return (S[0] - trX) / (m * (m - 1.0)) + (S[2] - trY) / (n * (n - 1.0)) -
           2.0 * S[1] / (m * n);
}


// MFMA Gram path (smmd_gram.hip): used for d > 32, or for every d when the
// environment sets SMMD_MMD_GRAM=1 (parity tests of the two paths)
struct GramArgs {
    const float *X;
    const float *Y;
    float *Zp;            // ws [Rp][dp]
    float *sq;            // ws [Rp]
    float *C;             // ws [rows_p][Rp]
    double *slab;         // ws [blocks][8]
    unsigned *counter;    // ws header
    int m, n, d, R, Rp, dp;
    int nrows, nxr, x_begin, y_begin;
    int tanh_in, trace_mode, need_grad, biased, has_const, kind;
    double const_diag;
    float gw_same_x, gw_same_y, gw_cross;
    float *out_sums;
    float *out_mmd2;
    float *grad_x;
    float *grad_y;
    KParams kp;
};

size_t gram_ws_bytes(int m, int n, int d);
smmd_status gram_mmd2_launch(const GramArgs &g, void *ws_body, hipStream_t s);

// 2-D tiled row x column-chunk path (smmd_mmd_tile.hip) for d <= 8
struct TileArgs {
    const float *X;
    const float *Y;
    int m, n, d;
    int nrows, nxr, x_begin, y_begin;
    int tanh_in, trace_mode, need_grad, biased, has_const;
    double const_diag;
    float gw_same_x, gw_same_y, gw_cross;
    float *grad_x;
    float *grad_y;
    float *out_sums;
    float *out_mmd2;
    KParams kp;
    // filled by tile_mmd2_launch
    int n_rt, n_ch, cpw, rows_pad;
    float *part;          // [n_ch][d + 1][rows_pad] per-chunk row partials
    double *blk_sums;     // [n_rt * n_ch][8], one record per workgroup
    unsigned *rt_counter; // [n_rt], in the workspace header
    unsigned *g_counter;
};

// Every smmd_mmd2_fwd path keeps its arrival counters in the first
// MMD_WS_HEADER bytes of the caller's workspace (zero at rest: each path
// resets what it used), its data after it, so one workspace serves all paths.
constexpr size_t MMD_WS_HEADER = 16384;
constexpr int TILE_MAX_RT = (int)(MMD_WS_HEADER / sizeof(unsigned)) - 64;
bool tile_supported(int d);
size_t tile_ws_bytes(int rows, int cols, int d);      // body bytes (after the header)
struct ScaledLossArgs;
// q != nullptr: the fused SMMD loss launch (smmd_smmd_loss_fwd), q->nblocks
// squared-norm blocks after the tile grid
smmd_status tile_mmd2_launch(TileArgs a, int kind, void *ws, hipStream_t s,
                             const ScaledLossArgs *q = nullptr);

}  // namespace smmd
