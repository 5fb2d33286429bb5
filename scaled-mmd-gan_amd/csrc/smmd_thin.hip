// smmd_thin.hip -- 3x3 stride-1 SAME convolutions with a thin side (<= 4
// channels) on gfx950 / MI355X: the critic's first layer (3 -> dim) and the
// generator's last (dim -> 3), with their input and weight gradients.
//
// Reference layers: snops.conv2d / resnet Conv2D at stride 1 SAME
// (gan/core/snops.py:69-90, gan/core/resnet/ops/conv2d.py:16-39; the critics'
// first conv, gan/core/architecture.py:395-407, :410-434) and snops.deconv2d
// at stride 1 SAME (gan/core/snops.py:104-126; the generators' last layer,
// architecture.py:178-208, :211-230).
//
// MIOpen runs these at 3-6x their HBM time on MI355X (its implicit-GEMM
// solvers transpose the 64-channel side to NHWC and tile for wide K; the
// thin side leaves most of a GEMM tile empty).  Here every kernel streams the
// wide tensor once and keeps the thin side on chip:
//
//   thin_in   (ci <= 4): a thread owns two output pixels and gathers their
//             9 ci taps once; the coefficients sit in LDS as output-channel
//             pairs, so each broadcast 16-byte LDS read feeds four packed FMAs
//             (v_pk_fma_f32); one coalesced row store per channel (the output
//             is the HBM traffic).
//   thin_out  (co <= 4, W <= 64): a lane owns one column of a TR-row tile; per
//             input channel it loads TR + 2 rows (coalesced, the next channel's
//             in flight), takes the left and right columns from its
//             neighbours (DPP wave shifts), and runs packed FMAs over output
//             channel pairs; the block's 4 waves split the input channels and
//             add their partial tiles in LDS in wave order.
//   wgrad     (min(ci, co) <= 4, W <= 64): an [CW x pixels] x [pixels x 9 CT]
//             product on the f32 matrix cores (v_mfma_f32_32x32x2_f32), rows
//             of the wide tensor and the expanded thin taps staged in LDS one
//             step ahead; per-block partials go to a slab that a second launch
//             adds in order.  (A VALU variant serves other widths.)
//
// Taps: t = 3 kh + kw reads the input at (h + kh - 1, w + kw - 1), zero outside.
// Weight modes (A[o][i][t] is the coefficient of input channel i, tap t in
// output channel o):
//   mode 0: A[o][i][t] = w[o][i][t]      w [co, ci, 3, 3]   (the forward)
//   mode 1: A[o][i][t] = w[i][o][8 - t]  w [ci, co, 3, 3]   (the input
//           gradient of a conv whose weight is w, = a stride-1 transposed conv)
// Every sum has a fixed order: results are bit-identical run to run.
#include "smmd_common.hpp"

namespace smmd {

constexpr int TH_T = 256;       // threads per block
constexpr int TO_TR = 4;        // thin_out: output rows per block
constexpr int WG_CG = 2;        // wgrad: wide channels per wave
constexpr int WG_RC = 64;       // wgrad: rows per wave (an image chunk)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int MODE>
__device__ __forceinline__ float wcoef(const float *__restrict__ w, int o, int i, int t, int CI,
                                       int CO) {
    return MODE == 0 ? w[((size_t)o * CI + i) * 9 + t] : w[((size_t)i * CO + o) * 9 + (8 - t)];
}

// ---- thin_in: y[n][o][p] = b[o] + sum_{i < CT, t} A[o][i][t] x[n][i][p + d(t)] ----
// A thread owns two pixels, p and p + 256, of the block's 512.  The block
// stages the coefficients of 64 output channels at a time in LDS as (o, o + 1)
// pairs, two taps per 16-byte word: one broadcast LDS read feeds four packed
// FMAs (v_pk_fma_f32: two output channels x two pixels).
constexpr int TI_PX = 2;                        // pixels per thread

template <int CT>
__device__ __forceinline__ void thin_in_gather(const float *__restrict__ x, int64_t gp,
                                               int64_t total, int HW, int H, int W,
                                               float (&xin)[(CT * 9 + 1) & ~1]) {
    constexpr int J = CT * 9;
    const bool live = gp < total;
    const int n = live ? (int)(gp / HW) : 0;
    const int p = live ? (int)(gp - (int64_t)n * HW) : 0;
    const int h = p / W, c = p - h * W;
#pragma unroll
    for (int i = 0; i < CT; ++i) {
        const float *xi = x + ((size_t)n * CT + i) * HW;
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int hh = h + kh - 1;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int ww = c + kw - 1;
                xin[i * 9 + kh * 3 + kw] =
                    (live && hh >= 0 && hh < H && ww >= 0 && ww < W) ? xi[hh * W + ww] : 0.f;
            }
        }
    }
    if (J & 1) xin[J] = 0.f;
}

template <int CT, int MODE>
__global__ __launch_bounds__(TH_T) void thin_in_kernel(const float *__restrict__ x,
                                                        const float *__restrict__ w,
                                                        const float *__restrict__ bias,
                                                        float *__restrict__ y, int N, int CO,
                                                        int H, int W) {
    constexpr int OC = 64;                      // output channels per LDS chunk
    constexpr int J = CT * 9, JP = (J + 1) & ~1, JQ = JP / 2;
    __shared__ float4 wl[(OC / 2) * JQ];        // {A[o][j], A[o+1][j], A[o][j+1], A[o+1][j+1]}
    __shared__ f2 bl[OC / 2];
    const int HW = H * W;
    const int64_t total = (int64_t)N * HW;
    const int64_t g0 = (int64_t)blockIdx.x * (TH_T * TI_PX) + threadIdx.x;
    const int64_t g1 = g0 + TH_T;
    float xa[JP], xb[JP];
    thin_in_gather<CT>(x, g0, total, HW, H, W, xa);
    thin_in_gather<CT>(x, g1, total, HW, H, W, xb);
    const bool la = g0 < total, lb = g1 < total;
    float *ya = y, *yb = y;
    if (la) {
        const int n = (int)(g0 / HW);
        ya = y + (size_t)n * CO * HW + (g0 - (int64_t)n * HW);
    }
    if (lb) {
        const int n = (int)(g1 / HW);
        yb = y + (size_t)n * CO * HW + (g1 - (int64_t)n * HW);
    }
    for (int o0 = 0; o0 < CO; o0 += OC) {
        __syncthreads();                        // the previous chunk's readers are done
        for (int e = threadIdx.x; e < (OC / 2) * JQ; e += TH_T) {
            const int op = e / JQ, jq = e - op * JQ;
            const int o = o0 + 2 * op;
            float a[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int oo = o + (u & 1), j = 2 * jq + (u >> 1);
                const int i = j / 9, t = j - i * 9;
                a[u] = (oo < CO && j < J) ? wcoef<MODE>(w, oo, i, t, CT, CO) : 0.f;
            }
            wl[e] = make_float4(a[0], a[1], a[2], a[3]);
        }
        if (threadIdx.x < OC / 2) {
            const int o = o0 + 2 * threadIdx.x;
            f2 b;
            b.x = (bias && o < CO) ? bias[o] : 0.f;
            b.y = (bias && o + 1 < CO) ? bias[o + 1] : 0.f;
            bl[threadIdx.x] = b;
        }
        __syncthreads();
        if (la) {
            const int npair = (min(OC, CO - o0) + 1) >> 1;
            for (int op = 0; op < npair; ++op) {
                f2 acca = bl[op], accb = acca;
                const float4 *wp = wl + op * JQ;
#pragma unroll
                for (int q = 0; q < JQ; ++q) {
                    const float4 c4 = wp[q];
                    const f2 w0 = f2{c4.x, c4.y}, w1 = f2{c4.z, c4.w};
                    acca = __builtin_elementwise_fma(w0, f2{xa[2 * q], xa[2 * q]}, acca);
                    accb = __builtin_elementwise_fma(w0, f2{xb[2 * q], xb[2 * q]}, accb);
                    acca = __builtin_elementwise_fma(w1, f2{xa[2 * q + 1], xa[2 * q + 1]}, acca);
                    accb = __builtin_elementwise_fma(w1, f2{xb[2 * q + 1], xb[2 * q + 1]}, accb);
                }
                const int o = o0 + 2 * op;
                ya[(size_t)o * HW] = acca.x;
                if (o + 1 < CO) ya[(size_t)(o + 1) * HW] = acca.y;
                if (lb) {
                    yb[(size_t)o * HW] = accb.x;
                    if (o + 1 < CO) yb[(size_t)(o + 1) * HW] = accb.y;
                }
            }
        }
    }
}

// left / right neighbour column of a row value (lane = column; zero outside):
// DPP whole-wave shifts, lane 0 (wave_shr) / lane 63 (wave_shl) get 0
__device__ __forceinline__ float from_left(float v, int) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                 0x138, 0xf, 0xf, false));
}

__device__ __forceinline__ float from_right(float v, int) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                                 0x130, 0xf, 0xf, false));
}

// ---- thin_out: y[n][o < CT][p] = b[o] + sum_{i < CI, t} A[o][i][t] x[n][i][p + d(t)] ----
// Coefficients of 64 input channels at a time in LDS as {A[0..3][i][t]}
// (one broadcast 16-byte read per tap); output channels advance in packed
// pairs (o0, o1), (o2, o3).
template <int CT, int MODE>
__global__ __launch_bounds__(TH_T) void thin_out_kernel(const float *__restrict__ x,
                                                         const float *__restrict__ w,
                                                         const float *__restrict__ bias,
                                                         float *__restrict__ y, int N, int CI,
                                                         int H, int W) {
    constexpr int TR = TO_TR;
    constexpr int IC = 64;                      // input channels per LDS chunk
    __shared__ float4 wl[IC * 9];
    __shared__ float red[4][TR * CT][SMMD_WAVE];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tiles = (H + TR - 1) / TR;
    const int n = blockIdx.x / tiles, h0 = (blockIdx.x - n * tiles) * TR;
    const int HW = H * W;
    const bool col = lane < W;
    f2 a01[TR], a23[TR];
#pragma unroll
    for (int r = 0; r < TR; ++r) {
        a01[r] = f2{0.f, 0.f};
        a23[r] = f2{0.f, 0.f};
    }
    for (int i0 = 0; i0 < CI; i0 += IC) {
        __syncthreads();
        for (int e = threadIdx.x; e < IC * 9; e += TH_T) {
            const int ii = e / 9, t = e - ii * 9, i = i0 + ii;
            float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < CI) {
                q.x = wcoef<MODE>(w, 0, i, t, CI, CT);
                if (CT > 1) q.y = wcoef<MODE>(w, 1, i, t, CI, CT);
                if (CT > 2) q.z = wcoef<MODE>(w, 2, i, t, CI, CT);
                if (CT > 3) q.w = wcoef<MODE>(w, 3, i, t, CI, CT);
            }
            wl[e] = q;
        }
        __syncthreads();
        // wave wv takes the chunk's input channels wv, wv + 4, ... in order;
        // the next channel's rows are loaded while this one computes
        const int i1 = min(CI, i0 + IC);
        float nv[TR + 2];
        auto load_rows = [&](int i, float (&dst)[TR + 2]) {
            const float *xi = x + ((size_t)n * CI + i) * HW;
#pragma unroll
            for (int r = 0; r < TR + 2; ++r) {
                const int hh = h0 + r - 1;
                dst[r] = (col && i < i1 && hh >= 0 && hh < H) ? xi[hh * W + lane] : 0.f;
            }
        };
        load_rows(i0 + wv, nv);
        for (int i = i0 + wv; i < i1; i += 4) {
            float v[TR + 2], vl[TR + 2], vr[TR + 2];
#pragma unroll
            for (int r = 0; r < TR + 2; ++r) v[r] = nv[r];
            load_rows(i + 4, nv);
#pragma unroll
            for (int r = 0; r < TR + 2; ++r) {
                vl[r] = from_left(v[r], lane);
                vr[r] = from_right(v[r], lane);
            }
            const float4 *wq = wl + (i - i0) * 9;
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    const float4 q = wq[kh * 3 + kw];
                    const f2 q01 = f2{q.x, q.y}, q23 = f2{q.z, q.w};
#pragma unroll
                    for (int r = 0; r < TR; ++r) {
                        const float s = kw == 0 ? vl[r + kh] : (kw == 1 ? v[r + kh] : vr[r + kh]);
                        const f2 sv = f2{s, s};
                        a01[r] = __builtin_elementwise_fma(q01, sv, a01[r]);
                        if (CT > 2) a23[r] = __builtin_elementwise_fma(q23, sv, a23[r]);
                    }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < TR; ++r) {
        red[wv][r * CT + 0][lane] = a01[r].x;
        if (CT > 1) red[wv][r * CT + 1][lane] = a01[r].y;
        if (CT > 2) red[wv][r * CT + 2][lane] = a23[r].x;
        if (CT > 3) red[wv][r * CT + 3][lane] = a23[r].y;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < TR * CT * SMMD_WAVE; e += TH_T) {
        const int j = e / SMMD_WAVE, l = e - j * SMMD_WAVE;
        const int r = j / CT, o = j - r * CT;
        const int hh = h0 + r;
        if (l < W && hh < H) {
            float s = red[0][j][l];
            s += red[1][j][l];
            s += red[2][j][l];
            s += red[3][j][l];
            if (bias) s += bias[o];
            y[((size_t)n * CT + o) * HW + hh * W + l] = s;
        }
    }
}

// ---- wgrad: R[c][k][t] = sum_{n, p} Wd[n][c][p] Th[n][k][p + d(t)] ----------
// Block = 4 waves; wave (blockIdx.y * 4 + wv) takes wide channels
// [cg * CG, cg * CG + CG) of image n, rows [r0, r0 + RC).  Its wave sums go to
// part[((n * chunks + chunk) * CW + c) * CT * 9 + k * 9 + t].
template <int CT>
__global__ __launch_bounds__(TH_T) void thin_wgrad_kernel(const float *__restrict__ wd,
                                                           const float *__restrict__ th,
                                                           float *__restrict__ part, int N,
                                                           int CW, int H, int W, int chunks) {
    constexpr int CG = WG_CG;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int cg = blockIdx.y * 4 + wv;
    const int c0 = cg * CG;
    if (c0 >= CW) return;                  // no block-level sync below
    const int n = blockIdx.x / chunks, chunk = blockIdx.x - n * chunks;
    const int r0 = chunk * WG_RC, r1 = min(H, r0 + WG_RC);
    const int HW = H * W;
    const bool col = lane < W;
    const float *tn = th + (size_t)n * CT * HW;
    const float *wn = wd + (size_t)n * CW * HW;
    float acc[CG][CT][9];
#pragma unroll
    for (int g = 0; g < CG; ++g)
#pragma unroll
        for (int k = 0; k < CT; ++k)
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[g][k][t] = 0.f;
    // rolling window of thin rows h - 1, h, h + 1 (centre, left, right columns)
    float tc[CT][3], tl[CT][3], tr[CT][3];
#pragma unroll
    for (int k = 0; k < CT; ++k) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int hh = r0 - 1 + j;
            const float v = (col && hh >= 0 && hh < H) ? tn[(size_t)k * HW + hh * W + lane] : 0.f;
            tc[k][j + 1] = v;
            tl[k][j + 1] = from_left(v, lane);
            tr[k][j + 1] = from_right(v, lane);
        }
    }
    for (int h = r0; h < r1; ++h) {
        float g[CG];
#pragma unroll
        for (int q = 0; q < CG; ++q) {
            const int c = c0 + q;
            g[q] = (col && c < CW) ? wn[(size_t)c * HW + h * W + lane] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < CT; ++k) {
            const int hh = h + 1;
            const float v = (col && hh < H) ? tn[(size_t)k * HW + hh * W + lane] : 0.f;
            tc[k][0] = tc[k][1];
            tc[k][1] = tc[k][2];
            tc[k][2] = v;
            tl[k][0] = tl[k][1];
            tl[k][1] = tl[k][2];
            tl[k][2] = from_left(v, lane);
            tr[k][0] = tr[k][1];
            tr[k][1] = tr[k][2];
            tr[k][2] = from_right(v, lane);
        }
#pragma unroll
        for (int q = 0; q < CG; ++q) {
#pragma unroll
            for (int k = 0; k < CT; ++k) {
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    acc[q][k][kh * 3 + 0] = fmaf(g[q], tl[k][kh], acc[q][k][kh * 3 + 0]);
                    acc[q][k][kh * 3 + 1] = fmaf(g[q], tc[k][kh], acc[q][k][kh * 3 + 1]);
                    acc[q][k][kh * 3 + 2] = fmaf(g[q], tr[k][kh], acc[q][k][kh * 3 + 2]);
                }
            }
        }
    }
    float *po = part + ((size_t)(n * chunks + chunk) * CW) * (CT * 9);
#pragma unroll
    for (int q = 0; q < CG; ++q) {
#pragma unroll
        for (int k = 0; k < CT; ++k) {
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const float s = wave_sum(acc[q][k][t]);
                if (lane == 0 && c0 + q < CW) po[(size_t)(c0 + q) * (CT * 9) + k * 9 + t] = s;
            }
        }
    }
}

// ---- wgrad on the f32 matrix cores --------------------------------------
// R[c][j] = sum_p Wd[c][p] B[j][p], B[j][p] = Th[k][p + d(t)] for j = 9 k + t
// (< 9 CT; columns 9 CT .. 31 are zero): an [CW x P] x [P x 32] product with
// K = the image pixels, on v_mfma_f32_32x32x2_f32 (fp32 products, fp32
// accumulation: a k-ordered fmaf chain per output).  Block = one image n and
// a band of WM_RB rows; its 4 waves are MT (= 32-channel M tiles) x RS (rows
// in flight).  Per step the block stages RS rows: A = Wd rows [MT 32 ch x 64
// px] and the expanded thin taps B [32 x 64 px], both [row][k] with a 65-float
// stride (conflict-free fragment reads), fetched one step ahead into
// registers.  A wave's 32 x 32 tile sums its rows; the RS waves of an M tile
// add in LDS in row order and write the block's [CW][9 CT] partial to the
// slab.  Needs W <= 64, W % 4 == 0, CW <= 128, 16-byte aligned Wd.
constexpr int WM_RB = 8;        // rows per block
constexpr int WM_LD = 65;       // LDS row stride (floats)

template <int CT, int MT>
__global__ __launch_bounds__(TH_T) void thin_wgrad_mfma_kernel(const float *__restrict__ wd,
                                                                const float *__restrict__ th,
                                                                float *__restrict__ part, int N,
                                                                int CW, int H, int W) {
    constexpr int RS = 4 / MT;                 // rows per step
    constexpr int AQ = RS * MT * 32 * 16;      // float4 of the A stage
    constexpr int AQT = AQ / TH_T;             // per thread (8)
    constexpr int BE = RS * 32 * 64;           // B stage elements
    constexpr int BET = BE / TH_T;             // per thread
    constexpr int J = CT * 9;
    __shared__ float As[RS][MT * 32][WM_LD];
    __shared__ float Bs[RS][32][WM_LD];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int mt = wv % MT, rs = wv / MT;
    const int bands = (H + WM_RB - 1) / WM_RB;
    const int n = blockIdx.x / bands, hb = (blockIdx.x - n * bands) * WM_RB;
    const int he = min(H, hb + WM_RB);
    const int HW = H * W;
    const float *wn = wd + (size_t)n * CW * HW;
    const float *tn = th + (size_t)n * CT * HW;
    float4 ra[AQT];
    float rb[BET];
    auto fetch = [&](int h0) {
#pragma unroll
        for (int q = 0; q < AQT; ++q) {
            const int e = threadIdx.x + q * TH_T;
            const int px4 = e & 15, cc = (e >> 4) % (MT * 32), rr = (e >> 4) / (MT * 32);
            const int h = h0 + rr;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (h < he && cc < CW && px4 * 4 < W)
                v = *reinterpret_cast<const float4 *>(wn + (size_t)cc * HW + h * W + px4 * 4);
            ra[q] = v;
        }
#pragma unroll
        for (int q = 0; q < BET; ++q) {
            const int e = threadIdx.x + q * TH_T;
            const int pp = e & 63, j = (e >> 6) & 31, rr = e >> 11;
            const int h = h0 + rr;
            float v = 0.f;
            if (j < J && h < he && pp < W) {
                const int k = j / 9, t = j - k * 9, kh = t / 3, kw = t - kh * 3;
                const int hh = h + kh - 1, ww = pp + kw - 1;
                if (hh >= 0 && hh < H && ww >= 0 && ww < W) v = tn[(size_t)k * HW + hh * W + ww];
            }
            rb[q] = v;
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int q = 0; q < AQT; ++q) {
            const int e = threadIdx.x + q * TH_T;
            const int px4 = e & 15, cc = (e >> 4) % (MT * 32), rr = (e >> 4) / (MT * 32);
            float *d = &As[rr][cc][px4 * 4];
            d[0] = ra[q].x;
            d[1] = ra[q].y;
            d[2] = ra[q].z;
            d[3] = ra[q].w;
        }
#pragma unroll
        for (int q = 0; q < BET; ++q) {
            const int e = threadIdx.x + q * TH_T;
            Bs[e >> 11][(e >> 6) & 31][e & 63] = rb[q];
        }
    };
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    fetch(hb);
    for (int h0 = hb; h0 < he; h0 += RS) {
        stash();
        __syncthreads();
        if (h0 + RS < he) fetch(h0 + RS);       // next rows in flight
        const float *ar = &As[rs][mt * 32 + (lane & 31)][lane >> 5];
        const float *br = &Bs[rs][lane & 31][lane >> 5];
#pragma unroll
        for (int kk = 0; kk < 32; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * kk], br[2 * kk], acc, 0, 0, 0);
        __syncthreads();
    }
    // the RS waves of each M tile add their tiles in row order (LDS: reuse As)
    float *red = &As[0][0][0];                  // [RS][MT][16][64] floats <= As
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((rs * MT + mt) * 16 + r) * 64 + lane] = acc[r];
    __syncthreads();
    if (rs == 0) {
        float *po = part + (size_t)blockIdx.x * CW * J;
        const int j = lane & 31;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            float s = red[(mt * 16 + r) * 64 + lane];
#pragma unroll
            for (int q = 1; q < RS; ++q) s += red[((q * MT + mt) * 16 + r) * 64 + lane];
            const int c = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (c < CW && j < J) po[(size_t)c * J + j] = s;
        }
    }
}

// gw from the slab part[S][E] (E = CW * 9 CT): a block owns 64 outputs; its
// 16 waves' lanes sum the partials s = g, g + 16, ... of their output (g = the
// wave) in order, then wave 0 adds the 16 sums in order.
//   thin_in  (Th = x):  gw[o = c][i = k][t]
//   thin_out (Th = gy): gw[o = k][i = c][8 - t]
constexpr int WF_T = 1024;

__global__ __launch_bounds__(WF_T) void thin_wgrad_final_kernel(const float *__restrict__ part,
                                                                 int S, int CW, int CT,
                                                                 int thin_in,
                                                                 float *__restrict__ gw,
                                                                 int accum) {
    __shared__ double red[WF_T / 64][64];
    const int E = CW * CT * 9;
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + lane;
    double acc = 0.0;
    if (e < E) {
        const float *p = part + e;
        int s = g;
        for (; s + 7 * 16 < S; s += 8 * 16) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = p[(size_t)(s + 16 * k) * E];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += (double)v[k];
        }
        for (; s < S; s += 16) acc += (double)p[(size_t)s * E];
    }
    red[g][lane] = acc;
    __syncthreads();
    if (g == 0 && e < E) {
        double t = 0.0;
#pragma unroll
        for (int q = 0; q < WF_T / 64; ++q) t += red[q][lane];
        const int c = e / (CT * 9), kt = e - c * (CT * 9);
        const int k = kt / 9, tt = kt - k * 9;
        const size_t dst = thin_in ? ((size_t)c * CT + k) * 9 + tt
                                   : ((size_t)k * CW + c) * 9 + (8 - tt);
        gw[dst] = accum ? gw[dst] + (float)t : (float)t;   // accum: a later contribution
    }
}

inline int wgrad_chunks(int H) { return (H + WG_RC - 1) / WG_RC; }

template <int MODE>
smmd_status launch_thin(const float *x, const float *w, const float *bias, float *y, int N,
                        int CI, int CO, int H, int W, hipStream_t st) {
    if (CI <= 4) {
        const int64_t total = (int64_t)N * H * W;
        const int64_t blocks = (total + TH_T * TI_PX - 1) / (TH_T * TI_PX);
        if (blocks > 0x7fffffff) return SMMD_EINVAL;
        dim3 g((unsigned)blocks), b(TH_T);
        switch (CI) {
            case 1: thin_in_kernel<1, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CO, H, W); break;
            case 2: thin_in_kernel<2, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CO, H, W); break;
            case 3: thin_in_kernel<3, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CO, H, W); break;
            default: thin_in_kernel<4, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CO, H, W); break;
        }
        return last_launch_status();
    }
    if (CO > 4 || W > SMMD_WAVE) return SMMD_EUNSUPPORTED;
    const int64_t blocks = (int64_t)N * ((H + TO_TR - 1) / TO_TR);
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    dim3 g((unsigned)blocks), b(TH_T);
    switch (CO) {
        case 1: thin_out_kernel<1, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CI, H, W); break;
        case 2: thin_out_kernel<2, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CI, H, W); break;
        case 3: thin_out_kernel<3, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CI, H, W); break;
        default: thin_out_kernel<4, MODE><<<g, b, 0, st>>>(x, w, bias, y, N, CI, H, W); break;
    }
    return last_launch_status();
}

}  // namespace smmd

using namespace smmd;

extern "C" smmd_status smmd_conv3x3_thin(const float *x, const float *w, const float *bias,
                                         float *y, int n, int ci, int co, int h, int w_img,
                                         int mode, smmd_stream_t stream) {
    if (n < 0 || ci <= 0 || co <= 0 || h < 0 || w_img < 0 || (mode != 0 && mode != 1))
        return SMMD_EINVAL;
    if (ci > 4 && co > 4) return SMMD_EUNSUPPORTED;
    if ((int64_t)h * w_img > 0x7fffffff / 4) return SMMD_EINVAL;
    if (n == 0 || h == 0 || w_img == 0) return SMMD_OK;
    if (!x || !w || !y) return SMMD_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    return mode == 0 ? launch_thin<0>(x, w, bias, y, n, ci, co, h, w_img, st)
                     : launch_thin<1>(x, w, bias, y, n, ci, co, h, w_img, st);
}

extern "C" size_t smmd_conv3x3_thin_wgrad_workspace_bytes(int n, int ci, int co, int h,
                                                          int w_img) {
    if (n <= 0 || ci <= 0 || co <= 0 || h <= 0 || w_img <= 0) return 0;
    const int ct = ci <= 4 ? ci : co, cw = ci <= 4 ? co : ci;
    const int s = max(wgrad_chunks(h), (h + WM_RB - 1) / WM_RB);   // VALU / MFMA slab rows
    return (size_t)n * s * cw * ct * 9 * sizeof(float);
}

static smmd_status thin_wgrad_launch(const float *gy, const float *x, float *gw, int n, int ci,
                                     int co, int h, int w_img, void *ws, size_t ws_bytes,
                                     int accum, smmd_stream_t stream) {
    if (n < 0 || ci <= 0 || co <= 0 || h < 0 || w_img < 0) return SMMD_EINVAL;
    if (ci > 4 && co > 4) return SMMD_EUNSUPPORTED;
    if (w_img > SMMD_WAVE) return SMMD_EUNSUPPORTED;
    if (!gw) return SMMD_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n == 0 || h == 0 || w_img == 0) {
        const size_t bytes = (size_t)ci * co * 9 * sizeof(float);
        return accum ? SMMD_OK : hip_status(hipMemsetAsync(gw, 0, bytes, st));
    }
    if (!gy || !x) return SMMD_EINVAL;
    const int thin_in = ci <= 4;
    const int ct = thin_in ? ci : co, cw = thin_in ? co : ci;
    const float *wd = thin_in ? gy : x;       // the wide tensor, streamed once
    const float *tt = thin_in ? x : gy;       // the thin tensor, shifted
    const int E = cw * ct * 9;
    // the MFMA kernel's B tile is one 32-column N tile: J = 9 ct taps must fit
    // (ct <= 3); a 4-channel thin side takes the VALU kernel
    const bool mfma = ct * 9 <= 32 && (w_img % 4) == 0 && cw <= 128 &&
                      (reinterpret_cast<uintptr_t>(wd) & 15) == 0;
    int S;
    if (mfma) {
        const int bands = (h + WM_RB - 1) / WM_RB;
        S = n * bands;
        if ((int64_t)n * bands > 0x7fffffff) return SMMD_EINVAL;
        if (!ws || ws_bytes < (size_t)S * E * sizeof(float)) return SMMD_EWORKSPACE;
        float *part = static_cast<float *>(ws);
        dim3 g((unsigned)S), b(TH_T);
#define SMMD_WG_MFMA(CTV, MTV) \
    thin_wgrad_mfma_kernel<CTV, MTV><<<g, b, 0, st>>>(wd, tt, part, n, cw, h, w_img)
#define SMMD_WG_MT(CTV)                                   \
    do {                                                  \
        if (cw <= 32) SMMD_WG_MFMA(CTV, 1);               \
        else if (cw <= 64) SMMD_WG_MFMA(CTV, 2);          \
        else SMMD_WG_MFMA(CTV, 4);                        \
    } while (0)
        switch (ct) {
            case 1: SMMD_WG_MT(1); break;
            case 2: SMMD_WG_MT(2); break;
            default: SMMD_WG_MT(3); break;
        }
#undef SMMD_WG_MT
#undef SMMD_WG_MFMA
    } else {
        const int chunks = wgrad_chunks(h);
        S = n * chunks;
        if (!ws || ws_bytes < (size_t)S * E * sizeof(float)) return SMMD_EWORKSPACE;
        float *part = static_cast<float *>(ws);
        const int groups = (cw + WG_CG - 1) / WG_CG;
        dim3 g((unsigned)S, (unsigned)((groups + 3) / 4)), b(TH_T);
        switch (ct) {
            case 1: thin_wgrad_kernel<1><<<g, b, 0, st>>>(wd, tt, part, n, cw, h, w_img, chunks); break;
            case 2: thin_wgrad_kernel<2><<<g, b, 0, st>>>(wd, tt, part, n, cw, h, w_img, chunks); break;
            case 3: thin_wgrad_kernel<3><<<g, b, 0, st>>>(wd, tt, part, n, cw, h, w_img, chunks); break;
            default: thin_wgrad_kernel<4><<<g, b, 0, st>>>(wd, tt, part, n, cw, h, w_img, chunks); break;
        }
    }
    smmd_status e = last_launch_status();
    if (e != SMMD_OK) return e;
    // gy's spatial shift for a thin output side: the kernel shifted the thin
    // tensor by +d(t); gw[o][i][t] = sum_q x[i][q] gy[o][q - d(t)] = R[i][o][8 - t]
    thin_wgrad_final_kernel<<<dim3((E + 63) / 64), dim3(WF_T), 0, st>>>(
        static_cast<const float *>(ws), S, cw, ct, thin_in, gw, accum);
    return last_launch_status();
}

extern "C" smmd_status smmd_conv3x3_thin_wgrad(const float *gy, const float *x, float *gw, int n,
                                               int ci, int co, int h, int w_img, void *ws,
                                               size_t ws_bytes, smmd_stream_t stream) {
    return thin_wgrad_launch(gy, x, gw, n, ci, co, h, w_img, ws, ws_bytes, 0, stream);
}

extern "C" smmd_status smmd_conv3x3_thin_wgrad_acc(const float *gy, const float *x, float *gw,
                                                   int n, int ci, int co, int h, int w_img,
                                                   void *ws, size_t ws_bytes,
                                                   smmd_stream_t stream) {
    return thin_wgrad_launch(gy, x, gw, n, ci, co, h, w_img, ws, ws_bytes, 1, stream);
}
