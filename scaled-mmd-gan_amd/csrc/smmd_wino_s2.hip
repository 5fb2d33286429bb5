// smmd_wino_s2.hip -- 4x4 stride-2 pad-1 convolutions (the folded ConvMeanPool
// layers of the critic, gan/core/resnet/block.py:63-66 as one strided conv,
// convops.fold_pool_weight) as polyphase Winograd F(2x2, 2x2) on the f32 MFMA.
//
// Split x into its four 2 x 2 phases and W' into four 2 x 2 taps: the conv is
// the sum over (c, phase) of 2 x 2 stride-1 correlations, i.e. one F(2x2, 2x2)
// problem with 4 C reduction channels: 9 point products per 2 x 2 output tile
// and (phase channel, k) pair, against 16 multiplies of the direct conv
// (1.78x fewer).  For output tile (ty, tx) and phase (pi, pj) the 3 x 3 input
// tile is x rows 4ty-1+pi+2a, cols 4tx-1+pj+2b (a, b in 0..2), the filter
// g[a][b] = W'[k][c][2a+pi][2b+pj] (a, b in 0..1).
//
//   V = B^T d B,  B^T = [[1,-1,0],[0,1,0],[0,-1,1]]
//   U = G g G^T,  G   = [[1,0],[1,1],[0,1]]
//   y = A^T M A,  A^T = [[1,1,0],[0,1,1]]
//
// Block: 64 tiles x 64 output channels, 4 waves, wave (kh, th) the 32 x 32
// quadrant for all 9 points (9 f32x16 accumulators); chunks of 8 phase
// channels (2 input channels x 4 phases) through a double-buffered 36 KB LDS
// stage, so two workgroups fit a CU.
#include "smmd_common.hpp"
#include "smmd_ldsdma.hpp"

namespace smmd {

namespace {

constexpr int S2_T = 256;
constexpr int S2_TB = 64;
constexpr int S2_KB = 64;
constexpr int S2_CC = 2;                     // input channels per chunk (8 phase channels)
constexpr int S2_STAGE = 9 * 8 * 64;         // floats per V (and per U) stage
// + the block's 64 biases (the epilogue reads them from LDS: a global load
// there would wait, in order, for every earlier store)
constexpr size_t S2_LDS = 2 * 2 * S2_STAGE * sizeof(float) + S2_KB * sizeof(float);

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

// neighbour lanes' values, 0 where the source lane is outside the wave
// (bound_ctrl: no preset of the destination; every VALU instruction costs
// SIMD time beside the f32 MFMA, profiles/r12/mfma_valu_coissue.txt)
__device__ __forceinline__ float s2_from_left(float v) {    // lane l gets lane l-1's v
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138,
                                                              0xf, 0xf, true));
}

__device__ __forceinline__ float s2_from_right(float v) {   // lane l gets lane l+1's v
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130,
                                                              0xf, 0xf, true));
}

// buffer access: a wave-uniform base in the descriptor, the lane's 32-bit
// byte offset in one VGPR (no 64-bit address arithmetic per access; tensors
// under 2 GiB, the *_supported checks: the range is 0x7fffffff bytes and
// S2_OOB = 2^31 its out-of-range sentinel); an offset past the range reads zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t s2_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0x7fffffff, 0x00020000);
}
constexpr uint32_t S2_OOB = 0x80000000u;

// The 16 taps of filter q of W': with sig NULL read from w [q][16]; else w is
// the raw weight of a spectrally normalised layer and the taps are those of
// W_eff = (W / sigma) * s (sn.py:43, snops.py:84), pool-folded from the raw
// 3 x 3 filter w [q][9] when fold (ConvMeanPool, block.py:63-66):
// W'[a][b] = 1/4 sum_{i,j in 0..1} W_eff[a-i][b-j] -- the SN refresh's P3
// arithmetic (smmd_sn.hip snf_p3, no contraction), so U is bit-identical to
// the transform of the W_eff / W' that P3 would have written.
__device__ __forceinline__ void s2_taps(const float *__restrict__ w, int64_t q, int fold,
                                        const float *__restrict__ sig,
                                        const float *__restrict__ sc, float (&f)[16]) {
#pragma clang fp contract(off)
    if (!sig) {
        const float *s = w + q * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) f[i] = s[i];
        return;
    }
    const float sigma = sig[0], scale = sc ? sc[0] : 1.f;
    if (!fold) {
        const float *s = w + q * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) f[i] = (s[i] / sigma) * scale;
        return;
    }
    const float *s = w + q * 9;
    float k[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) k[j] = (s[j] / sigma) * scale;
#pragma unroll
    for (int si = 0; si < 4; ++si)
#pragma unroll
        for (int ti = 0; ti < 4; ++ti) {
            float acc = 0.f;
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const int uu = si - a, vv = ti - b;
                    if (uu >= 0 && uu < 3 && vv >= 0 && vv < 3) acc += k[uu * 3 + vv];
                }
            f[si * 4 + ti] = acc * 0.25f;
        }
}

// U for (ko, ci): 4 phases x 9 points, stored u[kb][chunk][p9][h2][k64][c4]
// with phase channel pc = 4 (ci & 1) + 2 pi + pj = 4 h + c4
__global__ void s2_filter_kernel(const float *__restrict__ w, int KO, int CI,
                                 float *__restrict__ u, const float *__restrict__ sig,
                                 const float *__restrict__ sc, int fold) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)KO * CI) return;
    const int ko = (int)(idx % KO), ci = (int)(idx / KO);
    float f[16];
    s2_taps(w, (int64_t)ko * CI + ci, fold, sig, sc, f);
    const int kb = ko >> 6, kl = ko & 63, cc = ci >> 1, h = ci & 1;
    const int64_t base = ((int64_t)kb * (CI >> 1) + cc) * 9;
    float r[9][4];                    // [point][phase 2 pi + pj]
#pragma unroll
    for (int pi = 0; pi < 2; ++pi)
#pragma unroll
        for (int pj = 0; pj < 2; ++pj) {
            const float g00 = f[(pi) * 4 + pj], g01 = f[(pi) * 4 + 2 + pj];
            const float g10 = f[(2 + pi) * 4 + pj], g11 = f[(2 + pi) * 4 + 2 + pj];
            // Gg: rows (g0, g0 + g1, g1) over a, columns b
            const float t[3][2] = {{g00, g01}, {g00 + g10, g01 + g11}, {g10, g11}};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                r[i * 3 + 0][2 * pi + pj] = t[i][0];
                r[i * 3 + 1][2 * pi + pj] = t[i][0] + t[i][1];
                r[i * 3 + 2][2 * pi + pj] = t[i][1];
            }
        }
    // one float4 (the four phases) per point; consecutive lanes, consecutive ko
    float4 *u4 = reinterpret_cast<float4 *>(u);
#pragma unroll
    for (int p = 0; p < 9; ++p)
        u4[((base + p) * 2 + h) * 64 + kl] = make_float4(r[p][0], r[p][1], r[p][2], r[p][3]);
}

struct S2Geom {
    int N, C, K, H, W, TW, Timg;   // H, W: the input's; output H/2 x W/2
    int64_t T, slab;
    // the pair form (smmd_wino4x4s2_conv2): y = conv(x, U) + conv(x2, U2),
    // the input-channel loop running over both inputs
    const float *x2, *u2;
};

// The MFMA stream of one chunk, shared by the forward and the transposed
// kernel: 9 points x 4 MFMAs on the wave's 32 x 32 quadrant, point p's
// accumulator chained in c4 order (the accumulation order of every point is
// that of the unsliced loop, so the results are bit-identical to it).  Point
// p + 1's fragments are read right after point p's first MFMA, so three
// MFMAs (192 cycles) cover the LDS latency instead of none.  After every
// MFMA `slice(K)` (K = 4 p + m) issues that slot's piece of the next chunk's
// work (the transform and the V stores: the f32 MFMA holds the SIMD's VALU,
// so the pieces cost their issue time wherever they go, but inside the
// stream their load and store latencies are covered); sched_barrier pins
// the order.  The first fragments are read by the caller before it issues
// the next chunk's loads.
template <typename Slice>
__device__ __forceinline__ void s2_mfma_chunk(f32x16 (&acc)[9], const float4 *U, const float4 *V,
                                              int ua, int vb, float4 a, float4 b, Slice &&slice) {
#pragma unroll
    for (int p = 0; p < 9; ++p) {
        const float4 ca = a, cb = b;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(ca[m], cb[m], acc[p], 0, 0, 0);
            if (m == 0 && p < 8) {
                a = U[((p + 1) * 2) * 64 + ua];
                b = V[((p + 1) * 2) * 64 + vb];
            }
            slice(p * 4 + m);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// first MFMA slot of the transform slices: the rows were issued at the top
// of the chunk, 20 MFMAs (~1300 cycles) earlier
#ifndef S2_SLOT
#define S2_SLOT 20
#endif

// ACC: y += the result (smmd_wino4x4s2_conv_acc, one slab only)
template <bool EDGE, bool ACC>
__global__ __launch_bounds__(S2_T, 2) void s2_conv_kernel(
    const float *__restrict__ x, const float *__restrict__ u, const float *__restrict__ bias,
    float *__restrict__ y, S2Geom g) {
    extern __shared__ float4 s2_lds[];
    float4 *const Vs = s2_lds;                         // [2][p9][h2][t64]  (float4 = c4)
    float4 *const Us = s2_lds + 2 * (S2_STAGE / 4);    // [2][p9][h2][k64]
    float *const Bs = reinterpret_cast<float *>(s2_lds + 4 * (S2_STAGE / 4));   // [k64]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kb = blockIdx.y;
    const int64_t tile0 = (int64_t)blockIdx.x * S2_TB;
    const int nch1 = g.C / S2_CC;                       // chunks per input
    const int nch = g.x2 ? 2 * nch1 : nch1;             // over both inputs
    const int c0 = (int)((int64_t)nch * blockIdx.z / gridDim.z);
    const int nchunk = (int)((int64_t)nch * (blockIdx.z + 1) / gridDim.z) - c0;
    y += (int64_t)blockIdx.z * g.slab;

    // transform role: lane = tile; wave w = input channel e = w >> 1 of the
    // chunk and row phase pi = w & 1, both column phases
    const int e = w >> 1, pi = w & 1;
    const int64_t gt = tile0 + lane;
    const bool tok = gt < g.T;
    int tn = 0, tty = 0, ttx = 0;
    if (tok) {
        tn = (int)(gt / g.Timg);
        const int r = (int)(gt - (int64_t)tn * g.Timg);
        tty = r / g.TW;
        ttx = r - tty * g.TW;
    }
    const int64_t HW = (int64_t)g.H * g.W;
    // the lane's three patch rows: byte offsets from chunk cc's wave-uniform
    // base (input 2: the distance between the two tensors), a row outside the
    // image past the buffer range (reads zeros)
    uint32_t xo[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int yy = 4 * tty - 1 + pi + 2 * a;
        xo[a] = (yy < 0 || yy >= g.H)
                    ? S2_OOB
                    : (uint32_t)((((int64_t)tn * g.C + e) * HW + (int64_t)yy * g.W + 4 * ttx) * 4);
    }
    const int64_t x2shift = g.x2 ? (int64_t)(reinterpret_cast<uintptr_t>(g.x2) -
                                             reinterpret_cast<uintptr_t>(x)) : 0;
    auto xshift = [&](int cc) -> int64_t {      // bytes from chunk 0 of input 1
        const int c = c0 + cc;
        return c < nch1 ? (int64_t)c * S2_CC * HW * 4
                        : x2shift + (int64_t)(c - nch1) * S2_CC * HW * 4;
    };
    auto xchunk = [&](int cc) -> const float * {   // the lane's image and channel (EDGE)
        return reinterpret_cast<const float *>(
            reinterpret_cast<const char *>(x + ((int64_t)tn * g.C + e) * HW) + xshift(cc));
    };
    auto uchunk = [&](int cc) -> const float4 * {
        const int c = c0 + cc;
        return reinterpret_cast<const float4 *>(c < nch1 ? u : g.u2) +
               ((int64_t)kb * nch1 + (c < nch1 ? c : c - nch1)) * (S2_STAGE / 4);
    };

    f4v raw[3];
    auto load_rows = [&](int cc) {
        const __amdgpu_buffer_rsrc_t rs =
            s2_rsrc(reinterpret_cast<const char *>(x) + xshift(cc));
#pragma unroll
        for (int a = 0; a < 3; ++a)
            raw[a] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, xo[a], 0, 0));
    };
    // the filter stage (18 KiB, contiguous in u) by LDS-DMA: wave w moves
    // pieces w, w + 4, ... of 1 KiB (waves 0 and 1 five, 2 and 3 four)
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const uint32_t us_lds = lds_addr(Us);
    auto load_u = [&](int cc) {
        const float4 *sb = uchunk(cc);
        const uint32_t dst = us_lds + (uint32_t)(cc & 1) * (S2_STAGE * 4);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int piece = wu + 4 * i;
            if (piece < S2_STAGE / 256)
                glds16((uint32_t)(piece * 64 + lane) * 16, sb, dst + (uint32_t)piece * 1024);
        }
    };
    // the transform: V = B^T d B of the lane's tile for its (channel, row
    // phase) and both column phases, as row i's three points (v0: column
    // phase 0, v1: phase 1); t = B^T over the rows (the column-factored form:
    // the own columns packed, the outer columns from the neighbour lanes by
    // DPP with the image-edge zero applied at the source lane)
    f4v t[3];
    float d0[3][3], d1[3][3];        // EDGE: the whole tile's d, B^T applied
    auto xf_cols = [&](int cc) {
        if constexpr (!EDGE) {
            (void)cc;
            t[0] = raw[0] - raw[1];
            t[1] = raw[1];
            t[2] = raw[2] - raw[1];
        } else {
            const float *xc = xchunk(cc);
            // rows: columns 4tx-1 .. 4tx+4; pj = 0 takes (-1, 1, 3), pj = 1 (0, 2, 4)
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const int yy = 4 * tty - 1 + pi + 2 * a;
                const bool row = yy >= 0 && yy < g.H;     // (outside: loaded as zeros)
                const float c0v = raw[a].x, c1v = raw[a].y, c2v = raw[a].z, c3v = raw[a].w;
                float L = s2_from_left(c3v), R = s2_from_right(c0v);
                if (ttx > 0 && lane == 0) L = row ? xc[(int64_t)yy * g.W + 4 * ttx - 1] : 0.f;
                if (ttx < g.TW - 1 && lane == 63) R = row ? xc[(int64_t)yy * g.W + 4 * ttx + 4] : 0.f;
                L = ttx == 0 ? 0.f : L;
                R = ttx == g.TW - 1 ? 0.f : R;
                d0[a][0] = L;   d0[a][1] = c1v; d0[a][2] = c3v;
                d1[a][0] = c0v; d1[a][1] = c2v; d1[a][2] = R;
            }
#pragma unroll
            for (int b = 0; b < 3; ++b) {      // B^T d per column
                const float t00 = d0[0][b] - d0[1][b], t01 = d0[1][b], t02 = d0[2][b] - d0[1][b];
                const float t10 = d1[0][b] - d1[1][b], t11 = d1[1][b], t12 = d1[2][b] - d1[1][b];
                d0[0][b] = t00; d0[1][b] = t01; d0[2][b] = t02;
                d1[0][b] = t10; d1[1][b] = t11; d1[2][b] = t12;
            }
        }
    };
    const bool eL = ttx == 0, eR = ttx == g.TW - 1;
    // row i of V (points 3i .. 3i + 2) into stage buffer buf
    auto xf_row = [&](int i, int buf) {
        float v0[3], v1[3];
        if constexpr (!EDGE) {
            const float ws = eR ? 0.f : t[i].w, xs = eL ? 0.f : t[i].x;
            v0[0] = s2_from_left(ws) - t[i].y;      // columns (L, 1, 3)
            v0[1] = t[i].y;
            v0[2] = t[i].w - t[i].y;
            v1[0] = t[i].x - t[i].z;                // columns (0, 2, R)
            v1[1] = t[i].z;
            v1[2] = s2_from_right(xs) - t[i].z;
        } else {
            v0[0] = d0[i][0] - d0[i][1];
            v0[1] = d0[i][1];
            v0[2] = d0[i][2] - d0[i][1];
            v1[0] = d1[i][0] - d1[i][1];
            v1[1] = d1[i][1];
            v1[2] = d1[i][2] - d1[i][1];
        }
        float2 *const Vl = reinterpret_cast<float2 *>(Vs + buf * (S2_STAGE / 4)) +
                           (e * 64 + lane) * 2 + pi;
#pragma unroll
        for (int j = 0; j < 3; ++j)
            Vl[(3 * i + j) * 256] = make_float2(v0[j], v1[j]);      // point p: + p * 2 KB
    };

    f32x16 acc[9];
#pragma unroll
    for (int p = 0; p < 9; ++p) acc[p] = f32x16{};

    const int th = w & 1, kh = w >> 1, hl = lane >> 5, l32 = lane & 31;
    const int ua = hl * 64 + kh * 32 + l32, vb = hl * 64 + th * 32 + l32;

    // chunk 0 staged before the loop
    const float bias_k = (bias && tid < S2_KB) ? bias[kb * S2_KB + tid] : 0.f;
    load_u(0);
    load_rows(0);
    xf_cols(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) xf_row(i, 0);
    if (tid < S2_KB) Bs[tid] = bias_k;
    dma_wait_all();
    __syncthreads();
    for (int cc = 0;; ++cc) {
        const bool more = cc + 1 < nchunk;
        const int buf = cc & 1, nbuf = buf ^ 1;
        const float4 *U = Us + buf * (S2_STAGE / 4);
        const float4 *V = Vs + buf * (S2_STAGE / 4);
        // the first fragments' reads go out before the next chunk's loads
        const float4 a0 = U[ua], b0 = V[vb];
        __builtin_amdgcn_sched_barrier(0);
        if (more) {
#ifndef S2_NO_DMA        // (S2_NO_*: timing-only diagnostic builds, wrong results)
            load_u(cc + 1);
#endif
            __builtin_amdgcn_sched_barrier(0);
#ifndef S2_NO_ROWS
            load_rows(cc + 1);
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
        s2_mfma_chunk(acc, U, V, ua, vb, a0, b0, [&](int K) {
#ifdef S2_NO_XFORM
            return;
#endif
            if (!more) return;
            if (K == S2_SLOT) {
                // (an empty asm on the rows: their arithmetic cannot be
                // hoisted above this slot, so their wait lands here)
                asm volatile("" : "+v"(raw[0]), "+v"(raw[1]), "+v"(raw[2]));
                xf_cols(cc + 1);
            } else if (K == S2_SLOT + 2 || K == S2_SLOT + 4 || K == S2_SLOT + 6) {
                xf_row((K - S2_SLOT - 2) >> 1, nbuf);
            }
        });
        if (!more) break;
        dma_wait_all();                     // chunk cc + 1's filter stage landed
        __syncthreads();
    }

    // epilogue: C_p[k][tile]; output tile (2ty, 2tx) of y [N, K, H/2, W/2];
    // rows in pairs (r, r + 1: channels k, k + 1, adjacent registers) for
    // packed adds, buffer stores at the lane's fixed offsets plus a uniform
    // per-channel offset
    const int64_t et = tile0 + th * 32 + l32;
    if (et >= g.T) return;
    const int en = (int)(et / g.Timg);
    const int er = (int)(et - (int64_t)en * g.Timg);
    const int ety = er / g.TW, etx = er - ety * g.TW;
    const int Ho = g.H / 2, Wo = g.W / 2;
    typedef float f2v __attribute__((ext_vector_type(2)));
    typedef unsigned u2v __attribute__((ext_vector_type(2)));
    const int kl0 = kh * 32 + 4 * hl;                       // k - 64 kb of row 0
    const uint32_t o0 = (uint32_t)(((((int64_t)en * g.K + kb * S2_KB + kl0) * Ho + 2 * ety) * Wo +
                                     2 * etx) * 4);
    const uint32_t o1 = o0 + (uint32_t)Wo * 4;
    const uint32_t hw4 = (uint32_t)Ho * (uint32_t)Wo * 4;
    const __amdgpu_buffer_rsrc_t ys = s2_rsrc(y);
    // ACC: the earlier values, all loaded before the first store (a load
    // after a store to the same buffer would wait for it: one latency per row
    // pair instead of one per block)
    f2v yo[16][2];
    if constexpr (ACC) {
#pragma unroll
        for (int r = 0; r < 16; r += 2)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t so = (uint32_t)((r & 3) + 8 * (r >> 2) + h) * hw4;
                yo[r + h][0] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(ys, o0, so, 0));
                yo[r + h][1] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(ys, o1, so, 0));
            }
    }
#ifdef S2_NO_EPI
    for (int r = 0; r < 2; r += 2) {
#else
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
#endif
        const int kr = (r & 3) + 8 * (r >> 2);
        f2v m[9];
#pragma unroll
        for (int p = 0; p < 9; ++p) m[p] = f2v{acc[p][r], acc[p][r + 1]};
        // rows: s_a[j] = m[a][j] + m[a+1][j]
        f2v s0[3], s1[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            s0[j] = m[j] + m[3 + j];
            s1[j] = m[3 + j] + m[6 + j];
        }
        const f2v b = *reinterpret_cast<const f2v *>(Bs + kl0 + kr);
        f2v y00 = s0[0] + s0[1] + b, y01 = s0[1] + s0[2] + b;
        f2v y10 = s1[0] + s1[1] + b, y11 = s1[1] + s1[2] + b;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t so = (uint32_t)(kr + h) * hw4;
            if constexpr (ACC) {    // the earlier contribution + this one (autograd's sum)
                const f2v a = yo[r + h][0], c = yo[r + h][1];
                y00[h] = a.x + y00[h];
                y01[h] = a.y + y01[h];
                y10[h] = c.x + y10[h];
                y11[h] = c.y + y11[h];
            }
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, f2v{y00[h], y01[h]}), ys, o0, so, 0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, f2v{y10[h], y11[h]}), ys, o1, so, 0);
        }
    }
}

// ---- the transposed conv: dx = conv_transpose2d(gy, W', stride 2, pad 1) ----
// (the input gradient of the 4x4 stride-2 conv; also the generator's folded
// UpsampleConv, a transposed conv with K [cin, cout, 4, 4]).  Output phase
// (qi, qj) of dx is a 2 x 2 stride-1 correlation of gy: dx[2r+qi][2s+qj] =
// sum_k sum_{a,b in 0..1} gy[k][r-1+qi+a][s-1+qj+b] W'[k][c][3-qi-2a][3-qj-2b],
// one F(2x2, 2x2) problem per phase with K reduction channels.  Block: one
// phase (s2_xcd_order), 64 phase tiles x 64 output channels; as the
// forward kernel otherwise (chunks of 8 k, 9 accumulators per wave).

// U for the transposed conv: ut[q4][cb][kchunk][p9][h2][c64][k4], from W' [K][C][4][4];
// a thread owns one c and four consecutive k, so each (phase, point) is one
// float4 store and consecutive lanes (consecutive c) store consecutive 16 bytes
__global__ void s2t_filter_kernel(const float *__restrict__ w, int K, int C,
                                  float *__restrict__ u, const float *__restrict__ sig,
                                  const float *__restrict__ sc, int fold) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)(K >> 2) * C) return;
    const int c = (int)(idx % C), kq = (int)(idx / C);
    const int cb = c >> 6, cl = c & 63, kc = kq >> 1, h = kq & 1;
    const int64_t per_phase = (int64_t)C * K * 9;
    float f[4][16];
#pragma unroll
    for (int e = 0; e < 4; ++e) s2_taps(w, (int64_t)(4 * kq + e) * C + c, fold, sig, sc, f[e]);
    float4 *u4 = reinterpret_cast<float4 *>(u);
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int qj = 0; qj < 2; ++qj) {
            float r[9][4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                // g[a][b] = W'[3 - qi - 2a][3 - qj - 2b]
                const float g00 = f[e][(3 - qi) * 4 + 3 - qj], g01 = f[e][(3 - qi) * 4 + 1 - qj];
                const float g10 = f[e][(1 - qi) * 4 + 3 - qj], g11 = f[e][(1 - qi) * 4 + 1 - qj];
                const float t[3][2] = {{g00, g01}, {g00 + g10, g01 + g11}, {g10, g11}};
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    r[i * 3 + 0][e] = t[i][0];
                    r[i * 3 + 1][e] = t[i][0] + t[i][1];
                    r[i * 3 + 2][e] = t[i][1];
                }
            }
            const int64_t base =
                ((qi * 2 + qj) * per_phase + ((int64_t)cb * (K >> 3) + kc) * 9 * 512) / 4;
#pragma unroll
            for (int p = 0; p < 9; ++p)
                u4[base + (p * 2 + h) * 64 + cl] = make_float4(r[p][0], r[p][1], r[p][2], r[p][3]);
        }
}

struct S2TGeom {
    int N, K, C, Hg, Wg, TW, Timg;  // gy [N, K, Hg, Wg]; dx [N, C, 2Hg, 2Wg]; tiles of a phase
    int64_t T, slab;
    int CB, S;                      // channel blocks (C / 64), K slices
    // smmd_wino4x4s2t_conv_mask: dx = (mask <= 0 ? 0 : dx), mask of dx's shape
    // (the conv's input, a ReLU output: its producer's mask applied here)
    const float *mask;
};

// The block's work from its 1-D id, XCD-aware: blocks b and b + 8 share an
// XCD and its L2 (MI355X_MICROARCH.md, dispatch; for speed only, any
// placement is correct), so XCD x takes the x-th contiguous range of a
// logical order.  Tile-major ((tile block, slice, channel block), phase): the
// four phase blocks and the channel blocks of one tile block -- which read
// the same gy rows and write interleaved columns of the same dx lines -- run
// together on one L2 (a phase writes every other 4-byte column; on separate
// L2s each line went to HBM up to four times, each partial write read back
// first: 128 -> 64 MB written on the 64-channel fold layer at batch 64).
// (Measured and not kept: filter-major, (phase, channel block, slice) outer
// and tile blocks inner, 1-6 % slower on all four fold layers even where the
// filter outweighs gy and dx.)
__device__ __forceinline__ uint32_t s2_xcd_order(uint32_t L, uint32_t n) {
    const uint32_t q = n >> 3, r = n & 7, x = L & 7, j = L >> 3;
    return x < r ? x * (q + 1) + j : r * (q + 1) + (x - r) * q + j;
}

// the body for output phase (QI, QJ): the phase is a compile-time constant, so
// its row and column picks cost no per-lane selects (every VALU instruction
// costs SIMD time beside the f32 MFMA, profiles/r12/mfma_valu_coissue.txt)
template <bool EDGE, int QI, int QJ>
__device__ __forceinline__ void s2t_body(const float *__restrict__ gy, const float *__restrict__ u,
                                         const float *__restrict__ bias, float *__restrict__ dx,
                                         const S2TGeom &g, int64_t tb, int cb, int sl) {
    extern __shared__ float4 s2_lds[];
    float4 *const Vs = s2_lds;
    float4 *const Us = s2_lds + 2 * (S2_STAGE / 4);
    float *const Bs = reinterpret_cast<float *>(s2_lds + 4 * (S2_STAGE / 4));   // [c64]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int q = QI * 2 + QJ, qi = QI, qj = QJ;
    const int THg = g.Hg >> 1;           // phase tile rows per image
    const int S = g.S;
    const int64_t tile0 = tb * S2_TB;
    const int nch = g.K / 8;
    const int c0 = (int)((int64_t)nch * sl / S);
    const int nchunk = (int)((int64_t)nch * (sl + 1) / S) - c0;
    dx += (int64_t)sl * g.slab;

    // transform role: lane = tile, wave w = k channels 2w, 2w+1 of the chunk
    const int64_t gt = tile0 + lane;
    const bool tok = gt < g.T;
    int tn = 0, tty = 0, ttx = 0;
    if (tok) {
        tn = (int)(gt / g.Timg);
        const int r = (int)(gt - (int64_t)tn * g.Timg);
        tty = r / g.TW;
        ttx = r - tty * g.TW;
    }
    const int64_t HW = (int64_t)g.Hg * g.Wg;
    const float *gn = gy + ((int64_t)tn * g.K + (int64_t)c0 * 8 + 2 * w) * HW;
    const float4 *ub = reinterpret_cast<const float4 *>(u) + (int64_t)q * g.C * g.K * 9 / 4 +
                       ((int64_t)cb * nch + c0) * (S2_STAGE / 4);

    // the rows by buffer loads: chunk cc's base (k = 8 (c0 + cc)) uniform, the
    // lane's offsets fixed; a row outside the image reads zeros
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v raw[2][3];
    uint32_t roff[2][3];
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const int yy = 2 * tty - 1 + qi + a;
            roff[e][a] = (yy < 0 || yy >= g.Hg)
                             ? S2_OOB
                             : (uint32_t)((((int64_t)tn * g.K + 2 * w + e) * HW +
                                           (int64_t)yy * g.Wg + 2 * ttx) * 4);
        }
    auto load_rows = [&](int cc) {
        const __amdgpu_buffer_rsrc_t rs = s2_rsrc(gy + ((int64_t)c0 + cc) * 8 * HW);
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int a = 0; a < 3; ++a)
                raw[e][a] = __builtin_bit_cast(
                    f2v, __builtin_amdgcn_raw_buffer_load_b64(rs, roff[e][a], 0, 0));
    };
    // the filter stage (18 KiB, contiguous in u) by LDS-DMA, as the forward's
    const int wu = __builtin_amdgcn_readfirstlane(w);
    const uint32_t us_lds = lds_addr(Us);
    auto load_u = [&](int cc) {
        const float4 *sb = ub + (int64_t)cc * (S2_STAGE / 4);
        const uint32_t dst = us_lds + (uint32_t)(cc & 1) * (S2_STAGE * 4);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int piece = wu + 4 * i;
            if (piece < S2_STAGE / 256)
                glds16((uint32_t)(piece * 64 + lane) * 16, sb, dst + (uint32_t)piece * 1024);
        }
    };
    // the transform of the lane's phase tile for both k channels: t = B^T
    // over the rows (column-factored: the own two columns packed, the outer
    // column from the neighbour lane by DPP, its image-edge zero applied at
    // the source lane: a lane at its row's right edge passes 0 to the right,
    // one at the left edge 0 to the left); EDGE: d with B^T applied
    f2v t[2][3];
    float dd[2][3][3];
    const bool eL = ttx == 0, eR = ttx == g.TW - 1;
    auto xf_cols = [&](int cc) {
        if constexpr (!EDGE) {
            (void)cc;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                t[e][0] = raw[e][0] - raw[e][1];
                t[e][1] = raw[e][1];
                t[e][2] = raw[e][2] - raw[e][1];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const float *gc = gn + ((int64_t)cc * 8 + e) * HW;
                float (&d)[3][3] = dd[e];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const int yy = 2 * tty - 1 + qi + a;
                    // rows 2ty - 1 (phase row 0) and 2ty + 2 (phase row 1) can be
                    // outside the image (loaded as zeros); a tile past the end is
                    // never stored
                    const bool row = (a == 0 && qi == 0) ? tty > 0
                                     : (a == 2 && qi == 1) ? tty < THg - 1 : true;
                    const float cx = raw[e][a].x, cy = raw[e][a].y;
                    float L = s2_from_left(cy), R = s2_from_right(cx);
                    if (ttx > 0 && lane == 0) L = row ? gc[(int64_t)yy * g.Wg + 2 * ttx - 1] : 0.f;
                    if (ttx < g.TW - 1 && lane == 63)
                        R = row ? gc[(int64_t)yy * g.Wg + 2 * ttx + 2] : 0.f;
                    L = ttx == 0 ? 0.f : L;
                    R = ttx == g.TW - 1 ? 0.f : R;
                    // columns 2tx - 1 + qj + b
                    d[a][0] = qj ? cx : L;
                    d[a][1] = qj ? cy : cx;
                    d[a][2] = qj ? R : cy;
                }
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    const float t0 = d[0][b] - d[1][b], t2 = d[2][b] - d[1][b];
                    d[0][b] = t0;
                    d[2][b] = t2;
                }
            }
        }
    };
    // row i of V (points 3i .. 3i + 2), both k channels, into stage buffer buf
    auto xf_row = [&](int i, int buf) {
        float v[2][3];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            if constexpr (!EDGE) {
                if (qj == 0) {          // columns (L, x, y)
                    const float ys = eR ? 0.f : t[e][i].y;
                    v[e][0] = s2_from_left(ys) - t[e][i].x;
                    v[e][1] = t[e][i].x;
                    v[e][2] = t[e][i].y - t[e][i].x;
                } else {                // columns (x, y, R)
                    const float xs = eL ? 0.f : t[e][i].x;
                    v[e][0] = t[e][i].x - t[e][i].y;
                    v[e][1] = t[e][i].y;
                    v[e][2] = s2_from_right(xs) - t[e][i].y;
                }
            } else {
                v[e][0] = dd[e][i][0] - dd[e][i][1];
                v[e][1] = dd[e][i][1];
                v[e][2] = dd[e][i][2] - dd[e][i][1];
            }
        }
        float2 *const Vl = reinterpret_cast<float2 *>(Vs + buf * (S2_STAGE / 4)) +
                           ((w >> 1) * 64 + lane) * 2 + (w & 1);
#pragma unroll
        for (int j = 0; j < 3; ++j)
            Vl[(3 * i + j) * 256] = make_float2(v[0][j], v[1][j]);  // point p: + p * 2 KB
    };

    f32x16 acc[9];
#pragma unroll
    for (int p = 0; p < 9; ++p) acc[p] = f32x16{};

    const int th = w & 1, kh = w >> 1, hl = lane >> 5, l32 = lane & 31;
    const int ua = hl * 64 + kh * 32 + l32, vb = hl * 64 + th * 32 + l32;

    const float bias_c = (bias && tid < 64) ? bias[cb * 64 + tid] : 0.f;
    load_u(0);
    load_rows(0);
    xf_cols(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) xf_row(i, 0);
    if (tid < 64) Bs[tid] = bias_c;
    dma_wait_all();
    __syncthreads();
    for (int cc = 0;; ++cc) {
        const bool more = cc + 1 < nchunk;
        const int buf = cc & 1, nbuf = buf ^ 1;
        const float4 *U = Us + buf * (S2_STAGE / 4);
        const float4 *V = Vs + buf * (S2_STAGE / 4);
        const float4 a0 = U[ua], b0 = V[vb];
        __builtin_amdgcn_sched_barrier(0);
        if (more) {
#ifndef S2_NO_DMA
            load_u(cc + 1);
#endif
            __builtin_amdgcn_sched_barrier(0);
#ifndef S2_NO_ROWS
            load_rows(cc + 1);
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
        s2_mfma_chunk(acc, U, V, ua, vb, a0, b0, [&](int K) {
#ifdef S2_NO_XFORM
            return;
#endif
            if (!more) return;
            if (K == S2_SLOT) {
                asm volatile("" : "+v"(raw[0][0]), "+v"(raw[0][1]), "+v"(raw[0][2]),
                             "+v"(raw[1][0]), "+v"(raw[1][1]), "+v"(raw[1][2]));
                xf_cols(cc + 1);
            } else if (K == S2_SLOT + 2 || K == S2_SLOT + 4 || K == S2_SLOT + 6) {
                xf_row((K - S2_SLOT - 2) >> 1, nbuf);
            }
        });
        if (!more) break;
        dma_wait_all();
        __syncthreads();
    }

    // epilogue: phase tile (ty, tx) -> dx rows 2 (2ty + a) + qi, cols 2 (2tx + b) + qj;
    // buffer stores at the lane's fixed offsets plus a uniform per-channel
    // offset
    const int64_t et = tile0 + th * 32 + l32;
    if (et >= g.T) return;
    const int en = (int)(et / g.Timg);
    const int er = (int)(et - (int64_t)en * g.Timg);
    const int ety = er / g.TW, etx = er - ety * g.TW;
    const int Hx = 2 * g.Hg, Wx = 2 * g.Wg;
    const int cl0 = kh * 32 + 4 * hl;                       // c - 64 cb of row 0
    const uint32_t o0 = (uint32_t)(((((int64_t)en * g.C + cb * 64 + cl0) * Hx + 4 * ety + qi) * Wx +
                                     4 * etx + qj) * 4);
    const uint32_t o1 = o0 + (uint32_t)Wx * 8;            // output row + 2
    const uint32_t hw4 = (uint32_t)Hx * (uint32_t)Wx * 4;
    const __amdgpu_buffer_rsrc_t ds = s2_rsrc(dx);
    // the mask's 64 values of the lane, all loaded before the first store (the
    // stage's registers are free here): one latency per block instead of one
    // per output row pair
    float mk[16][4];
    const bool masked = g.mask != nullptr;
    if (masked) {
        const __amdgpu_buffer_rsrc_t ms = s2_rsrc(g.mask);
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t so = (uint32_t)((r & 3) + 8 * (r >> 2) + h) * hw4;
                mk[r + h][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ms, o0, so, 0));
                mk[r + h][1] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ms, o0 + 8, so, 0));
                mk[r + h][2] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ms, o1, so, 0));
                mk[r + h][3] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ms, o1 + 8, so, 0));
            }
        }
    }
#ifdef S2_NO_EPI
    for (int r = 0; r < 2; r += 2) {
#else
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
#endif
        const int cr = (r & 3) + 8 * (r >> 2);              // c - c of row 0
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float m[9];
#pragma unroll
            for (int p = 0; p < 9; ++p) m[p] = acc[p][r + h];
            float s0[3], s1[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                s0[j] = m[j] + m[3 + j];
                s1[j] = m[3 + j] + m[6 + j];
            }
            const float b = Bs[cl0 + cr + h];
            float v[4] = {s0[0] + s0[1] + b, s0[1] + s0[2] + b, s1[0] + s1[1] + b,
                          s1[1] + s1[2] + b};
            if (masked) {               // threshold_backward(v, mask, 0)'s select
#pragma unroll
                for (int i = 0; i < 4; ++i) v[i] = mk[r + h][i] <= 0.f ? 0.f : v[i];
            }
            const uint32_t so = (uint32_t)(cr + h) * hw4;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[0]), ds, o0, so, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[1]), ds, o0 + 8, so, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[2]), ds, o1, so, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v[3]), ds, o1 + 8, so, 0);
        }
    }
}

template <bool EDGE>
__global__ __launch_bounds__(S2_T, 2) void s2t_conv_kernel(
    const float *__restrict__ gy, const float *__restrict__ u, const float *__restrict__ bias,
    float *__restrict__ dx, S2TGeom g) {
    uint32_t W = s2_xcd_order(blockIdx.x, gridDim.x);
    const int q = (int)(W & 3);         // the block's output phase (wave-uniform)
    W >>= 2;
    const int cb = (int)(W % (uint32_t)g.CB);
    W /= (uint32_t)g.CB;
    const int sl = (int)(W % (uint32_t)g.S);
    const int64_t tb = W / (uint32_t)g.S;
    switch (q) {
    case 0: s2t_body<EDGE, 0, 0>(gy, u, bias, dx, g, tb, cb, sl); break;
    case 1: s2t_body<EDGE, 0, 1>(gy, u, bias, dx, g, tb, cb, sl); break;
    case 2: s2t_body<EDGE, 1, 0>(gy, u, bias, dx, g, tb, cb, sl); break;
    default: s2t_body<EDGE, 1, 1>(gy, u, bias, dx, g, tb, cb, sl); break;
    }
}

// (mask: the transposed conv's ReLU mask, applied after the bias)
__global__ void s2_reduce_kernel(const float *__restrict__ part, const float *__restrict__ bias,
                                 float *__restrict__ y, int64_t n4, int S, int K, int HW,
                                 const float *__restrict__ mask, int acc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    const float4 *p4 = reinterpret_cast<const float4 *>(part);
    const float4 mv = mask ? reinterpret_cast<const float4 *>(mask)[i] : float4{};
    float4 s = p4[i];
    for (int z = 1; z < S; ++z) {
        const float4 t = p4[i + z * n4];
        s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
    if (bias) {
        const float b = bias[(int)((i * 4 / HW) % K)];
        s.x += b; s.y += b; s.z += b; s.w += b;
    }
    if (mask) {
        s.x = mv.x <= 0.f ? 0.f : s.x;
        s.y = mv.y <= 0.f ? 0.f : s.y;
        s.z = mv.z <= 0.f ? 0.f : s.z;
        s.w = mv.w <= 0.f ? 0.f : s.w;
    }
    if (acc) {                  // y += the result
        const float4 o = reinterpret_cast<const float4 *>(y)[i];
        s = make_float4(o.x + s.x, o.y + s.y, o.z + s.z, o.w + s.w);
    }
    reinterpret_cast<float4 *>(y)[i] = s;
}

}  // namespace

// reduction slices: one workgroup per CU at least, at least 4 (8) chunks
// per slice.  Targets measured on the SNResNet-64 layers (conv / transposed,
// us): 256 workgroups 115 / 120 / 119 / 112 and 132 / 118 / 124 / 129; 512:
// 112 / 123 / 121 / 112 and 140 / 123 / 136 / 123; 1024 slower
static int s2_target() { return 256; }

static int s2t_slices(int64_t blocks, int nch) {
    int S = 1;
    while (blocks * S < s2_target() && nch / (2 * S) >= 4) S *= 2;
    return S;
}

static int s2_slices(int64_t blocks, int nch, int HWo) {
    int S = 1;
    while (blocks * S < s2_target() && nch / (2 * S) >= 8 && HWo % 4 == 0) S *= 2;
    return S;
}

}  // namespace smmd

using namespace smmd;

extern "C" int smmd_wino4x4s2_supported(int n, int ci, int ko, int h, int w_img) {
    return n > 0 && ci > 0 && ko > 0 && ci % S2_CC == 0 && ko % S2_KB == 0 && h > 0 &&
           w_img > 0 && h % 4 == 0 && w_img % 4 == 0 && (int64_t)n * ci * h * w_img < (1ll << 29) &&
           (int64_t)n * ko * h * w_img < (1ll << 31);   // x, y (n ko h w / 4) under 2 GiB (buffer offsets)
}

extern "C" size_t smmd_wino4x4s2_filter_bytes(int ko, int ci) {
    if (ko <= 0 || ci <= 0) return 0;
    return (size_t)36 * ko * ci * sizeof(float);
}

extern "C" smmd_status smmd_wino4x4s2_filter(const float *w, int ko, int ci, float *u,
                                             size_t u_bytes, smmd_stream_t stream) {
    if (ko <= 0 || ci <= 0 || !w || !u) return SMMD_EINVAL;
    if (ko % S2_KB || ci % S2_CC) return SMMD_EUNSUPPORTED;
    if (reinterpret_cast<uintptr_t>(u) & 15) return SMMD_EINVAL;
    if (u_bytes < smmd_wino4x4s2_filter_bytes(ko, ci)) return SMMD_EWORKSPACE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n = (int64_t)ko * ci;
    s2_filter_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(w, ko, ci, u,
                                                                             nullptr, nullptr, 0);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino4x4s2_filter_sn(const float *w, const float *sigma,
                                                const float *s, int fold, int ko, int ci,
                                                float *u, size_t u_bytes, smmd_stream_t stream) {
    if (ko <= 0 || ci <= 0 || !w || !u || !sigma || (fold != 0 && fold != 1)) return SMMD_EINVAL;
    if (ko % S2_KB || ci % S2_CC) return SMMD_EUNSUPPORTED;
    if (reinterpret_cast<uintptr_t>(u) & 15) return SMMD_EINVAL;
    if (u_bytes < smmd_wino4x4s2_filter_bytes(ko, ci)) return SMMD_EWORKSPACE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n = (int64_t)ko * ci;
    s2_filter_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(w, ko, ci, u,
                                                                             sigma, s, fold);
    return last_launch_status();
}

extern "C" size_t smmd_wino4x4s2_workspace_bytes(int n, int ci, int ko, int h, int w_img) {
    if (!smmd_wino4x4s2_supported(n, ci, ko, h, w_img)) return 0;
    const int64_t T = (int64_t)n * (h / 4) * (w_img / 4);
    const int S = s2_slices(((T + S2_TB - 1) / S2_TB) * (ko / S2_KB), ci / S2_CC,
                            (h / 2) * (w_img / 2));
    return S > 1 ? (size_t)S * n * ko * (h / 2) * (w_img / 2) * sizeof(float) : 0;
}

static smmd_status s2_conv(const float *x, const float *u, const float *x2, const float *u2,
                           const float *bias, float *y, int n, int ci, int ko, int h, int w_img,
                           void *ws, size_t ws_bytes, smmd_stream_t stream, int acc = 0) {
    if (n < 0 || ci <= 0 || ko <= 0 || h < 0 || w_img < 0) return SMMD_EINVAL;
    if (n == 0 || h == 0 || w_img == 0) return SMMD_OK;
    if (!x || !u || !y || (!x2 != !u2)) return SMMD_EINVAL;
    if (!smmd_wino4x4s2_supported(n, ci, ko, h, w_img)) return SMMD_EUNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) |
         reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(x2) |
         reinterpret_cast<uintptr_t>(u2)) & 15)
        return SMMD_EINVAL;
    const int pair = x2 ? 2 : 1;
    S2Geom g;
    g.x2 = x2;
    g.u2 = u2;
    g.N = n; g.C = ci; g.K = ko; g.H = h; g.W = w_img;
    g.TW = w_img / 4;
    g.Timg = (h / 4) * g.TW;
    g.T = (int64_t)n * g.Timg;
    const int64_t tb = (g.T + S2_TB - 1) / S2_TB;
    if (tb > 0x7fffffff) return SMMD_EINVAL;
    const int HWo = (h / 2) * (w_img / 2);
    const int S = s2_slices(tb * (ko / S2_KB), pair * ci / S2_CC, HWo);
    const int64_t total = (int64_t)n * ko * HWo;
    float *out = y;
    if (S > 1) {
        if (!ws || ws_bytes < (size_t)S * total * sizeof(float)) return SMMD_EWORKSPACE;
        if (reinterpret_cast<uintptr_t>(ws) & 15) return SMMD_EINVAL;
        out = static_cast<float *>(ws);
    }
    static bool attr = false;
    if (!attr) {
        const void *ks[4] = {reinterpret_cast<const void *>(s2_conv_kernel<false, false>),
                             reinterpret_cast<const void *>(s2_conv_kernel<true, false>),
                             reinterpret_cast<const void *>(s2_conv_kernel<false, true>),
                             reinterpret_cast<const void *>(s2_conv_kernel<true, true>)};
        for (const void *k : ks)
            if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)S2_LDS) !=
                hipSuccess)
                return SMMD_EHIP;
        attr = true;
    }
    g.slab = S > 1 ? total : 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)tb, (unsigned)(ko / S2_KB), (unsigned)S);
    const float *b1 = S > 1 ? nullptr : bias;
    const bool ka = acc && S == 1;      // sliced: the reduction adds
    auto k = 64 % g.TW == 0 ? (ka ? s2_conv_kernel<false, true> : s2_conv_kernel<false, false>)
                            : (ka ? s2_conv_kernel<true, true> : s2_conv_kernel<true, false>);
    k<<<grid, dim3(S2_T), S2_LDS, st>>>(x, u, b1, out, g);
    smmd_status e = last_launch_status();
    if (e != SMMD_OK || S == 1) return e;
    const int64_t n4 = total / 4;
    s2_reduce_kernel<<<dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st>>>(out, bias, y, n4,
                                                                              S, ko, HWo, nullptr,
                                                                              acc);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino4x4s2_conv(const float *x, const float *u, const float *bias,
                                           float *y, int n, int ci, int ko, int h, int w_img,
                                           void *ws, size_t ws_bytes, smmd_stream_t stream) {
    return s2_conv(x, u, nullptr, nullptr, bias, y, n, ci, ko, h, w_img, ws, ws_bytes, stream);
}

// y += conv(x, W') + bias: a later gradient contribution summed into an
// earlier one where autograd would add the two (convops._ConvBackward, the
// double backward's gradient of a gradient both a block's main path and its
// shortcut read)
extern "C" smmd_status smmd_wino4x4s2_conv_acc(const float *x, const float *u, const float *bias,
                                               float *y, int n, int ci, int ko, int h, int w_img,
                                               void *ws, size_t ws_bytes, smmd_stream_t stream) {
    return s2_conv(x, u, nullptr, nullptr, bias, y, n, ci, ko, h, w_img, ws, ws_bytes, stream, 1);
}

extern "C" size_t smmd_wino4x4s2_conv2_workspace_bytes(int n, int ci, int ko, int h, int w_img) {
    if (!smmd_wino4x4s2_supported(n, ci, ko, h, w_img)) return 0;
    const int64_t T = (int64_t)n * (h / 4) * (w_img / 4);
    const int S = s2_slices(((T + S2_TB - 1) / S2_TB) * (ko / S2_KB), 2 * ci / S2_CC,
                            (h / 2) * (w_img / 2));
    return S > 1 ? (size_t)S * n * ko * (h / 2) * (w_img / 2) * sizeof(float) : 0;
}

extern "C" smmd_status smmd_wino4x4s2_conv2(const float *x, const float *u, const float *x2,
                                            const float *u2, const float *bias, float *y, int n,
                                            int ci, int ko, int h, int w_img, void *ws,
                                            size_t ws_bytes, smmd_stream_t stream) {
    if (!x2 || !u2) return SMMD_EINVAL;
    return s2_conv(x, u, x2, u2, bias, y, n, ci, ko, h, w_img, ws, ws_bytes, stream);
}

extern "C" int smmd_wino4x4s2t_supported(int n, int k, int c, int hg, int wg) {
    return n > 0 && k > 0 && c > 0 && k % 8 == 0 && c % 64 == 0 && hg > 0 && wg > 0 &&
           hg % 2 == 0 && wg % 2 == 0 && (int64_t)n * k * hg * wg < (1ll << 29) &&
           (int64_t)n * c * 4 * hg * wg < (1ll << 29);   // gy, dx under 2 GiB (buffer offsets)
}

extern "C" smmd_status smmd_wino4x4s2t_filter(const float *w, int k, int c, float *u,
                                              size_t u_bytes, smmd_stream_t stream) {
    if (k <= 0 || c <= 0 || !w || !u) return SMMD_EINVAL;
    if (k % 8 || c % 64) return SMMD_EUNSUPPORTED;
    if (reinterpret_cast<uintptr_t>(u) & 15) return SMMD_EINVAL;
    if (u_bytes < smmd_wino4x4s2_filter_bytes(k, c)) return SMMD_EWORKSPACE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n = (int64_t)(k / 4) * c;
    s2t_filter_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(w, k, c, u,
                                                                              nullptr, nullptr, 0);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino4x4s2t_filter_sn(const float *w, const float *sigma,
                                                 const float *s, int fold, int k, int c,
                                                 float *u, size_t u_bytes, smmd_stream_t stream) {
    if (k <= 0 || c <= 0 || !w || !u || !sigma || (fold != 0 && fold != 1)) return SMMD_EINVAL;
    if (k % 8 || c % 64) return SMMD_EUNSUPPORTED;
    if (reinterpret_cast<uintptr_t>(u) & 15) return SMMD_EINVAL;
    if (u_bytes < smmd_wino4x4s2_filter_bytes(k, c)) return SMMD_EWORKSPACE;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t n = (int64_t)(k / 4) * c;
    s2t_filter_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(w, k, c, u,
                                                                              sigma, s, fold);
    return last_launch_status();
}

extern "C" size_t smmd_wino4x4s2t_workspace_bytes(int n, int k, int c, int hg, int wg) {
    if (!smmd_wino4x4s2t_supported(n, k, c, hg, wg)) return 0;
    const int64_t T = (int64_t)n * (hg / 2) * (wg / 2);
    const int S = s2t_slices(((T + S2_TB - 1) / S2_TB) * (c / 64) * 4, k / 8);
    return S > 1 ? (size_t)S * n * c * 4 * hg * wg * sizeof(float) : 0;
}

// dx [n, c, 2 hg, 2 wg] = conv_transpose2d(gy [n, k, hg, wg], W' [k, c, 4, 4], stride 2, pad 1) + bias
static smmd_status s2t_launch(const float *gy, const float *u, const float *bias,
                              const float *mask, float *dx, int n, int k, int c, int hg, int wg,
                              void *ws, size_t ws_bytes, smmd_stream_t stream) {
    if (n < 0 || k <= 0 || c <= 0 || hg < 0 || wg < 0) return SMMD_EINVAL;
    if (n == 0 || hg == 0 || wg == 0) return SMMD_OK;
    if (!gy || !u || !dx) return SMMD_EINVAL;
    if (!smmd_wino4x4s2t_supported(n, k, c, hg, wg)) return SMMD_EUNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(gy) | reinterpret_cast<uintptr_t>(dx) |
         reinterpret_cast<uintptr_t>(u) | reinterpret_cast<uintptr_t>(mask)) & 15)
        return SMMD_EINVAL;
    S2TGeom g;
    g.N = n; g.K = k; g.C = c; g.Hg = hg; g.Wg = wg;
    g.TW = wg / 2;
    g.Timg = (hg / 2) * g.TW;
    g.T = (int64_t)n * g.Timg;
    const int64_t tb = (g.T + S2_TB - 1) / S2_TB;
    if (tb > 0x7fffffff) return SMMD_EINVAL;
    const int S = s2t_slices(tb * (c / 64) * 4, k / 8);
    const int64_t total = (int64_t)n * c * 4 * hg * wg;
    float *out = dx;
    if (S > 1) {
        if (!ws || ws_bytes < (size_t)S * total * sizeof(float)) return SMMD_EWORKSPACE;
        if (reinterpret_cast<uintptr_t>(ws) & 15) return SMMD_EINVAL;
        out = static_cast<float *>(ws);
    }
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(s2t_conv_kernel<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)S2_LDS) != hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void *>(s2t_conv_kernel<true>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)S2_LDS) != hipSuccess)
            return SMMD_EHIP;
        attr = true;
    }
    g.slab = S > 1 ? total : 0;
    g.CB = c / 64;
    g.S = S;
    g.mask = S > 1 ? nullptr : mask;           // several slices: the final sum masks

    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t nblk = tb * (c / 64) * 4 * S;
    if (nblk > 0x7fffffff) return SMMD_EINVAL;
    const dim3 grid((unsigned)nblk);
    const float *b1 = S > 1 ? nullptr : bias;
    if (64 % g.TW == 0)
        s2t_conv_kernel<false><<<grid, dim3(S2_T), S2_LDS, st>>>(gy, u, b1, out, g);
    else
        s2t_conv_kernel<true><<<grid, dim3(S2_T), S2_LDS, st>>>(gy, u, b1, out, g);
    smmd_status e = last_launch_status();
    if (e != SMMD_OK || S == 1) return e;
    const int64_t n4 = total / 4;
    s2_reduce_kernel<<<dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st>>>(
        out, bias, dx, n4, S, c, 4 * hg * wg, mask, 0);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino4x4s2t_conv(const float *gy, const float *u, const float *bias,
                                            float *dx, int n, int k, int c, int hg, int wg,
                                            void *ws, size_t ws_bytes, smmd_stream_t stream) {
    return s2t_launch(gy, u, bias, nullptr, dx, n, k, c, hg, wg, ws, ws_bytes, stream);
}

extern "C" smmd_status smmd_wino4x4s2t_conv_mask(const float *gy, const float *u,
                                                 const float *bias, const float *mask, float *dx,
                                                 int n, int k, int c, int hg, int wg, void *ws,
                                                 size_t ws_bytes, smmd_stream_t stream) {
    if (!mask) return SMMD_EINVAL;
    return s2t_launch(gy, u, bias, mask, dx, n, k, c, hg, wg, ws, ws_bytes, stream);
}
