// smmd_wino_wgrad.hip -- the weight gradient of the 3x3 stride-1 SAME
// convolution as Winograd F(2x2, 3x3) on the f32 MFMA (TF's
// Conv2DBackpropFilter of snops.conv2d / resnet Conv2D, gan/core/snops.py:69-90,
// for the wide 3x3 layers of gan/core/resnet/block.py:38-50).
//
// The forward kernel (smmd_wino.hip) computes y_t = A^T (sum_c U_p V_p) A per
// 2 x 2 output tile t.  Its adjoint in U is
//   dU_p[k][c] = sum_t dM_p[k][t] V_p[c][t],   dM = A dY_t A^T,  V = B^T d_t B,
// and dW = G^T dU G: 16 point GEMMs that reduce over the tiles (2.25x fewer
// multiplies than the direct weight gradient).
//
// Block: 64 k x 64 c x a slice of the tiles, 4 waves; wave (kh, ch) owns the
// 32 x 32 (k, c) quadrant for all 16 points (16 f32x16 accumulators).  Tiles
// go 8 per chunk (4 MFMA k-steps of 2) through double-buffered LDS:
// dM [p][h][k64][t4] and V [p][h][c64][t4].  Transform role: lane = channel
// (k for dM, c for V), wave w = the chunk's tiles 2w, 2w+1 (horizontal
// neighbours: TW is even).  Each slice writes its partial dU [K][C][16] to the
// workspace; smmd_wino3x3_wgrad adds the slices in order (in groups of 16 first
// when there are more than 32) and applies G^T . G.
#include "smmd_common.hpp"

namespace smmd {

namespace {

constexpr int WG_T = 256;
constexpr int WG_TC = 8;                       // tiles per chunk
constexpr int WG_STAGE = 16 * WG_TC * 64;      // floats per dM (and per V) stage
constexpr size_t WG_LDS = 2 * 2 * WG_STAGE * sizeof(float);   // 128 KB

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f2v __attribute__((ext_vector_type(2)));

// one v_pk_add_f32 each (VOP3P: op_sel / op_sel_hi pick each source's half for
// the low / high result, neg_lo / neg_hi negate it; written as vector ops the
// compiler folded none of this and regrouped the pairs with v_mov), the same
// IEEE adds as the scalar forms.  Their results feed MFMAs a k-step later, and
// overwrite operands whose MFMAs issued at least two MFMAs earlier.
// (r.x + r.y, r.x - r.y)
__device__ __forceinline__ f2v wg_pm(f2v r) {
    f2v o;
    asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(o) : "v"(r));
    return o;
}
// (t0 - t2, t1 + t2) from t01, t23
__device__ __forceinline__ f2v wg_b01(f2v t01, f2v t23) {
    f2v o;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,0] neg_lo:[0,1]"
        : "=v"(o) : "v"(t01), "v"(t23));
    return o;
}
// (t2 - t1, t1 - t3) = (-t1 + t2, t1 + -t3)
__device__ __forceinline__ f2v wg_b23(f2v t01, f2v t23) {
    f2v o;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]"
        : "=v"(o) : "v"(t01), "v"(t23));
    return o;
}

struct WgGeom {
    int N, C, K, H, W, TW, Timg;
    int64_t T;
    int chunks_per_slice;
};

__global__ __launch_bounds__(WG_T, 1) void wino_wgrad_kernel(
    const float *__restrict__ x, const float *__restrict__ gy, float *__restrict__ part, WgGeom g) {
    extern __shared__ float4 wg_lds[];
    float4 *const Ms = wg_lds;                        // [2][p][h][k64]  (float4 = t4)
    float4 *const Vs = wg_lds + 2 * (WG_STAGE / 4);   // [2][p][h][c64]

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kb = blockIdx.x, cb = blockIdx.y, sl = blockIdx.z;
    const int64_t HW = (int64_t)g.H * g.W;
    const int64_t nchunks_all = (g.T + WG_TC - 1) / WG_TC;
    const int64_t ch0 = (int64_t)sl * g.chunks_per_slice;
    const int nchunk = (int)min((int64_t)g.chunks_per_slice, nchunks_all - ch0);
    const int kk = kb * 64 + lane, cc = cb * 64 + lane;    // this lane's channels

    float4 gr[2];       // gy rows 2ty, 2ty+1, cols 2tx0 .. 2tx0+3 (the wave's two tiles)
    float2 xr[4][4];    // x rows 2ty-1 .. 2ty+2, cols 2tx0-2 .. 2tx0+5 as four float2
    int ty = 0, tx0 = 0, tn = 0;
    bool tv = false;
    auto geom = [&](int64_t chunk) {
        const int64_t t = chunk * WG_TC + 2 * w;           // first of the wave's two tiles
        tv = t < g.T;
        tn = 0; ty = 0; tx0 = 0;
        if (tv) {
            tn = (int)(t / g.Timg);
            const int r = (int)(t - (int64_t)tn * g.Timg);
            ty = r / g.TW;
            tx0 = r - ty * g.TW;
        }
    };
    auto load = [&](int64_t chunk) {
        geom(chunk);
        const float *gp = gy + ((int64_t)tn * g.K + kk) * HW + (int64_t)(2 * ty) * g.W + 2 * tx0;
        gr[0] = *reinterpret_cast<const float4 *>(gp);
        gr[1] = *reinterpret_cast<const float4 *>(gp + g.W);
        const float *xp = x + ((int64_t)tn * g.C + cc) * HW;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int yy = min(max(2 * ty - 1 + i, 0), g.H - 1);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int xx = min(max(2 * tx0 - 2 + 2 * q, 0), g.W - 2);
                xr[i][q] = *reinterpret_cast<const float2 *>(xp + (int64_t)yy * g.W + xx);
            }
        }
    };
    auto store = [&](int buf) {
        float *M = reinterpret_cast<float *>(Ms + buf * (WG_STAGE / 4));
        float *V = reinterpret_cast<float *>(Vs + buf * (WG_STAGE / 4));
#pragma unroll
        for (int e = 0; e < 2; ++e) {                      // the wave's tiles 2w + e
            const int tl = 2 * w + e;                       // tile within the chunk
            const int h = tl >> 2, t4 = tl & 3;
            // dM = A dY A^T, A = [[1,0],[1,1],[1,-1],[0,-1]]
            const float d00 = tv ? (e ? gr[0].z : gr[0].x) : 0.f;
            const float d01 = tv ? (e ? gr[0].w : gr[0].y) : 0.f;
            const float d10 = tv ? (e ? gr[1].z : gr[1].x) : 0.f;
            const float d11 = tv ? (e ? gr[1].w : gr[1].y) : 0.f;
            const float r0[2] = {d00, d01}, r1[2] = {d00 + d10, d01 + d11};
            const float r2[2] = {d00 - d10, d01 - d11}, r3[2] = {-d10, -d11};
            const float *rr[4] = {r0, r1, r2, r3};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float a = rr[i][0], b = rr[i][1];
                const float m[4] = {a, a + b, a - b, -b};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    M[(((i * 4 + j) * 2 + h) * 64 + lane) * 4 + t4] = m[j];
            }
            // V = B^T d B of the x patch: rows 2ty-1+i, cols 2(tx0+e)-1+j
            float d[4][4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int yy = 2 * ty - 1 + i;
                const bool row = tv && yy >= 0 && yy < g.H;
                // cols 2tx0 - 2 .. 2tx0 + 5 held as xr[i][0..3]; tile e needs
                // 2tx0 + 2e - 1 .. 2tx0 + 2e + 2, i.e. offsets 2e + 1 .. 2e + 4
                float c8[8] = {xr[i][0].x, xr[i][0].y, xr[i][1].x, xr[i][1].y,
                               xr[i][2].x, xr[i][2].y, xr[i][3].x, xr[i][3].y};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int col = 2 * tx0 + 2 * e - 1 + j;
                    d[i][j] = (row && col >= 0 && col < g.W) ? c8[2 * e + 1 + j] : 0.f;
                }
            }
            float t[4][4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                t[0][j] = d[0][j] - d[2][j];
                t[1][j] = d[1][j] + d[2][j];
                t[2][j] = d[2][j] - d[1][j];
                t[3][j] = d[1][j] - d[3][j];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float v[4] = {t[i][0] - t[i][2], t[i][1] + t[i][2], t[i][2] - t[i][1],
                                    t[i][1] - t[i][3]};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    V[(((i * 4 + j) * 2 + h) * 64 + lane) * 4 + t4] = v[j];
            }
        }
    };

    f32x16 acc[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) acc[p] = f32x16{};

    const int ch = w & 1, kh = w >> 1, hl = lane >> 5, l32 = lane & 31;
    auto mfma_chunk = [&](int buf) {
        const float4 *M = Ms + buf * (WG_STAGE / 4);
        const float4 *V = Vs + buf * (WG_STAGE / 4);
#pragma unroll
        for (int p = 0; p < 16; ++p) {
            const float4 a = M[(p * 2 + hl) * 64 + kh * 32 + l32];
            const float4 b = V[(p * 2 + hl) * 64 + ch * 32 + l32];
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, acc[p], 0, 0, 0);
            acc[p] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, acc[p], 0, 0, 0);
        }
    };

    if (nchunk > 0) {
        load(ch0);
        store(0);
        __syncthreads();
        for (int c = 0; c + 1 < nchunk; ++c) {
            load(ch0 + c + 1);
            __builtin_amdgcn_sched_barrier(0);
            mfma_chunk(c & 1);
            __builtin_amdgcn_sched_barrier(0);
            store((c + 1) & 1);
            __syncthreads();
        }
        mfma_chunk((nchunk - 1) & 1);
    }

    // partial dU of this slice: part[sl][k][c][16], k rows (r & 3) + 8 (r >> 2) + 4 hl
    float *out = part + (int64_t)sl * g.K * g.C * 16;
    const int c = cb * 64 + ch * 32 + l32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int k = kb * 64 + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
        float4 *o = reinterpret_cast<float4 *>(out + ((int64_t)k * g.C + c) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            o[q] = make_float4(acc[4 * q][r], acc[4 * q + 1][r], acc[4 * q + 2][r],
                               acc[4 * q + 3][r]);
    }
}

// the first level of the slice reduction: out[g] = sum of slices g*G .. g*G+G-1
// in order, one thread per (group, float4 of dU): the many-slice layers (the
// 64-channel layer has 512) read their partials at the full width of the chip
__global__ void wino_wgrad_group_kernel(const float4 *__restrict__ part, int S, int G,
                                        int64_t nf4, int ngroups, float4 *__restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nf4 * ngroups) return;
    const int gi = (int)(idx / nf4);
    const int64_t f = idx - (int64_t)gi * nf4;
    const int s0 = gi * G, s1 = min(S, s0 + G);
    float4 a = part[(int64_t)s0 * nf4 + f];
    for (int s = s0 + 1; s < s1; ++s) {
        const float4 v = part[(int64_t)s * nf4 + f];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    out[idx] = a;
}

// dW[k][c] = G^T (sum over slices, in order, of dU) G, G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]]
__global__ void wino_wgrad_final_kernel(const float *__restrict__ part, int S, int K, int C,
                                        float *__restrict__ dw, int acc) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)K * C) return;
    float u[16];
    const float4 *p4 = reinterpret_cast<const float4 *>(part + idx * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float4 v = p4[q];
        u[4 * q] = v.x; u[4 * q + 1] = v.y; u[4 * q + 2] = v.z; u[4 * q + 3] = v.w;
    }
    const int64_t slab = (int64_t)K * C * 4;
    for (int s = 1; s < S; ++s) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 v = p4[s * slab + q];
            u[4 * q] += v.x; u[4 * q + 1] += v.y; u[4 * q + 2] += v.z; u[4 * q + 3] += v.w;
        }
    }
    // rows: t[a][j] = sum_i G[i][a] u[i][j]
    float t[3][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        t[0][j] = u[j] + 0.5f * (u[4 + j] + u[8 + j]);
        t[1][j] = 0.5f * (u[4 + j] - u[8 + j]);
        t[2][j] = 0.5f * (u[4 + j] + u[8 + j]) + u[12 + j];
    }
    float *o = dw + idx * 9;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float v0 = t[a][0] + 0.5f * (t[a][1] + t[a][2]);
        const float v1 = 0.5f * (t[a][1] - t[a][2]);
        const float v2 = 0.5f * (t[a][1] + t[a][2]) + t[a][3];
        o[a * 3 + 0] = acc ? o[a * 3 + 0] + v0 : v0;
        o[a * 3 + 1] = acc ? o[a * 3 + 1] + v1 : v1;
        o[a * 3 + 2] = acc ? o[a * 3 + 2] + v2 : v2;
    }
}


// ---------------------------------------------------------------------------
// r11 form: coalesced row loads staged through LDS, the transforms computed per
// lane straight into the MFMA operand registers (no transformed tiles in LDS),
// two waves per SIMD.
//
// A chunk is 16 tiles forming a rectangle of one image: RT = 16 / CT tile rows
// x CT tile columns (CT = 16 for tile rows of 16 or more tiles, else the whole
// row).  Its raw inputs -- gy rows 2ty0 .. 2ty0 + 2RT - 1 and x rows 2ty0 - 1 ..
// 2ty0 + 2RT, each 2CT columns wide (+ one halo column either side for x) --
// are buffer-loaded row by row (consecutive lanes along a row, float4; rows
// and halos outside the image read as zeros through the descriptor's range
// check) while the previous chunk's MFMAs run, then stored to the other LDS
// buffer.
//
// Block: 64 k x 64 c, 8 waves; wave w owns the (kh, ch) = ((w >> 1) & 1, w & 1)
// 32 x 32 quadrant for the 8 points of half ph = w >> 2 (rows i = 2 ph, 2 ph + 1
// of the 4 x 4 transform): 8 accumulators (128 AGPRs), so two waves share a
// SIMD and hide each other's LDS waits.  MFMA k-step s (2 tiles, tau = 2 s +
// lane / 32): lane (k or c = lane % 32, tau) reads its 2 x 2 gy tile and the 3 x
// 4 x rows its half needs from LDS (dword-pair reads; odd channel strides, so
// each 32-lane half hits 32 distinct banks), forms its half of dM = A dY A^T
// and V = B^T d B in registers and feeds them to its 8 point MFMAs as the A / B
// operands.  The next k-step's transform is sliced between this one's MFMAs;
// one barrier per chunk, before its last k-step.  Epilogue: the ph = 1 waves
// hand their accumulators to the ph = 0 waves through LDS, which apply G^T . G
// (the 16 points of one (k, c) are one lane's register r) and write the
// slice's partial dW [K][C][9]; smmd_wino3x3_wgrad adds the slices in order.
// ---------------------------------------------------------------------------
constexpr int WG2_T = 512;
constexpr int wg2_odd(int n) { return n | 1; }   // round up to odd

template <int CT>
struct Wg2 {
    static constexpr int RT = 16 / CT;               // tile rows per chunk
    static constexpr int XR = 2 * RT + 2;            // x rows staged
    static constexpr int XRS = 2 * CT + 6;           // x row stride (>= 2 CT + 4)
    static constexpr int XS = wg2_odd(XR * XRS);     // x channel stride (odd)
    static constexpr int GR = 2 * RT;                // gy rows
    static constexpr int GRS = 2 * CT + 2;           // gy row stride
    static constexpr int GS = wg2_odd(GR * GRS);     // gy channel stride (odd)
    static constexpr int STAGE = 64 * (XS + GS);     // floats per buffer
    static constexpr size_t LDS = 2 * STAGE * sizeof(float);
    static constexpr int XF4 = 64 * XR * (CT / 2);   // x float4 per chunk
    static constexpr int GF4 = 64 * GR * (CT / 2);   // gy float4 per chunk
    static constexpr int NX = (XF4 + WG2_T - 1) / WG2_T;
    static constexpr int NG = (GF4 + WG2_T - 1) / WG2_T;
    static constexpr int NH = 64 * XR * 2 / WG2_T;   // halo floats per thread (CT = 16)
};
static_assert(Wg2<16>::LDS <= 160 * 1024 && Wg2<4>::LDS <= 160 * 1024, "LDS budget");
static_assert(Wg2<16>::LDS >= 4 * 64 * 64 * sizeof(float), "epilogue hand-off fits");
static_assert(Wg2<16>::NH * WG2_T == 64 * Wg2<16>::XR * 2, "halo split");

// the body for the waves of transform half PH (rows 2 PH, 2 PH + 1 of the
// 4 x 4 transforms): a compile-time constant, so the half's picks cost no
// per-lane selects (every VALU instruction costs SIMD time beside the f32
// MFMA, profiles/r12/mfma_valu_coissue.txt)
template <int CT, int PH>
__device__ __forceinline__ void wgrad2_body(const float *__restrict__ x,
                                            const float *__restrict__ gy,
                                            float *__restrict__ part, const WgGeom &g) {
    using P = Wg2<CT>;
    extern __shared__ float4 wg2_lds4[];
    float *const lds = reinterpret_cast<float *>(wg2_lds4);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kb = blockIdx.x, cb = blockIdx.y, sl = blockIdx.z;
    const int64_t HW = (int64_t)g.H * g.W;
    const int64_t nchunks_all = g.T / 16;
    const int64_t ch0 = (int64_t)sl * g.chunks_per_slice;
    const int nchunk = (int)min((int64_t)g.chunks_per_slice, nchunks_all - ch0);
    const int cpi = g.Timg / 16;                      // chunks per image
    const int segs = g.TW / CT;                       // chunks across a tile row
    // CT == 16: halo columns loaded every chunk (zero at the image edges, so
    // a tile row of exactly 16 tiles stores zeros); CT < 16 covers whole
    // rows, whose halo columns are zero once for all
    constexpr bool halo = CT == 16;

    // Global reads are buffer loads: a row or halo column outside the image
    // gets an offset past the descriptor's range, which the hardware returns
    // as zeros, so no select waits on a load before the chunk's MFMAs.  A
    // thread whose index passes the chunk's count repeats the last element
    // (same value, same LDS slot): no branch.
    float4 xr[P::NX], gr[P::NG];
    float hr[P::NH > 0 ? P::NH : 1];
    constexpr uint32_t OOB = 0x80000000u;
    const uint32_t plane = (uint32_t)HW * 4u;
    auto gload = [&](int64_t chunk64) {
        // 32-bit (the chunk count is far below 2^31): the 64-bit division
        // was ~130 scalar instructions per chunk
        const uint32_t chunk = (uint32_t)chunk64;
        const int n = (int)(chunk / (uint32_t)cpi);
        const int q = (int)(chunk - (uint32_t)n * (uint32_t)cpi);
        const int ty0 = (q / segs) * P::RT, tx0 = (q % segs) * CT;
        const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(x + ((int64_t)n * g.C + cb * 64) * HW), 0, 64 * plane, 0x00020000);
        const __amdgpu_buffer_rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(gy + ((int64_t)n * g.K + kb * 64) * HW), 0, 64 * plane, 0x00020000);
#pragma unroll
        for (int i = 0; i < P::NX; ++i) {
            const int idx = min(i * WG2_T + tid, P::XF4 - 1);
            const int f = idx % (CT / 2), rc = idx / (CT / 2);
            const int r = rc % P::XR, c = rc / P::XR;
            const int yy = 2 * ty0 - 1 + r;
            const uint32_t off = (yy >= 0 && yy < g.H)
                                     ? c * plane + (uint32_t)(yy * g.W + 2 * tx0 + 4 * f) * 4u
                                     : OOB;
            xr[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xs, off, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < P::NG; ++i) {
            const int idx = min(i * WG2_T + tid, P::GF4 - 1);
            const int f = idx % (CT / 2), rk = idx / (CT / 2);
            const int r = rk % P::GR, k = rk / P::GR;
            const uint32_t off = k * plane + (uint32_t)((2 * ty0 + r) * g.W + 2 * tx0 + 4 * f) * 4u;
            gr[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(gs, off, 0, 0));
        }
        if (halo) {
#pragma unroll
            for (int i = 0; i < P::NH; ++i) {
                const int idx = i * WG2_T + tid;
                const int side = idx & 1, rc = idx >> 1;
                const int r = rc % P::XR, c = rc / P::XR;
                const int yy = 2 * ty0 - 1 + r;
                const int col = side ? 2 * tx0 + 2 * CT : 2 * tx0 - 1;
                const bool in = yy >= 0 && yy < g.H && (side ? tx0 + CT < g.TW : tx0 > 0);
                const uint32_t off = in ? c * plane + (uint32_t)(yy * g.W + col) * 4u : OOB;
                hr[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xs, off, 0, 0));
            }
        }
    };
    // x stage: X[c][r][j], j <-> column 2 tx0 - 2 + j; gy stage: Gd[k][r][col - 2 tx0]
    auto lstore = [&](int buf) {
        float *X = lds + buf * P::STAGE;
        float *Gd = X + 64 * P::XS;
#pragma unroll
        for (int i = 0; i < P::NX; ++i) {
            const int idx = min(i * WG2_T + tid, P::XF4 - 1);
            const int f = idx % (CT / 2), rc = idx / (CT / 2);
            const int r = rc % P::XR, c = rc / P::XR;
            float *d = X + c * P::XS + r * P::XRS + 2 + 4 * f;    // 4-byte aligned only
            d[0] = xr[i].x; d[1] = xr[i].y; d[2] = xr[i].z; d[3] = xr[i].w;
        }
#pragma unroll
        for (int i = 0; i < P::NG; ++i) {
            const int idx = min(i * WG2_T + tid, P::GF4 - 1);
            const int f = idx % (CT / 2), rk = idx / (CT / 2);
            const int r = rk % P::GR, k = rk / P::GR;
            float *d = Gd + k * P::GS + r * P::GRS + 4 * f;
            d[0] = gr[i].x; d[1] = gr[i].y; d[2] = gr[i].z; d[3] = gr[i].w;
        }
        if (halo) {
#pragma unroll
            for (int i = 0; i < P::NH; ++i) {
                const int idx = i * WG2_T + tid;
                const int side = idx & 1, rc = idx >> 1;
                const int r = rc % P::XR, c = rc / P::XR;
                X[c * P::XS + r * P::XRS + (side ? 2 * CT + 2 : 1)] = hr[i];
            }
        }
    };

    constexpr int ph = PH;
    const int kh = (w >> 1) & 1, ch = w & 1, hl = lane >> 5, l32 = lane & 31;
    // the lane's raw inputs of k-step s from buffer buf: x rows 2 ty + ph ..
    // 2 ty + ph + 2 of the 4 x 4 patch (channel c = ch 32 + l32) and the 2 x 2
    // gy tile (k = kh 32 + l32) of tile tau = 2 s + hl
    auto lds_read = [&](int buf, int s, float (&d)[12], float (&gv)[4]) {
        const float *X = lds + buf * P::STAGE;
        const float *Gd = X + 64 * P::XS;
        const int tau = 2 * s + hl;
        const int ty = tau / CT, tx = tau % CT;
        const float *xc = X + (ch * 32 + l32) * P::XS + (2 * ty + ph) * P::XRS + 2 * tx + 1;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) d[i * 4 + j] = xc[i * P::XRS + j];
        const float *gk = Gd + (kh * 32 + l32) * P::GS + (2 * ty) * P::GRS + 2 * tx;
        gv[0] = gk[0]; gv[1] = gk[1]; gv[2] = gk[P::GRS]; gv[3] = gk[P::GRS + 1];
    };
    // slice q of this wave's half of the transforms (after MFMA q of the
    // current k-step): a = rows 2 ph, 2 ph + 1 of dM' = A' dY A'^T, b = the
    // same rows of V = B^T d B (d = the patch rows ph .. ph + 2 read above).
    // A' = [[1,0],[1,1],[1,-1],[0,1]] is A = [[1,0],[1,1],[1,-1],[0,-1]] with
    // its last row negated, so dM'_ij = s_i s_j dM_ij (s_3 = -1, else 1) needs
    // no negations; the epilogue undoes the signs, bit for bit (negation is
    // exact and rounding symmetric)
    // Packed: the patch and gy rows arrive as column pairs (ds_read2_b32), so
    // each slice is v_pk_add_f32 on them (8 + 3 per k-step; scalar adds on
    // pairs the compiler regrouped cost ~9 v_mov per k-step besides)
    auto tslice = [&](int q, const float (&d)[12], const float (&gv)[4], f2v (&t)[4],
                      float (&a)[8], float (&b)[8]) {
#ifdef WG2_NO_XFORM       // timing-only diagnostic (wrong results): the LDS reads kept
        if (q == 0) {
#pragma unroll
            for (int i = 0; i < 12; ++i) asm volatile("" ::"v"(d[i]));
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(gv[i]));
        }
        return;
#endif
        if (q == 1) {
            // rows of A' dY: ph 0 (g01, g01 + g23), ph 1 (g01 - g23, g23); each
            // row R gives (R.x, R.x + R.y, R.x - R.y, R.y)
            const f2v g01 = {gv[0], gv[1]}, g23 = {gv[2], gv[3]};
            const f2v r0 = ph ? g01 - g23 : g01, r1 = ph ? g23 : g01 + g23;
            const f2v p0 = wg_pm(r0), p1 = wg_pm(r1);
            a[0] = r0.x; a[1] = p0.x; a[2] = p0.y; a[3] = r0.y;
            a[4] = r1.x; a[5] = p1.x; a[6] = p1.y; a[7] = r1.y;
        } else if (q == 2 || q == 3) {   // t row q - 2: rows (2 ph, 2 ph + 1) of B^T d
            // ph 0: rows 0, 1 = (d0 - d2, d1 + d2); ph 1: rows 2, 3 = (d2 - d1, d1 - d3)
            const int r = q - 2;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f2v e0 = {d[0 * 4 + 2 * h], d[0 * 4 + 2 * h + 1]};
                const f2v e1 = {d[1 * 4 + 2 * h], d[1 * 4 + 2 * h + 1]};
                const f2v e2 = {d[2 * 4 + 2 * h], d[2 * 4 + 2 * h + 1]};
                t[2 * r + h] = r == 0 ? (ph ? e1 - e0 : e0 - e2) : (ph ? e0 - e2 : e1 + e2);
            }
        } else if (q == 4 || q == 5) {   // row of V = t B: (t0 - t2, t1 + t2, t2 - t1, t1 - t3)
            const int i = q - 4;
            const f2v b01 = wg_b01(t[2 * i], t[2 * i + 1]), b23 = wg_b23(t[2 * i], t[2 * i + 1]);
            b[i * 4 + 0] = b01.x; b[i * 4 + 1] = b01.y;
            b[i * 4 + 2] = b23.x; b[i * 4 + 3] = b23.y;
        }
    };

    f32x16 acc[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = f32x16{};

    if (!halo) {      // whole rows: the halo columns are outside the image, zero once
        for (int i = tid; i < 2 * 64 * P::XR; i += WG2_T) {
            const int buf = i / (64 * P::XR), rc = i % (64 * P::XR);
            float *X = lds + buf * P::STAGE + (rc / P::XR) * P::XS + (rc % P::XR) * P::XRS;
            X[1] = 0.f;
            X[2 * CT + 2] = 0.f;
        }
    }
    if (nchunk > 0) {
        gload(ch0);
        lstore(0);
        __syncthreads();
        // the MFMA operands, double-buffered: k-step s reads set s & 1 and
        // forms the next k-step's into the other (a copy of the next set into
        // one fixed set cost ~80 v_mov per 64 MFMAs)
        float oa[2][8], ob[2][8];
        {
            float d[12], gv[4];
            f2v t[4];
            lds_read(0, 0, d, gv);
#pragma unroll
            for (int q = 0; q < 8; ++q) tslice(q, d, gv, t, oa[0], ob[0]);
        }
        for (int c = 0; c < nchunk; ++c) {
            const int buf = c & 1;
            // The schedule is pinned with sched_barrier: k-step s issues the
            // next k-step's LDS reads, then its 8 MFMAs, each followed by one
            // slice of the next transform.  The next chunk's global loads go
            // out at step 0, its LDS stores at step 5 (the other buffer), the
            // barrier before step 7's reads.  The last chunk loads, stores and
            // reads its own inputs once more (into the idle buffer, unused),
            // so the body has no branch.
            gload(ch0 + min(c + 1, nchunk - 1));
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int cur = s & 1, nxt = cur ^ 1;   // 8 k-steps: set 0 at every chunk start
                float d[12], gv[4];
                f2v t[4];
                if (s == 7) __syncthreads();             // every wave stored chunk c + 1
                __builtin_amdgcn_sched_barrier(0);
                lds_read(s < 7 ? buf : buf ^ 1, (s + 1) & 7, d, gv);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(oa[cur][q], ob[cur][q], acc[q],
                                                                  0, 0, 0);
                    tslice(q, d, gv, t, oa[nxt], ob[nxt]);
                    if (s == 5 && q == 0) lstore(buf ^ 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    }

    // the ph = 1 waves' points (i = 2, 3) to the ph = 0 waves, 8 registers r
    // at a time: E[wq][pl][rr][lane], wq = w & 3
    __syncthreads();
    float *out = part + (int64_t)sl * g.K * g.C * 9;
    const int c = cb * 64 + ch * 32 + l32;
    float *E = lds + (w & 3) * (8 * 8 * 64);
#pragma unroll
    for (int rh = 0; rh < 2; ++rh) {
        if (ph == 1) {
#pragma unroll
            for (int pl = 0; pl < 8; ++pl)
#pragma unroll
                for (int rr = 0; rr < 8; ++rr) E[(pl * 8 + rr) * 64 + lane] = acc[pl][rh * 8 + rr];
        }
        __syncthreads();
        if (ph == 0) {
            // dW partial of this slice: part[sl][k][c][9] = G^T dU G,
            // G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]]; k rows (r & 3) + 8 (r >> 2) + 4 hl
#pragma unroll
            for (int rr = 0; rr < 8; ++rr) {
                const int r = rh * 8 + rr;
                const int k = kb * 64 + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
                float u[16];
#pragma unroll
                for (int p = 0; p < 8; ++p) {
                    u[p] = acc[p][r];
                    u[8 + p] = E[(p * 8 + rr) * 64 + lane];
                }
                // u holds dU' (u'_ij = s_i s_j u_ij, s_3 = -1): with T = the
                // row pass on u', t[a][j] = T[a][j] for j < 3 and -T[a][j]
                // for j = 3, so each sign lands on a subtraction that equals
                // the original addition bit for bit
                float t[3][4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    t[0][j] = u[j] + 0.5f * (u[4 + j] + u[8 + j]);
                    t[1][j] = 0.5f * (u[4 + j] - u[8 + j]);
                    t[2][j] = 0.5f * (u[4 + j] + u[8 + j]) - u[12 + j];
                }
                float *o = out + ((int64_t)k * g.C + c) * 9;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    o[a * 3 + 0] = t[a][0] + 0.5f * (t[a][1] + t[a][2]);
                    o[a * 3 + 1] = 0.5f * (t[a][1] - t[a][2]);
                    o[a * 3 + 2] = 0.5f * (t[a][1] + t[a][2]) - t[a][3];
                }
            }
        }
        __syncthreads();
    }
}

template <int CT>
__global__ __launch_bounds__(WG2_T, 1) void wino_wgrad2_kernel(
    const float *__restrict__ x, const float *__restrict__ gy, float *__restrict__ part, WgGeom g) {
    // waves 4..7 are half 1 (a wave-uniform, scalar branch)
    if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 8))
        wgrad2_body<CT, 1>(x, gy, part, g);
    else
        wgrad2_body<CT, 0>(x, gy, part, g);
}

// out[i] = sum of the S slabs of n4 float4 each, in slab order (the last
// level of the r11 slice reduction, straight into dW)
// (acc: out += the sum, the later contribution of a weight used twice: the
// same add autograd would run, convops._late_gw)
__global__ void wino_wgrad_sum_kernel(const float4 *__restrict__ part, int S, int64_t n4,
                                      float4 *__restrict__ out, int acc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    float4 a = part[i];
    for (int s = 1; s < S; ++s) {
        const float4 v = part[(int64_t)s * n4 + i];
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (acc) {
        const float4 o = out[i];
        a = make_float4(o.x + a.x, o.y + a.y, o.z + a.z, o.w + a.w);
    }
    out[i] = a;
}

}  // namespace

static int wgrad_slices(int blocks, int64_t nchunks) {
    int64_t S = (256 + blocks - 1) / blocks;
    S = min(S, max((int64_t)1, nchunks / 8));      // at least 8 chunks per slice
    return (int)max((int64_t)1, S);
}

constexpr int WG_GROUP = 16;                       // slices per first-level group

static int wgrad_groups(int S) { return S > 2 * WG_GROUP ? (S + WG_GROUP - 1) / WG_GROUP : 0; }

// the r11 kernel's chunk shape for a tile-row width (0: not tiled by it)
static int wgrad2_ct(int h, int w_img) {
    const int TW = w_img / 2, TH = h / 2;
    if (h % 2 || w_img % 2) return 0;
    if (TW >= 16 && TW % 16 == 0) return 16;
    if (TW == 8 && TH % 2 == 0) return 8;
    if (TW == 4 && TH % 4 == 0) return 4;
    return 0;
}

// SMMD_WINO_WGRAD_V1=1: the first form (lane = channel loads) for every shape
static bool wgrad_v1_forced() {
    const char *e = getenv("SMMD_WINO_WGRAD_V1");
    return e && e[0] == '1';
}

static int wgrad2_slices(int blocks, int64_t nchunks) {
    int64_t S = (256 + blocks - 1) / blocks;
    S = min(S, max((int64_t)1, nchunks / 4));      // at least 4 chunks (64 tiles) per slice
    return (int)max((int64_t)1, S);
}

}  // namespace smmd

using namespace smmd;

extern "C" int smmd_wino3x3_wgrad_supported(int n, int ci, int co, int h, int w_img) {
    return n > 0 && ci > 0 && co > 0 && ci % 64 == 0 && co % 64 == 0 && h > 0 && w_img > 0 &&
           h % 2 == 0 && w_img % 4 == 0 && (int64_t)n * (ci + co) * h * w_img < (1ll << 40) &&
           (int64_t)h * w_img < (1ll << 23);   // a 64-channel range of one image under 2 GiB
}

static size_t wgrad_v1_ws(int n, int ci, int co, int h, int w_img) {
    const int64_t T = (int64_t)n * (h / 2) * (w_img / 2);
    const int S = wgrad_slices((co / 64) * (ci / 64), (T + WG_TC - 1) / WG_TC);
    return (size_t)(S + wgrad_groups(S)) * co * ci * 16 * sizeof(float);
}

static size_t wgrad_v2_ws(int n, int ci, int co, int h, int w_img) {
    const int64_t T = (int64_t)n * (h / 2) * (w_img / 2);
    const int S = wgrad2_slices((co / 64) * (ci / 64), T / 16);
    return (size_t)(S + wgrad_groups(S)) * co * ci * 9 * sizeof(float);
}

extern "C" size_t smmd_wino3x3_wgrad_workspace_bytes(int n, int ci, int co, int h, int w_img) {
    if (!smmd_wino3x3_wgrad_supported(n, ci, co, h, w_img)) return 0;
    // either form may run (SMMD_WINO_WGRAD_V1 is read per call)
    const size_t a = wgrad_v1_ws(n, ci, co, h, w_img);
    const size_t b = wgrad2_ct(h, w_img) ? wgrad_v2_ws(n, ci, co, h, w_img) : 0;
    return a > b ? a : b;
}

template <int CT>
static smmd_status wgrad2_launch(const float *x, const float *gy, float *part, const WgGeom &g,
                                 int S, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(wino_wgrad2_kernel<CT>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)Wg2<CT>::LDS) != hipSuccess)
            return SMMD_EHIP;
        attr = true;
    }
    wino_wgrad2_kernel<CT><<<dim3((unsigned)(g.K / 64), (unsigned)(g.C / 64), (unsigned)S),
                             dim3(WG2_T), Wg2<CT>::LDS, st>>>(x, gy, part, g);
    return last_launch_status();
}

// gw [co, ci, 3, 3] = the weight gradient of conv(x [n, ci, h, w], W, stride 1,
// pad 1) at upstream gy [n, co, h, w]
static smmd_status wgrad3_launch(const float *x, const float *gy, float *gw, int n, int ci,
                                 int co, int h, int w_img, void *ws, size_t ws_bytes, int acc,
                                 smmd_stream_t stream) {
    if (n < 0 || ci <= 0 || co <= 0 || h < 0 || w_img < 0 || !gw) return SMMD_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n == 0 || h == 0 || w_img == 0)
        return acc ? SMMD_OK
                   : hip_status(hipMemsetAsync(gw, 0, (size_t)co * ci * 9 * sizeof(float), st));
    if (!x || !gy) return SMMD_EINVAL;
    if (!smmd_wino3x3_wgrad_supported(n, ci, co, h, w_img)) return SMMD_EUNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gy)) & 15) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_wino3x3_wgrad_workspace_bytes(n, ci, co, h, w_img))
        return SMMD_EWORKSPACE;
    if (reinterpret_cast<uintptr_t>(ws) & 15) return SMMD_EINVAL;
    WgGeom g;
    g.N = n; g.C = ci; g.K = co; g.H = h; g.W = w_img;
    g.TW = w_img / 2;
    g.Timg = (h / 2) * g.TW;
    g.T = (int64_t)n * g.Timg;
    const int blocks = (co / 64) * (ci / 64);
    const int64_t nkc = (int64_t)co * ci;
    float *part = static_cast<float *>(ws);
    smmd_status e;
    const int ct = wgrad_v1_forced() ? 0 : wgrad2_ct(h, w_img);
    if (ct) {
        const int64_t nchunks = g.T / 16;
        const int S = wgrad2_slices(blocks, nchunks);
        g.chunks_per_slice = (int)((nchunks + S - 1) / S);
        const int Sused = (int)((nchunks + g.chunks_per_slice - 1) / g.chunks_per_slice);
        e = ct == 16 ? wgrad2_launch<16>(x, gy, part, g, Sused, st)
            : ct == 8 ? wgrad2_launch<8>(x, gy, part, g, Sused, st)
                      : wgrad2_launch<4>(x, gy, part, g, Sused, st);
        if (e != SMMD_OK) return e;
        const int64_t nf4 = nkc * 9 / 4;
        const int ng = wgrad_groups(Sused);
        int Sfin = Sused;
        if (ng > 0) {                              // two levels: groups of WG_GROUP slices, in order
            float *grp = part + (size_t)S * nkc * 9;
            const int64_t nt = nf4 * ng;
            wino_wgrad_group_kernel<<<dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st>>>(
                reinterpret_cast<const float4 *>(part), Sused, WG_GROUP, nf4, ng,
                reinterpret_cast<float4 *>(grp));
            e = last_launch_status();
            if (e != SMMD_OK) return e;
            part = grp;
            Sfin = ng;
        }
        wino_wgrad_sum_kernel<<<dim3((unsigned)((nf4 + 255) / 256)), dim3(256), 0, st>>>(
            reinterpret_cast<const float4 *>(part), Sfin, nf4, reinterpret_cast<float4 *>(gw),
            acc);
        return last_launch_status();
    }
    const int64_t nchunks = (g.T + WG_TC - 1) / WG_TC;
    const int S = wgrad_slices(blocks, nchunks);
    g.chunks_per_slice = (int)((nchunks + S - 1) / S);
    const int Sused = (int)((nchunks + g.chunks_per_slice - 1) / g.chunks_per_slice);
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(wino_wgrad_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)WG_LDS) != hipSuccess)
            return SMMD_EHIP;
        attr = true;
    }
    wino_wgrad_kernel<<<dim3((unsigned)(co / 64), (unsigned)(ci / 64), (unsigned)Sused), dim3(WG_T),
                        WG_LDS, st>>>(x, gy, part, g);
    e = last_launch_status();
    if (e != SMMD_OK) return e;
    const int ng = wgrad_groups(Sused);
    if (ng > 0) {                                  // two-level: groups of WG_GROUP slices, in order
        float *grp = part + (size_t)S * co * ci * 16;
        const int64_t nf4 = nkc * 4, nt = nf4 * ng;
        wino_wgrad_group_kernel<<<dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st>>>(
            reinterpret_cast<const float4 *>(part), Sused, WG_GROUP, nf4, ng,
            reinterpret_cast<float4 *>(grp));
        e = last_launch_status();
        if (e != SMMD_OK) return e;
        part = grp;
    }
    wino_wgrad_final_kernel<<<dim3((unsigned)((nkc + 255) / 256)), dim3(256), 0, st>>>(
        part, ng > 0 ? ng : Sused, co, ci, gw, acc);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino3x3_wgrad(const float *x, const float *gy, float *gw, int n,
                                          int ci, int co, int h, int w_img, void *ws,
                                          size_t ws_bytes, smmd_stream_t stream) {
    return wgrad3_launch(x, gy, gw, n, ci, co, h, w_img, ws, ws_bytes, 0, stream);
}

extern "C" smmd_status smmd_wino3x3_wgrad_acc(const float *x, const float *gy, float *gw, int n,
                                              int ci, int co, int h, int w_img, void *ws,
                                              size_t ws_bytes, smmd_stream_t stream) {
    return wgrad3_launch(x, gy, gw, n, ci, co, h, w_img, ws, ws_bytes, 1, stream);
}
