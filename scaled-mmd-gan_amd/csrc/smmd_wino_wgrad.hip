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
                                        float *__restrict__ dw) {
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
        o[a * 3 + 0] = t[a][0] + 0.5f * (t[a][1] + t[a][2]);
        o[a * 3 + 1] = 0.5f * (t[a][1] - t[a][2]);
        o[a * 3 + 2] = 0.5f * (t[a][1] + t[a][2]) + t[a][3];
    }
}

}  // namespace

static int wgrad_slices(int blocks, int64_t nchunks) {
    int64_t S = (256 + blocks - 1) / blocks;
    S = min(S, max((int64_t)1, nchunks / 8));      // at least 8 chunks per slice
    return (int)max((int64_t)1, S);
}

constexpr int WG_GROUP = 16;                       // slices per first-level group

static int wgrad_groups(int S) { return S > 2 * WG_GROUP ? (S + WG_GROUP - 1) / WG_GROUP : 0; }

}  // namespace smmd

using namespace smmd;

extern "C" int smmd_wino3x3_wgrad_supported(int n, int ci, int co, int h, int w_img) {
    return n > 0 && ci > 0 && co > 0 && ci % 64 == 0 && co % 64 == 0 && h > 0 && w_img > 0 &&
           h % 2 == 0 && w_img % 4 == 0 && (int64_t)n * (ci + co) * h * w_img < (1ll << 40);
}

extern "C" size_t smmd_wino3x3_wgrad_workspace_bytes(int n, int ci, int co, int h, int w_img) {
    if (!smmd_wino3x3_wgrad_supported(n, ci, co, h, w_img)) return 0;
    const int64_t T = (int64_t)n * (h / 2) * (w_img / 2);
    const int S = wgrad_slices((co / 64) * (ci / 64), (T + WG_TC - 1) / WG_TC);
    return (size_t)(S + wgrad_groups(S)) * co * ci * 16 * sizeof(float);
}

// gw [co, ci, 3, 3] = the weight gradient of conv(x [n, ci, h, w], W, stride 1,
// pad 1) at upstream gy [n, co, h, w]
extern "C" smmd_status smmd_wino3x3_wgrad(const float *x, const float *gy, float *gw, int n,
                                          int ci, int co, int h, int w_img, void *ws,
                                          size_t ws_bytes, smmd_stream_t stream) {
    if (n < 0 || ci <= 0 || co <= 0 || h < 0 || w_img < 0 || !gw) return SMMD_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n == 0 || h == 0 || w_img == 0)
        return hip_status(hipMemsetAsync(gw, 0, (size_t)co * ci * 9 * sizeof(float), st));
    if (!x || !gy) return SMMD_EINVAL;
    if (!smmd_wino3x3_wgrad_supported(n, ci, co, h, w_img)) return SMMD_EUNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gy)) & 15) return SMMD_EINVAL;
    WgGeom g;
    g.N = n; g.C = ci; g.K = co; g.H = h; g.W = w_img;
    g.TW = w_img / 2;
    g.Timg = (h / 2) * g.TW;
    g.T = (int64_t)n * g.Timg;
    const int64_t nchunks = (g.T + WG_TC - 1) / WG_TC;
    const int blocks = (co / 64) * (ci / 64);
    const int S = wgrad_slices(blocks, nchunks);
    g.chunks_per_slice = (int)((nchunks + S - 1) / S);
    const int Sused = (int)((nchunks + g.chunks_per_slice - 1) / g.chunks_per_slice);
    if (!ws || ws_bytes < (size_t)(S + wgrad_groups(S)) * co * ci * 16 * sizeof(float))
        return SMMD_EWORKSPACE;
    if (reinterpret_cast<uintptr_t>(ws) & 15) return SMMD_EINVAL;
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(wino_wgrad_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)WG_LDS) != hipSuccess)
            return SMMD_EHIP;
        attr = true;
    }
    float *part = static_cast<float *>(ws);
    wino_wgrad_kernel<<<dim3((unsigned)(co / 64), (unsigned)(ci / 64), (unsigned)Sused), dim3(WG_T),
                        WG_LDS, st>>>(x, gy, part, g);
    smmd_status e = last_launch_status();
    if (e != SMMD_OK) return e;
    const int64_t nkc = (int64_t)co * ci;
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
        part, ng > 0 ? ng : Sused, co, ci, gw);
    return last_launch_status();
}
