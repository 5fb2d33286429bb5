// smmd_wino_s2_wgrad.hip -- the weight gradient of the 4x4 stride-2 pad-1
// convolution (the critic's folded ConvMeanPool layers, gan/core/resnet/
// block.py:63-66 as one strided conv; with the roles of x and gy swapped, the
// generator's folded UpsampleConv, block.py:53-60) as polyphase Winograd
// F(2x2, 2x2) on the f32 MFMA: TF's Conv2DBackpropFilter of those layers
// (snops.py:69-90), 1.78x fewer multiplies than the direct weight gradient.
//
// The forward kernel (smmd_wino_s2.hip) computes, per 2 x 2 output tile t and
// x phase (pi, pj), y_t = A^T (sum_{c, phase} U_p V_p) A with
//   V = B^T d B,  B^T = [[1,-1,0],[0,1,0],[0,-1,1]],  d[a][b] = x[4ty-1+pi+2a][4tx-1+pj+2b]
//   U = G g G^T,  G   = [[1,0],[1,1],[0,1]],          g[a][b] = W'[k][c][2a+pi][2b+pj]
//   y = A^T M A,  A^T = [[1,1,0],[0,1,1]].
// Its adjoint in U: dU_p[k][c'] = sum_t dM_p[k][t] V_p[c'][t] with dM = A dY A^T
// (c' = (c, phase): 4 C reduction columns), then dg = G^T dU G is the phase's
// 2 x 2 tap block of dW'.
//
// Block: 64 k x 16 c (64 phase columns c' = 4 c + 2 pi + pj), 8 waves: wave w
// owns the (kh, ch) = ((w >> 1) & 1, w & 1) 32 x 32 quadrant for all 9 points
// (9 accumulators, 144 VGPRs) and the k-steps of parity tp = w >> 2, so two
// waves share a SIMD.  A chunk is 16 output tiles of whole tile rows (one or
// more images); its x rows (with one zero column either side) and gy rows are
// buffer-loaded row by row (consecutive lanes along a row; rows outside the
// image read as zeros through the descriptor's range check), stored to the
// other LDS buffer mid-chunk.  k-step s = 2 tiles (tau = 2s + lane / 32):
// lane (k or c' = lane % 32, tau) reads its 2 x 2 gy tile and its phase's 3 x 3
// patch (stride 2 in x) from LDS and forms dM and V in registers, sliced
// between the previous k-step's MFMAs.  Epilogue: the tp = 1 waves hand their
// accumulators to the tp = 0 waves through LDS, which apply G^T . G and write
// the slice's partial dW' [K][C][16]; the slices are added in order.
#include "smmd_common.hpp"

namespace smmd {

namespace {

constexpr int W2_T = 512;
typedef float f32x16 __attribute__((ext_vector_type(16)));

// chunk geometry: CT tile columns (= the whole tile row), RT tile rows per
// image, NI images; CT * RT * NI = 16 tiles
template <int CT, int RT>
struct S2w {
    static constexpr int NI = 16 / (CT * RT);
    static constexpr int TPI = CT * RT;                  // tiles per image in the chunk
    static constexpr int XR = 4 * RT + 2;                // x rows per image (4 ty0 - 1 ..)
    static constexpr int XRS = 4 * CT + 2;               // x row stride: = 2 mod 4
    static constexpr int XS = ((NI * XR * XRS + 3) & ~7) + 4;   // channel stride: = 4 mod 8
    static constexpr int GRS = 2 * CT;                   // gy row stride
    static constexpr int GS = (NI * 2 * RT * 2 * CT) | 1;       // gy channel stride (odd)
    static constexpr int STAGE = 16 * XS + 64 * GS;
    static constexpr size_t LDS = 2 * STAGE * sizeof(float);
    static constexpr int XF4 = 16 * NI * XR * CT;        // x float4 per chunk (4 CT cols a row)
    static constexpr int GF4 = 64 * NI * (TPI);          // gy float4 per chunk (4 TPI floats)
    static constexpr int NX = (XF4 + W2_T - 1) / W2_T;
    static constexpr int NG = (GF4 + W2_T - 1) / W2_T;
    static_assert(CT * RT * NI == 16, "16 tiles per chunk");
    static_assert(XS >= NI * XR * XRS && XS % 8 == 4, "x channel stride");
    static_assert(XRS % 4 == 2, "x row stride");
    static_assert(LDS >= 4 * 9 * 8 * 64 * sizeof(float), "epilogue hand-off fits");
    static_assert(LDS <= 160 * 1024, "LDS budget");
};

struct S2wGeom {
    int N, C, K, H, W;          // x [N, C, H, W], gy [N, K, H/2, W/2]
    int TH, TW, Timg;           // output tiles
    int64_t T;
    int chunks_per_slice;
};

template <int CT, int RT>
__global__ __launch_bounds__(W2_T, 1) void s2_wgrad_kernel(
    const float *__restrict__ x, const float *__restrict__ gy, float *__restrict__ part,
    S2wGeom g) {
    using P = S2w<CT, RT>;
    extern __shared__ float4 s2w_lds4[];
    float *const lds = reinterpret_cast<float *>(s2w_lds4);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int kb = blockIdx.x, cb = blockIdx.y, sl = blockIdx.z;
    const int HW = g.H * g.W, Ho = g.H / 2, Wo = g.W / 2, HWo = Ho * Wo;
    const int64_t nchunks_all = g.T / 16;
    const int64_t ch0 = (int64_t)sl * g.chunks_per_slice;
    const int nchunk = (int)min((int64_t)g.chunks_per_slice, nchunks_all - ch0);
    const int cpi = g.Timg >= 16 ? g.Timg / 16 : 1;     // chunks per image (NI == 1)

    // buffer loads: rows outside the image read as zeros (offset past the range)
    float4 xr[P::NX], gr[P::NG];
    constexpr uint32_t OOB = 0x80000000u;
    auto gload = [&](int64_t chunk) {
        int n0, ty0;
        if (P::NI > 1) {
            n0 = (int)(chunk * P::NI);
            ty0 = 0;
        } else {                  // 32-bit: a 64-bit division is ~130 scalar instructions
            const uint32_t ch32 = (uint32_t)chunk;
            n0 = (int)(ch32 / (uint32_t)cpi);
            ty0 = (int)(ch32 - (uint32_t)n0 * (uint32_t)cpi) * RT;
        }
        const uint32_t xrange = (uint32_t)(((P::NI - 1) * g.C + 16) * HW) * 4u;
        const uint32_t grange = (uint32_t)(((P::NI - 1) * g.K + 64) * HWo) * 4u;
        const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(x + ((int64_t)n0 * g.C + cb * 16) * HW), 0, xrange, 0x00020000);
        const __amdgpu_buffer_rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(gy + ((int64_t)n0 * g.K + kb * 64) * HWo), 0, grange, 0x00020000);
#pragma unroll
        for (int i = 0; i < P::NX; ++i) {
            const int idx = min(i * W2_T + tid, P::XF4 - 1);
            const int f = idx % CT, rr = idx / CT;
            const int r = rr % P::XR, ci = rr / P::XR;
            const int c = ci % 16, img = ci / 16;
            const int yy = 4 * ty0 - 1 + r;
            const uint32_t off = (yy >= 0 && yy < g.H)
                                     ? (uint32_t)((img * g.C + c) * HW + yy * g.W + 4 * f) * 4u
                                     : OOB;
            xr[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xs, off, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < P::NG; ++i) {
            const int idx = min(i * W2_T + tid, P::GF4 - 1);
            const int f = idx % P::TPI, ki = idx / P::TPI;
            const int k = ki % 64, img = ki / 64;
            const uint32_t off =
                (uint32_t)((img * g.K + k) * HWo + (2 * ty0) * Wo + 4 * f) * 4u;
            gr[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(gs, off, 0, 0));
        }
    };
    // x stage X[c][img][r][j] (j <-> image column j - 1); gy stage Gd[k][img][row][col]
    auto lstore = [&](int buf) {
        float *X = lds + buf * P::STAGE;
        float *Gd = X + 16 * P::XS;
#pragma unroll
        for (int i = 0; i < P::NX; ++i) {
            const int idx = min(i * W2_T + tid, P::XF4 - 1);
            const int f = idx % CT, rr = idx / CT;
            const int r = rr % P::XR, ci = rr / P::XR;
            const int c = ci % 16, img = ci / 16;
            float *d = X + c * P::XS + (img * P::XR + r) * P::XRS + 1 + 4 * f;
            d[0] = xr[i].x; d[1] = xr[i].y; d[2] = xr[i].z; d[3] = xr[i].w;
        }
#pragma unroll
        for (int i = 0; i < P::NG; ++i) {
            const int idx = min(i * W2_T + tid, P::GF4 - 1);
            const int f = idx % P::TPI, ki = idx / P::TPI;
            const int k = ki % 64, img = ki / 64;
            float *d = Gd + k * P::GS + img * (4 * P::TPI) + 4 * f;
            d[0] = gr[i].x; d[1] = gr[i].y; d[2] = gr[i].z; d[3] = gr[i].w;
        }
    };

    const int tp = w >> 2, kh = (w >> 1) & 1, ch = w & 1, hl = lane >> 5, l32 = lane & 31;
    const int cp = ch * 32 + l32;                      // this lane's phase column
    const int cl = cp >> 2, pi = (cp >> 1) & 1, pj = cp & 1;
    // the lane's raw inputs of k-step s: the phase's 3 x 3 patch (stride 2)
    // and the 2 x 2 gy tile of tile tau = 2 s + hl
    auto lds_read = [&](int buf, int s, float (&d)[9], float (&gv)[4]) {
        const float *X = lds + buf * P::STAGE;
        const float *Gd = X + 16 * P::XS;
        const int tau = 2 * s + hl;
        const int img = tau / P::TPI, loc = tau % P::TPI;
        const int ty = loc / CT, tx = loc % CT;
        const float *xc = X + cl * P::XS + (img * P::XR + 4 * ty + pi) * P::XRS + 4 * tx + pj;
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) d[a * 3 + b] = xc[(2 * a) * P::XRS + 2 * b];
        const float *gk = Gd + (kh * 32 + l32) * P::GS + img * (4 * P::TPI) + (2 * ty) * P::GRS +
                          2 * tx;
        gv[0] = gk[0]; gv[1] = gk[1]; gv[2] = gk[P::GRS]; gv[3] = gk[P::GRS + 1];
    };
    // slice q (after MFMA q): a = dM = A dY A^T, b = V = B^T d B
    auto tslice = [&](int q, const float (&d)[9], const float (&gv)[4], float (&t)[9],
                      float (&a)[9], float (&b)[9]) {
        if (q == 1) {
            // rows of A dY: (y0, y0 + y1, y1); then columns the same way
            const float r0[2] = {gv[0], gv[1]};
            const float r1[2] = {gv[0] + gv[2], gv[1] + gv[3]};
            const float r2[2] = {gv[2], gv[3]};
            a[0] = r0[0]; a[1] = r0[0] + r0[1]; a[2] = r0[1];
            a[3] = r1[0]; a[4] = r1[0] + r1[1]; a[5] = r1[1];
            a[6] = r2[0]; a[7] = r2[0] + r2[1]; a[8] = r2[1];
        } else if (q == 2) {             // t = B^T d: rows (d0 - d1, d1, d2 - d1)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                t[j] = d[j] - d[3 + j];
                t[3 + j] = d[3 + j];
                t[6 + j] = d[6 + j] - d[3 + j];
            }
        } else if (q == 3) {             // V = t B: columns (t0 - t1, t1, t2 - t1)
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                b[i * 3 + 0] = t[i * 3 + 0] - t[i * 3 + 1];
                b[i * 3 + 1] = t[i * 3 + 1];
                b[i * 3 + 2] = t[i * 3 + 2] - t[i * 3 + 1];
            }
        }
    };

    f32x16 acc[9];
#pragma unroll
    for (int p = 0; p < 9; ++p) acc[p] = f32x16{};

    // the zero columns either side of every x row, both buffers
    for (int i = tid; i < 2 * 16 * P::NI * P::XR; i += W2_T) {
        const int buf = i / (16 * P::NI * P::XR), rc = i % (16 * P::NI * P::XR);
        const int c = rc / (P::NI * P::XR), row = rc % (P::NI * P::XR);
        float *X = lds + buf * P::STAGE + c * P::XS + row * P::XRS;
        X[0] = 0.f;
        X[4 * CT + 1] = 0.f;
    }
    if (nchunk > 0) {
        gload(ch0);
        lstore(0);
        __syncthreads();
        // the MFMA operands, double-buffered: k-step m reads set m & 1 and
        // forms the next k-step's into the other (no copy into a fixed set)
        float oa[2][9], ob[2][9];
        {
            float d[9], gv[4], t[9];
            lds_read(0, tp, d, gv);
#pragma unroll
            for (int q = 0; q < 9; ++q) tslice(q, d, gv, t, oa[0], ob[0]);
        }
        for (int c = 0; c < nchunk; ++c) {
            const int buf = c & 1;
            // this wave's k-steps s = 2 m + tp, m = 0..3; the next chunk's
            // loads at m = 0, its LDS stores and the barrier before m = 3's
            // reads (which fetch the next chunk's first k-step)
            gload(ch0 + min(c + 1, nchunk - 1));
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int cur = m & 1, nxt = cur ^ 1;   // 4 k-steps: set 0 at every chunk start
                float d[9], gv[4], t[9];
                if (m == 3) {
                    lstore(buf ^ 1);
                    __syncthreads();                 // every wave stored chunk c + 1
                }
                __builtin_amdgcn_sched_barrier(0);
                lds_read(m < 3 ? buf : buf ^ 1, m < 3 ? 2 * (m + 1) + tp : tp, d, gv);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(oa[cur][q], ob[cur][q], acc[q],
                                                                  0, 0, 0);
                    tslice(q, d, gv, t, oa[nxt], ob[nxt]);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    }

    // tp = 1 hands its accumulators to tp = 0: E[wq][p][rr][lane], 8 registers r
    // at a time (72 KB)
    __syncthreads();
    float *out = part + (int64_t)sl * g.K * g.C * 16;
    const int c = cb * 16 + cl;
    float *E = lds + (w & 3) * (9 * 8 * 64);
#pragma unroll
    for (int rh = 0; rh < 2; ++rh) {
        if (tp == 1) {
#pragma unroll
            for (int p = 0; p < 9; ++p)
#pragma unroll
                for (int rr = 0; rr < 8; ++rr) E[(p * 8 + rr) * 64 + lane] = acc[p][rh * 8 + rr];
        }
        __syncthreads();
        if (tp == 0) {
#pragma unroll
            for (int rr = 0; rr < 8; ++rr) {
                const int r = rh * 8 + rr;
                const int k = kb * 64 + kh * 32 + (r & 3) + 8 * (r >> 2) + 4 * hl;
                float u[9];
#pragma unroll
                for (int p = 0; p < 9; ++p) u[p] = acc[p][r] + E[(p * 8 + rr) * 64 + lane];
                // dg = G^T dU G, G = [[1,0],[1,1],[0,1]]
                float tt[2][3];
#pragma unroll
                for (int j = 0; j < 3; ++j) {
                    tt[0][j] = u[j] + u[3 + j];
                    tt[1][j] = u[3 + j] + u[6 + j];
                }
                float *o = out + ((int64_t)k * g.C + c) * 16;
#pragma unroll
                for (int a = 0; a < 2; ++a) {
                    o[(2 * a + pi) * 4 + pj] = tt[a][0] + tt[a][1];
                    o[(2 * a + pi) * 4 + 2 + pj] = tt[a][1] + tt[a][2];
                }
            }
        }
        __syncthreads();
    }
}

// out[i] = sum of the S slabs of n4 float4 each, in slab order
// (acc: out += the sum, a weight's later gradient contribution)
__global__ void s2w_sum_kernel(const float4 *__restrict__ part, int S, int64_t n4,
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

// the first level for many slices: out[g] = slices g G .. g G + G - 1, in order
__global__ void s2w_group_kernel(const float4 *__restrict__ part, int S, int G, int64_t nf4,
                                 int ngroups, float4 *__restrict__ out) {
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

constexpr int S2W_GROUP = 16;
int s2w_groups(int S) { return S > 2 * S2W_GROUP ? (S + S2W_GROUP - 1) / S2W_GROUP : 0; }

// (CT, RT) of the chunk for output tile grid TH x TW (0: not tiled)
int s2w_shape(int TH, int TW, int *rt) {
    if (TW == 16) { *rt = 1; return 16; }
    if (TW == 8 && TH % 2 == 0) { *rt = 2; return 8; }
    if (TW == 4 && TH % 4 == 0) { *rt = 4; return 4; }
    if (TW == 2 && TH == 2) { *rt = 2; return 2; }
    return 0;
}

int s2w_slices(int blocks, int64_t nchunks) {
    int64_t S = (256 + blocks - 1) / blocks;
    S = min(S, max((int64_t)1, nchunks / 4));      // at least 4 chunks (64 tiles) per slice
    return (int)max((int64_t)1, S);
}

template <int CT, int RT>
smmd_status s2w_launch(const float *x, const float *gy, float *part, const S2wGeom &g, int S,
                       hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(s2_wgrad_kernel<CT, RT>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)S2w<CT, RT>::LDS) != hipSuccess)
            return SMMD_EHIP;
        attr = true;
    }
    s2_wgrad_kernel<CT, RT><<<dim3((unsigned)(g.K / 64), (unsigned)(g.C / 16), (unsigned)S),
                              dim3(W2_T), S2w<CT, RT>::LDS, st>>>(x, gy, part, g);
    return last_launch_status();
}

}  // namespace

}  // namespace smmd

using namespace smmd;

extern "C" int smmd_wino4x4s2_wgrad_supported(int n, int ci, int co, int h, int w_img) {
    int rt = 0;
    return n > 0 && ci > 0 && co > 0 && ci % 16 == 0 && co % 64 == 0 && h > 0 && w_img > 0 &&
           h % 4 == 0 && w_img % 4 == 0 && s2w_shape(h / 4, w_img / 4, &rt) != 0 &&
           (int64_t)n * (h / 4) * (w_img / 4) % 16 == 0 &&
           (int64_t)4 * ci * h * w_img * 4 < (1ll << 31) &&
           (int64_t)4 * co * h * w_img < (1ll << 31) && (int64_t)n * (ci + co) * h * w_img < (1ll << 40);
}

extern "C" size_t smmd_wino4x4s2_wgrad_workspace_bytes(int n, int ci, int co, int h, int w_img) {
    if (!smmd_wino4x4s2_wgrad_supported(n, ci, co, h, w_img)) return 0;
    const int64_t T = (int64_t)n * (h / 4) * (w_img / 4);
    const int S = s2w_slices((co / 64) * (ci / 16), T / 16);
    return (size_t)(S + s2w_groups(S)) * co * ci * 16 * sizeof(float);
}

// gw [co, ci, 4, 4] = the weight gradient of conv(x [n, ci, h, w], W', stride 2,
// pad 1) at upstream gy [n, co, h/2, w/2]
static smmd_status s2w_launch_all(const float *x, const float *gy, float *gw, int n, int ci,
                                  int co, int h, int w_img, void *ws, size_t ws_bytes, int acc,
                                  smmd_stream_t stream) {
    if (n < 0 || ci <= 0 || co <= 0 || h < 0 || w_img < 0 || !gw) return SMMD_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (n == 0 || h == 0 || w_img == 0)
        return acc ? SMMD_OK
                   : hip_status(hipMemsetAsync(gw, 0, (size_t)co * ci * 16 * sizeof(float), st));
    if (!x || !gy) return SMMD_EINVAL;
    if (!smmd_wino4x4s2_wgrad_supported(n, ci, co, h, w_img)) return SMMD_EUNSUPPORTED;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(gy) |
         reinterpret_cast<uintptr_t>(gw)) & 15)
        return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_wino4x4s2_wgrad_workspace_bytes(n, ci, co, h, w_img))
        return SMMD_EWORKSPACE;
    if (reinterpret_cast<uintptr_t>(ws) & 15) return SMMD_EINVAL;
    S2wGeom g;
    g.N = n; g.C = ci; g.K = co; g.H = h; g.W = w_img;
    g.TH = h / 4; g.TW = w_img / 4;
    g.Timg = g.TH * g.TW;
    g.T = (int64_t)n * g.Timg;
    int rt = 0;
    const int ct = s2w_shape(g.TH, g.TW, &rt);
    const int blocks = (co / 64) * (ci / 16);
    const int64_t nchunks = g.T / 16;
    const int S = s2w_slices(blocks, nchunks);
    g.chunks_per_slice = (int)((nchunks + S - 1) / S);
    const int Sused = (int)((nchunks + g.chunks_per_slice - 1) / g.chunks_per_slice);
    float *part = static_cast<float *>(ws);
    smmd_status e = ct == 16 ? s2w_launch<16, 1>(x, gy, part, g, Sused, st)
                    : ct == 8 ? s2w_launch<8, 2>(x, gy, part, g, Sused, st)
                    : ct == 4 ? s2w_launch<4, 4>(x, gy, part, g, Sused, st)
                              : s2w_launch<2, 2>(x, gy, part, g, Sused, st);
    if (e != SMMD_OK) return e;
    const int64_t nf4 = (int64_t)co * ci * 4;
    const int ng = s2w_groups(Sused);
    int Sfin = Sused;
    if (ng > 0) {
        float *grp = part + (size_t)S * co * ci * 16;
        const int64_t nt = nf4 * ng;
        s2w_group_kernel<<<dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st>>>(
            reinterpret_cast<const float4 *>(part), Sused, S2W_GROUP, nf4, ng,
            reinterpret_cast<float4 *>(grp));
        e = last_launch_status();
        if (e != SMMD_OK) return e;
        part = grp;
        Sfin = ng;
    }
    s2w_sum_kernel<<<dim3((unsigned)((nf4 + 255) / 256)), dim3(256), 0, st>>>(
        reinterpret_cast<const float4 *>(part), Sfin, nf4, reinterpret_cast<float4 *>(gw), acc);
    return last_launch_status();
}

extern "C" smmd_status smmd_wino4x4s2_wgrad(const float *x, const float *gy, float *gw, int n,
                                            int ci, int co, int h, int w_img, void *ws,
                                            size_t ws_bytes, smmd_stream_t stream) {
    return s2w_launch_all(x, gy, gw, n, ci, co, h, w_img, ws, ws_bytes, 0, stream);
}

extern "C" smmd_status smmd_wino4x4s2_wgrad_acc(const float *x, const float *gy, float *gw,
                                                int n, int ci, int co, int h, int w_img,
                                                void *ws, size_t ws_bytes,
                                                smmd_stream_t stream) {
    return s2w_launch_all(x, gy, gw, n, ci, co, h, w_img, ws, ws_bytes, 1, stream);
}
