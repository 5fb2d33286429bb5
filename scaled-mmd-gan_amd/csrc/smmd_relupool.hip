// smmd_relupool.hip -- the two consumers of a critic down-block's input, fused
// (gfx950 / MI355X): the main path's ReLU and the shortcut's 2x2 mean pool
// read the block input once, and their backward is one pass.
//
// Reference: gan/core/resnet/block.py:44 (tf.nn.relu of the block input, bn
// off in the critic: mode ''), :69-71 (MeanPoolConv: add_n of the four strided
// slices / 4, then the 1x1 conv), :50 (shortcut + output, so the input's
// gradient is the sum of the two paths' gradients).
//
//   mask_pool     (u; m) -> (u s_m(m), pool(u s_p(m)))     u = (x + bx) (+ (y + by))
//   mask_pool_adj (a, b; m) -> a s_m(m) + s_p(m) up(b) / 4  its adjoint (the backward)
// with s(m) = 1 where m > 0, else the slope (s_m: 0, the ReLU; s_p: 1, or the
// leaky ReLU's 0.2 when the block input is lrelu of the first conv's output,
// architecture.py:393 -- then relu(lrelu(h)) = relu(h) and the block's input
// is never written).  y: the previous block's two paths, added here instead
// of in a separate pass (block.py:50 feeding the next block); bx, by: their
// convolutions' per-channel biases (snops.py:89-90), added here too.
//
// Each is linear in its first arguments with m a constant, and each is the
// other's backward, so every order of the double backward is these two
// kernels.  The arithmetic is that of the torch ops they replace, in their
// order: threshold_backward's select, avg_pool2d's ((x00 + x01) + x10) + x11
// then / 4, and the one add of the two path gradients (commutative), so the
// results are bit-identical to relu + avg_pool2d and to their backward.
//
// HBM-bound elementwise work: a thread owns a 2-row x 4-column patch of one
// [H, W] plane (two float4 per input row pair, one float2 of the pooled side).
#include "smmd_common.hpp"

namespace smmd {

constexpr int RP_T = 256;

// x s(m): x where m > 0, else x * slope (0 for the ReLU; 1: x unchanged)
__device__ __forceinline__ float msel(float m, float x, float slope) {
    return m > 0.f ? x : (slope == 0.f ? 0.f : (slope == 1.f ? x : x * slope));
}

__device__ __forceinline__ float4 msel4(float4 m, float4 x, float slope) {
    return make_float4(msel(m.x, x.x, slope), msel(m.y, x.y, slope), msel(m.z, x.z, slope),
                       msel(m.w, x.w, slope));
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ float4 addb(float4 a, float b) {
    return make_float4(a.x + b, a.y + b, a.z + b, a.w + b);
}

__global__ __launch_bounds__(RP_T) void mask_pool_kernel(const float *__restrict__ x,
                                                         const float *__restrict__ y,
                                                         const float *__restrict__ bx,
                                                         const float *__restrict__ by, int C,
                                                         const float *__restrict__ m,
                                                         float slope_m, float slope_p,
                                                         int64_t patches, int H, int W,
                                                         float *__restrict__ out_m,
                                                         float *__restrict__ out_p) {
    const int64_t t = (int64_t)blockIdx.x * RP_T + threadIdx.x;
    if (t >= patches) return;
    const int wq = W >> 2, hh = H >> 1;
    const int j = (int)(t % wq);
    const int64_t r = t / wq;                 // plane * hh + i
    const int i = (int)(r % hh);
    const int64_t plane = r / hh;
    const size_t o0 = ((size_t)plane * H + 2 * i) * W + 4 * j;
    float4 x0 = *reinterpret_cast<const float4 *>(x + o0);
    float4 x1 = *reinterpret_cast<const float4 *>(x + o0 + W);
    const int c = (bx || by) ? (int)(plane % C) : 0;
    if (bx) {                                 // conv output + its bias
        const float b = bx[c];
        x0 = addb(x0, b);
        x1 = addb(x1, b);
    }
    if (y) {                                  // the residual sum, x + y
        float4 y0 = *reinterpret_cast<const float4 *>(y + o0);
        float4 y1 = *reinterpret_cast<const float4 *>(y + o0 + W);
        if (by) {
            const float b = by[c];
            y0 = addb(y0, b);
            y1 = addb(y1, b);
        }
        x0 = add4(x0, y0);
        x1 = add4(x1, y1);
    }
    float4 m0 = x0, m1 = x1;                  // m NULL: the mask is the input itself
    if (m) {
        m0 = *reinterpret_cast<const float4 *>(m + o0);
        m1 = *reinterpret_cast<const float4 *>(m + o0 + W);
    }
    if (out_m) {
        *reinterpret_cast<float4 *>(out_m + o0) = msel4(m0, x0, slope_m);
        *reinterpret_cast<float4 *>(out_m + o0 + W) = msel4(m1, x1, slope_m);
    }
    if (out_p) {
#pragma clang fp contract(off)
        const float4 q0 = msel4(m0, x0, slope_p), q1 = msel4(m1, x1, slope_p);
        const float p0 = (((q0.x + q0.y) + q1.x) + q1.y) / 4.f;   // block.py:71 mean
        const float p1 = (((q0.z + q0.w) + q1.z) + q1.w) / 4.f;
        const size_t op = ((size_t)plane * hh + i) * (W >> 1) + 2 * j;
        *reinterpret_cast<float2 *>(out_p + op) = make_float2(p0, p1);
    }
}

__global__ __launch_bounds__(RP_T) void mask_pool_adj_kernel(const float *__restrict__ a,
                                                             const float *__restrict__ b,
                                                             const float *__restrict__ m,
                                                             float slope_m, float slope_p,
                                                             int64_t patches, int H, int W,
                                                             float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * RP_T + threadIdx.x;
    if (t >= patches) return;
    const int wq = W >> 2, hh = H >> 1;
    const int j = (int)(t % wq);
    const int64_t r = t / wq;
    const int i = (int)(r % hh);
    const int64_t plane = r / hh;
    const size_t o0 = ((size_t)plane * H + 2 * i) * W + 4 * j;
    const float4 m0 = *reinterpret_cast<const float4 *>(m + o0);
    const float4 m1 = *reinterpret_cast<const float4 *>(m + o0 + W);
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    if (a) {
        s0 = msel4(m0, *reinterpret_cast<const float4 *>(a + o0), slope_m);
        s1 = msel4(m1, *reinterpret_cast<const float4 *>(a + o0 + W), slope_m);
    }
    if (b) {
        const size_t op = ((size_t)plane * hh + i) * (W >> 1) + 2 * j;
        const float2 bb = *reinterpret_cast<const float2 *>(b + op);
        const float q0 = bb.x * 0.25f, q1 = bb.y * 0.25f;   // up(b / 4): block.py:71 adjoint
        const float4 u0 = msel4(m0, make_float4(q0, q0, q1, q1), slope_p);
        const float4 u1 = msel4(m1, make_float4(q0, q0, q1, q1), slope_p);
        s0 = a ? add4(s0, u0) : u0;
        s1 = a ? add4(s1, u1) : u1;
    }
    *reinterpret_cast<float4 *>(out + o0) = s0;
    *reinterpret_cast<float4 *>(out + o0 + W) = s1;
}

// a generator up block's output (block.py:50 with the UpsampleConv shortcut,
// block.py:53-60, whose 1x1 conv runs before the nearest upsample):
// out = up(s + bs) + (h + bh), s at half resolution.  The unfused ops' order:
// bias adds, the upsample copy, then the one add.
__global__ __launch_bounds__(RP_T) void up_add_kernel(const float *__restrict__ s,
                                                      const float *__restrict__ bs,
                                                      const float *__restrict__ h,
                                                      const float *__restrict__ bh, int C,
                                                      int64_t patches, int H, int W,
                                                      float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * RP_T + threadIdx.x;
    if (t >= patches) return;
    const int wq = W >> 2, hh = H >> 1;
    const int j = (int)(t % wq);
    const int64_t r = t / wq;
    const int i = (int)(r % hh);
    const int64_t plane = r / hh;
    const int c = (int)(plane % C);
    const size_t o0 = ((size_t)plane * H + 2 * i) * W + 4 * j;
    const size_t op = ((size_t)plane * hh + i) * (W >> 1) + 2 * j;
    float2 ss = *reinterpret_cast<const float2 *>(s + op);
    if (bs) {
        const float b = bs[c];
        ss.x += b;
        ss.y += b;
    }
    float4 h0 = *reinterpret_cast<const float4 *>(h + o0);
    float4 h1 = *reinterpret_cast<const float4 *>(h + o0 + W);
    if (bh) {
        const float b = bh[c];
        h0 = addb(h0, b);
        h1 = addb(h1, b);
    }
    const float4 u = make_float4(ss.x, ss.x, ss.y, ss.y);
    *reinterpret_cast<float4 *>(out + o0) = add4(u, h0);
    *reinterpret_cast<float4 *>(out + o0 + W) = add4(u, h1);
}

// The critic's tail (architecture.py:430-433, _forward_chained): y[r] =
// sum_i lrelu(a[r][i] + b[r][i]) over the hw pixels of each (n, c) row, and in
// mask mode (mu set) the adjoint of the backward below: y[r] = sum_i (a + b)
// * s(mu + mv) with s(h) = 1 for h > 0 else slope (leaky_relu_backward's
// select).  One thread per row, float4 loads, the row summed in pixel order.
__global__ __launch_bounds__(RP_T) void row_lrelu_sum_kernel(
    const float *__restrict__ a, const float *__restrict__ b, const float *__restrict__ mu,
    const float *__restrict__ mv, float *__restrict__ y, int64_t rows, int hw, float slope) {
    const int64_t r = (int64_t)blockIdx.x * RP_T + threadIdx.x;
    if (r >= rows) return;
    const size_t o = (size_t)r * hw;
    float acc = 0.f;
    for (int i = 0; i < hw; i += 4) {
        float4 t = *reinterpret_cast<const float4 *>(a + o + i);
        if (b) t = add4(t, *reinterpret_cast<const float4 *>(b + o + i));
        float tv[4] = {t.x, t.y, t.z, t.w};
        if (mu) {
            float4 h = *reinterpret_cast<const float4 *>(mu + o + i);
            if (mv) h = add4(h, *reinterpret_cast<const float4 *>(mv + o + i));
            const float hv[4] = {h.x, h.y, h.z, h.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += hv[j] > 0.f ? tv[j] : tv[j] * slope;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) acc += tv[j] > 0.f ? tv[j] : tv[j] * slope;
        }
    }
    y[r] = acc;
}

// the tail's backward: out[r][i] = g[r] * s(mu + mv) (the row sum's broadcast,
// then leaky_relu_backward: h > 0 ? g : g * slope, bit-identical to them)
__global__ __launch_bounds__(RP_T) void row_lrelu_bcast_kernel(
    const float *__restrict__ g, const float *__restrict__ mu, const float *__restrict__ mv,
    float *__restrict__ out, int64_t rows, int hw, float slope) {
    const int64_t r = (int64_t)blockIdx.x * RP_T + threadIdx.x;
    if (r >= rows) return;
    const size_t o = (size_t)r * hw;
    const float gv = g[r], gs = gv * slope;
    for (int i = 0; i < hw; i += 4) {
        float4 h = *reinterpret_cast<const float4 *>(mu + o + i);
        if (mv) h = add4(h, *reinterpret_cast<const float4 *>(mv + o + i));
        *reinterpret_cast<float4 *>(out + o + i) =
            make_float4(h.x > 0.f ? gv : gs, h.y > 0.f ? gv : gs, h.z > 0.f ? gv : gs,
                        h.w > 0.f ? gv : gs);
    }
}

static bool rp_shape_ok(int64_t planes, int H, int W) {
    return planes >= 0 && H > 0 && W > 0 && (H % 2) == 0 && (W % 4) == 0;
}

static bool al16(const void *p) { return p == nullptr || ((uintptr_t)p & 15) == 0; }
static bool al8(const void *p) { return p == nullptr || ((uintptr_t)p & 7) == 0; }

}  // namespace smmd

using namespace smmd;

extern "C" smmd_status smmd_mask_pool2(const float *x, const float *y, const float *bx,
                                       const float *by, int C, const float *m, float slope_m,
                                       float slope_p, int64_t planes, int H, int W,
                                       float *out_masked, float *out_pool,
                                       smmd_stream_t stream) {
    if (!rp_shape_ok(planes, H, W) || !x || (!out_masked && !out_pool)) return SMMD_EINVAL;
    if ((by && !y) || ((bx || by) && (C < 1 || planes % C != 0))) return SMMD_EINVAL;
    if (!al16(x) || !al16(y) || !al16(m) || !al16(out_masked) || !al8(out_pool)) return SMMD_EINVAL;
    const int64_t patches = planes * (H / 2) * (W / 4);
    if (patches == 0) return SMMD_OK;
    const int64_t blocks = (patches + RP_T - 1) / RP_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipLaunchKernelGGL(mask_pool_kernel, dim3((unsigned)blocks), dim3(RP_T), 0,
                       (hipStream_t)stream, x, y, bx, by, C, m, slope_m, slope_p, patches, H, W,
                       out_masked, out_pool);
    return last_launch_status();
}

extern "C" smmd_status smmd_mask_pool2_adj(const float *a, const float *b, const float *m,
                                           float slope_m, float slope_p, int64_t planes, int H,
                                           int W, float *out, smmd_stream_t stream) {
    if (!rp_shape_ok(planes, H, W) || !out || !m || (!a && !b)) return SMMD_EINVAL;
    if (!al16(a) || !al16(m) || !al16(out) || !al8(b)) return SMMD_EINVAL;
    const int64_t patches = planes * (H / 2) * (W / 4);
    if (patches == 0) return SMMD_OK;
    const int64_t blocks = (patches + RP_T - 1) / RP_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipLaunchKernelGGL(mask_pool_adj_kernel, dim3((unsigned)blocks), dim3(RP_T), 0,
                       (hipStream_t)stream, a, b, m, slope_m, slope_p, patches, H, W, out);
    return last_launch_status();
}

extern "C" smmd_status smmd_up_add(const float *s, const float *bs, const float *h,
                                   const float *bh, int C, int64_t planes, int H, int W,
                                   float *out, smmd_stream_t stream) {
    if (!rp_shape_ok(planes, H, W) || !s || !h || !out || C < 1 || planes % C != 0)
        return SMMD_EINVAL;
    if (!al8(s) || !al16(h) || !al16(out)) return SMMD_EINVAL;
    const int64_t patches = planes * (H / 2) * (W / 4);
    if (patches == 0) return SMMD_OK;
    const int64_t blocks = (patches + RP_T - 1) / RP_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipLaunchKernelGGL(up_add_kernel, dim3((unsigned)blocks), dim3(RP_T), 0, (hipStream_t)stream,
                       s, bs, h, bh, C, patches, H, W, out);
    return last_launch_status();
}

extern "C" smmd_status smmd_row_lrelu_sum(const float *a, const float *b, const float *mu,
                                          const float *mv, float *y, int64_t rows, int hw,
                                          float slope, smmd_stream_t stream) {
    if (!a || !y || rows < 0 || hw <= 0 || hw % 4 != 0 || (mv && !mu)) return SMMD_EINVAL;
    if (!al16(a) || !al16(b) || !al16(mu) || !al16(mv)) return SMMD_EINVAL;
    if (rows == 0) return SMMD_OK;
    const int64_t blocks = (rows + RP_T - 1) / RP_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipLaunchKernelGGL(row_lrelu_sum_kernel, dim3((unsigned)blocks), dim3(RP_T), 0,
                       (hipStream_t)stream, a, b, mu, mv, y, rows, hw, slope);
    return last_launch_status();
}

extern "C" smmd_status smmd_row_lrelu_bcast(const float *g, const float *mu, const float *mv,
                                            float *out, int64_t rows, int hw, float slope,
                                            smmd_stream_t stream) {
    if (!g || !mu || !out || rows < 0 || hw <= 0 || hw % 4 != 0) return SMMD_EINVAL;
    if (!al16(mu) || !al16(mv) || !al16(out)) return SMMD_EINVAL;
    if (rows == 0) return SMMD_OK;
    const int64_t blocks = (rows + RP_T - 1) / RP_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipLaunchKernelGGL(row_lrelu_bcast_kernel, dim3((unsigned)blocks), dim3(RP_T), 0,
                       (hipStream_t)stream, g, mu, mv, out, rows, hw, slope);
    return last_launch_status();
}
