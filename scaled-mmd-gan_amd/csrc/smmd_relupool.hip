// smmd_relupool.hip -- the two consumers of a critic down-block's input, fused
// (gfx950 / MI355X): the main path's ReLU and the shortcut's 2x2 mean pool
// read the block input once, and their backward is one pass.
//
// Reference: gan/core/resnet/block.py:44 (tf.nn.relu of the block input, bn
// off in the critic: mode ''), :69-71 (MeanPoolConv: add_n of the four strided
// slices / 4, then the 1x1 conv), :50 (shortcut + output, so the input's
// gradient is the sum of the two paths' gradients).
//
//   mask_pool     (x; m) -> (x [m > 0], pool(x))        forward, m = x: (relu, pool)
//   mask_pool_adj (a, b; m) -> a [m > 0] + up(b) / 4    its adjoint (the backward)
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

__device__ __forceinline__ float msel(float m, float x) { return m > 0.f ? x : 0.f; }

__global__ __launch_bounds__(RP_T) void mask_pool_kernel(const float *__restrict__ x,
                                                         const float *__restrict__ m,
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
    const float4 x0 = *reinterpret_cast<const float4 *>(x + o0);
    const float4 x1 = *reinterpret_cast<const float4 *>(x + o0 + W);
    if (out_m) {
        float4 m0 = x0, m1 = x1;
        if (m != x) {
            m0 = *reinterpret_cast<const float4 *>(m + o0);
            m1 = *reinterpret_cast<const float4 *>(m + o0 + W);
        }
        *reinterpret_cast<float4 *>(out_m + o0) =
            make_float4(msel(m0.x, x0.x), msel(m0.y, x0.y), msel(m0.z, x0.z), msel(m0.w, x0.w));
        *reinterpret_cast<float4 *>(out_m + o0 + W) =
            make_float4(msel(m1.x, x1.x), msel(m1.y, x1.y), msel(m1.z, x1.z), msel(m1.w, x1.w));
    }
    if (out_p) {
#pragma clang fp contract(off)
        const float p0 = (((x0.x + x0.y) + x1.x) + x1.y) / 4.f;   // block.py:71 mean
        const float p1 = (((x0.z + x0.w) + x1.z) + x1.w) / 4.f;
        const size_t op = ((size_t)plane * hh + i) * (W >> 1) + 2 * j;
        *reinterpret_cast<float2 *>(out_p + op) = make_float2(p0, p1);
    }
}

__global__ __launch_bounds__(RP_T) void mask_pool_adj_kernel(const float *__restrict__ a,
                                                             const float *__restrict__ b,
                                                             const float *__restrict__ m,
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
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    if (a) {
        const float4 a0 = *reinterpret_cast<const float4 *>(a + o0);
        const float4 a1 = *reinterpret_cast<const float4 *>(a + o0 + W);
        const float4 m0 = *reinterpret_cast<const float4 *>(m + o0);
        const float4 m1 = *reinterpret_cast<const float4 *>(m + o0 + W);
        s0 = make_float4(msel(m0.x, a0.x), msel(m0.y, a0.y), msel(m0.z, a0.z), msel(m0.w, a0.w));
        s1 = make_float4(msel(m1.x, a1.x), msel(m1.y, a1.y), msel(m1.z, a1.z), msel(m1.w, a1.w));
    }
    if (b) {
        const size_t op = ((size_t)plane * hh + i) * (W >> 1) + 2 * j;
        const float2 bb = *reinterpret_cast<const float2 *>(b + op);
        const float q0 = bb.x * 0.25f, q1 = bb.y * 0.25f;   // up(b / 4): block.py:71 adjoint
        if (a) {
            s0.x += q0; s0.y += q0; s0.z += q1; s0.w += q1;
            s1.x += q0; s1.y += q0; s1.z += q1; s1.w += q1;
        } else {
            s0 = make_float4(q0, q0, q1, q1);
            s1 = s0;
        }
    }
    *reinterpret_cast<float4 *>(out + o0) = s0;
    *reinterpret_cast<float4 *>(out + o0 + W) = s1;
}

static bool rp_shape_ok(int64_t planes, int H, int W) {
    return planes >= 0 && H > 0 && W > 0 && (H % 2) == 0 && (W % 4) == 0;
}

static bool al16(const void *p) { return p == nullptr || ((uintptr_t)p & 15) == 0; }
static bool al8(const void *p) { return p == nullptr || ((uintptr_t)p & 7) == 0; }

}  // namespace smmd

using namespace smmd;

extern "C" smmd_status smmd_mask_pool2(const float *x, const float *m, int64_t planes, int H,
                                       int W, float *out_masked, float *out_pool,
                                       smmd_stream_t stream) {
    if (!rp_shape_ok(planes, H, W) || !x || (out_masked && !m) || (!out_masked && !out_pool))
        return SMMD_EINVAL;
    if (!al16(x) || !al16(m) || !al16(out_masked) || !al8(out_pool)) return SMMD_EINVAL;
    const int64_t patches = planes * (H / 2) * (W / 4);
    if (patches == 0) return SMMD_OK;
    const int64_t blocks = (patches + RP_T - 1) / RP_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipLaunchKernelGGL(mask_pool_kernel, dim3((unsigned)blocks), dim3(RP_T), 0,
                       (hipStream_t)stream, x, m, patches, H, W, out_masked, out_pool);
    return last_launch_status();
}

extern "C" smmd_status smmd_mask_pool2_adj(const float *a, const float *b, const float *m,
                                           int64_t planes, int H, int W, float *out,
                                           smmd_stream_t stream) {
    if (!rp_shape_ok(planes, H, W) || !out || (!a && !b) || (a && !m)) return SMMD_EINVAL;
    if (!al16(a) || !al16(m) || !al16(out) || !al8(b)) return SMMD_EINVAL;
    const int64_t patches = planes * (H / 2) * (W / 4);
    if (patches == 0) return SMMD_OK;
    const int64_t blocks = (patches + RP_T - 1) / RP_T;
    if (blocks > 0x7fffffff) return SMMD_EINVAL;
    hipLaunchKernelGGL(mask_pool_adj_kernel, dim3((unsigned)blocks), dim3(RP_T), 0,
                       (hipStream_t)stream, a, b, m, patches, H, W, out);
    return last_launch_status();
}
