// smmd_bias.hip -- bias gradient of a convolution: db[c] = sum_{n, h, w} gy[n, c, h, w]
// (gfx950 / MI355X).
//
// Reference: the TF autodiff of tf.nn.bias_add in snops.conv2d / resnet
// Conv2D (gan/core/snops.py:89-90, gan/core/resnet/ops/conv2d.py:37-39), i.e.
// BiasAddGrad over NHWC; here over the NCHW tensor the MIOpen convolutions use.
// An HBM stream: every element of gy read once (4 B), 4 B written per channel.
//
// Stage 1: block (c, s) sums its contiguous chunk of rows n of channel c (each
// row is HW contiguous floats, float4 loads when HW % 4 == 0 and the base is
// 16-B aligned) into one float,
// fixed order (per-thread sums, then the fixed wave/block tree).  Rows shorter
// than the block are packed several per step so every lane loads.
// Stage 2: one thread per channel adds its S partials in order.  S is chosen
// so stage 1 has >= 2048 blocks (8 per CU) whenever N allows; from 512
// channels on S = 1 and stage 1 writes the result (one launch).
#include "smmd_common.hpp"

namespace smmd {

constexpr int CS_T = 256;

__global__ __launch_bounds__(CS_T) void chan_sum_partial_kernel(const float *__restrict__ gy,
                                                                int N, int C, int HW, int S,
                                                                int vec, float *__restrict__ part) {
    const int c = blockIdx.x, s = blockIdx.y;
    const int R = (N + S - 1) / S;                      // rows n in [n0, n1) of this block
    const int n0 = s * R, n1 = min(N, n0 + R);
    float acc = 0.f;
    const bool v4 = vec != 0;                           // HW % 4 == 0 and gy 16-B aligned
    const int w = v4 ? (HW >> 2) : HW;                  // row width in load units
    if (w >= CS_T) {
        for (int n = n0; n < n1; ++n) {
            const float *row = gy + ((size_t)n * C + c) * HW;
            if (v4) {
                const float4 *r4 = reinterpret_cast<const float4 *>(row);
                for (int i = threadIdx.x; i < w; i += CS_T) {
                    const float4 x = r4[i];
                    acc += (x.x + x.y) + (x.z + x.w);
                }
            } else {
                for (int i = threadIdx.x; i < w; i += CS_T) acc += row[i];
            }
        }
    } else {
        // short rows: the block covers rpi rows per step, thread t owns
        // column t % w of row t / w, so every lane loads
        const int rpi = CS_T / w;
        const int r = threadIdx.x / w, col = threadIdx.x - r * w;
        if (r < rpi) {
            for (int n = n0 + r; n < n1; n += rpi) {
                const float *row = gy + ((size_t)n * C + c) * HW;
                if (v4) {
                    const float4 x = reinterpret_cast<const float4 *>(row)[col];
                    acc += (x.x + x.y) + (x.z + x.w);
                } else {
                    acc += row[col];
                }
            }
        }
    }
    __shared__ float red[CS_T / SMMD_WAVE];
    acc = block_sum<CS_T / SMMD_WAVE>(acc, red);
    if (threadIdx.x == 0) part[(size_t)s * C + c] = acc;     // [S][C]: coalesced final
}

__global__ __launch_bounds__(256) void chan_sum_final_kernel(const float *__restrict__ part,
                                                             int C, int S,
                                                             float *__restrict__ out) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    // partials of channel c at stride C: a wave's loads of one s are one
    // coalesced run, and the unrolled loads are all in flight before the adds
    const float *p = part + c;
    float acc = 0.f;
    int s = 0;
    for (; s + 8 <= S; s += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[(size_t)(s + k) * C];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k];
    }
    for (; s < S; ++s) acc += p[(size_t)s * C];
    out[c] = acc;
}

inline int chan_sum_split(int N, int C) {
    if (C >= 512) return 1;        // >= 2 blocks per CU already: one launch, no partials
    int S = (2048 + C - 1) / C;
    if (S > N) S = N;
    if (S < 1) S = 1;
    return S;
}

}  // namespace smmd

using namespace smmd;

extern "C" size_t smmd_channel_sum_workspace_bytes(int N, int C) {
    if (N <= 0 || C <= 0) return 0;
    return (size_t)C * chan_sum_split(N, C) * sizeof(float);
}

extern "C" smmd_status smmd_channel_sum(const float *gy, int N, int C, int HW, float *out,
                                        void *ws, size_t ws_bytes, smmd_stream_t stream) {
    if (N < 0 || C < 0 || HW < 0) return SMMD_EINVAL;
    if (C == 0) return SMMD_OK;
    if (!out) return SMMD_EINVAL;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (N == 0 || HW == 0) {
        if (hipMemsetAsync(out, 0, (size_t)C * sizeof(float), st) != hipSuccess) return SMMD_EHIP;
        return SMMD_OK;
    }
    if (!gy) return SMMD_EINVAL;
    // float4 rows need HW % 4 == 0 and a 16-B aligned base (a contiguous view
    // with a storage offset may not be): otherwise the scalar-load path
    const int vec = ((HW & 3) == 0 && (reinterpret_cast<uintptr_t>(gy) & 15) == 0) ? 1 : 0;
    const int S = chan_sum_split(N, C);
    if (!ws || ws_bytes < (size_t)C * S * sizeof(float)) return SMMD_EWORKSPACE;
    if (S > 65535) return SMMD_EINVAL;
    if (S == 1) {                  // each block owns a whole channel: write the result
        chan_sum_partial_kernel<<<dim3(C, 1), dim3(CS_T), 0, st>>>(gy, N, C, HW, 1, vec, out);
        return last_launch_status();
    }
    float *part = static_cast<float *>(ws);
    chan_sum_partial_kernel<<<dim3(C, S), dim3(CS_T), 0, st>>>(gy, N, C, HW, S, vec, part);
    smmd_status e = last_launch_status();
    if (e != SMMD_OK) return e;
    chan_sum_final_kernel<<<dim3((C + 255) / 256), dim3(256), 0, st>>>(part, C, S, out);
    return last_launch_status();
}
