// smmd_bnrelu.hip -- training-mode batch norm + ReLU of the generator
// (gfx950 / MI355X): the forward, with or without the record its backward
// needs, and that backward (the generator step).
//
// Reference: tf.layers.batch_normalization(training=True, momentum=0.9,
// epsilon=1e-5) then tf.nn.relu (gan/core/snops.py:31-40 batch_norm,
// resnet/ops/batchnorm.py:10-18, resnet/block.py:42-47 Normalize + relu,
// architecture.py:178-208 bn4 + relu): y = relu((x - mean) / sqrt(var + eps)
// * gamma + beta) with the batch's per-channel mean and biased variance over
// (N, H, W), the moving averages updated with the unbiased variance (torch's
// BatchNorm2d convention, momentum 0.1 = TF's 0.9 decay).
//
// Two launches over [N, C, HW] NCHW fp32, the grid (C, S) of the channel sum
// (smmd_bias.hip): (1) block (c, s) sums and sums the squares of its rows of
// channel c, shifted by its first element (float4 loads, per-thread float,
// block tree in double) into a
// [S][C] double slab; (2) block (c, s) reduces channel c's S partials in a
// fixed order (every block of the channel the same way), forms
// scale = gamma / sqrt(var + eps), applies relu(((x - k) - (mean - k)) * scale
// + beta) to its rows, and block (c, 0) updates the moving
// averages.  HBM: one read for the statistics, one read + one write to apply.
#include "smmd_common.hpp"

namespace smmd {

constexpr int BN_T = 256;

__device__ __forceinline__ void bn_rows(int N, int S, int s, int &n0, int &n1) {
    const int R = (N + S - 1) / S;
    n0 = s * R;
    n1 = min(N, n0 + R);
}

__global__ __launch_bounds__(BN_T) void bn_stats_kernel(const float *__restrict__ x, int N, int C,
                                                        int HW, int S,
                                                        double *__restrict__ part) {
    const int c = blockIdx.x, s = blockIdx.y;
    int n0, n1;
    bn_rows(N, S, s, n0, n1);
    const int w4 = HW >> 2;
    // rows shorter than the block are packed rpi per step (lane t: row t / w4,
    // column t % w4), so every lane loads on the small maps too
    const int rpi = w4 >= BN_T ? 1 : BN_T / w4;
    const int r = w4 >= BN_T ? 0 : (int)threadIdx.x / w4;
    const int col = w4 >= BN_T ? (int)threadIdx.x : (int)threadIdx.x - r * w4;
    const int step = w4 >= BN_T ? BN_T : w4;     // column stride within a row
    // shifted sums: every thread subtracts the channel's first element k
    // (x[0, c, 0], one cached load), so sum (x - k)^2 does not cancel
    // against the mean when |mean| >> std (a sample lies within a few std
    // of the mean); apply adds k back
    const float k = x[(size_t)c * HW];
    float a = 0.f, q = 0.f;
    if (r < rpi) {
        for (int n = n0 + r; n < n1; n += rpi) {
            const float4 *row = reinterpret_cast<const float4 *>(x + ((size_t)n * C + c) * HW);
            for (int i = col; i < w4; i += step) {
                const float4 v = row[i];
                const float dx = v.x - k, dy = v.y - k, dz = v.z - k, dw = v.w - k;
                a += (dx + dy) + (dz + dw);
                q = fmaf(dx, dx, q);
                q = fmaf(dy, dy, q);
                q = fmaf(dz, dz, q);
                q = fmaf(dw, dw, q);
            }
        }
    }
    __shared__ double red[BN_T / SMMD_WAVE];
    const double sa = block_sum<BN_T / SMMD_WAVE>((double)a, red);
    const double sq = block_sum<BN_T / SMMD_WAVE>((double)q, red);
    if (threadIdx.x == 0) {
        part[((size_t)s * C + c) * 2 + 0] = sa;
        part[((size_t)s * C + c) * 2 + 1] = sq;
    }
}

__global__ __launch_bounds__(BN_T) void bn_apply_kernel(const float *__restrict__ x, int N, int C,
                                                        int HW, int S,
                                                        const double *__restrict__ part,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ beta,
                                                        float *__restrict__ run_mean,
                                                        float *__restrict__ run_var,
                                                        float momentum, float eps,
                                                        float *__restrict__ y,
                                                        float *__restrict__ save) {
    const int c = blockIdx.x, s = blockIdx.y;
    __shared__ float sh[4];
    if (threadIdx.x < SMMD_WAVE) {
        // fixed order: lane-strided over the S partials, then the wave tree
        double a = 0.0, q = 0.0;
        for (int k = threadIdx.x; k < S; k += SMMD_WAVE) {
            a += part[((size_t)k * C + c) * 2 + 0];
            q += part[((size_t)k * C + c) * 2 + 1];
        }
        a = wave_sum(a);
        q = wave_sum(q);
        if (threadIdx.x == 0) {
            const double cnt = (double)N * (double)HW;
            const double ms = a / cnt;                   // mean of x - k
            const double mean = (double)x[(size_t)c * HW] + ms;
            double var = q / cnt - ms * ms;
            if (var < 0.0) var = 0.0;
            const double inv = 1.0 / sqrt(var + (double)eps);
            const double g = gamma ? (double)gamma[c] : 1.0;
            const double b = beta ? (double)beta[c] : 0.0;
            sh[0] = (float)(g * inv);
            sh[1] = (float)b;
            sh[2] = x[(size_t)c * HW];                  // the shift k
            sh[3] = (float)ms;                           // mean - k
            if (s == 0 && save) {                        // for smmd_bn_relu_bwd
                save[4 * c + 0] = sh[2];
                save[4 * c + 1] = sh[3];
                save[4 * c + 2] = (float)inv;
                save[4 * c + 3] = sh[0];
            }
            if (s == 0 && run_mean && run_var) {
                const double unb = cnt > 1.0 ? var * cnt / (cnt - 1.0) : var;
                run_mean[c] = (float)((1.0 - momentum) * (double)run_mean[c] + momentum * mean);
                run_var[c] = (float)((1.0 - momentum) * (double)run_var[c] + momentum * unb);
            }
        }
    }
    __syncthreads();
    // y = relu(((x - k) - (mean - k)) * scale + beta): x - k is exact (both
    // near the mean), so no x * scale term cancels against mean * scale
    const float sc = sh[0], bb = sh[1], k = sh[2], ms = sh[3];
    int n0, n1;
    bn_rows(N, S, s, n0, n1);
    const int w4 = HW >> 2;
    const int rpi = w4 >= BN_T ? 1 : BN_T / w4;  // short rows packed, as in the statistics
    const int r = w4 >= BN_T ? 0 : (int)threadIdx.x / w4;
    const int col = w4 >= BN_T ? (int)threadIdx.x : (int)threadIdx.x - r * w4;
    const int step = w4 >= BN_T ? BN_T : w4;
    if (r >= rpi) return;
    for (int n = n0 + r; n < n1; n += rpi) {
        const size_t off = ((size_t)n * C + c) * HW;
        const float4 *row = reinterpret_cast<const float4 *>(x + off);
        float4 *out = reinterpret_cast<float4 *>(y + off);
        for (int i = col; i < w4; i += step) {
            const float4 v = row[i];
            out[i] = make_float4(fmaxf(fmaf((v.x - k) - ms, sc, bb), 0.f),
                                 fmaxf(fmaf((v.y - k) - ms, sc, bb), 0.f),
                                 fmaxf(fmaf((v.z - k) - ms, sc, bb), 0.f),
                                 fmaxf(fmaf((v.w - k) - ms, sc, bb), 0.f));
        }
    }
}

// ---- backward of relu(batch_norm(x)) (training mode) ------------------------
// With z = xhat gamma + beta (the forward's value: the same float ops from the
// saved {k, mean - k, 1/sqrt(var + eps), gamma / sqrt(var + eps)}), so the ReLU
// mask is the forward's bit for bit), gz = gy [z > 0], M = N HW:
//   dbeta = sum gz,  dgamma = sum gz xhat,
//   dx = gamma inv (gz - dbeta / M - xhat dgamma / M)
// Pass 1 (grid (C, S)): per-block (sum gz, sum gz xhat) in double to a slab;
// pass 2: every block reduces its channel's partials in a fixed order, block
// (c, 0) writes dgamma, dbeta, all write dx.  HBM: x, gy read twice, dx once.
__device__ __forceinline__ void bn_bwd_elem(float x, float g, float k, float ms, float inv,
                                            float sc, float bb, float &gz, float &xh) {
    const float xm = (x - k) - ms;
    gz = (fmaf(xm, sc, bb) > 0.f) ? g : 0.f;
    xh = xm * inv;
}

__global__ __launch_bounds__(BN_T) void bn_bwd_stats_kernel(const float *__restrict__ x,
                                                            const float *__restrict__ gy, int N,
                                                            int C, int HW, int S,
                                                            const float *__restrict__ save,
                                                            const float *__restrict__ beta,
                                                            double *__restrict__ part) {
    const int c = blockIdx.x, s = blockIdx.y;
    int n0, n1;
    bn_rows(N, S, s, n0, n1);
    const int w4 = HW >> 2;
    const int rpi = w4 >= BN_T ? 1 : BN_T / w4;
    const int r = w4 >= BN_T ? 0 : (int)threadIdx.x / w4;
    const int col = w4 >= BN_T ? (int)threadIdx.x : (int)threadIdx.x - r * w4;
    const int step = w4 >= BN_T ? BN_T : w4;
    const float k = save[4 * c + 0], ms = save[4 * c + 1], inv = save[4 * c + 2];
    const float sc = save[4 * c + 3], bb = beta ? beta[c] : 0.f;
    float a = 0.f, q = 0.f;
    if (r < rpi) {
        for (int n = n0 + r; n < n1; n += rpi) {
            const size_t off = ((size_t)n * C + c) * HW;
            const float4 *xr = reinterpret_cast<const float4 *>(x + off);
            const float4 *gr = reinterpret_cast<const float4 *>(gy + off);
            for (int i = col; i < w4; i += step) {
                const float4 v = xr[i], g = gr[i];
                float gz, xh;
                bn_bwd_elem(v.x, g.x, k, ms, inv, sc, bb, gz, xh); a += gz; q = fmaf(gz, xh, q);
                bn_bwd_elem(v.y, g.y, k, ms, inv, sc, bb, gz, xh); a += gz; q = fmaf(gz, xh, q);
                bn_bwd_elem(v.z, g.z, k, ms, inv, sc, bb, gz, xh); a += gz; q = fmaf(gz, xh, q);
                bn_bwd_elem(v.w, g.w, k, ms, inv, sc, bb, gz, xh); a += gz; q = fmaf(gz, xh, q);
            }
        }
    }
    __shared__ double red[BN_T / SMMD_WAVE];
    const double sa = block_sum<BN_T / SMMD_WAVE>((double)a, red);
    const double sq = block_sum<BN_T / SMMD_WAVE>((double)q, red);
    if (threadIdx.x == 0) {
        part[((size_t)s * C + c) * 2 + 0] = sa;
        part[((size_t)s * C + c) * 2 + 1] = sq;
    }
}

__global__ __launch_bounds__(BN_T) void bn_bwd_apply_kernel(
    const float *__restrict__ x, const float *__restrict__ gy, int N, int C, int HW, int S,
    const double *__restrict__ part, const float *__restrict__ save,
    const float *__restrict__ beta, float *__restrict__ gx, float *__restrict__ ggamma,
    float *__restrict__ gbeta) {
    const int c = blockIdx.x, s = blockIdx.y;
    __shared__ float sh[2];
    if (threadIdx.x < SMMD_WAVE) {
        double a = 0.0, q = 0.0;
        for (int j = threadIdx.x; j < S; j += SMMD_WAVE) {
            a += part[((size_t)j * C + c) * 2 + 0];
            q += part[((size_t)j * C + c) * 2 + 1];
        }
        a = wave_sum(a);
        q = wave_sum(q);
        if (threadIdx.x == 0) {
            const double cnt = (double)N * (double)HW;
            sh[0] = (float)(a / cnt);
            sh[1] = (float)(q / cnt);
            if (s == 0) {
                if (gbeta) gbeta[c] = (float)a;
                if (ggamma) ggamma[c] = (float)q;
            }
        }
    }
    __syncthreads();
    const float mb = sh[0], mq = sh[1];
    const float k = save[4 * c + 0], ms = save[4 * c + 1], inv = save[4 * c + 2];
    const float sc = save[4 * c + 3], bb = beta ? beta[c] : 0.f;
    int n0, n1;
    bn_rows(N, S, s, n0, n1);
    const int w4 = HW >> 2;
    const int rpi = w4 >= BN_T ? 1 : BN_T / w4;
    const int r = w4 >= BN_T ? 0 : (int)threadIdx.x / w4;
    const int col = w4 >= BN_T ? (int)threadIdx.x : (int)threadIdx.x - r * w4;
    const int step = w4 >= BN_T ? BN_T : w4;
    if (r >= rpi) return;
    for (int n = n0 + r; n < n1; n += rpi) {
        const size_t off = ((size_t)n * C + c) * HW;
        const float4 *xr = reinterpret_cast<const float4 *>(x + off);
        const float4 *gr = reinterpret_cast<const float4 *>(gy + off);
        float4 *out = reinterpret_cast<float4 *>(gx + off);
        for (int i = col; i < w4; i += step) {
            const float4 v = xr[i], g = gr[i];
            float gz, xh;
            float4 o;
            bn_bwd_elem(v.x, g.x, k, ms, inv, sc, bb, gz, xh); o.x = sc * ((gz - mb) - xh * mq);
            bn_bwd_elem(v.y, g.y, k, ms, inv, sc, bb, gz, xh); o.y = sc * ((gz - mb) - xh * mq);
            bn_bwd_elem(v.z, g.z, k, ms, inv, sc, bb, gz, xh); o.z = sc * ((gz - mb) - xh * mq);
            bn_bwd_elem(v.w, g.w, k, ms, inv, sc, bb, gz, xh); o.w = sc * ((gz - mb) - xh * mq);
            out[i] = o;
        }
    }
}

inline int bn_split(int N, int C) {
    if (C >= 512) return 1;
    int S = (2048 + C - 1) / C;
    if (S > N) S = N;
    return S < 1 ? 1 : S;
}

}  // namespace smmd

using namespace smmd;

extern "C" size_t smmd_bn_relu_workspace_bytes(int N, int C) {
    if (N <= 0 || C <= 0) return 0;
    return (size_t)bn_split(N, C) * C * 2 * sizeof(double);
}

extern "C" smmd_status smmd_bn_relu_fwd_save(const float *x, int N, int C, int HW,
                                             const float *gamma, const float *beta,
                                             float *running_mean, float *running_var,
                                             float momentum, float eps, float *y, float *save,
                                             void *ws, size_t ws_bytes, smmd_stream_t stream) {
    if (!x || !y || N < 1 || C < 1 || HW < 4 || (HW & 3)) return SMMD_EINVAL;
    if (((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return SMMD_EINVAL;
    const int S = bn_split(N, C);
    if (S > 65535) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_bn_relu_workspace_bytes(N, C)) return SMMD_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    double *part = static_cast<double *>(ws);
    hipLaunchKernelGGL(bn_stats_kernel, dim3(C, S), dim3(BN_T), 0, st, x, N, C, HW, S, part);
    smmd_status e = last_launch_status();
    if (e != SMMD_OK) return e;
    hipLaunchKernelGGL(bn_apply_kernel, dim3(C, S), dim3(BN_T), 0, st, x, N, C, HW, S,
                       (const double *)part, gamma, beta, running_mean, running_var, momentum,
                       eps, y, save);
    return last_launch_status();
}

extern "C" smmd_status smmd_bn_relu_fwd(const float *x, int N, int C, int HW, const float *gamma,
                                        const float *beta, float *running_mean,
                                        float *running_var, float momentum, float eps, float *y,
                                        void *ws, size_t ws_bytes, smmd_stream_t stream) {
    return smmd_bn_relu_fwd_save(x, N, C, HW, gamma, beta, running_mean, running_var, momentum,
                                 eps, y, nullptr, ws, ws_bytes, stream);
}

extern "C" smmd_status smmd_bn_relu_bwd(const float *x, const float *gy, int N, int C, int HW,
                                        const float *beta, const float *save, float *gx,
                                        float *ggamma, float *gbeta, void *ws, size_t ws_bytes,
                                        smmd_stream_t stream) {
    if (!x || !gy || !gx || !save || N < 1 || C < 1 || HW < 4 || (HW & 3)) return SMMD_EINVAL;
    if (((uintptr_t)x & 15) || ((uintptr_t)gy & 15) || ((uintptr_t)gx & 15)) return SMMD_EINVAL;
    const int S = bn_split(N, C);
    if (S > 65535) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_bn_relu_workspace_bytes(N, C)) return SMMD_EWORKSPACE;
    hipStream_t st = (hipStream_t)stream;
    double *part = static_cast<double *>(ws);
    hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3(C, S), dim3(BN_T), 0, st, x, gy, N, C, HW, S,
                       save, beta, part);
    smmd_status e = last_launch_status();
    if (e != SMMD_OK) return e;
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(C, S), dim3(BN_T), 0, st, x, gy, N, C, HW, S,
                       (const double *)part, save, beta, gx, ggamma, gbeta);
    return last_launch_status();
}
