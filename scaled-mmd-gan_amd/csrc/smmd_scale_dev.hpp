// smmd_scale_dev.hpp -- device code of the scaled loss shared by its own
// launches (smmd_scale.hip) and the fused MMD^2 + scaled-loss launch
// (smmd_mmd_tile.hip): the per-(row, chunk) squared-norm partials of the
// Jacobian and the one-block finalize (J, nD, scale, losses).
//
// Reference: gan/core/ops.py:228-233 (squared_norm_jacobian),
// gan/core/model.py:366-403 (add_scaling), gan/core/smmd.py:21-23, :40-42.
#pragma once
#include "smmd_common.hpp"

namespace smmd {

constexpr int SQ_CHUNK = 4096;   // floats per block of the squared-norm pass
// workspace header: the arrival ticket (word 0) and, 256 B apart, the 8 shard
// counters of the fused loss launch's two-level ticket
constexpr int SQ_SHARDS = 8;
constexpr int SQ_SHARD_STRIDE = 64;              // unsigned words (256 B)
constexpr size_t SQ_WS_HEADER = 4096;

struct ScaledLossArgs {
    const float *jac;
    int64_t per_sample;
    int nchunk, vec;
    double *part;        // ws + SQ_WS_HEADER: [rows * nchunk] partials
    unsigned *counter;   // ws + 0: arrival ticket (zero at rest)
    int n_cols, b, b_total, dof, variant, sqrt_scale;
    const float *feat;
    const float *base_loss;
    float sc;
    float *out;
    float *per_sample_out;
    int nblocks;         // squared-norm blocks (rows * nchunk)
    // the all-gather mode's fused loss (smmd_smmd_loss_fwd_gathered): J and nD
    // are not reduced from the Jacobian here but summed, in rank order, from
    // the gathered per-rank partials stats[r * stats_stride + {0, 1}]
    // (ops.scaling_partials of every rank, carried by the feature all-gather)
    const float *stats;              // NULL: J / nD from the Jacobian partials
    int stats_world, stats_stride;
};
// (host code zero-fills a ScaledLossArgs before setting its fields: a field
// added later must read as "off", never as stack garbage)

// ---- per-(row, chunk) partial sum of squares of block `blk` (256 threads):
// a thread's (up to) four float4 loads are issued before its fmas (one memory
// round trip, not four); the fma chain runs in index order either way --------
__device__ __forceinline__ double sqnorm_block(const ScaledLossArgs &a, int blk) {
    const float *__restrict__ jac = a.jac;
    const int64_t per_sample = a.per_sample;
    const int nchunk = a.nchunk, vec = a.vec;
    const int row = blk / nchunk, ch = blk % nchunk;
    const float *p = jac + (size_t)row * per_sample;
    const int64_t b0 = (int64_t)ch * SQ_CHUNK;
    const int64_t e0 = (b0 + SQ_CHUNK < per_sample) ? b0 + SQ_CHUNK : per_sample;
    float acc = 0.f;
    if (vec) {
        constexpr int Q = SQ_CHUNK / 1024;
        float4 x[Q];
#pragma unroll
        for (int k = 0; k < Q; ++k) {
            const int64_t i = b0 + threadIdx.x * 4 + k * 1024;
            x[k] = (i < e0) ? *reinterpret_cast<const float4 *>(p + i)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < Q; ++k) {
            if (b0 + threadIdx.x * 4 + k * 1024 < e0) {
                acc = fmaf(x[k].x, x[k].x, acc);
                acc = fmaf(x[k].y, x[k].y, acc);
                acc = fmaf(x[k].z, x[k].z, acc);
                acc = fmaf(x[k].w, x[k].w, acc);
            }
        }
    } else {
        for (int64_t i = b0 + threadIdx.x; i < e0; i += 256) acc = fmaf(p[i], p[i], acc);
    }
    __shared__ double red[4];
    return block_sum<4>((double)acc, red);
}

// ---- finalize: per-sample norms, J, nD, scale, losses (one 256-thread block;
// partials summed in fixed order).  base: the loss being scaled. ------------
constexpr int SQ_FIN_LDS = 2048;    // partials staged through LDS (16 KiB)

// pre: the partials already staged in LDS by the caller (the fused loss
// launch), or nullptr to load them here.
__device__ __forceinline__ void scaled_loss_final(const ScaledLossArgs &a, float base,
                                                  const double *pre = nullptr) {
    const double *__restrict__ part = a.part;
    const int n_cols = a.n_cols, b = a.b, b_total = a.b_total, nchunk = a.nchunk;
    const float *feat = a.feat;
    const int dof = a.dof, variant = a.variant, sqrt_scale = a.sqrt_scale;
    const float sc = a.sc;
    float *out = a.out, *per_sample_out = a.per_sample_out;
    __shared__ double red[4];
    __shared__ double pl[SQ_FIN_LDS];
    const int tot = n_cols * b * nchunk;
    const bool staged = pre == nullptr && tot <= SQ_FIN_LDS;
    if (staged) {
        // every partial loaded with 8 loads in flight per thread (one memory
        // round trip for the configs' 64 x 3 partials), then summed from LDS
        for (int i0 = threadIdx.x; i0 < tot; i0 += 256 * 8) {
            double t[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int i = i0 + j * 256;
                t[j] = (i < tot) ? part[i] : 0.0;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (i0 + j * 256 < tot) pl[i0 + j * 256] = t[j];
        }
        __syncthreads();
    }
    const double *src = pre ? pre : (staged ? pl : part);
    double jsum = 0.0;
    for (int s = threadIdx.x; s < b; s += 256) {
        double ps = 0.0;
        for (int c = 0; c < n_cols; ++c) {          // ops.py:232 sum over columns
            const double *q = src + ((size_t)c * b + s) * nchunk;
            double t = 0.0;
            for (int k = 0; k < nchunk; ++k) t += q[k];
            ps += t;
        }
        if (per_sample_out) per_sample_out[s] = (float)ps;
        jsum += ps;
    }
    jsum = block_sum<4>(jsum, red);
    double nd = 0.0;
    if (variant == 1 && feat) {
        double fs = 0.0;
        for (int i = threadIdx.x; i < b * dof; i += 256) fs += (double)feat[i] * (double)feat[i];
        fs = block_sum<4>(fs, red);
        nd = fs / ((double)b_total * dof);              // model.py:385
    }
    if (threadIdx.x == 0) {
        float J = (float)(jsum / (double)b_total);       // model.py:384
        float nD = (float)nd;
        if (a.stats) {
            // the gathered partials (each already / b_total), summed in rank
            // order as collectives.StepExchange does: the same bits
            J = a.stats[0];
            nD = a.stats[1];
            for (int r = 1; r < a.stats_world; ++r) {
                J = J + a.stats[(size_t)r * a.stats_stride];
                nD = nD + a.stats[(size_t)r * a.stats_stride + 1];
            }
        }
        const float q = (variant == 1) ? (J + nD) : J;  // model.py:387-390
        const float scale = 1.f / (sc * q + 1.f);
        const float f = sqrt_scale ? sqrtf(scale) : scale;   // smmd.py:22 / :41
        const float g = base * f;
        out[0] = g;
        out[1] = -g;
        out[2] = scale;
        out[3] = J;
        out[4] = nD;
        out[5] = base;
        out[6] = 0.f;
        out[7] = 0.f;
    }
}

}  // namespace smmd
