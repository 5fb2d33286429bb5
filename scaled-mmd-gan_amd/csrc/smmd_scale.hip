// smmd_scale.hip -- scaling regulariser of the SMMD/SWGAN loss and the
// TF-semantics clip + Adam update, gfx950 (MI355X).  All HBM-bound.
//
// Reference: gan/core/ops.py:228-233 (squared_norm_jacobian),
// gan/core/model.py:366-403 (add_scaling), gan/core/smmd.py:21-23, :40-42
// (apply_scaling), gan/core/model.py:444-468 (clip_by_norm + Adam).
#include "smmd_scale_dev.hpp"
#include "smmd_sn_tile.hpp"

#include <stdlib.h>

namespace smmd {

// ---- the squared-norm pass; the last block to arrive runs the finalize
// (per-sample norms, J, nD, scale, losses) ------------------------------------
__global__ __launch_bounds__(256) void sqnorm_partial_kernel(ScaledLossArgs a) {
    const double s = sqnorm_block(a, blockIdx.x);
    __shared__ int last;
    if (threadIdx.x < 64) {      // wave 0: publish the partial write-through, then the ticket
        if (threadIdx.x == 0) store_wt(a.part + blockIdx.x, s);
        const int l = wave_ticket(a.counter, gridDim.x);
        if (threadIdx.x == 0) last = l;
    }
    __syncthreads();
    if (!last) return;
    acquire_block();
    scaled_loss_final(a, a.base_loss ? a.base_loss[0] : 0.f);
    ticket_reset(a.counter);
}

// ---- backward: d base, d jac, d feat ---------------------------------------
__global__ void scaled_loss_finalize_kernel(float *out, float sc, int variant, int sqrt_scale) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const float q = (variant == 1) ? (out[3] + out[4]) : out[3];
        const float scale = 1.f / (sc * q + 1.f);
        const float g = out[5] * (sqrt_scale ? sqrtf(scale) : scale);
        out[0] = g;
        out[1] = -g;
        out[2] = scale;
    }
}

// Optional MMD part (the fused SMMD loss, smmd_smmd_loss_bwd): base = mmd2,
// so dX, dY = (g_mmd2 + go f) * the forward's unit gradients gxu, gyu.
struct MmdBwdPart {
    const float *g_mmd2;           // upstream gradient of the mmd2 output (may be null)
    const float *gxu, *gyu;        // d mmd2 / dX, dY of the forward
    int64_t nx, ny;
    float *dX, *dY;
};

__global__ __launch_bounds__(256) void scaled_loss_bwd_kernel(
    const float *__restrict__ jac, int64_t n_jac, int b, const float *__restrict__ feat,
    int64_t n_feat, int dof, const float *fwd_out, float sc, int variant, int sqrt_scale,
    const float *g_loss_grad, float *d_base, float *__restrict__ gjac, float *__restrict__ gfeat,
    int vec, MmdBwdPart mp) {
    const float go = g_loss_grad ? g_loss_grad[0] : 1.f;
    const float scale = fwd_out[2];
    const float base = fwd_out[5];
    const float f = sqrt_scale ? sqrtf(scale) : scale;
    const float fp = sqrt_scale ? 0.5f / sqrtf(scale) : 1.f;
    const float coefq = go * base * fp * (-sc * scale * scale);   // dL/dQ
    const float cj = coefq * (2.f / (float)b);
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t nth = (size_t)gridDim.x * blockDim.x;
    if (tid == 0 && d_base) d_base[0] = go * f;
    if (mp.dX) {
        const float dm = (mp.g_mmd2 ? mp.g_mmd2[0] : 0.f) + go * f;
        for (size_t i = tid; i < (size_t)mp.nx; i += nth) mp.dX[i] = mp.gxu[i] * dm;
        for (size_t i = tid; i < (size_t)mp.ny; i += nth) mp.dY[i] = mp.gyu[i] * dm;
    }
    if (!gjac) {
        // no Jacobian gradient wanted (a generator step: jac is a constant)
    } else if (vec) {
        const int64_t n4 = n_jac / 4;
        for (size_t i = tid; i < (size_t)n4; i += nth) {
            const float4 x = reinterpret_cast<const float4 *>(jac)[i];
            float4 o;
            o.x = cj * x.x; o.y = cj * x.y; o.z = cj * x.z; o.w = cj * x.w;
            reinterpret_cast<float4 *>(gjac)[i] = o;
        }
        for (size_t i = (size_t)n4 * 4 + tid; i < (size_t)n_jac; i += nth) gjac[i] = cj * jac[i];
    } else {
        for (size_t i = tid; i < (size_t)n_jac; i += nth) gjac[i] = cj * jac[i];
    }
    if (gfeat && feat) {
        const float cf = (variant == 1) ? coefq * (2.f / ((float)b * (float)dof)) : 0.f;
        for (size_t i = tid; i < (size_t)n_feat; i += nth) gfeat[i] = cf * feat[i];
    }
}

// ---------------------------------------------------------------------------
// flat multi-tensor clip / Adam.  Tensors are [off[i], off[i+1]) of one flat
// buffer.  The norm pass cuts each tensor into OPT_SQ_CHUNK-element blocks
// (one double partial each); the update / clip pass into OPT_UP_CHUNK-element
// blocks, small enough that the ~2.5k blocks of a 10 M-parameter critic spread
// evenly over 256 CUs (16 K-element blocks left 105 CUs with one block more
// than the rest), each thread issuing all of its loads before any update.
// ---------------------------------------------------------------------------
constexpr int OPT_SQ_CHUNK = 8192;
constexpr int OPT_UP_CHUNK = 4096;
constexpr int OPT_SQ_IT = OPT_SQ_CHUNK / 4 / 256;   // float4 per thread, full block
constexpr int OPT_UP_IT = OPT_UP_CHUNK / 4 / 256;
constexpr int OPT_MAX = 96;     // tensors per launch set (kernel-arg budget)

struct OptTable {
    int n;
    int total_blocks;            // blocks of the pass this table drives
    int chunk;                   // elements per block of that pass
    int64_t off[OPT_MAX + 1];
    int blk[OPT_MAX + 1];        // first block of each tensor (this pass)
    int sblk[OPT_MAX + 1];       // first norm-pass block of each tensor (partial slab)
    unsigned char skip[OPT_MAX]; // tensor updated elsewhere (the SN-fused update)
};

__device__ __forceinline__ int opt_find(const OptTable &t, int b) {
    int lo = 0, hi = t.n - 1;
    while (lo < hi) {                 // last i with blk[i] <= b
        const int mid = (lo + hi + 1) >> 1;
        if (t.blk[mid] <= b) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// every tensor range [off[i], off[i+1]) of the flat buffer is walked as float4
// when all offsets are multiples of 4 and the buffers 16-byte aligned (vec);
// FlatAdam pads its tensors to that.
__device__ __forceinline__ void opt_range(const OptTable &t, int ti, int b, int64_t &lo,
                                          int64_t &hi) {
    lo = t.off[ti] + (int64_t)(b - t.blk[ti]) * t.chunk;
    hi = (lo + t.chunk < t.off[ti + 1]) ? lo + t.chunk : t.off[ti + 1];
}

__global__ __launch_bounds__(256) void opt_sqsum_kernel(OptTable t, const float *__restrict__ g,
                                                        float gscale, int vec,
                                                        double *__restrict__ part) {
    const int ti = opt_find(t, blockIdx.x);
    if (t.skip[ti]) return;     // a tensor whose norm comes from elsewhere (G-direct SN)
    int64_t lo, hi;
    opt_range(t, ti, blockIdx.x, lo, hi);
    float acc0 = 0.f, acc1 = 0.f;
    if (vec && hi - lo == OPT_SQ_CHUNK) {     // full block: every load in flight at once
        const float4 *g4 = reinterpret_cast<const float4 *>(g) + lo / 4 + threadIdx.x;
        float4 x[OPT_SQ_IT];
#pragma unroll
        for (int k = 0; k < OPT_SQ_IT; ++k) x[k] = g4[k * 256];
#pragma unroll
        for (int k = 0; k < OPT_SQ_IT; ++k) {
            acc0 = fmaf(x[k].x * gscale, x[k].x * gscale, acc0);
            acc1 = fmaf(x[k].y * gscale, x[k].y * gscale, acc1);
            acc0 = fmaf(x[k].z * gscale, x[k].z * gscale, acc0);
            acc1 = fmaf(x[k].w * gscale, x[k].w * gscale, acc1);
        }
    } else if (vec) {
        const float4 *g4 = reinterpret_cast<const float4 *>(g);
        for (int64_t i = lo / 4 + threadIdx.x; i < hi / 4; i += 256) {
            const float4 x = g4[i];
            acc0 = fmaf(x.x * gscale, x.x * gscale, acc0);
            acc1 = fmaf(x.y * gscale, x.y * gscale, acc1);
            acc0 = fmaf(x.z * gscale, x.z * gscale, acc0);
            acc1 = fmaf(x.w * gscale, x.w * gscale, acc1);
        }
    } else {
        for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
            const float x = g[i] * gscale;
            acc0 = fmaf(x, x, acc0);
        }
    }
    __shared__ double red[4];
    const double s = block_sum<4>((double)acc0 + (double)acc1, red);
    if (threadIdx.x == 0) part[t.sblk[ti] + (blockIdx.x - t.blk[ti])] = s;
}

__device__ __forceinline__ float clip_factor(const OptTable &t, int ti, const double *part,
                                             float clip, float *sh) {
    return clip_factor_slab(part, t.sblk[ti], t.sblk[ti + 1], clip, sh);
}

__global__ __launch_bounds__(256) void opt_clip_kernel(OptTable t, float *__restrict__ g,
                                                       const double *__restrict__ part, float clip,
                                                       int vec) {
    const int ti = opt_find(t, blockIdx.x);
    __shared__ float sh[1];
    const float f = clip_factor(t, ti, part, clip, sh);
    int64_t lo, hi;
    opt_range(t, ti, blockIdx.x, lo, hi);
    if (vec) {
        float4 *g4 = reinterpret_cast<float4 *>(g);
        for (int64_t i = lo / 4 + threadIdx.x; i < hi / 4; i += 256) {
            float4 x = g4[i];
            x.x *= f; x.y *= f; x.z *= f; x.w *= f;
            g4[i] = x;
        }
    } else {
        for (int64_t i = lo + threadIdx.x; i < hi; i += 256) g[i] = g[i] * f;
    }
}

struct AdamArgs {
    float *p, *m, *v;
    const float *g;
    const double *part;     // norm-pass partials
    const float *lr_t_dev;  // non-NULL: lr_t read at execution time (graph replay)
    float clip;             // > 0: per-tensor clip_by_norm
    int vec;
    int norm_inblock;       // every tensor one update block: its norm summed in the block
    AdamK k;                // k.f set per tensor
};

__device__ __forceinline__ AdamK adam_k(const AdamArgs &a) {
    AdamK k = a.k;
    if (a.lr_t_dev) k.lr_t = a.lr_t_dev[0];
    return k;
}

// update block b of the table (blocks of skipped tensors return at once)
__device__ __forceinline__ void opt_adam_block(const OptTable &t, int b, const AdamArgs &a) {
    const int ti = opt_find(t, b);
    if (t.skip[ti]) return;             // block-uniform
    float *__restrict__ p = a.p;
    float *__restrict__ m = a.m;
    float *__restrict__ v = a.v;
    const float *__restrict__ g = a.g;
    const int vec = a.vec;
    __shared__ float sh[1];
    AdamK k = adam_k(a);
    int64_t lo, hi;
    opt_range(t, ti, b, lo, hi);
    if (!(a.clip > 0.f)) {
        k.f = 1.f;
    } else if (a.norm_inblock) {
        // the whole tensor is this block's range: its norm here, no norm pass
        __shared__ double red[4];
        float acc = 0.f;
        for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
            const float x = g[i] * k.gscale;
            acc = fmaf(x, x, acc);
        }
        const float ss = (float)block_sum<4>((double)acc, red);
        const float inv = (ss > 0.f) ? rsqrtf(ss) : INFINITY;
        k.f = a.clip * fminf(inv, 1.f / a.clip);
    } else {
        k.f = clip_factor(t, ti, a.part, a.clip, sh);
    }
    if (vec && hi - lo == OPT_UP_CHUNK) {     // full block: 4 x OPT_UP_IT float4 loads in flight
        const int64_t b4 = lo / 4 + threadIdx.x;
        float4 *p4 = reinterpret_cast<float4 *>(p) + b4;
        const float4 *g4 = reinterpret_cast<const float4 *>(g) + b4;
        float4 *m4 = reinterpret_cast<float4 *>(m) + b4;
        float4 *v4 = reinterpret_cast<float4 *>(v) + b4;
        float4 pp[OPT_UP_IT], gg[OPT_UP_IT], mm[OPT_UP_IT], vv[OPT_UP_IT];
#pragma unroll
        for (int j = 0; j < OPT_UP_IT; ++j) {
            gg[j] = g4[j * 256];
            pp[j] = p4[j * 256];
            mm[j] = ld_nt(m4 + j * 256);
            vv[j] = ld_nt(v4 + j * 256);
        }
#pragma unroll
        for (int j = 0; j < OPT_UP_IT; ++j) {
            k.upd(pp[j].x, gg[j].x, mm[j].x, vv[j].x);
            k.upd(pp[j].y, gg[j].y, mm[j].y, vv[j].y);
            k.upd(pp[j].z, gg[j].z, mm[j].z, vv[j].z);
            k.upd(pp[j].w, gg[j].w, mm[j].w, vv[j].w);
            p4[j * 256] = pp[j];
            st_nt(m4 + j * 256, mm[j]);
            st_nt(v4 + j * 256, vv[j]);
        }
    } else if (vec) {
        float4 *p4 = reinterpret_cast<float4 *>(p);
        const float4 *g4 = reinterpret_cast<const float4 *>(g);
        float4 *m4 = reinterpret_cast<float4 *>(m);
        float4 *v4 = reinterpret_cast<float4 *>(v);
        for (int64_t i = lo / 4 + threadIdx.x; i < hi / 4; i += 256) {
            float4 pp = p4[i], mm = m4[i], vv = v4[i];
            const float4 gg = g4[i];
            k.upd(pp.x, gg.x, mm.x, vv.x);
            k.upd(pp.y, gg.y, mm.y, vv.y);
            k.upd(pp.z, gg.z, mm.z, vv.z);
            k.upd(pp.w, gg.w, mm.w, vv.w);
            p4[i] = pp;
            m4[i] = mm;
            v4[i] = vv;
        }
    } else {
        for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
            float pp = p[i], mm = m[i], vv = v[i];
            k.upd(pp, g[i], mm, vv);
            p[i] = pp;
            m[i] = mm;
            v[i] = vv;
        }
    }
}

__global__ __launch_bounds__(256) void opt_adam_kernel(OptTable t, AdamArgs a) {
    opt_adam_block(t, blockIdx.x, a);
}

// one launch for a critic update with SN layers: the SN weight tiles first
// (tile-shaped, with the next power iteration's P1), then the blocks of every
// other tensor
template <int H, bool GD = false>
__global__ __launch_bounds__(256) void opt_adam_sn_kernel(OptTable t, SnAdamTable st,
                                                          AdamArgs a) {
    if ((int)blockIdx.x < st.total_tiles)
        sn_adam_tile<H, GD>(st, blockIdx.x, adam_k(a), a.part, a.clip);
    else
        opt_adam_block(t, blockIdx.x - st.total_tiles, a);
}

// row groups of the fused SN tile (env SMMD_SN_ADAM_H = 1 | 2 | 4, default 2)
static int sn_adam_groups() {
    const char *e = getenv("SMMD_SN_ADAM_H");
    return (e && (e[0] == '1' || e[0] == '4')) ? e[0] - '0' : 2;
}
static_assert(sizeof(OptTable) + sizeof(SnAdamTable) + sizeof(AdamArgs) <= 4000,
              "kernel argument budget");

static AdamArgs adam_args(float *p, const float *g, float *m, float *v, const void *ws,
                          float gscale, float clip, double lr_t, float b1, float b2, float eps,
                          int vec) {
    AdamArgs a;
    a.p = p;
    a.m = m;
    a.v = v;
    a.g = g;
    a.part = (const double *)ws;
    a.lr_t_dev = nullptr;
    a.clip = clip;
    a.vec = vec;
    a.norm_inblock = 0;
    a.k.gscale = gscale;
    a.k.f = 1.f;
    a.k.lr_t = (float)lr_t;
    a.k.b1c = 1.f - b1;
    a.k.b2c = 1.f - b2;
    a.k.eps = eps;
    return a;
}

// the update pass skips skipped tensors' blocks without launching them: a
// skipped tensor keeps one block (the map stays strictly increasing) that
// returns at once
static int opt_vec(const int64_t *off, int n, const void *a, const void *b, const void *c,
                   const void *d) {
    for (int i = 0; i <= n; ++i)
        if (off[i] % 4) return 0;
    const uintptr_t al = (uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)d;
    return (al % 16) == 0;
}

// blocks of a tensor of n elements at `chunk` elements per block (an empty
// tensor keeps one block so the block -> tensor map stays strictly increasing)
static int64_t opt_blocks(int64_t n, int chunk) { return n == 0 ? 1 : (n + chunk - 1) / chunk; }

// table of tensors [first, first + count) for a pass of `chunk`-element blocks
static bool build_opt(const int64_t *off, int first, int count, int chunk, OptTable &t,
                      const unsigned char *skip = nullptr) {
    memset(&t, 0, sizeof(t));
    t.n = count;
    t.chunk = chunk;
    int64_t blocks = 0, sblocks = 0;
    for (int i = 0; i <= count; ++i) {
        t.off[i] = off[first + i];
        if (i > 0 && t.off[i] < t.off[i - 1]) return false;
    }
    for (int i = 0; i < count; ++i) {
        t.blk[i] = (int)blocks;
        t.sblk[i] = (int)sblocks;
        const int64_t n = t.off[i + 1] - t.off[i];
        blocks += skip && skip[first + i] ? 1 : opt_blocks(n, chunk);
        t.skip[i] = skip && skip[first + i] ? 1 : 0;
        sblocks += opt_blocks(n, OPT_SQ_CHUNK);
        if (blocks > INT32_MAX / 2) return false;
    }
    t.blk[count] = (int)blocks;
    t.sblk[count] = (int)sblocks;
    t.total_blocks = (int)blocks;
    return true;
}

}  // namespace smmd

using namespace smmd;

extern "C" {

size_t smmd_scaled_loss_workspace_bytes(int rows, int64_t per_sample) {
    if (rows < 1 || per_sample < 1) return 0;
    const int64_t nchunk = (per_sample + SQ_CHUNK - 1) / SQ_CHUNK;
    return SQ_WS_HEADER + align_up((size_t)rows * nchunk * sizeof(double), 256);   // tickets + partials
}

smmd_status smmd_scaled_loss_fwd(const float *jac, int n_cols, int b, int b_total,
                                 int64_t per_sample, const float *feat, int dof,
                                 const float *base_loss, float sc,
                                 int variant, int sqrt_scale, float *out, float *per_sample_out,
                                 void *ws, size_t ws_bytes, smmd_stream_t stream) {
    if (!jac || !out || n_cols < 1 || b < 1 || per_sample < 1) return SMMD_EINVAL;
    if (b_total < 1) b_total = b;
    if (variant != 0 && variant != 1) return SMMD_EINVAL;
    if (variant == 1 && (!feat || dof < 1)) return SMMD_EINVAL;
    const int rows = n_cols * b;
    if (!ws || ws_bytes < smmd_scaled_loss_workspace_bytes(rows, per_sample)) return SMMD_EWORKSPACE;
    const int nchunk = (int)((per_sample + SQ_CHUNK - 1) / SQ_CHUNK);
    const int vec = (per_sample % 4 == 0) && ((uintptr_t)jac % 16 == 0);
    ScaledLossArgs a;
    memset(&a, 0, sizeof(a));        // every field not set below (stats: none) is zero
    a.jac = jac;
    a.per_sample = per_sample;
    a.nchunk = nchunk;
    a.vec = vec;
    // ticket first, at a fixed offset: a cached workspace reused for fewer rows
    // must not find its counter inside an earlier call's partials
    a.counter = (unsigned *)ws;
    a.part = (double *)((char *)ws + SQ_WS_HEADER);
    a.n_cols = n_cols;
    a.b = b;
    a.b_total = b_total;
    a.dof = dof;
    a.variant = variant;
    a.sqrt_scale = sqrt_scale;
    a.feat = feat;
    a.base_loss = base_loss;
    a.sc = sc;
    a.out = out;
    a.per_sample_out = per_sample_out;
    a.nblocks = rows * nchunk;
    hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(rows * nchunk), dim3(256), 0,
                       (hipStream_t)stream, a);
    return last_launch_status();
}

smmd_status smmd_scaled_loss_finalize(float *out, float sc, int variant, int sqrt_scale,
                                      smmd_stream_t stream) {
    if (!out || (variant != 0 && variant != 1)) return SMMD_EINVAL;
    hipLaunchKernelGGL(scaled_loss_finalize_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                       out, sc, variant, sqrt_scale);
    return last_launch_status();
}

smmd_status smmd_scaled_loss_bwd(const float *jac, int n_cols, int b, int b_total,
                                 int64_t per_sample, const float *feat, int dof,
                                 const float *fwd_out, float sc,
                                 int variant, int sqrt_scale, const float *g_loss_grad,
                                 float *d_base, float *gjac, float *gfeat, smmd_stream_t stream) {
    if (!jac || !fwd_out || !gjac || n_cols < 1 || b < 1 || per_sample < 1) return SMMD_EINVAL;
    if (variant == 1 && (!feat || !gfeat || dof < 1)) return SMMD_EINVAL;
    if (b_total < 1) b_total = b;
    const int64_t n_jac = (int64_t)n_cols * b * per_sample;
    const int vec = ((uintptr_t)jac % 16 == 0) && ((uintptr_t)gjac % 16 == 0);
    int64_t blocks = (n_jac / 4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    MmdBwdPart mp;
    memset(&mp, 0, sizeof(mp));
    hipLaunchKernelGGL(scaled_loss_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, jac, n_jac, b_total, feat, (int64_t)b * (dof > 0 ? dof : 0),
                       dof, fwd_out, sc, variant, sqrt_scale, g_loss_grad, d_base, gjac, gfeat, vec,
                       mp);
    return last_launch_status();
}

smmd_status smmd_smmd_loss_bwd(const float *jac, int n_cols, int b, int64_t per_sample,
                               const float *feat, int dof, const float *fwd_out, float sc,
                               int variant, int sqrt_scale, const float *g_loss_grad,
                               const float *g_mmd2_grad, const float *gx_unit, int m,
                               const float *gy_unit, int n, int d, float *gjac, float *gfeat,
                               float *dX, float *dY, smmd_stream_t stream) {
    return smmd_smmd_loss_bwd_ex(jac, n_cols, b, b, per_sample, feat, dof, fwd_out, sc, variant,
                                 sqrt_scale, g_loss_grad, g_mmd2_grad, gx_unit, m, gy_unit, n, d,
                                 gjac, gfeat, dX, dY, stream);
}

smmd_status smmd_smmd_loss_bwd_ex(const float *jac, int n_cols, int b, int b_total,
                                  int64_t per_sample, const float *feat, int dof,
                                  const float *fwd_out, float sc, int variant, int sqrt_scale,
                                  const float *g_loss_grad, const float *g_mmd2_grad,
                                  const float *gx_unit, int m, const float *gy_unit, int n, int d,
                                  float *gjac, float *gfeat, float *dX, float *dY,
                                  smmd_stream_t stream) {
    if (!jac || !fwd_out || !g_loss_grad || n_cols < 1 || b < 1 || per_sample < 1)
        return SMMD_EINVAL;
    if (b_total < 1) b_total = b;
    if (!gx_unit || !gy_unit || !dX || !dY || m < 1 || n < 1 || d < 1) return SMMD_EINVAL;
    if (variant != 0 && variant != 1) return SMMD_EINVAL;
    if (variant == 1 && gfeat && (!feat || dof < 1)) return SMMD_EINVAL;
    const int64_t n_jac = (int64_t)n_cols * b * per_sample;
    const int vec = ((uintptr_t)jac % 16 == 0) && ((uintptr_t)gjac % 16 == 0);
    // without gjac (a generator step) only the small dX / dY loops run
    int64_t blocks = gjac ? (n_jac / 4 + 255) / 256 : ((int64_t)(m + n) * d + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    MmdBwdPart mp;
    mp.g_mmd2 = g_mmd2_grad;
    mp.gxu = gx_unit;
    mp.gyu = gy_unit;
    mp.nx = (int64_t)m * d;
    mp.ny = (int64_t)n * d;
    mp.dX = dX;
    mp.dY = dY;
    hipLaunchKernelGGL(scaled_loss_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, jac, n_jac, b_total, feat,
                       (int64_t)b * (dof > 0 ? dof : 0), dof, fwd_out, sc, variant, sqrt_scale,
                       g_loss_grad, nullptr, gjac, gfeat, vec, mp);
    return last_launch_status();
}

size_t smmd_opt_workspace_bytes(const int64_t *offsets, int n_tensors) {
    if (!offsets || n_tensors < 1) return 0;
    int64_t blocks = 0;
    for (int i = 0; i < n_tensors; ++i) blocks += opt_blocks(offsets[i + 1] - offsets[i], OPT_SQ_CHUNK);
    return align_up((size_t)blocks * sizeof(double) + 256, 256);
}

smmd_status smmd_clip_by_norm_flat(float *grad, const int64_t *offsets, int n_tensors,
                                   float clip_norm, void *ws, size_t ws_bytes,
                                   smmd_stream_t stream) {
    if (!grad || !offsets || n_tensors < 1 || !(clip_norm > 0.f)) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_opt_workspace_bytes(offsets, n_tensors)) return SMMD_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    for (int first = 0; first < n_tensors; first += OPT_MAX) {
        const int count = (n_tensors - first < OPT_MAX) ? n_tensors - first : OPT_MAX;
        OptTable ts, tu;
        if (!build_opt(offsets, first, count, OPT_SQ_CHUNK, ts) ||
            !build_opt(offsets, first, count, OPT_UP_CHUNK, tu))
            return SMMD_EINVAL;
        const int vec = opt_vec(offsets + first, count, grad, grad, grad, grad);
        hipLaunchKernelGGL(opt_sqsum_kernel, dim3(ts.total_blocks), dim3(256), 0, s, ts,
                           (const float *)grad, 1.f, vec, (double *)ws);
        hipLaunchKernelGGL(opt_clip_kernel, dim3(tu.total_blocks), dim3(256), 0, s, tu, grad,
                           (const double *)ws, clip_norm, vec);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

// tf.train.AdamOptimizer: lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t)
static double adam_lr_t(float lr, float beta1, float beta2, int64_t step) {
    return (double)lr * sqrt(1.0 - pow((double)beta2, (double)step)) /
           (1.0 - pow((double)beta1, (double)step));
}

static smmd_status adam_flat_impl(float *param, const float *grad, float *m, float *v,
                                  const int64_t *offsets, int n_tensors, float grad_scale,
                                  float clip_norm, double lr_t, const float *lr_t_dev,
                                  float beta1, float beta2, float eps, void *ws, size_t ws_bytes,
                                  hipStream_t s) {
    if (!param || !grad || !m || !v || !offsets || n_tensors < 1) return SMMD_EINVAL;
    if (clip_norm > 0.f && (!ws || ws_bytes < smmd_opt_workspace_bytes(offsets, n_tensors)))
        return SMMD_EWORKSPACE;
    for (int first = 0; first < n_tensors; first += OPT_MAX) {
        const int count = (n_tensors - first < OPT_MAX) ? n_tensors - first : OPT_MAX;
        OptTable ts, tu;
        if (!build_opt(offsets, first, count, OPT_SQ_CHUNK, ts) ||
            !build_opt(offsets, first, count, OPT_UP_CHUNK, tu))
            return SMMD_EINVAL;
        const int vec = opt_vec(offsets + first, count, param, grad, m, v);
        if (clip_norm > 0.f)
            hipLaunchKernelGGL(opt_sqsum_kernel, dim3(ts.total_blocks), dim3(256), 0, s, ts, grad,
                               grad_scale, vec, (double *)ws);
        AdamArgs aa = adam_args(param, grad, m, v, ws, grad_scale, clip_norm, lr_t, beta1, beta2,
                                eps, vec);
        aa.lr_t_dev = lr_t_dev;
        hipLaunchKernelGGL(opt_adam_kernel, dim3(tu.total_blocks), dim3(256), 0, s, tu, aa);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

smmd_status smmd_adam_flat(float *param, const float *grad, float *m, float *v,
                           const int64_t *offsets, int n_tensors, float grad_scale,
                           float clip_norm, float lr, float beta1, float beta2, float eps,
                           int64_t step, void *ws, size_t ws_bytes, smmd_stream_t stream) {
    if (step < 1) return SMMD_EINVAL;
    return adam_flat_impl(param, grad, m, v, offsets, n_tensors, grad_scale, clip_norm,
                          adam_lr_t(lr, beta1, beta2, step), nullptr, beta1, beta2, eps, ws,
                          ws_bytes, (hipStream_t)stream);
}

static smmd_status adam_flat_sn_impl(float *param, const float *grad, float *m, float *v,
                                     const int64_t *offsets, int n_tensors, float grad_scale,
                                     float clip_norm, double lr_t, const float *lr_t_dev,
                                     float beta1, float beta2, float eps, void *ws,
                                     size_t ws_bytes, const smmd_sn_layer *layers,
                                     const int32_t *sn_tensor, int n_layers, void *sn_ws,
                                     size_t sn_ws_bytes, hipStream_t s, int gdirect = 0) {
    if (!param || !grad || !m || !v || !offsets || n_tensors < 1) return SMMD_EINVAL;
    if (!layers || !sn_tensor || n_layers < 1 || n_layers > SMMD_SN_MAX_LAYERS) return SMMD_EINVAL;
    if (n_tensors > OPT_MAX) return SMMD_EUNSUPPORTED;     // one partial slab for every tensor
    if (clip_norm > 0.f && (!ws || ws_bytes < smmd_opt_workspace_bytes(offsets, n_tensors)))
        return SMMD_EWORKSPACE;
    unsigned char skip[OPT_MAX] = {0};
    for (int i = 0; i < n_layers; ++i) {
        const int ti = sn_tensor[i];
        if (ti < 0 || ti >= n_tensors || skip[ti]) return SMMD_EINVAL;
        skip[ti] = 1;
    }
    OptTable ts, tu;
    // G-direct: the SN tensors' norms come from their grad-stats records, so
    // the norm pass skips them too (their flat gradient is never formed)
    if (!build_opt(offsets, 0, n_tensors, OPT_SQ_CHUNK, ts, gdirect ? skip : nullptr) ||
        !build_opt(offsets, 0, n_tensors, OPT_UP_CHUNK, tu, skip))
        return SMMD_EINVAL;
    const int vec = opt_vec(offsets, n_tensors, param, grad, m, v);
    SnAdamHost h;
    h.param = param;
    h.m = m;
    h.v = v;
    h.grad = grad;
    h.offsets = offsets;
    h.sblk = ts.sblk;
    h.gdirect = gdirect;
    SnAdamTable snt;
    const smmd_status r = sn_adam_table(layers, sn_tensor, n_layers, h, sn_ws, sn_ws_bytes, snt);
    if (r != SMMD_OK) return r;
    // G-direct with every other tensor within one update block (the critics'
    // biases and scales): each block sums its tensor's norm itself and the
    // norm-pass launch goes away
    int inblock = gdirect;
    for (int i = 0; i < n_tensors && inblock; ++i)
        if (!skip[i] && offsets[i + 1] - offsets[i] > OPT_UP_CHUNK) inblock = 0;
    if (clip_norm > 0.f && !inblock)
        hipLaunchKernelGGL(opt_sqsum_kernel, dim3(ts.total_blocks), dim3(256), 0, s, ts, grad,
                           grad_scale, vec, (double *)ws);
    AdamArgs aa = adam_args(param, grad, m, v, ws, grad_scale, clip_norm, lr_t, beta1, beta2, eps,
                            vec);
    aa.lr_t_dev = lr_t_dev;
    aa.norm_inblock = inblock;
    const dim3 grid(snt.total_tiles + tu.total_blocks);
    const int hg = sn_adam_groups();
    if (gdirect) {     // H = 2: the fold staging of H = 1 would not fit beside it
        hipLaunchKernelGGL((opt_adam_sn_kernel<2, true>), grid, dim3(256), 0, s, tu, snt, aa);
        return last_launch_status();
    }
    if (hg == 1)
        hipLaunchKernelGGL(opt_adam_sn_kernel<1>, grid, dim3(256), 0, s, tu, snt, aa);
    else if (hg == 4)
        hipLaunchKernelGGL(opt_adam_sn_kernel<4>, grid, dim3(256), 0, s, tu, snt, aa);
    else
        hipLaunchKernelGGL(opt_adam_sn_kernel<2>, grid, dim3(256), 0, s, tu, snt, aa);
    return last_launch_status();
}

smmd_status smmd_adam_flat_sn(float *param, const float *grad, float *m, float *v,
                              const int64_t *offsets, int n_tensors, float grad_scale,
                              float clip_norm, float lr, float beta1, float beta2, float eps,
                              int64_t step, void *ws, size_t ws_bytes,
                              const smmd_sn_layer *layers, const int32_t *sn_tensor,
                              int n_layers, void *sn_ws, size_t sn_ws_bytes,
                              smmd_stream_t stream) {
    if (step < 1) return SMMD_EINVAL;
    return adam_flat_sn_impl(param, grad, m, v, offsets, n_tensors, grad_scale, clip_norm,
                             adam_lr_t(lr, beta1, beta2, step), nullptr, beta1, beta2, eps, ws,
                             ws_bytes, layers, sn_tensor, n_layers, sn_ws, sn_ws_bytes,
                             (hipStream_t)stream);
}

smmd_status smmd_adam_flat_ex(float *param, const float *grad, float *m, float *v,
                              const int64_t *offsets, int n_tensors, float grad_scale,
                              float clip_norm, const float *lr_t, float beta1, float beta2,
                              float eps, void *ws, size_t ws_bytes,
                              const smmd_sn_layer *layers, const int32_t *sn_tensor,
                              int n_layers, void *sn_ws, size_t sn_ws_bytes,
                              smmd_stream_t stream) {
    if (!lr_t) return SMMD_EINVAL;
    if (n_layers == 0)
        return adam_flat_impl(param, grad, m, v, offsets, n_tensors, grad_scale, clip_norm, 0.0,
                              lr_t, beta1, beta2, eps, ws, ws_bytes, (hipStream_t)stream);
    return adam_flat_sn_impl(param, grad, m, v, offsets, n_tensors, grad_scale, clip_norm, 0.0,
                             lr_t, beta1, beta2, eps, ws, ws_bytes, layers, sn_tensor, n_layers,
                             sn_ws, sn_ws_bytes, (hipStream_t)stream);
}

smmd_status smmd_adam_flat_sn2(float *param, const float *grad, float *m, float *v,
                               const int64_t *offsets, int n_tensors, float grad_scale,
                               float clip_norm, float lr, float beta1, float beta2, float eps,
                               int64_t step, const float *lr_t, void *ws, size_t ws_bytes,
                               const smmd_sn_layer *layers, const int32_t *sn_tensor,
                               int n_layers, void *sn_ws, size_t sn_ws_bytes, int flags,
                               smmd_stream_t stream) {
    if (flags & ~SMMD_ADAM_SN_GDIRECT) return SMMD_EINVAL;
    if (!lr_t && step < 1) return SMMD_EINVAL;
    return adam_flat_sn_impl(param, grad, m, v, offsets, n_tensors, grad_scale, clip_norm,
                             lr_t ? 0.0 : adam_lr_t(lr, beta1, beta2, step), lr_t, beta1, beta2,
                             eps, ws, ws_bytes, layers, sn_tensor, n_layers, sn_ws, sn_ws_bytes,
                             (hipStream_t)stream, (flags & SMMD_ADAM_SN_GDIRECT) ? 1 : 0);
}

}  // extern "C"
