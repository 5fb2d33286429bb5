// smmd_mmd_tile.hip -- fused pairwise MMD^2 + unit gradient on a 2-D grid of
// (64-row tile) x (column chunk) workgroups, for feature widths d <= 8 (the
// configs' d = 1 above all).
//
// Reference: gan/core/mmd.py:18-188 (kernels), :194-220 (estimator) and TF's
// autodiff of them.
//
// Layout.  A workgroup is 4 waves.  Lane l of every wave owns local row
// r = 64 * tile + l of Z = [X rows; Y rows]; wave w sweeps its own run of
// `cpw` columns of the chunk, so a workgroup covers 64 rows x 4 cpw columns.
// The column loop index is wave-uniform, so a column's features are scalar
// loads (8 columns per s_load, the next batch in flight while this one is
// computed) and every lane evaluates K(z_r, z_c) with the column in SGPRs:
// no LDS, no cross-lane traffic inside the sweep.  Per-row gradient
// accumulators are reduced over the 4 waves in LDS (fixed order w0..w3),
// published per chunk write-through to a slab, and the last-arriving chunk of
// each row tile sums the chunks in chunk order (CDNA4 guide G16: sc1 stores,
// drain, ticket, acquire).  Block sums go up the same two levels (chunk ->
// row tile -> all), each level one load per lane and a fixed butterfly.
// Deterministic: every sum has a fixed order whatever the arrival order.
//
// Kernel evaluation: the Gaussian and rational-quadratic families take fast
// forms with the term count a template constant (parameters in SGPRs):
// exp(c R) = exp2(c log2(e) R) on v_exp_f32, (1 + R / (2a))^-a =
// exp2(-a log2(1 + R / (2a))) on v_log_f32 / v_exp_f32, and the derivative's
// division by q as one v_rcp_f32 (about 1 ulp each; the parity tests hold
// them to the oracle at the fp32 tolerances).
#include "smmd_common.hpp"
#include "smmd_kern.hpp"
#include "smmd_scale_dev.hpp"

#include <stdlib.h>

namespace smmd {

constexpr int TILE_ROWS = 64;
constexpr int TILE_WAVES = 4;

template <int DT>
__device__ __forceinline__ float tdot(const float (&a)[DT], const float (&b)[DT]) {
    float s = a[0] * b[0];
#pragma unroll
    for (int k = 1; k < DT; ++k) s = fmaf(a[k], b[k], s);
    return s;
}

// Per pair: K, and (al, be) with dK/dz_i = al z_i + be (z_i - z_j).
// NT > 0: Gaussian / RQ mixture of NT terms in the fast form; NT == 0: the
// shared evaluator of smmd_kern.hpp (runtime term count; distance, dot).
template <int KIND, int NT>
struct PairEval {
    float p0[NT > 0 ? NT : 1], p1[NT > 0 ? NT : 1], p2[NT > 0 ? NT : 1];
    float add_dot;
    __device__ __forceinline__ void init(const KParams &kp) {
        add_dot = kp.add_dot;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            if (KIND == SMMD_KIND_RBF) {
                p0[t] = kp.c1[t] * 1.4426950408889634f;   // -gamma log2(e)
                p1[t] = kp.wt[t];
                p2[t] = 2.f * kp.c1[t];                   // d/draw, x2 (d raw / d z)
            } else {
                p0[t] = 1.f / kp.c1[t];                   // 1 / (2 alpha)
                p1[t] = kp.c2[t];                         // -alpha
                p2[t] = kp.wt[t];
            }
        }
    }
    __device__ __forceinline__ void eval(const KParams &kp, float raw, float dot, float sqi,
                                         float sqc, float &K, float &al, float &be) const {
        if (NT == 0) {
            Kern<KIND>::eval(kp, raw, dot, sqi, sqc, K, al, be);
        } else if (KIND == SMMD_KIND_RBF) {     // mmd.py:55-116
            const float R = fmaxf(raw, 0.f);
            float k = 0.f, dk = 0.f;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float e = p1[t] * __builtin_amdgcn_exp2f(p0[t] * R);
                k += e;
                dk = fmaf(p2[t], e, dk);
            }
            K = k;
            al = 0.f;
            be = (raw >= 0.f) ? dk : 0.f;         // tf.maximum: ties pass the gradient
        } else {                                  // RQ, mmd.py:143-188
            const float R = fmaxf(raw, 0.f);
            float k = 0.f, dk = 0.f;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float q = fmaf(R, p0[t], 1.f);
                const float e = p2[t] * __builtin_amdgcn_exp2f(p1[t] * __builtin_amdgcn_logf(q));
                k += e;
                // d e / dR = e * (-alpha) / (q * 2 alpha)
                dk = fmaf(e * (p1[t] * p0[t]), __builtin_amdgcn_rcpf(q), dk);
            }
            if (add_dot > 0.f) k = fmaf(add_dot, dot, k);
            K = k;
            al = add_dot;
            be = ((raw >= 0.f) ? 2.f * dk : 0.f) - add_dot;
        }
    }
};

template <int DT, bool TANH>
__device__ __forceinline__ void load_cols(const float *__restrict__ S, int dd, int j,
                                          float (&zb)[8][DT]) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int k = 0; k < DT; ++k) zb[u][k] = (k < dd) ? S[(size_t)(j + u) * dd + k] : 0.f;
}

// One column range [j0, j1) of one side (X or Y columns).  The column index
// is wave-uniform, so the column features are scalar loads: 8 columns per
// batch, the next batch's load issued before this batch is evaluated.
template <int DT, int KIND, int NT, bool TANH, bool GRAD>
__device__ __forceinline__ void sweep(const KParams &kp, const PairEval<KIND, NT> &pe,
                                      const float *__restrict__ S, int d, int j0, int j1,
                                      const float (&zi)[DT], float sqi, float w, float &sumK,
                                      float &aacc, float (&acc)[DT]) {
    const int dd = (DT == 1) ? 1 : d;
    auto pair = [&](const float (&zc0)[DT]) {
        float zc[DT];
#pragma unroll
        for (int k = 0; k < DT; ++k) zc[k] = TANH ? tanhf(zc0[k]) : zc0[k];
        const float sqc = tdot<DT>(zc, zc);
        const float dot = tdot<DT>(zi, zc);
        const float raw = (-2.f * dot + sqi) + sqc;      // mmd.py:67 order
        float K, al, be;
        pe.eval(kp, raw, dot, sqi, sqc, K, al, be);
        sumK += K;
        if (GRAD) {
            if (KIND != SMMD_KIND_RBF) aacc = fmaf(w, al, aacc);
            const float c = w * be;
#pragma unroll
            for (int k = 0; k < DT; ++k) acc[k] = fmaf(c, zi[k] - zc[k], acc[k]);
        }
    };
    int j = j0;
    if (j + 8 <= j1) {
        float nb[8][DT];
        load_cols<DT, TANH>(S, dd, j, nb);
        for (; j + 8 <= j1; j += 8) {
            float cb[8][DT];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int k = 0; k < DT; ++k) cb[u][k] = nb[u][k];
            if (j + 16 <= j1) load_cols<DT, TANH>(S, dd, j + 8, nb);
#pragma unroll
            for (int u = 0; u < 8; ++u) pair(cb[u]);
        }
    }
    for (; j < j1; ++j) {
        float zc[DT];
#pragma unroll
        for (int k = 0; k < DT; ++k) zc[k] = (k < dd) ? S[(size_t)j * dd + k] : 0.f;
        pair(zc);
    }
}

// lane 0 publishes a 6-double record write-through (one lane, constant
// indices: a per-lane pick would index S dynamically and put it in scratch)
__device__ __forceinline__ void publish6(double *rec, const double (&S)[6], int lane) {
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) store_wt(rec + k, S[k]);
    }
}

// (no private arrays may be indexed by a lane-dependent value here: the
// compiler then moves them to LDS, addressed through the dispatch packet --
// a scalar load from the host-side queue measured at ~10 us per launch)
// The body of workgroup `bid` of the grid.  FUSED (the SMMD loss launch
// below): every workgroup publishes its sums record (lane 0 of wave 0,
// write-through) and no grid ticket is taken here -- the launch's loss ticket
// collects the records; the row tiles' gradient tickets work as usual.
template <int DT, int KIND, int NT, bool TANH, bool GRAD, bool FUSED = false>
__device__ __forceinline__ void mmd2_tile_body(const TileArgs &a, const float *__restrict__ X,
                                               const float *__restrict__ Y, int bid) {
    constexpr int NV = DT + 1;                 // acc[DT], aacc
    __shared__ float lds_v[TILE_WAVES][NV][TILE_ROWS];
    __shared__ double lds_s[TILE_WAVES][6];
    __shared__ double lds_s2[TILE_WAVES][6];
    __shared__ int lds_flag[2];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ch = bid % a.n_ch;               // column chunk
    const int rt = bid / a.n_ch;               // row tile
    const int r = rt * TILE_ROWS + lane;
    const bool active = r < a.nrows;
    const bool isx = r < a.nxr;
    const int ri = isx ? a.x_begin + r : a.y_begin + (r - a.nxr);
    PairEval<KIND, NT> pe;
    pe.init(a.kp);

    float zi[DT];
#pragma unroll
    for (int k = 0; k < DT; ++k) zi[k] = 0.f;
    if (active) {
        const float *p = (isx ? X : Y) + (size_t)ri * a.d;
#pragma unroll
        for (int k = 0; k < DT; ++k) zi[k] = (k < a.d) ? p[k] : 0.f;
        if (TANH) {
#pragma unroll
            for (int k = 0; k < DT; ++k) zi[k] = tanhf(zi[k]);
        }
    }
    const float sqi = tdot<DT>(zi, zi);
    const float wX = isx ? a.gw_same_x : a.gw_cross;    // weight of an X column
    const float wY = isx ? a.gw_cross : a.gw_same_y;    // weight of a Y column

    // this wave's columns: [c0, c1) of the global column list [X; Y]
    const int c0 = (ch * TILE_WAVES + w) * a.cpw;
    const int c1 = min(c0 + a.cpw, a.m + a.n);
    float sX = 0.f, sY = 0.f, tr = 0.f, aacc = 0.f;
    float acc[DT];
#pragma unroll
    for (int k = 0; k < DT; ++k) acc[k] = 0.f;
    if (c0 < c1) {
        const int xe = min(c1, a.m);
        if (c0 < xe)
            sweep<DT, KIND, NT, TANH, GRAD>(a.kp, pe, X, a.d, c0, xe, zi, sqi, wX, sX, aacc, acc);
        const int ys = max(c0, a.m);
        if (ys < c1)
            sweep<DT, KIND, NT, TANH, GRAD>(a.kp, pe, Y, a.d, ys - a.m, c1 - a.m, zi, sqi, wY, sY,
                                            aacc, acc);
        // the diagonal pair of this row, if its column is in this run: the
        // trace, and (trace mode) its gradient term taken back out
        const int dcol = isx ? ri : a.m + ri;
        if (active && dcol >= c0 && dcol < c1) {
            const float dot = tdot<DT>(zi, zi);
            const float raw = (-2.f * dot + sqi) + sqi;
            float K, al, be;
            pe.eval(a.kp, raw, dot, sqi, sqi, K, al, be);
            tr = K;
            if (GRAD && a.trace_mode) aacc = fmaf(-(isx ? wX : wY), al, aacc);
        }
    }
    if (!active) { sX = sY = tr = aacc = 0.f; }

    // ---- reduce the 4 waves: sums (double, w0..w3) and per-row values -----
    {
        // S = {s_xx, s_xy, s_yy, t_xx, t_yy, s_yx}
        float v6[6] = {isx ? sX : 0.f, isx ? sY : 0.f, isx ? 0.f : sY,
                       isx ? tr : 0.f, isx ? 0.f : tr, isx ? 0.f : sX};
#pragma unroll
        for (int k = 0; k < 6; ++k) v6[k] = wave_sum(v6[k]);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) lds_s[w][k] = (double)v6[k];
        }
        if (GRAD) {
#pragma unroll
            for (int k = 0; k < DT; ++k) lds_v[w][k][lane] = acc[k];
            lds_v[w][DT][lane] = aacc;
        }
    }
    __syncthreads();
    double S[6];
    float v[NV];
#pragma unroll
    for (int k = 0; k < 6; ++k) S[k] = ((lds_s[0][k] + lds_s[1][k]) + lds_s[2][k]) + lds_s[3][k];
    if (GRAD) {
#pragma unroll
        for (int k = 0; k < NV; ++k)
            v[k] = ((lds_v[0][k][lane] + lds_v[1][k][lane]) + lds_v[2][k][lane]) +
                   lds_v[3][k][lane];
    }
    const int nb = a.n_rt * a.n_ch;
    // the row tile's ticket exists only when there are gradients to gather
    // over several chunks; every counter taken is reset by its last taker
    const bool rt_ticket = GRAD && a.n_ch > 1;
    bool rt_last = GRAD, g_last = !FUSED;
    if (FUSED) {
        // the sums record for the loss ticket's last taker; the row tile's
        // gradient ticket as below
        if (w == 0) {
            if (rt_ticket) {
#pragma unroll
                for (int k = 0; k < NV; ++k)
                    store_wt(a.part + ((size_t)ch * NV + k) * a.rows_pad + r, v[k]);
            }
            publish6(a.blk_sums + (size_t)bid * 8, S, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            unsigned prev = 0;
            if (lane == 0 && rt_ticket)
                prev = __hip_atomic_fetch_add(a.rt_counter + rt, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
            prev = __shfl(prev, 0, SMMD_WAVE);
            if (lane == 0) lds_flag[0] = GRAD && (!rt_ticket || prev == (unsigned)a.n_ch - 1);
        }
        __syncthreads();
        rt_last = lds_flag[0] != 0;
        if (!rt_last) return;
        if (rt_ticket) acquire_block();
    } else if (nb > 1) {
        // publish (wave 0): this chunk's per-row partials and the block's sums,
        // write-through; drain; then BOTH tickets at once -- the row tile's
        // (lane 0) and the whole grid's (lane 1) -- so the gradient and the
        // estimator reductions run side by side, not one after the other
        if (w == 0) {
            if (rt_ticket) {
#pragma unroll
                for (int k = 0; k < NV; ++k)
                    store_wt(a.part + ((size_t)ch * NV + k) * a.rows_pad + r, v[k]);
            }
            publish6(a.blk_sums + (size_t)bid * 8, S, lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            unsigned prev = 0;
            if (lane == 0 && rt_ticket)
                prev = __hip_atomic_fetch_add(a.rt_counter + rt, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 1)
                prev = __hip_atomic_fetch_add(a.g_counter, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
            const unsigned p_rt = __shfl(prev, 0, SMMD_WAVE), p_g = __shfl(prev, 1, SMMD_WAVE);
            if (lane == 0) {
                lds_flag[0] = GRAD && (!rt_ticket || p_rt == (unsigned)a.n_ch - 1);
                lds_flag[1] = p_g == (unsigned)nb - 1;
            }
        }
        __syncthreads();
        rt_last = lds_flag[0] != 0;
        g_last = lds_flag[1] != 0;
        if (!rt_last && !g_last) return;
        acquire_block();                       // every wave reads other blocks' data
    }

    if (!FUSED && g_last && nb > 1) {          // 256 threads over the block records
        double tt[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        for (int b = threadIdx.x; b < nb; b += TILE_ROWS * TILE_WAVES) {
#pragma unroll
            for (int k = 0; k < 6; ++k) tt[k] += a.blk_sums[(size_t)b * 8 + k];
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) tt[k] = wave_sum(tt[k]);
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) lds_s2[w][k] = tt[k];
        }
    }
    if (!FUSED && nb > 1) __syncthreads();

    // the row tile's last chunk: its rows' gradients, chunks summed in order
    if (w == 0 && rt_last) {
        if (rt_ticket) {
#pragma unroll
            for (int k = 0; k < NV; ++k) v[k] = 0.f;
            int c = 0;
            for (; c + 4 <= a.n_ch; c += 4) {      // 4 chunks' loads in flight
                float q[4][NV];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < NV; ++k)
                        q[u][k] = a.part[((size_t)(c + u) * NV + k) * a.rows_pad + r];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int k = 0; k < NV; ++k) v[k] += q[u][k];
            }
            for (; c < a.n_ch; ++c) {
#pragma unroll
                for (int k = 0; k < NV; ++k) v[k] += a.part[((size_t)c * NV + k) * a.rows_pad + r];
            }
            if (lane == 0)
                __hip_atomic_store(a.rt_counter + rt, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (GRAD && active) {
            float *gp = isx ? a.grad_x + (size_t)r * a.d : a.grad_y + (size_t)(r - a.nxr) * a.d;
#pragma unroll
            for (int k = 0; k < DT; ++k) {
                if (k < a.d) {
                    float gk = fmaf(v[DT], zi[k], v[k]);
                    if (TANH) gk *= 1.f - zi[k] * zi[k];
                    gp[k] = gk;
                }
            }
        }
    }

    // the grid's last block: the estimator from every block's sums
    if (!FUSED && w == 0 && g_last && lane == 0) {
        if (nb > 1) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                S[k] = ((lds_s2[0][k] + lds_s2[1][k]) + lds_s2[2][k]) + lds_s2[3][k];
            __hip_atomic_store(a.g_counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (a.out_sums) {
#pragma unroll
            for (int k = 0; k < 6; ++k) store_wt(a.out_sums + k, (float)S[k]);
            store_wt(a.out_sums + 6, 0.f);
            store_wt(a.out_sums + 7, 0.f);
        }
        if (a.out_mmd2)
            store_wt(a.out_mmd2, (float)estimator(S, (double)a.m, (double)a.n, a.biased,
                                                  a.has_const, a.const_diag));
    }
}

template <int DT, int KIND, int NT, bool TANH, bool GRAD>
__global__ __launch_bounds__(TILE_ROWS * TILE_WAVES) void mmd2_tile_kernel(
    TileArgs a, const float *__restrict__ X, const float *__restrict__ Y) {
    mmd2_tile_body<DT, KIND, NT, TANH, GRAD>(a, X, Y, blockIdx.x);
}

// The scaled SMMD loss in ONE launch (smmd_smmd_loss_fwd): workgroups
// [0, nb) run the MMD^2 tile sweep above, the rest the Jacobian's
// squared-norm partials (smmd_scale_dev.hpp); every workgroup publishes its
// record and takes the ONE loss ticket, and its last taker forms the
// estimator from the nb sums records (the order of the unfused grid's last
// block), then the scaled-loss finalize with base = that estimator.  Two
// dependent launches with two ticket levels each become one launch with one.
template <int DT, int KIND, int NT, bool TANH, bool GRAD>
__global__ __launch_bounds__(TILE_ROWS * TILE_WAVES) void smmd_loss_kernel(
    TileArgs a, const float *__restrict__ X, const float *__restrict__ Y, ScaledLossArgs q) {
    static_assert(TILE_ROWS * TILE_WAVES == 256, "the norm blocks are 256 threads");
    const int nb = a.n_rt * a.n_ch;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ int last;
    if ((int)blockIdx.x < nb) {
        mmd2_tile_body<DT, KIND, NT, TANH, GRAD, true>(a, X, Y, blockIdx.x);
    } else {
        const int blk = blockIdx.x - nb;
        const double s = sqnorm_block(q, blk);
        if (threadIdx.x == 0) store_wt(q.part + blk, s);
    }
    if (w == 0) {                              // the wave whose lane 0 published
        const int l = wave_ticket(q.counter, gridDim.x);
        if (lane == 0) last = l;
    }
    __syncthreads();
    if (!last) return;
    // The last taker.  Every record and partial it reads was stored
    // write-through (sc1) by one lane of its workgroup, drained, then that
    // lane added to this ONE counter: with sc1 loads of every handed-off byte
    // no agent acquire is needed (MI355X_MICROARCH hand-off table, row 1; an
    // acquire costs ~1.7 us).  Records and partials are loaded together, all
    // in flight before the first use; past one pass of either, the acquire
    // and plain loads as usual.
    const int tot = q.n_cols * q.b * q.nchunk;
    const bool fast = nb <= TILE_ROWS * TILE_WAVES && tot <= SQ_FIN_LDS;
    __shared__ double pl[SQ_FIN_LDS];
    __shared__ double s2[TILE_WAVES][6];
    __shared__ float base;
    double tt[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (fast) {
        const int tid = threadIdx.x;
        if (tid < nb) {
#pragma unroll
            for (int k = 0; k < 6; ++k)
                tt[k] = __hip_atomic_load(a.blk_sums + (size_t)tid * 8 + k, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
        }
        double t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int i = tid + j * 256;
            t[j] = (i < tot) ? __hip_atomic_load(q.part + i, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0.0;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (tid + j * 256 < tot) pl[tid + j * 256] = t[j];
    } else {
        acquire_block();
        for (int b = threadIdx.x; b < nb; b += TILE_ROWS * TILE_WAVES) {
#pragma unroll
            for (int k = 0; k < 6; ++k) tt[k] += a.blk_sums[(size_t)b * 8 + k];
        }
    }
    // the estimator: the records summed as the unfused grid's last block does
#pragma unroll
    for (int k = 0; k < 6; ++k) tt[k] = wave_sum(tt[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) s2[w][k] = tt[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double S[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) S[k] = ((s2[0][k] + s2[1][k]) + s2[2][k]) + s2[3][k];
        if (a.out_sums) {
#pragma unroll
            for (int k = 0; k < 6; ++k) a.out_sums[k] = (float)S[k];
            a.out_sums[6] = 0.f;
            a.out_sums[7] = 0.f;
        }
        const float e = (float)estimator(S, (double)a.m, (double)a.n, a.biased, a.has_const,
                                         a.const_diag);
        a.out_mmd2[0] = e;
        base = e;
    }
    __syncthreads();
    scaled_loss_final(q, base, fast ? pl : nullptr);
    ticket_reset(q.counter);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// Grid: 64-row tiles x column chunks of 4 runs of cpw columns.  Aim for ~512
// workgroups (2048 waves, 8 per CU) on large problems, but give every wave at
// least 32 columns: below that the per-chunk publish and the reductions cost
// more than the sweep (tools/hip/mmd_abi_bench.cpp on MI355X, rbf fwd + grad,
// 2 x 2048 rows: 18.7 us at 512 workgroups, 22.6 at 1024, 34 at 2048).
// SMMD_TILE_BLOCKS / SMMD_TILE_MINCPW override both (tuning runs).
constexpr int TILE_TARGET_BLOCKS = 512;
constexpr int TILE_MIN_CPW = 32;
// The fused loss launch at small N (<= 256 rows): the sweep is on its
// critical path while the row tiles' gradient combines are not (nothing in
// the launch waits for them), so columns go 8 per wave: 4x the waves
constexpr int TILE_FUSED_MIN_CPW = 8;
constexpr int TILE_FUSED_SMALL_ROWS = 256;

static int env_int(const char *k, int dflt) {
    const char *e = getenv(k);
    return (e && e[0]) ? atoi(e) : dflt;
}

static void tile_shape(int rows, int cols, int &n_rt, int &n_ch, int &cpw, int min_cpw) {
    n_rt = (rows + TILE_ROWS - 1) / TILE_ROWS;
    int mincpw = env_int("SMMD_TILE_MINCPW", min_cpw);
    if (mincpw < min_cpw) mincpw = min_cpw;
    const int max_ch = (cols + TILE_WAVES * mincpw - 1) / (TILE_WAVES * mincpw);
    const int target = env_int("SMMD_TILE_BLOCKS", TILE_TARGET_BLOCKS);
    int ch = (target + n_rt - 1) / n_rt;
    if (ch > max_ch) ch = max_ch;
    if (ch < 1) ch = 1;
    cpw = (cols + TILE_WAVES * ch - 1) / (TILE_WAVES * ch);
    cpw = (cpw + 7) / 8 * 8;                    // whole 8-column batches
    n_ch = (cols + TILE_WAVES * cpw - 1) / (TILE_WAVES * cpw);
}

static int tile_dt(int d) {
    if (d <= 1) return 1;
    if (d <= 2) return 2;
    if (d <= 4) return 4;
    if (d <= 8) return 8;
    return 0;
}

bool tile_supported(int d) { return tile_dt(d) != 0; }

size_t tile_ws_bytes(int rows, int cols, int d) {
    const int dt = tile_dt(d);
    if (!dt) return 0;
    // a bound over every local row count <= rows (the row-sharded calls):
    // tile_shape never gives more tiles or chunks than these
    const int n_rt = (rows + TILE_ROWS - 1) / TILE_ROWS;
    int n_ch = (cols + TILE_WAVES * TILE_MIN_CPW - 1) / (TILE_WAVES * TILE_MIN_CPW);
    if (rows <= TILE_FUSED_SMALL_ROWS)          // the fused loss launch's finer split
        n_ch = (cols + TILE_WAVES * TILE_FUSED_MIN_CPW - 1) / (TILE_WAVES * TILE_FUSED_MIN_CPW);
    const size_t rows_pad = (size_t)n_rt * TILE_ROWS;
    size_t b = align_up((size_t)n_rt * n_ch * 8 * sizeof(double), 256);
    b += align_up((size_t)n_ch * (dt + 1) * rows_pad * sizeof(float), 256);
    return b;
}

template <int DT, int KIND, int NT>
static void launch_tile_k(const TileArgs &a, hipStream_t s, const ScaledLossArgs *q) {
    const dim3 block(TILE_ROWS * TILE_WAVES);
    if (q) {                                   // the fused SMMD loss (with gradient)
        const dim3 grid(a.n_rt * a.n_ch + q->nblocks);
        if (a.tanh_in)
            hipLaunchKernelGGL((smmd_loss_kernel<DT, KIND, NT, true, true>), grid, block, 0, s, a, a.X, a.Y, *q);
        else
            hipLaunchKernelGGL((smmd_loss_kernel<DT, KIND, NT, false, true>), grid, block, 0, s, a, a.X, a.Y, *q);
        return;
    }
    const dim3 grid(a.n_rt * a.n_ch);
    if (a.tanh_in) {
        if (a.need_grad)
            hipLaunchKernelGGL((mmd2_tile_kernel<DT, KIND, NT, true, true>), grid, block, 0, s, a, a.X, a.Y);
        else
            hipLaunchKernelGGL((mmd2_tile_kernel<DT, KIND, NT, true, false>), grid, block, 0, s, a, a.X, a.Y);
    } else {
        if (a.need_grad)
            hipLaunchKernelGGL((mmd2_tile_kernel<DT, KIND, NT, false, true>), grid, block, 0, s, a, a.X, a.Y);
        else
            hipLaunchKernelGGL((mmd2_tile_kernel<DT, KIND, NT, false, false>), grid, block, 0, s, a, a.X, a.Y);
    }
}

// term counts with a compiled fast form: rbf (1), mix_rq* (3), mix_rbf (6)
template <int DT, int KIND>
static void launch_tile_terms(const TileArgs &a, hipStream_t s, const ScaledLossArgs *q) {
    switch (a.kp.n_terms) {
        case 1: launch_tile_k<DT, KIND, 1>(a, s, q); break;
        case 3: launch_tile_k<DT, KIND, 3>(a, s, q); break;
        case 6: launch_tile_k<DT, KIND, 6>(a, s, q); break;
        default: launch_tile_k<DT, KIND, 0>(a, s, q); break;
    }
}

template <int DT>
static bool launch_tile_dt(const TileArgs &a, int kind, hipStream_t s, const ScaledLossArgs *q) {
    switch (kind) {
        case SMMD_KIND_RBF: launch_tile_terms<DT, SMMD_KIND_RBF>(a, s, q); return true;
        case SMMD_KIND_RQ: launch_tile_terms<DT, SMMD_KIND_RQ>(a, s, q); return true;
        case SMMD_KIND_DISTANCE: launch_tile_k<DT, SMMD_KIND_DISTANCE, 0>(a, s, q); return true;
        case SMMD_KIND_DOT: launch_tile_k<DT, SMMD_KIND_DOT, 0>(a, s, q); return true;
    }
    return false;
}

// ws: the whole workspace; counters in its header (g_counter = word 0,
// rt_counter from byte 256), data from MMD_WS_HEADER
smmd_status tile_mmd2_launch(TileArgs a, int kind, void *ws, hipStream_t s,
                             const ScaledLossArgs *q) {
    const int dt = tile_dt(a.d);
    if (!dt) return SMMD_EUNSUPPORTED;
    tile_shape(a.nrows, a.m + a.n, a.n_rt, a.n_ch, a.cpw,
               (q && a.nrows <= TILE_FUSED_SMALL_ROWS) ? TILE_FUSED_MIN_CPW : TILE_MIN_CPW);
    if (a.n_rt > TILE_MAX_RT) return SMMD_EUNSUPPORTED;
    a.rows_pad = a.n_rt * TILE_ROWS;
    a.g_counter = (unsigned *)ws;
    a.rt_counter = (unsigned *)((char *)ws + 256);
    char *p = (char *)ws + MMD_WS_HEADER;
    a.blk_sums = (double *)p;
    p += align_up((size_t)a.n_rt * a.n_ch * 8 * sizeof(double), 256);
    a.part = (float *)p;
    bool ok = false;
    if (q && (!a.need_grad || (int64_t)a.n_rt * a.n_ch + q->nblocks > 0x7fffffff))
        return SMMD_EINVAL;
    switch (dt) {
        case 1: ok = launch_tile_dt<1>(a, kind, s, q); break;
        case 2: ok = launch_tile_dt<2>(a, kind, s, q); break;
        case 4: ok = launch_tile_dt<4>(a, kind, s, q); break;
        case 8: ok = launch_tile_dt<8>(a, kind, s, q); break;
    }
    if (!ok) return SMMD_EINVAL;
    return last_launch_status();
}

}  // namespace smmd
