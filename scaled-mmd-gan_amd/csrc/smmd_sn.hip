// smmd_sn.hip -- spectral normalisation of every SN layer of a network in one
// set of launches (gfx950 / MI355X).
//
// Reference: gan/core/sn.py:12-59 (power iteration, sigma, W_bar = W/sigma),
// gan/core/snops.py:82-84 (W_eff = s * W_bar), their TF autodiff (backward).
// The TF graph runs ~8 small ops per layer per discriminator call (2 GEMV,
// 2 norms, sigma, RealDiv, Mul, assign).  Here all layers are cut into
// 32 x 256 fp32 tiles (32 KiB) and one launch walks every tile of every layer:
//
//   P1  tile -> partial column sums  sum_rows u_n W[n, k]     (HBM pass 1)
//   P2  tile -> v_raw for its 256 columns from the P1 slab, then partial row
//       dots sum_cols v_raw_k W[n, k]                          (HBM pass 2,
//       usually served by the Infinity Cache: the net fits in 256 MiB)
//   R2  one block per layer: ||v_raw||, v, u_raw, ||u_raw||, u', sigma
//   P3  tile -> W_eff = (W / sigma) * s                        (read + write)
//
// Lanes own 4 consecutive columns (16-byte loads), waves own 8 rows, so a
// wave-instruction reads 1 KiB of one row.  All reductions have a fixed order.
//
// Measured alternative (not kept): P1 electing the last row tile of each column
// tile to reduce v_raw, and P2 electing the last tile of each layer to run R2
// (arrival tickets, write-through partials).  It removes the R2 launch but puts
// each reducer's serial chain of dependent L2 loads at the tail of its kernel:
// P1 11 -> 19 us, P2 + R2 20 -> 34 us on the SNResNet-64 critic.
#include "smmd_sn_tile.hpp"

#include <atomic>
#include <stdlib.h>

namespace smmd {

struct SnLayerDev {
    const float *W;
    float *W_eff;
    float *u;        // user u (read at iteration 0, written when update_u)
    float *v;
    float *sigma;
    const float *s;
    const float *G;
    float *gW;
    float *gs;
    float *p1;       // ws [nrt][K]
    float *vraw;     // ws [K]
    float *q2;       // ws [N][nctp] row partials, one contiguous 16-B aligned row per n
    float *ucur;     // ws [N]  u' of the last iteration
    float *dotp;     // ws [ntiles] backward partial <G, W>
    int N, K, nrt, nct;
    int nctp;        // nct rounded up to a multiple of 4
    int tile_begin;
    int vec;         // K % 4 == 0 and 16-byte aligned rows
};

struct SnTable {
    int n_layers;
    int total_tiles;
    int iter;        // current power iteration (0 -> read layer.u)
    int last_iter;
    int update_u;
    float eps;
    SnLayerDev L[SN_CHUNK];
};

// Layer of a tile: static-index scan of the (monotone) tile_begin fields, then
// readfirstlane so the index is provably wave-uniform and the descriptor is
// read with scalar loads instead of a dependent chain of vector loads.
__device__ __forceinline__ int find_layer(const SnTable &t, int tile) {
    int l = 0;
#pragma unroll
    for (int i = 1; i < SN_CHUNK; ++i)
        l += (i < t.n_layers && tile >= t.L[i].tile_begin) ? 1 : 0;
    return __builtin_amdgcn_readfirstlane(l);
}

__global__ __launch_bounds__(256) void sn_p1_kernel(SnTable t) {
    const int tile = blockIdx.x;
    const SnLayerDev L = t.L[find_layer(t, tile)];
    const int lt = tile - L.tile_begin;
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    const float *uin = (t.iter == 0) ? L.u : L.ucur;
    float4 wt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);
    p1_tile(uin, L.p1, L.N, L.K, rt, r0, c0, wt);
}

__global__ __launch_bounds__(256) void sn_p2_kernel(SnTable t) {
    const int tile = blockIdx.x;
    const SnLayerDev L = t.L[find_layer(t, tile)];
    const int lt = tile - L.tile_begin;
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;

    float4 wt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);   // issue the tile loads first

    // v_raw for this tile's columns: fixed-order sum over row tiles of P1
    __shared__ float vr[SN_TC];
    {
        const int c = ct * SN_TC + threadIdx.x;
        float s = 0.f;
        if (c < L.K) {
#pragma unroll 4
            for (int r = 0; r < L.nrt; ++r) s += L.p1[(size_t)r * L.K + c];
        }
        vr[threadIdx.x] = s;
        if (rt == 0 && c < L.K) L.vraw[c] = s;
    }
    __syncthreads();
    const float v0 = vr[lane * 4 + 0], v1 = vr[lane * 4 + 1];
    const float v2 = vr[lane * 4 + 2], v3 = vr[lane * 4 + 3];
    float part[SN_RPW];
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i)
        part[i] = fmaf(v3, wt[i].w, fmaf(v2, wt[i].z, fmaf(v1, wt[i].y, v0 * wt[i].x)));
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) part[i] = wave_sum(part[i]);
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < SN_RPW; ++i)
            if (r0 + i < L.N) L.q2[(size_t)(r0 + i) * L.nctp + ct] = part[i];
    }
}

// u_raw[n] * ||v_raw|| = sum over column tiles c < nct of q2[n][c], in order.
// The row is contiguous and 16-B aligned, so all of its loads are issued
// before the first add (the [nct][N] layout cost one L2 round trip per pair).
__device__ __forceinline__ float q2_row_sum(const SnLayerDev &L, int n) {
    const float4 *q = reinterpret_cast<const float4 *>(L.q2 + (size_t)n * L.nctp);
    const int n4 = L.nctp >> 2;
    float s = 0.f;
    for (int j0 = 0; j0 < n4; j0 += 8) {
        float4 b[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            b[j] = (j0 + j < n4) ? q[j0 + j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = (j0 + j) * 4;
            if (c + 0 < L.nct) s += b[j].x;
            if (c + 1 < L.nct) s += b[j].y;
            if (c + 2 < L.nct) s += b[j].z;
            if (c + 3 < L.nct) s += b[j].w;
        }
    }
    return s;
}

// norms, v, u', sigma of one layer (sn.py:12-13, :38-42) by one 1024-thread
// block, from v_raw [K] and the row partials q2.  With r_n = (W v_raw)_n:
//   nv = ||v_raw|| + eps, u_raw = r / nv, nu = ||u_raw|| + eps,
//   u' = u_raw / nu, sigma = u_raw . u' = ||u_raw||^2 / nu.
// Every input is loaded up front and the two norms share ONE block
// reduction (||u_raw||^2 = sum r_n^2 / nv^2), so the block makes one round
// of dependent global loads instead of four.
constexpr int EP_KREG = 8;    // v_raw values per thread kept in registers (K <= 8192)
constexpr int EP_NREG = 2;    // rows per thread kept in registers (N <= 2048)

__device__ void sn_layer_epilogue(const SnTable &t, const SnLayerDev &L, int last_iter,
                                  double *red) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float vr[EP_KREG], rs[EP_NREG];
#pragma unroll
    for (int j = 0; j < EP_KREG; ++j) {
        const int k = tid + j * 1024;
        vr[j] = (k < L.K) ? L.vraw[k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < EP_NREG; ++j) {
        const int n = tid + j * 1024;
        rs[j] = (n < L.N) ? q2_row_sum(L, n) : 0.f;
    }
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int j = 0; j < EP_KREG; ++j) a += (double)vr[j] * (double)vr[j];
    for (int k = tid + EP_KREG * 1024; k < L.K; k += 1024) {
        const double x = (double)L.vraw[k];
        a += x * x;
    }
#pragma unroll
    for (int j = 0; j < EP_NREG; ++j) b += (double)rs[j] * (double)rs[j];
    for (int n = tid + EP_NREG * 1024; n < L.N; n += 1024) {      // rare: N > 2048
        const float r = q2_row_sum(L, n);
        L.ucur[n] = r;
        b += (double)r * (double)r;
    }
    a = wave_sum(a);
    b = wave_sum(b);
    __syncthreads();
    if (lane == 0) {
        red[w] = a;
        red[16 + w] = b;
    }
    __syncthreads();
    double sa = 0.0, sb = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        sa += red[i];
        sb += red[16 + i];
    }
    const float nv = (float)sqrt(sa) + t.eps;                   // sn.py:13
    const double uu = sb / ((double)nv * (double)nv);           // ||u_raw||^2
    const float nu = (float)sqrt(uu) + t.eps;
#pragma unroll
    for (int j = 0; j < EP_KREG; ++j) {
        const int k = tid + j * 1024;
        if (k < L.K) L.v[k] = vr[j] / nv;
    }
    for (int k = tid + EP_KREG * 1024; k < L.K; k += 1024) L.v[k] = L.vraw[k] / nv;
    const bool upd = t.update_u && last_iter;
#pragma unroll
    for (int j = 0; j < EP_NREG; ++j) {
        const int n = tid + j * 1024;
        if (n < L.N) {
            const float un = (rs[j] / nv) / nu;                 // u' = l2n(v W)
            L.ucur[n] = un;
            if (upd) L.u[n] = un;
        }
    }
    for (int n = tid + EP_NREG * 1024; n < L.N; n += 1024) {
        const float un = (L.ucur[n] / nv) / nu;
        L.ucur[n] = un;
        if (upd) L.u[n] = un;
    }
    if (tid == 0) L.sigma[0] = (float)(uu / (double)nu);     // (v W) . u', sn.py:42
}

// R2: one 1024-thread block per layer runs the epilogue
__global__ __launch_bounds__(1024) void sn_r2_kernel(SnTable t) {
    __shared__ double red[32];
    sn_layer_epilogue(t, t.L[blockIdx.x], t.last_iter, red);
}

__global__ __launch_bounds__(256) void sn_p3_kernel(SnTable t) {
    const int tile = blockIdx.x;
    const SnLayerDev L = t.L[find_layer(t, tile)];
    if (!L.W_eff) return;
    const int lt = tile - L.tile_begin;
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    const float sigma = L.sigma[0];
    const float s = L.s ? L.s[0] : 1.f;
    float4 wt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);
    const bool full_cols = (c0 + 3 < L.K);
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) {
        const int r = r0 + i;
        if (r >= L.N) break;
        // W_bar = W / sigma (sn.py:43), then s * W_bar (snops.py:84)
        float4 o;
        o.x = (wt[i].x / sigma) * s;
        o.y = (wt[i].y / sigma) * s;
        o.z = (wt[i].z / sigma) * s;
        o.w = (wt[i].w / sigma) * s;
        float *p = L.W_eff + (size_t)r * L.K + c0;
        if (L.vec && full_cols) {
            *reinterpret_cast<float4 *>(p) = o;
        } else {
            if (c0 + 0 < L.K) p[0] = o.x;
            if (c0 + 1 < L.K) p[1] = o.y;
            if (c0 + 2 < L.K) p[2] = o.z;
            if (c0 + 3 < L.K) p[3] = o.w;
        }
    }
}

// backward A: partial <G, W> per tile
__global__ __launch_bounds__(256) void sn_bwd_a_kernel(SnTable t) {
    const int tile = blockIdx.x;
    const SnLayerDev L = t.L[find_layer(t, tile)];
    const int lt = tile - L.tile_begin;
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    float4 wt[SN_RPW], gt[SN_RPW];
    load_tile(L.W, L.N, L.K, L.vec, r0, c0, wt);
    load_tile(L.G, L.N, L.K, L.vec, r0, c0, gt);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) {
        acc = fmaf(gt[i].x, wt[i].x, acc);
        acc = fmaf(gt[i].y, wt[i].y, acc);
        acc = fmaf(gt[i].z, wt[i].z, acc);
        acc = fmaf(gt[i].w, wt[i].w, acc);
    }
    __shared__ float red[4];
    acc = block_sum<4>(acc, red);
    if (threadIdx.x == 0) L.dotp[lt] = acc;
}

// backward B: gW = (s G)/sigma - (s <G,W> / sigma^2) u' v^T ; gs = <G,W>/sigma
__global__ __launch_bounds__(256) void sn_bwd_b_kernel(SnTable t) {
    const int tile = blockIdx.x;
    const SnLayerDev L = t.L[find_layer(t, tile)];
    const int lt = tile - L.tile_begin;
    const int rt = lt / L.nct, ct = lt % L.nct;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r0 = rt * SN_TR + w * SN_RPW;
    const int c0 = ct * SN_TC + lane * 4;
    float4 gt[SN_RPW];
    load_tile(L.G, L.N, L.K, L.vec, r0, c0, gt);
    __shared__ float sh_d;
    if (w == 0) {
        const int nt = L.nrt * L.nct;
        double d = 0.0;
        for (int i = lane; i < nt; i += 64) d += (double)L.dotp[i];
        d = wave_sum(d);
        if (lane == 0) sh_d = (float)d;
    }
    __syncthreads();
    const float d = sh_d;                         // <G, W>
    const float sigma = L.sigma[0];
    const float s = L.s ? L.s[0] : 1.f;
    if (lt == 0 && threadIdx.x == 0 && L.gs) L.gs[0] = d / sigma;
    const float coef = (s * d) / (sigma * sigma);  // -dsigma factor
    float vv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) vv[k] = (c0 + k < L.K) ? L.v[c0 + k] : 0.f;
    const bool full_cols = (c0 + 3 < L.K);
#pragma unroll
    for (int i = 0; i < SN_RPW; ++i) {
        const int r = r0 + i;
        if (r >= L.N) break;
        const float cu = coef * L.ucur[r];
        float4 o;
        o.x = (s * gt[i].x) / sigma - cu * vv[0];
        o.y = (s * gt[i].y) / sigma - cu * vv[1];
        o.z = (s * gt[i].z) / sigma - cu * vv[2];
        o.w = (s * gt[i].w) / sigma - cu * vv[3];
        float *p = L.gW + (size_t)r * L.K + c0;
        if (L.vec && full_cols) {
            *reinterpret_cast<float4 *>(p) = o;
        } else {
            if (c0 + 0 < L.K) p[0] = o.x;
            if (c0 + 1 < L.K) p[1] = o.y;
            if (c0 + 2 < L.K) p[2] = o.z;
            if (c0 + 3 < L.K) p[3] = o.w;
        }
    }
}

// ---------------------------------------------------------------------------
// Resident path: one cooperative launch per call.  Every workgroup (one per
// CU, 1024 threads) loads its share of 32 x 256 tiles of every layer ONCE into
// registers and keeps them across the phases of the power iteration, which
// are separated by grid barriers:
//
//   A   resident tiles -> column partials (LDS reduce of the 16 waves) -> P1
//   A2  P1 -> v_raw, 256-column chunks spread over the grid
//   B   resident tiles . v_raw -> per-row partials q2
//   R   one workgroup per layer: the sn_r2 epilogue (norms, v, u', sigma)
//   C   resident tiles -> W_eff = (W / sigma) * s
//
// HBM traffic: one read of W and one write of W_eff (8 B per weight) instead
// of the three reads + one write of the P1/P2/P3 launch set.  The backward
// reads G and W once (the <G, W> partials), keeps G, and writes gW after one
// barrier: 12 B per weight instead of 20.
// ---------------------------------------------------------------------------
constexpr int SR_TR = 32;            // tile rows (thread: rows w and w + 16)
constexpr int SR_THREADS = 1024;
constexpr int SR_TMAX = 8;           // resident tiles per workgroup
constexpr int SR_GROUP = 4;          // tiles per LDS reduction round (64 KiB)
constexpr unsigned SR_SPIN_LIMIT = 1u << 22;   // ~0.2 s of polling, then give up

struct GridBarrier {
    unsigned count;   // arrivals of the current barrier (returns to 0)
    unsigned gen;     // completed barriers (monotone, wraps)
    unsigned err;     // set when a barrier timed out (grid not co-resident)
    unsigned pad;
};

// Self-resetting grid barrier for a cooperative (co-resident) launch.  The
// last arriver resets `count` and bumps `gen`; the others poll `gen`.  A
// bounded poll guarantees termination even if co-residency were violated.
__device__ __forceinline__ void grid_sync(GridBarrier *b, unsigned nblocks) {
    // every wave's global stores must have reached L2 before thread 0 writes
    // the L2 back (__syncthreads alone does not wait for vmcnt)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = __hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old =
            __hip_atomic_fetch_add(&b->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == nblocks - 1) {
            __hip_atomic_store(&b->count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&b->gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            unsigned spins = 0;
            while (__hip_atomic_load(&b->gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > SR_SPIN_LIMIT) {
                    __hip_atomic_store(&b->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

// Phase timestamps (s_memrealtime, 100 MHz) of blocks 0 and G-1 in the spare
// bytes of the 256-byte workspace header: u64 slots 2+i (block 0) and 16+i
// (last block).  One store per phase per block; read by tools/diag_sn_phases.py.
#define SR_STAMP(bar, i)                                                            \
    do {                                                                            \
        if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))   \
            reinterpret_cast<unsigned long long *>(bar)[(blockIdx.x ? 16 : 2) + (i)] = \
                __builtin_amdgcn_s_memrealtime();                                   \
    } while (0)

struct SrTile {
    int layer, rt, ct;
};

__device__ __forceinline__ SrTile sr_tile(const SnTable &t, int tile) {
    SrTile o;
    o.layer = find_layer(t, tile);
    const int lt = tile - t.L[o.layer].tile_begin;
    const int nct = t.L[o.layer].nct;
    o.rt = lt / nct;
    o.ct = lt - o.rt * nct;
    return o;
}

// raw buffer over [p, p + bytes): out-of-range loads return 0 without a branch
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sr_rsrc(const void *p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes,
                                             0x00020000);
}

__device__ __forceinline__ float4 sr_bload4(__amdgpu_buffer_rsrc_t r, int elem) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, elem * 4, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                       __uint_as_float(v.w));
}

// rows r0 and r0 + 16 of a tile, 4 columns at c0 (zero outside the matrix).
// vec layers (K % 4 == 0): two unconditional buffer loads (rows >= N are out of
// range and read 0; a float4 never straddles a row end), columns >= K masked.
__device__ __forceinline__ void sr_load(const float *__restrict__ base, int N, int K, int vec,
                                        int r0, int c0, float4 &a, float4 &b) {
    const int r1 = r0 + 16;
    if (vec) {
        const __amdgpu_buffer_rsrc_t rs = sr_rsrc(base, (unsigned)N * (unsigned)K * 4u);
        const float4 x = sr_bload4(rs, r0 * K + c0), y = sr_bload4(rs, r1 * K + c0);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        a = (c0 < K) ? x : z;
        b = (c0 < K) ? y : z;
        return;
    }
    float x[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (c0 + k < K) {
            if (r0 < N) x[k] = base[(size_t)r0 * K + c0 + k];
            if (r1 < N) x[4 + k] = base[(size_t)r1 * K + c0 + k];
        }
    }
    a = make_float4(x[0], x[1], x[2], x[3]);
    b = make_float4(x[4], x[5], x[6], x[7]);
}

__device__ __forceinline__ void sr_store(float *__restrict__ base, int N, int K, int vec, int r,
                                         int c0, float4 o) {
    if (r >= N) return;
    float *p = base + (size_t)r * K + c0;
    if (vec && c0 + 3 < K) {
        *reinterpret_cast<float4 *>(p) = o;
        return;
    }
    if (c0 + 0 < K) p[0] = o.x;
    if (c0 + 1 < K) p[1] = o.y;
    if (c0 + 2 < K) p[2] = o.z;
    if (c0 + 3 < K) p[3] = o.w;
}

// tile j of this block (strided over the grid), or false past the end
#define SR_FOR_TILES(j, q, L)                                                    \
    for (int j = 0; j < SR_TMAX; ++j)                                            \
        if (const int tile_ = blockIdx.x + j * gridDim.x; tile_ < t.total_tiles) \
            if (const SrTile q = sr_tile(t, tile_); true)                        \
                if (const SnLayerDev &L = t.L[q.layer]; true)

__global__ __launch_bounds__(SR_THREADS) void sn_resident_kernel(SnTable t, GridBarrier *bar,
                                                                 int num_iters) {
    const unsigned G = gridDim.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ float red[SR_GROUP][16][SN_TC];
    __shared__ double dred[32];

    SR_STAMP(bar, 0);
    float4 wa[SR_TMAX], wb[SR_TMAX];
#pragma unroll
    for (int j = 0; j < SR_TMAX; ++j) wa[j] = wb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    SR_FOR_TILES(j, q, L) {
        sr_load(L.W, L.N, L.K, L.vec, q.rt * SR_TR + w, q.ct * SN_TC + lane * 4, wa[j], wb[j]);
    }

    for (int it = 0; it < num_iters; ++it) {
        // ---- A: column partials of u^T W over the tile's 32 rows -> P1
#pragma unroll
        for (int g0 = 0; g0 < SR_TMAX; g0 += SR_GROUP) {
#pragma unroll
            for (int jj = 0; jj < SR_GROUP && g0 + jj < SR_TMAX; ++jj) {
                const int j = g0 + jj;
                const int tile = blockIdx.x + j * G;
                if (tile >= t.total_tiles) break;
                const SrTile q = sr_tile(t, tile);
                const SnLayerDev &L = t.L[q.layer];
                const float *uin = (it == 0) ? L.u : L.ucur;
                const int r0 = q.rt * SR_TR + w, r1 = r0 + 16;
                const float u0 = (r0 < L.N) ? uin[r0] : 0.f;
                const float u1 = (r1 < L.N) ? uin[r1] : 0.f;
                float4 acc;
                acc.x = fmaf(u1, wb[j].x, u0 * wa[j].x);
                acc.y = fmaf(u1, wb[j].y, u0 * wa[j].y);
                acc.z = fmaf(u1, wb[j].z, u0 * wa[j].z);
                acc.w = fmaf(u1, wb[j].w, u0 * wa[j].w);
                *reinterpret_cast<float4 *>(&red[jj][w][lane * 4]) = acc;
            }
            __syncthreads();
            {
                const int jj = threadIdx.x >> 8, c = threadIdx.x & 255;
                const int tile = blockIdx.x + (g0 + jj) * G;
                if (g0 + jj < SR_TMAX && tile < t.total_tiles) {
                    const SrTile q = sr_tile(t, tile);
                    const SnLayerDev &L = t.L[q.layer];
                    const int col = q.ct * SN_TC + c;
                    float s = 0.f;
#pragma unroll
                    for (int i = 0; i < 16; ++i) s += red[jj][i][c];
                    if (col < L.K) L.p1[(size_t)q.rt * L.K + col] = s;
                }
            }
            __syncthreads();
        }
        if (it == 0) SR_STAMP(bar, 1);
        grid_sync(bar, G);
        if (it == 0) SR_STAMP(bar, 2);

        // ---- A2: v_raw = sum over row tiles of P1; 256-column chunks, 4 per block
        for (int qi = blockIdx.x * 4 + (threadIdx.x >> 8); ; qi += G * 4) {
            int l = 0, cb = 0;
            for (; l < t.n_layers; ++l) {
                if (qi < cb + t.L[l].nct) break;
                cb += t.L[l].nct;
            }
            if (l >= t.n_layers) break;
            const SnLayerDev &L = t.L[l];
            const int col = (qi - cb) * SN_TC + (threadIdx.x & 255);
            if (col < L.K) {
                float s = 0.f;
#pragma unroll 8
                for (int r = 0; r < L.nrt; ++r) s += L.p1[(size_t)r * L.K + col];
                L.vraw[col] = s;
            }
        }
        if (it == 0) SR_STAMP(bar, 3);
        grid_sync(bar, G);
        if (it == 0) SR_STAMP(bar, 4);

        // ---- B: per-row partial dots with v_raw -> q2[row][ct]
#pragma unroll
        SR_FOR_TILES(j, q, L) {
            const int c0 = q.ct * SN_TC + lane * 4;
            const float v0 = (c0 + 0 < L.K) ? L.vraw[c0 + 0] : 0.f;
            const float v1 = (c0 + 1 < L.K) ? L.vraw[c0 + 1] : 0.f;
            const float v2 = (c0 + 2 < L.K) ? L.vraw[c0 + 2] : 0.f;
            const float v3 = (c0 + 3 < L.K) ? L.vraw[c0 + 3] : 0.f;
            float d0 = fmaf(v3, wa[j].w, fmaf(v2, wa[j].z, fmaf(v1, wa[j].y, v0 * wa[j].x)));
            float d1 = fmaf(v3, wb[j].w, fmaf(v2, wb[j].z, fmaf(v1, wb[j].y, v0 * wb[j].x)));
            d0 = wave_sum(d0);
            d1 = wave_sum(d1);
            if (lane == 0) {
                const int r0 = q.rt * SR_TR + w, r1 = r0 + 16;
                if (r0 < L.N) L.q2[(size_t)r0 * L.nctp + q.ct] = d0;
                if (r1 < L.N) L.q2[(size_t)r1 * L.nctp + q.ct] = d1;
            }
        }
        if (it == 0) SR_STAMP(bar, 5);
        grid_sync(bar, G);
        if (it == 0) SR_STAMP(bar, 6);

        // ---- R: norms, v, u', sigma (one workgroup per layer)
        const int last = (it == num_iters - 1);
        for (int l = blockIdx.x; l < t.n_layers; l += G) sn_layer_epilogue(t, t.L[l], last, dred);
        if (it == 0) SR_STAMP(bar, 7);
        grid_sync(bar, G);
        if (it == 0) SR_STAMP(bar, 8);
    }

    // ---- C: W_eff = (W / sigma) * s from the resident tiles
#pragma unroll
    SR_FOR_TILES(j, q, L) {
        if (!L.W_eff) continue;
        const float sigma = L.sigma[0];
        const float s = L.s ? L.s[0] : 1.f;
        const int r0 = q.rt * SR_TR + w, c0 = q.ct * SN_TC + lane * 4;
        float4 o;
        o.x = (wa[j].x / sigma) * s; o.y = (wa[j].y / sigma) * s;
        o.z = (wa[j].z / sigma) * s; o.w = (wa[j].w / sigma) * s;
        sr_store(L.W_eff, L.N, L.K, L.vec, r0, c0, o);
        o.x = (wb[j].x / sigma) * s; o.y = (wb[j].y / sigma) * s;
        o.z = (wb[j].z / sigma) * s; o.w = (wb[j].w / sigma) * s;
        sr_store(L.W_eff, L.N, L.K, L.vec, r0 + 16, c0, o);
    }
    SR_STAMP(bar, 9);
}

// backward: <G, W> partial per tile -> barrier -> per-layer sum (fixed order,
// every block redoes it for its layers) -> gW from the resident G tiles
__global__ __launch_bounds__(SR_THREADS) void sn_resident_bwd_kernel(SnTable t, GridBarrier *bar) {
    const unsigned G = gridDim.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ float dsh[SR_TMAX][16];
    __shared__ float dlay[SR_TMAX];

    float4 ga[SR_TMAX], gb[SR_TMAX];
#pragma unroll
    for (int j = 0; j < SR_TMAX; ++j) ga[j] = gb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    SR_FOR_TILES(j, q, L) {
        const int r0 = q.rt * SR_TR + w, c0 = q.ct * SN_TC + lane * 4;
        float4 wa, wb;
        sr_load(L.W, L.N, L.K, L.vec, r0, c0, wa, wb);
        sr_load(L.G, L.N, L.K, L.vec, r0, c0, ga[j], gb[j]);
        float acc = 0.f;
        acc = fmaf(ga[j].x, wa.x, acc); acc = fmaf(ga[j].y, wa.y, acc);
        acc = fmaf(ga[j].z, wa.z, acc); acc = fmaf(ga[j].w, wa.w, acc);
        acc = fmaf(gb[j].x, wb.x, acc); acc = fmaf(gb[j].y, wb.y, acc);
        acc = fmaf(gb[j].z, wb.z, acc); acc = fmaf(gb[j].w, wb.w, acc);
        acc = wave_sum(acc);
        if (lane == 0) dsh[j][w] = acc;
    }
    __syncthreads();
    // wave j publishes tile j's partial (sr_tile needs a wave-uniform tile)
    if (w < SR_TMAX) {
        const int j = w;
        const int tile = blockIdx.x + j * G;
        if (tile < t.total_tiles && lane == 0) {
            const SrTile q = sr_tile(t, tile);
            float s = 0.f;
            for (int i = 0; i < 16; ++i) s += dsh[j][i];
            t.L[q.layer].dotp[tile - t.L[q.layer].tile_begin] = s;
        }
    }
    grid_sync(bar, G);

    // per-layer <G, W>: wave j sums the dotp of tile j's layer (fixed order)
    if (w < SR_TMAX) {
        const int j = w;
        const int tile = blockIdx.x + j * G;
        if (tile < t.total_tiles) {
            const SrTile q = sr_tile(t, tile);
            const SnLayerDev &L = t.L[q.layer];
            const int nt = L.nrt * L.nct;
            double d = 0.0;
            for (int i = lane; i < nt; i += 64) d += (double)L.dotp[i];
            d = wave_sum(d);
            if (lane == 0) dlay[j] = (float)d;
        }
    }
    __syncthreads();
#pragma unroll
    SR_FOR_TILES(j, q, L) {
        const float d = dlay[j];                      // <G, W>
        const float sigma = L.sigma[0];
        const float s = L.s ? L.s[0] : 1.f;
        const int r0 = q.rt * SR_TR + w, c0 = q.ct * SN_TC + lane * 4;
        if (q.rt == 0 && q.ct == 0 && threadIdx.x == 0 && L.gs) L.gs[0] = d / sigma;
        const float coef = (s * d) / (sigma * sigma);
        float vv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) vv[k] = (c0 + k < L.K) ? L.v[c0 + k] : 0.f;
        const float cu0 = (r0 < L.N) ? coef * L.ucur[r0] : 0.f;
        const float cu1 = (r0 + 16 < L.N) ? coef * L.ucur[r0 + 16] : 0.f;
        float4 o;
        o.x = (s * ga[j].x) / sigma - cu0 * vv[0];
        o.y = (s * ga[j].y) / sigma - cu0 * vv[1];
        o.z = (s * ga[j].z) / sigma - cu0 * vv[2];
        o.w = (s * ga[j].w) / sigma - cu0 * vv[3];
        sr_store(L.gW, L.N, L.K, L.vec, r0, c0, o);
        o.x = (s * gb[j].x) / sigma - cu1 * vv[0];
        o.y = (s * gb[j].y) / sigma - cu1 * vv[1];
        o.z = (s * gb[j].z) / sigma - cu1 * vv[2];
        o.w = (s * gb[j].w) / sigma - cu1 * vv[3];
        sr_store(L.gW, L.N, L.K, L.vec, r0 + 16, c0, o);
    }
}
#undef SR_FOR_TILES

// ---------------------------------------------------------------------------
// host side: workspace carve and launch sets
// ---------------------------------------------------------------------------
static int ceil_div(int a, int b) { return (a + b - 1) / b; }

static size_t layer_ws_bytes(int N, int K) {
    // P1 / dotp sized for the finer (resident) row tiling, which also covers SN_TR
    const int nrt = ceil_div(N, SR_TR), nct = ceil_div(K, SN_TC);
    size_t b = 0;
    b += align_up((size_t)nrt * K * 4, 256);   // p1
    b += align_up((size_t)K * 4, 256);         // vraw
    b += align_up((size_t)((nct + 3) & ~3) * N * 4, 256);   // q2
    b += align_up((size_t)N * 4, 256);         // ucur
    b += align_up((size_t)nrt * nct * 4, 256); // dotp
    return b;
}

static bool build_table(const smmd_sn_layer *layers, int first, int count, char *ws,
                        SnTable &t, int tile_rows) {
    memset(&t, 0, sizeof(t));
    t.n_layers = count;
    int tiles = 0;
    // every chunk gets the workspace region of its layers (by global index)
    size_t off = 0;
    for (int i = 0; i < first; ++i) off += layer_ws_bytes(layers[i].N, layers[i].K);
    for (int i = 0; i < count; ++i) {
        const smmd_sn_layer &src = layers[first + i];
        if (!src.W || src.N < 1 || src.K < 1) return false;
        SnLayerDev &L = t.L[i];
        L.W = src.W;
        L.W_eff = src.W_eff;
        L.u = src.u;
        L.v = src.v;
        L.sigma = src.sigma;
        L.s = src.s;
        L.G = src.G;
        L.gW = src.gW;
        L.gs = src.gs;
        L.N = src.N;
        L.K = src.K;
        L.nrt = ceil_div(src.N, tile_rows);
        L.nct = ceil_div(src.K, SN_TC);
        L.tile_begin = tiles;
        tiles += L.nrt * L.nct;
        const uintptr_t al = (uintptr_t)src.W | (uintptr_t)(src.W_eff ? src.W_eff : src.W) |
                             (uintptr_t)(src.G ? src.G : src.W) | (uintptr_t)(src.gW ? src.gW : src.W);
        L.vec = (src.K % 4 == 0) && (al % 16 == 0);
        char *p = ws + off;
        const int nrt_max = ceil_div(src.N, SR_TR);
        L.p1 = (float *)p;   p += align_up((size_t)nrt_max * L.K * 4, 256);
        L.vraw = (float *)p; p += align_up((size_t)L.K * 4, 256);
        L.nctp = (L.nct + 3) & ~3;
        L.q2 = (float *)p;   p += align_up((size_t)L.nctp * L.N * 4, 256);
        L.ucur = (float *)p; p += align_up((size_t)L.N * 4, 256);
        L.dotp = (float *)p; p += align_up((size_t)nrt_max * L.nct * 4, 256);
        off += layer_ws_bytes(L.N, L.K);
    }
    t.total_tiles = tiles;
    return true;
}

static bool coop_launch() {
    const char *e = getenv("SMMD_SN_COOP");
    return !(e && e[0] == '0');
}

// The resident path is opt-in (SMMD_SN_RESIDENT=1): on MI355X its four grid
// barriers cost 15-20 us each and the cooperative launch ~20 us, so the
// single-launch kernel (1 read + 1 write of W, 120 us measured on the
// SNResNet-64 critic) loses to the launch set (3 reads + 1 write, 54 us).
static bool resident_enabled() {
    const char *e = getenv("SMMD_SN_RESIDENT");
    return e && e[0] == '1';
}

// co-resident 1024-thread blocks of a resident kernel on the current device
// (cached per device: the only host state the library keeps)
template <typename K>
static int coresident_blocks(K kernel, int slot) {
    static std::atomic<int> cache[2][64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int v = cache[slot][dev].load(std::memory_order_relaxed);
    if (v) return v;
    int cus = 0, per_cu = 0, coop = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, SR_THREADS, 0) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    v = coop ? cus * per_cu : 0;
    cache[slot][dev].store(v > 0 ? v : -1, std::memory_order_relaxed);
    return v > 0 ? v : -1;
}

// grid for the resident path, or 0 when it does not apply (too many layers
// for one table, more tiles than the registers of the co-resident grid hold)
template <typename K>
static int resident_grid(K kernel, int slot, int n_layers, const SnTable &t) {
    if (n_layers > SN_CHUNK || !resident_enabled()) return 0;
    const int cap = coresident_blocks(kernel, slot);
    if (cap <= 0) return 0;
    const int g = t.total_tiles < cap ? t.total_tiles : cap;
    if ((long)g * SR_TMAX < (long)t.total_tiles) return 0;
    return g;
}

smmd_status sn_adam_table(const smmd_sn_layer *layers, const int32_t *sn_tensor, int n_layers,
                          const SnAdamHost &a, void *sn_ws, size_t sn_ws_bytes, SnAdamTable &t) {
    if (n_layers < 1 || n_layers > SN_CHUNK) return SMMD_EUNSUPPORTED;
    if (!sn_ws || sn_ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    SnTable st;
    if (!build_table(layers, 0, n_layers, (char *)sn_ws + 256, st, SN_TR)) return SMMD_EINVAL;
    memset(&t, 0, sizeof(t));
    t.n_layers = n_layers;
    t.total_tiles = st.total_tiles;
    for (int i = 0; i < n_layers; ++i) {
        const smmd_sn_layer &src = layers[i];
        const int ti = sn_tensor[i];
        const int64_t off = a.offsets[ti];
        // the SN weight must be tensor ti of the flat buffer, N x K rows
        if (!src.u || src.W != a.param + off || a.offsets[ti + 1] - off < (int64_t)src.N * src.K)
            return SMMD_EINVAL;
        SnAdamLayerDev &L = t.L[i];
        L.p = const_cast<float *>(a.param) + off;
        L.m = const_cast<float *>(a.m) + off;
        L.v = const_cast<float *>(a.v) + off;
        L.g = a.grad + off;
        L.u = src.u;
        L.p1 = st.L[i].p1;
        L.N = src.N;
        L.K = src.K;
        L.nct = st.L[i].nct;
        L.tile_begin = st.L[i].tile_begin;
        const uintptr_t al = (uintptr_t)L.p | (uintptr_t)L.m | (uintptr_t)L.v | (uintptr_t)L.g;
        L.vec = (src.K % 4 == 0) && (al % 16 == 0);
        L.sb0 = a.sblk[ti];
        L.sb1 = a.sblk[ti + 1];
    }
    return SMMD_OK;
}

}  // namespace smmd

using namespace smmd;

extern "C" {

size_t smmd_sn_workspace_bytes(const smmd_sn_layer *layers, int n_layers) {
    if (!layers || n_layers < 1) return 0;
    size_t b = 256;
    for (int i = 0; i < n_layers; ++i) b += layer_ws_bytes(layers[i].N, layers[i].K);
    return b;
}

smmd_status smmd_sn_power_iter(const smmd_sn_layer *layers, int n_layers, int num_iters,
                               float eps, int update_u, void *ws, size_t ws_bytes,
                               smmd_stream_t stream) {
    return smmd_sn_power_iter_ex(layers, n_layers, num_iters, eps, update_u, 0, ws, ws_bytes,
                                 stream);
}

smmd_status smmd_sn_power_iter_ex(const smmd_sn_layer *layers, int n_layers, int num_iters,
                                  float eps, int update_u, int flags, void *ws, size_t ws_bytes,
                                  smmd_stream_t stream) {
    if (flags & ~SMMD_SN_P1_READY) return SMMD_EINVAL;
    if (!layers || n_layers < 1 || n_layers > SMMD_SN_MAX_LAYERS || num_iters < 1)
        return SMMD_EINVAL;
    for (int i = 0; i < n_layers; ++i)
        if (!layers[i].u || !layers[i].v || !layers[i].sigma) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    {
        SnTable t;
        if (n_layers <= SN_CHUNK) {
            if (!build_table(layers, 0, n_layers, (char *)ws + 256, t, SR_TR)) return SMMD_EINVAL;
            const int g = resident_grid(sn_resident_kernel, 0, n_layers, t);
            if (g > 0) {
                t.eps = eps;
                t.update_u = update_u ? 1 : 0;
                GridBarrier *bar = (GridBarrier *)ws;
                void *args[] = {&t, &bar, &num_iters};
                if (!coop_launch()) {   // diagnostic: plain launch of the same grid
                    hipLaunchKernelGGL(sn_resident_kernel, dim3(g), dim3(SR_THREADS), 0, s, t,
                                       bar, num_iters);
                    return last_launch_status();
                }
                return hip_status(hipLaunchCooperativeKernel((const void *)sn_resident_kernel,
                                                             dim3(g), dim3(SR_THREADS), args, 0, s));
            }
        }
    }
    for (int first = 0; first < n_layers; first += SN_CHUNK) {
        const int count = (n_layers - first < SN_CHUNK) ? n_layers - first : SN_CHUNK;
        SnTable t;
        if (!build_table(layers, first, count, (char *)ws + 256, t, SN_TR)) return SMMD_EINVAL;
        t.eps = eps;
        t.update_u = update_u ? 1 : 0;
        for (int it = 0; it < num_iters; ++it) {
            t.iter = it;
            t.last_iter = (it == num_iters - 1);
            if (it > 0 || !(flags & SMMD_SN_P1_READY))   // else written by smmd_adam_flat_sn
                hipLaunchKernelGGL(sn_p1_kernel, dim3(t.total_tiles), dim3(256), 0, s, t);
            hipLaunchKernelGGL(sn_p2_kernel, dim3(t.total_tiles), dim3(256), 0, s, t);
            hipLaunchKernelGGL(sn_r2_kernel, dim3(t.n_layers), dim3(1024), 0, s, t);
        }
        bool any_eff = false;
        for (int i = 0; i < count; ++i) any_eff |= (t.L[i].W_eff != nullptr);
        if (any_eff) hipLaunchKernelGGL(sn_p3_kernel, dim3(t.total_tiles), dim3(256), 0, s, t);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

smmd_status smmd_sn_weight_bwd(const smmd_sn_layer *layers, int n_layers, void *ws,
                               size_t ws_bytes, smmd_stream_t stream) {
    if (!layers || n_layers < 1 || n_layers > SMMD_SN_MAX_LAYERS) return SMMD_EINVAL;
    for (int i = 0; i < n_layers; ++i)
        if (!layers[i].G || !layers[i].gW || !layers[i].v || !layers[i].sigma) return SMMD_EINVAL;
    if (!ws || ws_bytes < smmd_sn_workspace_bytes(layers, n_layers)) return SMMD_EWORKSPACE;
    hipStream_t s = (hipStream_t)stream;
    if (n_layers <= SN_CHUNK) {
        SnTable t;
        if (!build_table(layers, 0, n_layers, (char *)ws + 256, t, SR_TR)) return SMMD_EINVAL;
        const int g = resident_grid(sn_resident_bwd_kernel, 1, n_layers, t);
        if (g > 0) {
            GridBarrier *bar = (GridBarrier *)ws;
            void *args[] = {&t, &bar};
            return hip_status(hipLaunchCooperativeKernel((const void *)sn_resident_bwd_kernel,
                                                         dim3(g), dim3(SR_THREADS), args, 0, s));
        }
    }
    for (int first = 0; first < n_layers; first += SN_CHUNK) {
        const int count = (n_layers - first < SN_CHUNK) ? n_layers - first : SN_CHUNK;
        SnTable t;
        if (!build_table(layers, first, count, (char *)ws + 256, t, SN_TR)) return SMMD_EINVAL;
        hipLaunchKernelGGL(sn_bwd_a_kernel, dim3(t.total_tiles), dim3(256), 0, s, t);
        hipLaunchKernelGGL(sn_bwd_b_kernel, dim3(t.total_tiles), dim3(256), 0, s, t);
        smmd_status st = last_launch_status();
        if (st != SMMD_OK) return st;
    }
    return SMMD_OK;
}

}  // extern "C"
