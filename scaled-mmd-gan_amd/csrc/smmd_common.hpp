// smmd_common.hpp -- shared device helpers for libsmmd_hip.so (gfx950 only).
//
// Wave = 64 lanes on CDNA4; every reduction below is written for that width
// and uses a fixed butterfly order so results are bit-reproducible.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/smmd_hip.h"

#define SMMD_WAVE 64

namespace smmd {

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, SMMD_WAVE);
    return x;
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, SMMD_WAVE);
    return x;
}

// Sum of one float per thread over a block of NW waves; result valid in all
// threads.  `red` is LDS scratch of >= NW floats.  Fixed order.
template <int NW>
__device__ __forceinline__ float block_sum(float x, float *red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    x = wave_sum(x);
    __syncthreads();
    if (lane == 0) red[w] = x;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += red[i];
    return t;
}

template <int NW>
__device__ __forceinline__ double block_sum(double x, double *red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    x = wave_sum(x);
    __syncthreads();
    if (lane == 0) red[w] = x;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += red[i];
    return t;
}

// ---- in-launch hand-off to a last-arriving workgroup (CDNA4 guide G16) -----
// Producers store the published words WRITE-THROUGH (sc1: a relaxed
// agent-scope atomic store), so no release fence (an L2 write-back per block,
// which made a 1233-block pass 4x slower); the storing wave drains, then lane 0
// takes a ticket.  The last arriver acquires once and reads with plain loads.
__device__ __forceinline__ void store_wt(float *p, float x) {
    __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void store_wt(double *p, double x) {
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(p),
                       (unsigned long long)__double_as_longlong(x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Called by every lane of the one wave that made all the write-through stores
// being published.  Returns 1 in every lane for the arrivals-th arriver.
__device__ __forceinline__ int wave_ticket(unsigned *ctr, unsigned arrivals) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = 0;
    if ((threadIdx.x & 63) == 0)
        prev = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __shfl(prev, 0, SMMD_WAVE);
    return prev == arrivals - 1;
}

// Last arriver: one lane's agent-scope acquire (drops this CU's stale L1
// lines), its drain, then the barrier; afterwards every wave may load.
__device__ __forceinline__ void acquire_block() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

__device__ __forceinline__ void ticket_reset(unsigned *ctr) {
    if (threadIdx.x == 0) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tf.train.AdamOptimizer element update (Eigen ApplyAdam), shared by the flat
// optimizer and the SN-fused update so both give the same bits:
//   m += (g - m)(1-b1); v += (g^2 - v)(1-b2); var -= lr_t m / (sqrt(v) + eps)
// Every operation rounds on its own: with contraction on, the compiler fused
// different products into the subtractions in the two kernels (g has several
// uses), and the updates differed in the last bit from the second step on.
struct AdamK {
    float gscale, f, lr_t, b1c, b2c, eps;   // f: clip factor; b1c = 1 - b1, b2c = 1 - b2
    __device__ __forceinline__ void upd(float &p, float g, float &m, float &v) const {
#pragma clang fp contract(off)
        g = (g * gscale) * f;
        m += (g - m) * b1c;
        v += (g * g - v) * b2c;
        p -= (m * lr_t) / (sqrtf(v) + eps);
    }
};

// One lane's share of a fixed-order strided sum: s = sum over j ascending of
// x[i0 + j * stride] for i0 + j * stride < i1, accumulated in double.  The
// loads of each batch of 16 are all issued before the first add, so a slab
// just written by another XCD costs one memory round trip per 16 terms instead
// of one per term (the sum, and so the bits, are those of the plain loop).
template <typename T>
__device__ __forceinline__ double strided_sum(const T *__restrict__ x, int i0, int i1,
                                              int stride) {
    constexpr int B = 16;
    double s = 0.0;
    for (int base = i0; base < i1; base += B * stride) {
        T t[B];
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const int i = base + j * stride;
            t[j] = (i < i1) ? x[i] : T(0);
        }
#pragma unroll
        for (int j = 0; j < B; ++j)
            if (base + j * stride < i1) s += (double)t[j];
    }
    return s;
}

// clip factor of tf.clip_by_norm (TF 1.x form): clip * min(rsqrt(ss), 1/clip),
// ss = the norm pass's double partials [b0, b1) summed by wave 0 in a fixed
// order; every thread of the block gets it (sh: one float of LDS)
__device__ __forceinline__ float clip_factor_slab(const double *part, int b0, int b1, float clip,
                                                  float *sh) {
    if (threadIdx.x < 64) {
        double s = strided_sum(part, b0 + (int)threadIdx.x, b1, 64);
        s = wave_sum(s);
        if (threadIdx.x == 0) {
            const float ss = (float)s;
            const float inv = (ss > 0.f) ? rsqrtf(ss) : INFINITY;
            sh[0] = clip * fminf(inv, 1.f / clip);
        }
    }
    __syncthreads();
    return sh[0];
}

// Work item of block b in a 1-D grid of n blocks, XCD-aware: the dispatcher
// deals blocks round-robin to the 8 XCDs (b and b + 8 share one and its L2;
// MI355X_MICROARCH.md, dispatch), so XCD x takes the x-th contiguous range of
// the work order.  A bijection on [0, n) for any n; placement is only speed.
__device__ __forceinline__ int xcd_order(int b, int n) {
    const int q = n >> 3, r = n & 7, x = b & 7, i = b >> 3;
    return x * q + (x < r ? x : r) + i;
}

inline smmd_status hip_status(hipError_t e) {
    return e == hipSuccess ? SMMD_OK : SMMD_EHIP;
}

inline smmd_status last_launch_status() {
    return hip_status(hipGetLastError());
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace smmd
