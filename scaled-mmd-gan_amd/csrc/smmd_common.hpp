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

inline smmd_status hip_status(hipError_t e) {
    return e == hipSuccess ? SMMD_OK : SMMD_EHIP;
}

inline smmd_status last_launch_status() {
    return hip_status(hipGetLastError());
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace smmd
