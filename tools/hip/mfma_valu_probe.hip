// Does independent VALU work issue in the shadow of v_mfma_f32_32x32x2_f32
// (f32 in, 64 cycles per SIMD) on gfx950?  One wave per SIMD (256-thread
// blocks, one block per CU), a loop of 16 MFMAs on 4 accumulators with F
// independent v_add_f32 / v_fma_f32 fillers after each MFMA; cycles per MFMA
// from s_memtime around the loop (median over blocks).  Also the same with
// v_mfma_f32_32x32x1_2b_f32 is not needed: the question is the f32 pipe.
//
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/hip/mfma_valu_probe.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int F>
__global__ __launch_bounds__(256, 1) void probe(float *out, unsigned long long *cyc, int iters) {
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = f32x16{};
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    float f[8];
    for (int i = 0; i < 8; ++i) f[i] = a + i;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
            for (int k = 0; k < F; ++k) f[k & 7] = __builtin_fmaf(f[k & 7], 1.0001f, 0.5f);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 16; ++j) s += acc[i][j];
    for (int i = 0; i < 8; ++i) s += f[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// two waves per SIMD (512-thread blocks): waves 0-3 issue only the MFMAs,
// waves 4-7 only F fillers per slot; cycles of each group per slot
template <int F>
__global__ __launch_bounds__(512, 1) void probe2(float *out, unsigned long long *cyc, int iters) {
    const int grp = threadIdx.x >> 8;
    f32x16 acc[4];
    for (int i = 0; i < 4; ++i) acc[i] = f32x16{};
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    float f[8];
    for (int i = 0; i < 8; ++i) f[i] = a + i;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (grp == 0) {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 3], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else {
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
#pragma unroll
                for (int k = 0; k < F; ++k) f[k & 7] = __builtin_fmaf(f[k & 7], 1.0001f, 0.5f);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 16; ++j) s += acc[i][j];
    for (int i = 0; i < 8; ++i) s += f[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
    if ((threadIdx.x & 255) == 0) cyc[2 * blockIdx.x + grp] = t1 - t0;
}

template <int F>
static void run2(float *out, unsigned long long *dcyc, int blocks, int iters) {
    probe2<F><<<blocks, 512>>>(out, dcyc, iters);
    probe2<F><<<blocks, 512>>>(out, dcyc, iters);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * blocks), m(blocks), v(blocks);
    (void)hipMemcpy(h.data(), dcyc, 2 * blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    for (int b = 0; b < blocks; ++b) { m[b] = h[2 * b]; v[b] = h[2 * b + 1]; }
    std::sort(m.begin(), m.end());
    std::sort(v.begin(), v.end());
    printf("two waves/SIMD, fillers/slot %2d: MFMA wave %6.1f, VALU wave %6.1f cycles per slot\n", F,
           (double)m[blocks / 2] / (16.0 * iters), (double)v[blocks / 2] / (16.0 * iters));
}

template <int F>
static void run(float *out, unsigned long long *dcyc, int blocks, int iters) {
    probe<F><<<blocks, 256>>>(out, dcyc, iters);
    probe<F><<<blocks, 256>>>(out, dcyc, iters);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(blocks);
    hipMemcpy(h.data(), dcyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    const double per = (double)h[blocks / 2] / (16.0 * iters);
    printf("fillers/MFMA %2d: %6.1f cycles per MFMA (ideal 64 if they co-issue; %5.1f if each filler adds 4)\n",
           F, per, 64.0 + 4.0 * F);
}

int main() {
    const int blocks = 256, iters = 2000;
    float *out;
    unsigned long long *cyc;
    hipMalloc(&out, blocks * 256 * sizeof(float));
    hipMalloc(&cyc, blocks * sizeof(unsigned long long));
    run<0>(out, cyc, blocks, iters);
    run<2>(out, cyc, blocks, iters);
    run<4>(out, cyc, blocks, iters);
    run<6>(out, cyc, blocks, iters);
    run<8>(out, cyc, blocks, iters);
    run<12>(out, cyc, blocks, iters);
    run<16>(out, cyc, blocks, iters);
    hipFree(out);
    hipFree(cyc);
    (void)hipMalloc(&out, blocks * 512 * sizeof(float));
    (void)hipMalloc(&cyc, 2 * blocks * sizeof(unsigned long long));
    run2<0>(out, cyc, blocks, iters);
    run2<4>(out, cyc, blocks, iters);
    run2<8>(out, cyc, blocks, iters);
    run2<16>(out, cyc, blocks, iters);
    hipFree(cyc);
    return 0;
}
