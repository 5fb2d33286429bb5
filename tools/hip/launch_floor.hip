// Launch-floor probe: back-to-back launches of (a) an empty kernel and (b) a
// kernel whose every lane loads one float and writes it back, for several
// grid sizes; mean time per launch from hipEvents around 200 launches.
//   hipcc --offload-arch=gfx950 -O3 tools/hip/launch_floor.hip -o /tmp/launch_floor
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void empty_kernel(int) {}

__global__ __launch_bounds__(256) void touch_kernel(const float *__restrict__ x, float *y, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = x[i] * 2.f;
}

__global__ __launch_bounds__(256) void lds_kernel(const float *__restrict__ x, float *y, int n) {
    __shared__ float s[4][64];
    const int i = blockIdx.x * 256 + threadIdx.x;
    s[threadIdx.x >> 6][threadIdx.x & 63] = (i < n) ? x[i] : 0.f;
    __syncthreads();
    if (threadIdx.x < 64 && i < n) y[i] = s[0][threadIdx.x] + s[1][threadIdx.x] + s[2][threadIdx.x] + s[3][threadIdx.x];
}

int main() {
    const int n = 1 << 22;
    float *x, *y;
    hipMalloc(&x, n * 4);
    hipMalloc(&y, n * 4);
    hipMemset(x, 0, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grids[] = {1, 2, 8, 32, 128, 256, 512, 1024, 4096};
    for (int kind = 0; kind < 3; ++kind) {
        for (int g : grids) {
            for (int w = 0; w < 20; ++w) {
                if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(g), dim3(256), 0, 0, 0);
                else if (kind == 1) hipLaunchKernelGGL(touch_kernel, dim3(g), dim3(256), 0, 0, x, y, n);
                else hipLaunchKernelGGL(lds_kernel, dim3(g), dim3(256), 0, 0, x, y, n);
            }
            hipDeviceSynchronize();
            hipEventRecord(a, 0);
            for (int it = 0; it < 200; ++it) {
                if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(g), dim3(256), 0, 0, 0);
                else if (kind == 1) hipLaunchKernelGGL(touch_kernel, dim3(g), dim3(256), 0, 0, x, y, n);
                else hipLaunchKernelGGL(lds_kernel, dim3(g), dim3(256), 0, 0, x, y, n);
            }
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("%s grid %5d: %.2f us/launch\n", kind == 0 ? "empty" : (kind == 1 ? "touch" : "lds  "), g,
                   ms * 1e3f / 200);
        }
    }
    return 0;
}
