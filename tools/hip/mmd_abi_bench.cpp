// smmd_mmd2_fwd timed from C++ through the C ABI (no Python in the loop):
// 200 back-to-back calls per size after warm-up, hipEvents around them.
//   hipcc --offload-arch=gfx950 -O2 tools/hip/mmd_abi_bench.cpp -Iinclude \
//         -Lscaled-mmd-gan_amd/lib -lsmmd_hip -o tools/hip/mmd_abi_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "smmd_hip.h"

int main(int argc, char **argv) {
    const int sizes[] = {64, 256, 512, 1024, 2048, 4096};
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int N : sizes) {
        const int d = 1;
        std::vector<float> h(2 * N);
        srand(1234);
        for (auto &v : h) v = (float)rand() / RAND_MAX * 4.f - 2.f;
        float *X, *Y, *sums, *out, *gx, *gy;
        void *ws;
        hipMalloc(&X, N * 4);
        hipMalloc(&Y, N * 4);
        hipMemcpy(X, h.data(), N * 4, hipMemcpyHostToDevice);
        hipMemcpy(Y, h.data() + N, N * 4, hipMemcpyHostToDevice);
        hipMalloc(&sums, 64);
        hipMalloc(&out, 64);
        hipMalloc(&gx, N * 4);
        hipMalloc(&gy, N * 4);
        const size_t wsb = smmd_mmd2_workspace_bytes(N, N, d);
        hipMalloc(&ws, wsb);
        hipMemset(ws, 0, wsb);
        smmd_kernel_desc k = {};
        k.kind = SMMD_KIND_RBF;
        k.n_terms = 1;
        k.param[0] = 1.0;
        k.wt[0] = 1.0;
        k.has_const_diag = 1;
        k.const_diag = 1.0;
        for (int w = 0; w < 20; ++w)
            smmd_mmd2_fwd(&k, X, N, Y, N, d, 0, 0, N, 0, N, sums, out, gx, gy, ws, wsb, 0);
        hipDeviceSynchronize();
        hipEventRecord(a, 0);
        const int iters = 200;
        for (int it = 0; it < iters; ++it)
            smmd_mmd2_fwd(&k, X, N, Y, N, d, 0, 0, N, 0, N, sums, out, gx, gy, ws, wsb, 0);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms, r;
        hipEventElapsedTime(&ms, a, b);
        hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
        printf("N %5d  %.2f us/call  mmd2 %.6g\n", N, ms * 1e3f / iters, r);
        hipFree(X); hipFree(Y); hipFree(sums); hipFree(out); hipFree(gx); hipFree(gy); hipFree(ws);
    }
    return 0;
}
