// Reproducer: the readback sequence of round 1's qsim_batch_avg_probabilities —
// hipMallocAsync -> kernel writes the buffer -> hipMemcpyAsync to PAGEABLE host memory -> hipFreeAsync
// -> hipStreamSynchronize — repeated on two streams.  argv[1] selects a variant: 0 as above;
// 1 pinned host memory; 2 hipMalloc/hipFree instead of the stream-ordered pool; 3 the free after
// the synchronisation.  Build: hipcc -O2 --offload-arch=gfx950 repro_pool_pageable.hip -o repro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 2; } } while (0)
__global__ void fill(double* p, size_t n, double tag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = tag + (double)i;
}
int main(int argc, char** argv) {
    const int v = argc > 1 ? std::atoi(argv[1]) : 0;
    hipStream_t s[2];
    for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    long bad = 0, calls = 0;
    for (size_t n : {size_t(1) << 12, size_t(1) << 16, size_t(1) << 20}) {
        std::vector<double> pageable(n);
        double* host = pageable.data();
        if (v == 1) CK(hipHostMalloc((void**)&host, n * sizeof(double), hipHostMallocDefault));
        for (int it = 0; it < 200; ++it) {
            hipStream_t st = s[it & 1];
            double* d = nullptr;
            if (v == 2) CK(hipMalloc((void**)&d, n * sizeof(double)));
            else CK(hipMallocAsync((void**)&d, n * sizeof(double), st));
            const double tag = 1e9 * (it + 1);
            hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, st, d, n, tag);
            CK(hipMemcpyAsync(host, d, n * sizeof(double), hipMemcpyDeviceToHost, st));
            if (v == 0 || v == 1) CK(hipFreeAsync(d, st));
            CK(hipStreamSynchronize(st));
            if (v == 2) CK(hipFree(d));
            if (v == 3) CK(hipFreeAsync(d, st));
            size_t wrong = 0;
            for (size_t i = 0; i < n; ++i) wrong += host[i] != tag + (double)i;
            ++calls;
            if (wrong && ++bad <= 3) printf("variant %d n=%zu it=%d: %zu wrong (e.g. %g for %g)\n", v, n, it, wrong, host[0], tag);
        }
        if (v == 1) CK(hipHostFree(host));
    }
    printf("variant %d: calls %ld, with a wrong host copy %ld\n", v, calls, bad);
    return bad ? 1 : 0;
}
