// Wave-dispatch ceiling: launch time of grids that do (almost) no work, for the block shapes the
// build kernel uses — is k_build (~4,096 x 1024-thread blocks per 4096^2 image) dispatch-bound?
//   hipcc -O3 --offload-arch=gfx950 -o tools/dispatch_bench tools/dispatch_bench.hip && tools/dispatch_bench
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* sink, int flag) {
    if (flag == 12345 && threadIdx.x == 0) sink[blockIdx.x] = 1;  // never true: no memory traffic
}

// one 16-B non-temporal store per lane (what a k_build wave's first level costs at minimum)
typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void k_store(f4* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    __builtin_nontemporal_store(f4{1.f, 2.f, 3.f, 4.f}, out + i);
}

int main() {
    int* sink;
    f4* out;
    hipMalloc(&sink, 1 << 24);
    hipMalloc(&out, (size_t)1 << 31);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int shapes[][2] = {{4096, 1024}, {8192, 512}, {16384, 256}, {65536, 64}, {32768, 1024}};
    for (auto& sh : shapes) {
        const int grid = sh[0], block = sh[1];
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(block), 0, 0, sink, 0);
        hipEventRecord(a);
        const int reps = 50;
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(block), 0, 0, sink, 0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = 1e3 * ms / reps, waves = (double)grid * block / 64;
        printf("{\"kernel\": \"empty\", \"grid\": %d, \"block\": %d, \"us\": %.2f, \"waves_per_us\": %.0f}\n", grid, block,
               us, waves / us);
        const size_t n = (size_t)grid * block;
        if (n * 16 <= ((size_t)1 << 31)) {
            hipEventRecord(a);
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_store, dim3(grid), dim3(block), 0, 0, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
            const double us2 = 1e3 * ms / reps;
            printf("{\"kernel\": \"store16B\", \"grid\": %d, \"block\": %d, \"us\": %.2f, \"GBps\": %.0f, \"waves_per_us\": %.0f}\n",
                   grid, block, us2, n * 16 / us2 / 1e3, waves / us2);
        }
    }
    return 0;
}
