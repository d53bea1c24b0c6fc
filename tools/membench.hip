// HBM ceilings for the pyramid's access pattern on MI355X (tools only, not the product):
// write-only, read-only and copy streams with 16-B lanes, plain vs non-temporal stores, and a
// "1 read : 5 write streams" kernel shaped like k_build (one int4 read, five float4 stores to five
// separate levels).  Prints one JSON line per case.
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench tools/membench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            return 1;                                                             \
        }                                                                         \
    } while (0)

template <bool NT>
__global__ void k_write(f4* __restrict__ p, long n) {
    const f4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        if constexpr (NT)
            __builtin_nontemporal_store(v, p + i);
        else
            p[i] = v;
    }
}

__global__ void k_read(const f4* __restrict__ p, long n, float* out) {
    f4 acc = {0, 0, 0, 0};
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) acc += p[i];
    if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1.f;
}

template <bool NT>
__global__ void k_copy(const f4* __restrict__ a, f4* __restrict__ b, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        if constexpr (NT)
            __builtin_nontemporal_store(a[i], b + i);
        else
            b[i] = a[i];
    }
}

// one block = one contiguous chunk of 256 lanes x PER float4 (non-persistent grid)
template <bool NT, int PER>
__global__ void k_write_chunk(f4* __restrict__ p) {
    const f4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    f4* q = p + (long)blockIdx.x * 256 * PER + threadIdx.x;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if constexpr (NT)
            __builtin_nontemporal_store(v, q + k * 256);
        else
            q[k * 256] = v;
    }
}

// in-place scale, one block = 256 lanes x PER float4, reads issued before writes; LNT = nt loads
template <bool NT, bool LNT, int PER>
__global__ void k_scale_chunk(f4* __restrict__ p) {
    f4* q = p + (long)blockIdx.x * 256 * PER + threadIdx.x;
    f4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = LNT ? __builtin_nontemporal_load(q + k * 256) : q[k * 256];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if constexpr (NT)
            __builtin_nontemporal_store(v[k] * 1.0001f, q + k * 256);
        else
            q[k * 256] = v[k] * 1.0001f;
    }
}

// out-of-place copy, one block = 256 lanes x PER float4
template <bool NT, int PER>
__global__ void k_copy_chunk(const f4* __restrict__ a, f4* __restrict__ b) {
    const long base = (long)blockIdx.x * 256 * PER + threadIdx.x;
    f4 v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = a[base + k * 256];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if constexpr (NT)
            __builtin_nontemporal_store(v[k], b + base + k * 256);
        else
            b[base + k * 256] = v[k];
    }
}

// n int4 reads, 5 x n float4 writes into 5 separate arrays (the k_build octave-0 shape)
template <bool NT>
__global__ void k_r1w5(const i4* __restrict__ in, f4* __restrict__ out, long n) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const f4 x = __builtin_convertvector(in[i], f4);
#pragma unroll
        for (int s = 0; s < 5; ++s) {
            const f4 v = x * (float)(s + 1);
            if constexpr (NT)
                __builtin_nontemporal_store(v, out + s * n + i);
            else
                out[s * n + i] = v;
        }
    }
}

template <class F>
float time_it(F&& launch, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(a);
        launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const long bytes = 512l << 20;  // 512 MiB per stream
    const long n = bytes / 16;
    f4 *a, *b;
    float* o;
    CHECK(hipMalloc(&a, bytes * 6));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&o, 16));
    CHECK(hipMemset(a, 0, bytes * 6));
    CHECK(hipMemset(b, 0, bytes));
    const int reps = 20;
    {
        const int grid = 0;
        auto rep = [&](const char* name, double moved, float ms) {
            printf("{\"case\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", name, grid, ms, moved / ms / 1e6);
        };
        rep("chunk4_nt", bytes, time_it([&] { k_write_chunk<true, 4><<<n / 1024, 256>>>(a); }, reps));
        rep("chunk4_plain", bytes, time_it([&] { k_write_chunk<false, 4><<<n / 1024, 256>>>(a); }, reps));
        rep("chunk16_nt", bytes, time_it([&] { k_write_chunk<true, 16><<<n / 4096, 256>>>(a); }, reps));
        rep("chunk1_nt", bytes, time_it([&] { k_write_chunk<true, 1><<<n / 256, 256>>>(a); }, reps));
        rep("scale1_nt", 2.0 * bytes, time_it([&] { k_scale_chunk<true, false, 1><<<n / 256, 256>>>(a); }, reps));
        rep("scale1_plain", 2.0 * bytes, time_it([&] { k_scale_chunk<false, false, 1><<<n / 256, 256>>>(a); }, reps));
        rep("scale1_ntld_nt", 2.0 * bytes, time_it([&] { k_scale_chunk<true, true, 1><<<n / 256, 256>>>(a); }, reps));
        rep("scale4_nt", 2.0 * bytes, time_it([&] { k_scale_chunk<true, false, 4><<<n / 1024, 256>>>(a); }, reps));
        rep("scale4_ntld_nt", 2.0 * bytes, time_it([&] { k_scale_chunk<true, true, 4><<<n / 1024, 256>>>(a); }, reps));
        rep("scale4_plain", 2.0 * bytes, time_it([&] { k_scale_chunk<false, false, 4><<<n / 1024, 256>>>(a); }, reps));
        rep("copy1_nt", 2.0 * bytes, time_it([&] { k_copy_chunk<true, 1><<<n / 256, 256>>>(b, a); }, reps));
        rep("copy4_nt", 2.0 * bytes, time_it([&] { k_copy_chunk<true, 4><<<n / 1024, 256>>>(b, a); }, reps));
        rep("copy4_plain", 2.0 * bytes, time_it([&] { k_copy_chunk<false, 4><<<n / 1024, 256>>>(b, a); }, reps));
        rep("chunk4_nt_2GB", 4.0 * bytes, time_it([&] { k_write_chunk<true, 4><<<4 * n / 1024, 256>>>(a); }, reps));
        rep("chunk4_plain_2GB", 4.0 * bytes, time_it([&] { k_write_chunk<false, 4><<<4 * n / 1024, 256>>>(a); }, reps));
    }
    for (int grid : {2048, 16384}) {
        const int blk = 256;
        auto rep = [&](const char* name, double moved, float ms) {
            printf("{\"case\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", name, grid, ms, moved / ms / 1e6);
        };
        rep("write_plain", bytes, time_it([&] { k_write<false><<<grid, blk>>>(a, n); }, reps));
        rep("write_nt", bytes, time_it([&] { k_write<true><<<grid, blk>>>(a, n); }, reps));
        rep("read", bytes, time_it([&] { k_read<<<grid, blk>>>(a, n, o); }, reps));
        rep("copy_plain", 2.0 * bytes, time_it([&] { k_copy<false><<<grid, blk>>>(a, b, n); }, reps));
        rep("copy_nt", 2.0 * bytes, time_it([&] { k_copy<true><<<grid, blk>>>(a, b, n); }, reps));
        const long n5 = n / 5;  // 5 output streams of 1/5 of 512 MiB... keep total writes = 512 MiB
        rep("r1w5_plain", 16.0 * n5 * 6, time_it([&] { k_r1w5<false><<<grid, blk>>>((const i4*)b, a, n5); }, reps));
        rep("r1w5_nt", 16.0 * n5 * 6, time_it([&] { k_r1w5<true><<<grid, blk>>>((const i4*)b, a, n5); }, reps));
    }
    return 0;
}
