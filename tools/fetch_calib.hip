// FETCH_SIZE calibration for the access widths the convolution extension's staging uses (tools
// only, not the product).  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of a
// wide (16 B / lane) coalesced streaming read; other widths are uncalibrated.  Each case below reads
// a buffer whose fetched-line count is known, one dispatch per case in a fixed order (printed), so
// per-dispatch counters of one rocprofv3 --pmc pass map to the cases:
//   b128        int4 per lane, contiguous                       (k_conv_blk octave 0)
//   b32_s1      one dword per lane, contiguous                  (every word of every line)
//   b32_s<K>    one dword per lane, K dwords apart, K = 2..32   (k_conv_blk octave o: K = 2^o)
// Lines touched: bytes / 128 for K <= 32 (every 128-B line holds at least one loaded dword);
// for K = 16 only every other 64-B half of a line is needed, for K = 32 one word per line.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int i4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));         \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

__global__ void k_b128(const i4* __restrict__ p, long n, int* out) {
    i4 acc = {0, 0, 0, 0};
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load(p + i);
    if (acc.x + acc.y + acc.z + acc.w == 0x12345) out[0] = 1;
}

__global__ void k_b32(const int* __restrict__ p, long n, int stride, int* out) {
    int acc = 0;  // thread i loads dword i * stride (n loads in all)
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        acc += __builtin_nontemporal_load(p + i * stride);
    if (acc == 0x12345) out[0] = 1;
}

int main() {
    const size_t bytes = size_t(1) << 30;  // 1 GiB: 4x the Infinity Cache
    int* buf = nullptr;
    int* out = nullptr;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 1, bytes));
    const long dwords = (long)(bytes / 4);
    const int grid = 256 * 16, block = 256;
    printf("{\"case\": \"b128\", \"lines\": %ld, \"bytes_of_lines\": %zu}\n", (long)(bytes / 128), bytes);
    hipLaunchKernelGGL(k_b128, dim3(grid), dim3(block), 0, 0, (const i4*)buf, dwords / 4, out);
    for (int stride : {1, 2, 4, 8, 16, 32}) {
        const long n = dwords / stride;
        printf("{\"case\": \"b32_s%d\", \"lines\": %ld, \"bytes_of_lines\": %zu, \"dwords_loaded\": %ld}\n", stride,
               (long)(bytes / 128), bytes, n);
        hipLaunchKernelGGL(k_b32, dim3(grid), dim3(block), 0, 0, (const int*)buf, n, stride, out);
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(buf));
    CHECK(hipFree(out));
    return 0;
}
