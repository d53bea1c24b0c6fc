// Write-alignment microbenchmark (round 5, for the convolution extension's 240-column tiles):
// does a 960-B wave store that starts mid-line (every other tile of k_conv_blk: 240 floats at
// 960 * tc bytes) write slower than a line-aligned 1-KiB one?  Same total bytes per pass, 5
// passes ("levels") per segment like the conv tile's five level stores, non-temporal 16-B stores.
//   mode 0: segment k = 1024 B at 1024 k (64 lanes), aligned
//   mode 1: segment k = 960 B at 960 k (60 lanes), adjacent segments share a line every other k
//   mode 2: segment k = 960 B at 1024 k (60 lanes, 64-B gap), never shares a line, partial lines
//   mode 3: segment k = 768 B at 768 k (48 lanes), line-aligned
// One wave per segment, 16 waves per block: segments 16 b .. 16 b + 15, so adjacent segments of one
// block share an XCD and blocks b, b+1 (adjacent 16-segment runs) run on different XCDs.
//   tools/wr_align [MiB per level, default 512]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(1024) k_write(float* __restrict__ out, long long level_floats, int seg_floats,
                                                int stride_floats, int lanes, long long segs) {
    const long long seg = (long long)blockIdx.x * 16 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (seg >= segs || lane >= lanes) return;
    const f4 v = {(float)seg, (float)lane, 1.f, 2.f};
    float* p = out + seg * stride_floats + 4 * lane;
#pragma unroll
    for (int s = 0; s < 5; ++s) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p + s * level_floats));
    (void)seg_floats;
}

int main(int argc, char** argv) {
    const long long mib = argc > 1 ? std::atoll(argv[1]) : 512;
    const long long level_floats = (mib << 20) / 4;
    float* buf = nullptr;
    if (hipMalloc(&buf, (size_t)level_floats * 4 * 5 + (1 << 20)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Mode {
        int seg, stride, lanes;
        const char* name;
    } modes[] = {{256, 256, 64, "1024B aligned"}, {240, 240, 60, "960B adjacent (mid-line starts)"},
                 {240, 256, 60, "960B at 1024 (gaps)"}, {192, 192, 48, "768B aligned"}};
    for (int rep = 0; rep < 3; ++rep)
        for (const Mode& m : modes) {
            const long long segs = level_floats / m.stride - 1;
            const long long bytes = segs * m.seg * 4 * 5;
            const unsigned grid = (unsigned)((segs + 15) / 16);
            for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_write, dim3(grid), dim3(1024), 0, 0, buf, level_floats, m.seg, m.stride, m.lanes, segs);
            hipEventRecord(e0, 0);
            const int it = 10;
            for (int i = 0; i < it; ++i)
                hipLaunchKernelGGL(k_write, dim3(grid), dim3(1024), 0, 0, buf, level_floats, m.seg, m.stride, m.lanes, segs);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            std::printf("{\"mode\": \"%s\", \"rep\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", m.name, rep, ms / it,
                        bytes / (ms / it * 1e-3) / 1e12);
        }
    hipFree(buf);
    return 0;
}
