// Speed-of-light probe for config 2's byte mix (tools only, not the product).  How fast can ANY
// kernel move exactly k_build's algorithmic bytes for one 4096² image (S = 2, O = 5: 67,108,864 B
// of int32 read, 446,955,520 B of float written) in one launch, on the product's pyramid backing?
//
// The "ideal build" kernel keeps k_build's work split but none of its arithmetic or geometry: one
// 1024-thread block per 4,096 input pixels (k_build's 16 x 256 tile), one int4 load per thread,
// five non-temporal float4 stores per thread into five level arrays (octave 0), then the block's
// 1/4096 share of octaves 1-4 as contiguous float4 stores.  Every store is a contiguous 16-KiB run
// per block and level, so this is an upper bound for k_build's 1-KiB row runs.
//
// Backings: "vmm2m" = one reserved range backed by separately created 2 MiB pieces (the product's
// default, csrc/gdp.hip alloc_spread); "malloc" = one hipMalloc.  Launches rotate over 5 buffer
// sets (2.57 GB, beyond the 256 MB Infinity Cache) as bench.py does; each launch is timed alone
// with HIP events.  Cases: ideal build per image (config 2's launch), the same kernel over 16
// images in one launch (a long launch, config 4's regime), a write-only stream of the same
// 514,064,384 B, and — for the in-place re-entry pass `k_levels` (`--op regen`) — an in-place
// read-modify-write of the 447 MB pyramid: one thread per 4-pixel group loading its five levels,
// then storing five (k_levels' shape without the windows), in 256-thread blocks; and a read-reuse
// probe (a 1 MiB / 64 MiB working set read 64 times per thread) that shows whether each backing
// is cached in L2 at all.  One JSON line per case.
//   make -C tools sol_c2 && tools/sol_c2 [launches]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

constexpr long kPix = 4096L * 4096L;                  // input pixels per image
constexpr long kIn = kPix * 4;                        // 67,108,864 B
constexpr long kOct0 = kPix * 4 * 5;                  // 335,544,320 B (5 scales)
constexpr long kRest = (kPix / 4 + kPix / 16 + kPix / 64 + kPix / 256) * 4 * 5;  // 111,411,200 B
constexpr long kOut = kOct0 + kRest;                  // 446,955,520 B
constexpr long kBlocks = kPix / 4096;                 // 4,096 tiles of 16 x 256
constexpr int kRestPerBlock = (int)(kRest / 16 / kBlocks);  // 1,700 float4
static_assert(kRest % (16 * kBlocks) == 0, "octaves 1-4 split evenly over the tiles");

// one block = one 4,096-pixel tile of image blockIdx.y
__global__ void __launch_bounds__(1024) k_ideal(const i4* __restrict__ in, f4* __restrict__ out, long in_stride,
                                                long out_stride) {
    const long b = blockIdx.y;
    const long t = (long)blockIdx.x * 1024 + threadIdx.x;
    const i4 x = in[b * in_stride + t];
    const f4 v = __builtin_convertvector(x, f4);
    f4* o = out + b * out_stride;
#pragma unroll
    for (int s = 0; s < 5; ++s) __builtin_nontemporal_store(v * (float)(s + 1), o + s * (kPix / 4) + t);
    f4* r = o + 5 * (kPix / 4) + (long)blockIdx.x * kRestPerBlock;
    for (int i = threadIdx.x; i < kRestPerBlock; i += 1024) __builtin_nontemporal_store(v, r + i);
}

// in-place five-level read-modify-write (k_levels' access shape): thread = one float4 of each level
__global__ void __launch_bounds__(256) k_rmw5(f4* __restrict__ pyr, long lev_f4, long n) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    f4 v[5];
#pragma unroll
    for (int s = 0; s < 5; ++s) v[s] = __builtin_nontemporal_load(pyr + s * lev_f4 + i);
#pragma unroll
    for (int s = 0; s < 4; ++s) __builtin_nontemporal_store(v[s] - v[s + 1], pyr + s * lev_f4 + i);
    __builtin_nontemporal_store(v[4], pyr + 4 * lev_f4 + i);
}

// cache probe: every thread reads `reps` float4s from a small working set (`ws` float4s, e.g. 1 MiB):
// served from L2 when the backing is cached there, from memory when it is not
__global__ void __launch_bounds__(256) k_reuse(const f4* __restrict__ p, long ws, int reps, float* sink) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    long i = ((long)blockIdx.x * 256 + threadIdx.x) % ws;
    for (int r = 0; r < reps; ++r) {
        acc += p[i];
        i += 4099 * 64;  // next line of another wave's block, wrapping in the working set
        if (i >= ws) i -= ws;
    }
    if (acc.x + acc.y + acc.z + acc.w == 1234.5f) sink[0] = 1.f;
}

// write-only: one float4 per thread, 1024-thread blocks
__global__ void __launch_bounds__(1024) k_write(f4* __restrict__ out, long n) {
    const long i = (long)blockIdx.x * 1024 + threadIdx.x;
    const f4 v = {1.f, 2.f, 3.f, (float)blockIdx.x};
    if (i < n) __builtin_nontemporal_store(v, out + i);
}

static char* alloc_vmm2m(size_t bytes) {
    const size_t two = 2u << 20;
    bytes = (bytes + two - 1) / two * two;
    int dev = 0;
    CHECK(hipGetDevice(&dev));
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    void* base = nullptr;
    CHECK(hipMemAddressReserve(&base, bytes, two, nullptr, 0));
    for (size_t off = 0; off < bytes; off += two) {
        hipMemGenericAllocationHandle_t h;
        CHECK(hipMemCreate(&h, two, &prop, 0));
        CHECK(hipMemMap(static_cast<char*>(base) + off, two, 0, h, 0));
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(base, bytes, &acc, 1));
    return static_cast<char*>(base);
}

struct Stats {
    double mean_ms, median_ms, min_ms;
};

template <class F>
static Stats time_launches(F&& launch, int n) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) launch(i);
    CHECK(hipDeviceSynchronize());
    std::vector<double> t;
    for (int i = 0; i < n; ++i) {
        CHECK(hipEventRecord(a, 0));
        launch(i);
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
    }
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    Stats s;
    s.mean_ms = std::accumulate(t.begin(), t.end(), 0.0) / t.size();
    std::sort(t.begin(), t.end());
    s.median_ms = t[t.size() / 2];
    s.min_ms = t[0];
    return s;
}

static void report(const char* kase, const char* backing, int images, double bytes, const Stats& s) {
    std::printf("{\"case\": \"%s\", \"backing\": \"%s\", \"images\": %d, \"bytes_per_launch\": %.0f, "
                "\"mean_ms\": %.5f, \"median_ms\": %.5f, \"min_ms\": %.5f, \"TBps_mean\": %.3f, \"frac_of_8TBps\": %.4f}\n",
                kase, backing, images, bytes, s.mean_ms, s.median_ms, s.min_ms, bytes / (s.mean_ms * 1e-3) / 1e12,
                bytes / (s.mean_ms * 1e-3) / 8e12);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const int launches = argc > 1 ? std::atoi(argv[1]) : 200;
    const int sets = 5;
    for (int backing = 0; backing < 2; ++backing) {
        const char* bname = backing == 0 ? "vmm2m" : "malloc";
        // per set: 1 image (input + pyramid); the 16-image case reuses the same memory as 16 x ...
        const long big = 16;
        const size_t in_bytes = (size_t)kIn * big, out_bytes = (size_t)kOut * big;
        char *in_base = nullptr, *out_base = nullptr;
        if (backing == 0) {
            in_base = alloc_vmm2m(in_bytes);
            out_base = alloc_vmm2m(out_bytes);
        } else {
            CHECK(hipMalloc(&in_base, in_bytes));
            CHECK(hipMalloc(&out_base, out_bytes));
        }
        CHECK(hipMemset(in_base, 1, in_bytes));
        CHECK(hipMemset(out_base, 0, out_bytes));
        // 1 image per launch, rotating over `sets` of the 16 slots spread across the buffer
        auto one = [&](int i) {
            const long slot = (long)(i % sets) * 3;  // slots 0, 3, 6, 9, 12
            hipLaunchKernelGGL(k_ideal, dim3(kBlocks, 1), dim3(1024), 0, 0,
                               reinterpret_cast<const i4*>(in_base + slot * kIn),
                               reinterpret_cast<f4*>(out_base + slot * kOut), kIn / 16, kOut / 16);
        };
        report("ideal_build_1img", bname, 1, (double)(kIn + kOut), time_launches(one, launches));
        auto sixteen = [&](int) {
            hipLaunchKernelGGL(k_ideal, dim3(kBlocks, big), dim3(1024), 0, 0, reinterpret_cast<const i4*>(in_base),
                               reinterpret_cast<f4*>(out_base), kIn / 16, kOut / 16);
        };
        report("ideal_build_16img", bname, 16, (double)(kIn + kOut) * big, time_launches(sixteen, launches / 10 + 5));
        const long wn = (kIn + kOut) / 16;
        auto wonly = [&](int i) {
            const long slot = (long)(i % sets) * 3;
            hipLaunchKernelGGL(k_write, dim3((unsigned)((wn + 1023) / 1024)), dim3(1024), 0, 0,
                               reinterpret_cast<f4*>(out_base + slot * kOut), wn);
        };
        report("write_only_1img", bname, 1, (double)(kIn + kOut), time_launches(wonly, launches));
        // the pyramid as five equal levels of kOut / 5 bytes, read and rewritten in place
        const long lev = kOut / 5 / 16;
        auto rmw = [&](int i) {
            const long slot = (long)(i % sets) * 3;
            hipLaunchKernelGGL(k_rmw5, dim3((unsigned)((lev + 255) / 256)), dim3(256), 0, 0,
                               reinterpret_cast<f4*>(out_base + slot * kOut), lev, lev);
        };
        report("inplace_rmw5_1img", bname, 1, 2.0 * (double)kOut, time_launches(rmw, launches));
        // L2 residency of the backing: 1 MiB and 64 MiB working sets read 64 times per thread
        for (long ws_mib : {1L, 64L}) {
            const long ws = (ws_mib << 20) / 16;
            const unsigned grid = 8192;
            const int reps = 64;
            auto reuse = [&](int) {
                hipLaunchKernelGGL(k_reuse, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const f4*>(out_base), ws, reps,
                                   reinterpret_cast<float*>(in_base));
            };
            report(ws_mib == 1 ? "reuse_read_1MiB_ws" : "reuse_read_64MiB_ws", bname, 0, 16.0 * grid * 256 * reps,
                   time_launches(reuse, 50));
        }
        CHECK(hipDeviceSynchronize());
        if (backing == 1) {
            CHECK(hipFree(in_base));
            CHECK(hipFree(out_base));
        }  // the VMM ranges live until exit
    }
    return 0;
}
