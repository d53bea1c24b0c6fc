// Which XCD (XCC) runs each workgroup of a launch shaped like k_build's (tools only, not the product).
// The tile order GDP_TUNE_TILE_ORDER = 1 assumes workgroup u runs on XCD u mod 8; this records the
// actual XCC_ID of every workgroup (s_getreg HW_REG_XCC_ID, written with a plain vector store) for
// grids of 1024- and 512-thread blocks and prints, per case, the fraction of workgroups with
// xcc == u mod 8 and the per-XCD workgroup counts.
//   hipcc --offload-arch=gfx950 -O3 -o tools/xcd_map tools/xcd_map.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                             \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));         \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

__global__ void k_xcc(unsigned* out, int spin) {
    if (threadIdx.x == 0) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        out[blockIdx.x] = xcc & 0xf;
    }
    // keep the workgroup resident a little, like a build unit (no memory traffic)
    for (int i = 0; i < spin; ++i) __builtin_amdgcn_s_sleep(2);
}

int main() {
    for (int block : {1024, 768, 512}) {
        for (int grid : {4096, 32448}) {
            unsigned* d = nullptr;
            CHECK(hipMalloc(&d, grid * sizeof(unsigned)));
            hipLaunchKernelGGL(k_xcc, dim3(grid), dim3(block), 0, 0, d, 64);
            CHECK(hipDeviceSynchronize());
            std::vector<unsigned> h(grid);
            CHECK(hipMemcpy(h.data(), d, grid * sizeof(unsigned), hipMemcpyDeviceToHost));
            CHECK(hipFree(d));
            long match = 0, cnt[16] = {0};
            for (int u = 0; u < grid; ++u) {
                match += h[u] == (unsigned)(u % 8);
                cnt[h[u] & 15]++;
            }
            printf("{\"block\": %d, \"grid\": %d, \"frac_xcc_eq_u_mod_8\": %.4f, \"per_xcc\": [", block, grid,
                   (double)match / grid);
            for (int x = 0; x < 8; ++x) printf("%s%ld", x ? ", " : "", cnt[x]);
            printf("], \"first16\": [");
            for (int u = 0; u < 16; ++u) printf("%s%u", u ? ", " : "", h[u]);
            printf("]}\n");
        }
    }
    return 0;
}
