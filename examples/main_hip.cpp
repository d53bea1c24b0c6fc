// The reference's driver (main.cpp:26-75) with the one-line include / class-name swap that the
// drop-in boundary promises: all-ones MAX x MAX image, n = 512, S = 2, GenerateDoG timed in a
// loop until >= 100 ms, mean ms printed.  Extra (optional) arguments make it a parity tool:
//     main_hip [n] [S] [input: ones | lcg:SEED] [dump.f32] [calls] [dog | mpi | mixed]
// writes the pyramid after `calls` GenerateDoG() calls (`mpi`: GenerateDoG_mpi(argc, argv) calls,
// main.cpp:68's method; `mixed`: GenerateDoG_mpi, GenerateDoG, GenerateDoG_mpi, ...) in the packed
// [o][s][r][c] layout.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>

#include "GaussDePyramid-HIP.h"

using namespace std;
const int MAX = 1024;
int n = 512;

int main(int argc, char* argv[]) {
    int S = 2;
    std::string input = "ones";
    if (argc > 1) n = std::atoi(argv[1]);
    if (argc > 2) S = std::atoi(argv[2]);
    if (argc > 3) input = argv[3];
    const int dim = n > MAX ? n : MAX;
    int** p = new int*[dim];
    uint32_t s = input.rfind("lcg:", 0) == 0 ? (uint32_t)std::strtoul(input.c_str() + 4, nullptr, 0) : 0;
    for (int i = 0; i < dim; ++i) {
        p[i] = new int[dim];
        for (int j = 0; j < dim; ++j) {
            if (input == "ones" || i >= n || j >= n) {
                p[i][j] = 1;
            } else {  // SURVEY.md Appendix A LCG over the n x n image, row-major
                s = s * 1664525u + 1013904223u;
                p[i][j] = (int)(s >> 24);
            }
        }
    }
    if (argc > 4) {  // parity mode
        const int calls = argc > 5 ? std::atoi(argv[5]) : 1;
        const std::string mode = argc > 6 ? argv[6] : "dog";
        GaussPyramid_hip g(p, n, S);
        for (int c = 0; c < calls; ++c) {
            if (mode == "mpi" || (mode == "mixed" && c % 2 == 0))
                g.GenerateDoG_mpi(argc, argv);
            else
                g.GenerateDoG();
        }
        FILE* f = std::fopen(argv[4], "wb");
        int len = n;
        for (int o = 0; o < gdp_octaves_for(n); ++o, len /= 2)
            for (int sc = 0; sc < S + 3; ++sc)
                for (int r = 0; r < len; ++r) std::fwrite(g.GaussPy[o][sc][r], sizeof(float), len, f);
        std::fclose(f);
        return 0;
    }
    // main.cpp:60-74: GenerateDoG_mpi called back to back (re-filtering, no GaussPyInit) until
    // >= 100 ms, mean ms printed.  First the drop-in default (GaussPy mirrored to host after every
    // call: PCIe-inclusive), then the device path alone (mirror_host = false).
    for (int mirror = 1; mirror >= 0; --mirror) {
        int times = 0;
        GaussPyramid_hip g(p, n, S);
        g.mirror_host = mirror != 0;
        std::chrono::duration<double, std::milli> elapsed{};
        while (elapsed.count() < 100) {
            auto start = std::chrono::high_resolution_clock::now();
            g.GenerateDoG_mpi(argc, argv);
            auto end = std::chrono::high_resolution_clock::now();
            elapsed += end - start;
            times += 1;
        }
        cout << float(elapsed.count()) / float(times) << (mirror ? " ms/call incl. GaussPy host mirror" : " ms/call device only")
             << endl;
    }
    return 0;
}
