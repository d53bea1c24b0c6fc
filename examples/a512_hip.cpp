// Parity driver of the AVX-512 drop-in classes (include/GaussDePyramid-HIP-AVX512.h): builds an
// n x n image, constructs the class the reference would (GaussPyramid_a512omp / _a512xp with the
// _hip suffix), calls <method> <calls> times and writes GaussPy in the packed [o][s][r][c] layout.
//     a512_hip <nomp_dynamic | GenerateDoG | xp.GenerateDoG> <n> <S> <ones | lcg:SEED> <calls> <out.f32>
// A bare `a512_hip` times GenerateDoG_nomp_dynamic on the reference's main.cpp input (all-ones,
// n = 512, S = 2) the way main.cpp:60-74 times its call: back to back until >= 100 ms.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>

#include "GaussDePyramid-HIP-AVX512.h"

template <class G>
static void write_pyramid(G& g, int n, int S, const char* path) {
    FILE* f = std::fopen(path, "wb");
    if (!f) std::exit(3);
    int len = n;
    for (int o = 0; o < gdp_octaves_for(n); ++o, len /= 2)
        for (int sc = 0; sc < S + 3; ++sc)
            for (int r = 0; r < len; ++r) std::fwrite(g.GaussPy[o][sc][r], sizeof(float), len, f);
    std::fclose(f);
}

int main(int argc, char* argv[]) {
    const std::string method = argc > 1 ? argv[1] : "time";
    const int n = argc > 2 ? std::atoi(argv[2]) : 512;
    const int S = argc > 3 ? std::atoi(argv[3]) : 2;
    const std::string input = argc > 4 ? argv[4] : "ones";
    const int calls = argc > 5 ? std::atoi(argv[5]) : 1;
    int** p = new int*[n];
    uint32_t s = input.rfind("lcg:", 0) == 0 ? (uint32_t)std::strtoul(input.c_str() + 4, nullptr, 0) : 0;
    for (int i = 0; i < n; ++i) {
        p[i] = new int[n];
        for (int j = 0; j < n; ++j) {
            if (input == "ones") {
                p[i][j] = 1;
            } else {  // SURVEY.md Appendix A LCG, row-major
                s = s * 1664525u + 1013904223u;
                p[i][j] = (int)(s >> 24);
            }
        }
    }
    if (method == "time") {
        counnt = 16;  // the reference's knob (GaussDePyramid-AVX512xOpenMP.h:18); no effect on the GPU
        GaussPyramid_a512omp_hip g(p, n, S);
        for (int mirror = 1; mirror >= 0; --mirror) {
            g.mirror_host = mirror != 0;
            int times = 0;
            std::chrono::duration<double, std::milli> elapsed{};
            while (elapsed.count() < 100) {
                g.GaussPyInit();  // untimed, as the reference's own timing (ref_harness, main.cpp:36-59)
                auto start = std::chrono::high_resolution_clock::now();
                g.GenerateDoG_nomp_dynamic();
                auto end = std::chrono::high_resolution_clock::now();
                elapsed += end - start;
                times += 1;
            }
            std::cout << float(elapsed.count()) / float(times)
                      << (mirror ? " ms/call incl. GaussPy host mirror" : " ms/call device only") << std::endl;
        }
    } else if (argc > 6 && method == "xp.GenerateDoG") {
        GaussPyramid_a512xp_hip g(p, n, S);
        for (int c = 0; c < calls; ++c) g.GenerateDoG();
        write_pyramid(g, n, S, argv[6]);
    } else if (argc > 6 && (method == "nomp_dynamic" || method == "GenerateDoG")) {
        GaussPyramid_a512omp_hip g(p, n, S);
        for (int c = 0; c < calls; ++c) {
            if (method == "nomp_dynamic")
                g.GenerateDoG_nomp_dynamic();
            else
                g.GenerateDoG();
        }
        write_pyramid(g, n, S, argv[6]);
    } else {
        std::fprintf(stderr, "usage: see the header of examples/a512_hip.cpp\n");
        return 2;
    }
    for (int i = 0; i < n; ++i) delete[] p[i];
    delete[] p;
    return 0;
}
