// mpitest.cpp's driver (:496-558) on the drop-in header: all-ones MAX x MAX image, n = 256,
// GaussPyInit(p) then GenerateDoG_mpi_omp(argc, argv).  Parity mode:
//     mpitest_hip [n] [lcg:SEED|ones] [dump.f32] [mpi|mpi_omp] [S]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "GaussDePyramid-HIP-mpitest.h"

int main(int argc, char* argv[]) {
    int** p = new int*[MAX];
    std::string input = argc > 2 ? argv[2] : "ones";
    int nn = argc > 1 ? std::atoi(argv[1]) : 256;
    uint32_t s = input.rfind("lcg:", 0) == 0 ? (uint32_t)std::strtoul(input.c_str() + 4, nullptr, 0) : 0;
    for (int i = 0; i < MAX; ++i) {
        p[i] = new int[MAX];
        for (int j = 0; j < MAX; ++j) {
            if (input == "ones" || i >= nn || j >= nn) {
                p[i][j] = 1;
            } else {
                s = s * 1664525u + 1013904223u;
                p[i][j] = (int)(s >> 24);
            }
        }
    }
    n = nn;
    if (argc > 5) S = std::atoi(argv[5]);
    GaussPyInit(p);
    if (argc > 4 && std::string(argv[4]) == "mpi")
        GenerateDoG_mpi(argc, argv);
    else
        GenerateDoG_mpi_omp(argc, argv);
    if (argc > 3) {
        FILE* f = std::fopen(argv[3], "wb");
        for (int o = 0; o < layer; ++o)
            for (int sc = 0; sc < S + 3; ++sc)
                for (int r = 0; r < (n >> o); ++r) std::fwrite(GaussPy[o][sc][r], sizeof(float), n >> o, f);
        std::fclose(f);
    }
    delete_mpi();
    return 0;
}
