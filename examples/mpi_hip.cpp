// main.cpp (:26-75) driving the MPI-variant drop-in (GaussDePyramid-HIP-mpi.h): all-ones MAX x MAX
// image, n = 512, S = 2, GenerateDoG_mpi in a >= 100 ms loop, mean ms printed by the collector.
// Launch with any MPI: `mpiexec -n <ranks> examples/mpi_hip` (one GPU per rank), or directly
// (MPI singleton, one rank).  Parity mode: mpi_hip [n] [lcg:SEED|ones] [dump.f32] [calls] [mixed]
// — `calls` GenerateDoG_mpi calls on the same object (default 1); with "mixed" a single-process
// GenerateDoG() runs between consecutive GenerateDoG_mpi calls; with "edit" the collector edits its
// GaussPy between them (level (0, 1) zeroed, row 3 of level (0, 0) scaled by -2: two-way state);
// a 7th argument "defer" turns the deferred download on first (DeferDownload(true)).
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "GaussDePyramid-HIP-mpi.h"

const int MAX = 1024;

int main(int argc, char* argv[]) {
    int n = argc > 1 ? std::atoi(argv[1]) : 512;
    std::string input = argc > 2 ? argv[2] : "ones";
    const int dim = n > MAX ? n : MAX;
    int** p = new int*[dim];
    uint32_t s = input.rfind("lcg:", 0) == 0 ? (uint32_t)std::strtoul(input.c_str() + 4, nullptr, 0) : 0;
    for (int i = 0; i < dim; ++i) {
        p[i] = new int[dim];
        for (int j = 0; j < dim; ++j) {
            if (input == "ones" || i >= n || j >= n) {
                p[i][j] = 1;
            } else {
                s = s * 1664525u + 1013904223u;
                p[i][j] = (int)(s >> 24);
            }
        }
    }
    GaussPyramid_hip_mpi g(p, n, 2);
    if (argc > 3) {  // parity mode: collective builds, the collector dumps its GaussPy
        const int calls = argc > 4 ? std::atoi(argv[4]) : 1;
        const bool mixed = argc > 5 && std::string(argv[5]) == "mixed";
        const bool edit = argc > 5 && std::string(argv[5]) == "edit";
        if (argc > 6 && std::string(argv[6]) == "defer") g.DeferDownload(true);
        for (int c = 0; c < calls; ++c) {
            if (c > 0 && mixed) g.GenerateDoG();
            if (c > 0 && edit && g.rank() == g.collector()) {
                for (int r = 0; r < n; ++r)
                    for (int k = 0; k < n; ++k) g.GaussPy[0][1][r][k] = 0.0f;
                for (int k = 0; k < n; ++k) g.GaussPy[0][0][3][k] *= -2.0f;
            }
            g.GenerateDoG_mgpu(argc, argv);  // = GenerateDoG_mpi (the SURVEY's name for the RCCL form)
        }
        if (g.rank() == g.collector()) {  // rank 0, or S+3 under the reference's role map (>= S+4 ranks)
            // rows through a local copy (a deferred page must be touched by the CPU, not write(2))
            FILE* f = std::fopen(argv[3], "wb");
            if (!f) return 3;
            float* row = new float[n];
            for (int o = 0, len = n; len; ++o, len /= 2)
                for (int sc = 0; sc < 5; ++sc)
                    for (int r = 0; r < len; ++r) {
                        for (int k = 0; k < len; ++k) row[k] = g.GaussPy[o][sc][r][k];
                        if (std::fwrite(row, sizeof(float), len, f) != (size_t)len) return 3;
                    }
            delete[] row;
            if (std::fclose(f) != 0) return 3;
        }
        return 0;
    }
    g.GenerateDoG_mpi(argc, argv);  // first call: MPI/RCCL communicator setup, not timed
    int times = 0;
    std::chrono::duration<double, std::milli> elapsed{};
    while (elapsed.count() < 100) {
        auto start = std::chrono::high_resolution_clock::now();
        g.GenerateDoG_mpi(argc, argv);
        auto end = std::chrono::high_resolution_clock::now();
        elapsed += end - start;
        times += 1;
    }
    if (g.rank() == g.collector()) std::printf("%g ms/call (collector, incl. gather + GaussPy host mirror)\n", elapsed.count() / times);
    return 0;
}
