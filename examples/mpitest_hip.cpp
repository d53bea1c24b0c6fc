// mpitest.cpp's driver (:496-558) on the drop-in header: all-ones MAX x MAX image, n = 256,
// GaussPyInit(p) then GenerateDoG_mpi_omp(argc, argv).  Parity mode:
//     mpitest_hip [n] [lcg:SEED|ones] [dump.f32] [mpi|mpi_omp] [S] [op ...]
// With ops (applied in order after the first GaussPyInit(p), replacing the one implicit
// GenerateDoG_* call) the global GaussPy is edited between calls, as a caller of mpitest.cpp's
// free functions may do (mpitest.cpp:128-133, :165 work on whatever GaussPy holds):
//   init | mpi | omp                       GaussPyInit(p) / GenerateDoG_mpi / GenerateDoG_mpi_omp
//   zero:O:S  neg:O:S  scale:O:S:R:F  set:O:S:R:C:V   edit level (O, S) of GaussPy
//   reseat:O:S:R                           point GaussPy[O][S][R] at a fresh copy of the row
//   mirror:0|1  dirty  syncdev  synchost   gdp_mpitest_mirror_host, _host_dirty, _SyncDevice(), _SyncHost()
//   defer:0|1  stale                       gdp_mpitest_defer_download; print `stale=<bytes>` to stderr
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "GaussDePyramid-HIP-mpitest.h"

static std::vector<std::string> split(const std::string& s) {
    std::vector<std::string> out;
    size_t a = 0;
    for (;;) {
        const size_t b = s.find(':', a);
        out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
        if (b == std::string::npos) return out;
        a = b + 1;
    }
}

static int apply(const std::string& spec, int** p, int argc, char** argv) {
    const std::vector<std::string> f = split(spec);
    const std::string& op = f[0];
    auto num = [&](size_t k) { return std::atoi(f.at(k).c_str()); };
    if (op == "init") GaussPyInit(p);
    else if (op == "mpi") GenerateDoG_mpi(argc, argv);
    else if (op == "omp") GenerateDoG_mpi_omp(argc, argv);
    else if (op == "mirror") gdp_mpitest_mirror_host = num(1) != 0;
    else if (op == "dirty") gdp_mpitest_host_dirty = true;
    else if (op == "syncdev") gdp_mpitest_SyncDevice();
    else if (op == "synchost") gdp_mpitest_SyncHost();
    else if (op == "defer") gdp_mpitest_defer_download = num(1) != 0;
    else if (op == "stale") std::fprintf(stderr, "stale=%lld\n", gdp_mpitest_stale_bytes());
    else if (op == "zero" || op == "neg" || op == "scale" || op == "set" || op == "reseat") {
        const int o = num(1), s = num(2), len = n >> o;
        if (op == "zero" || op == "neg") {
            for (int r = 0; r < len; ++r)
                for (int c = 0; c < len; ++c) GaussPy[o][s][r][c] = op == "zero" ? 0.0f : -GaussPy[o][s][r][c];
        } else if (op == "scale") {
            const float k = std::strtof(f.at(4).c_str(), nullptr);
            for (int c = 0; c < len; ++c) GaussPy[o][s][num(3)][c] *= k;
        } else if (op == "set") {
            GaussPy[o][s][num(3)][num(4)] = std::strtof(f.at(5).c_str(), nullptr);
        } else {  // leaked on purpose: delete_mpi frees only the rows it allocated
            float* row = new float[len];
            std::memcpy(row, GaussPy[o][s][num(3)], sizeof(float) * len);
            GaussPy[o][s][num(3)] = row;
        }
    } else {
        std::fprintf(stderr, "unknown op %s\n", spec.c_str());
        return 2;
    }
    return 0;
}

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
    if (argc > 6) {
        for (int i = 6; i < argc; ++i)
            if (apply(argv[i], p, argc, argv) != 0) return 2;
    } else if (argc > 4 && std::string(argv[4]) == "mpi") {
        GenerateDoG_mpi(argc, argv);
    } else {
        GenerateDoG_mpi_omp(argc, argv);
    }
    if (argc > 3) {
        // rows through a local copy: a long fwrite may pass the row to write(2), which fails on a
        // deferred page not fetched yet (the copy's reads fetch it)
        FILE* f = std::fopen(argv[3], "wb");
        if (!f) return 3;
        std::vector<float> row(n);
        for (int o = 0; o < layer; ++o)
            for (int sc = 0; sc < S + 3; ++sc)
                for (int r = 0; r < (n >> o); ++r) {
                    std::memcpy(row.data(), GaussPy[o][sc][r], sizeof(float) * (n >> o));
                    if (std::fwrite(row.data(), sizeof(float), n >> o, f) != (size_t)(n >> o)) return 3;
                }
        if (std::fclose(f) != 0) return 3;
    }
    delete_mpi();
    return 0;
}
