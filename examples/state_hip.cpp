// GaussPy as two-way state (GuassDePyramid.h:16): the reference's float**** IS the pyramid, and
// GaussFilter / GenerateDoG work on whatever the caller left in it (:122-131, :140-146).  This
// driver edits GaussPy / data on the host between calls of a drop-in class and dumps GaussPy, so a
// test can replay the same edits on the oracle and compare bit for bit.
//     state_hip <hip | a512omp | a512xp> <n> <S> <ones | lcg:SEED> <out.f32 | -> <op> ...
// ops (applied in order):
//   init | dog | mpi | nomp | filter:O          GaussPyInit / GenerateDoG / GenerateDoG_mpi /
//                                               GenerateDoG_nomp_dynamic / GaussFilter(O)
//   zero:O:S  neg:O:S  scale:O:S:R:F  set:O:S:R:C:V   edit level (O, S) of GaussPy on the host
//   data:R:C:V                                  edit the class's `data` copy of the image
//   reseat:O:S:R                                point GaussPy[O][S][R] at a fresh copy of the row
//   mirror:0|1  dirty  syncdev  synchost        mirror_host, host_dirty = true, SyncDevice, SyncHost
//   time:CALLS                                  time CALLS back-to-back GenerateDoG calls (stderr)
//   track:0|1                                   TrackWrites (write-tracked mirror, default on)
//   written                                     print `written=<bytes>` (the next upload) to stderr
//   defer:0|1  stale                            DeferDownload; print `stale=<bytes>` to stderr
//   read                                        read every GaussPy float once (fetches a deferred
//                                               mirror page by page; prints `read_ms=` to stderr)
//   readmt:T  negmt:O:S:T                       the read / neg:O:S from T threads at once, rows
//                                               interleaved (concurrent faults on the mirror)
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "GaussDePyramid-HIP-AVX512.h"

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

// class-specific methods; a call a class does not have is a usage error
static void call_mpi(GaussPyramid_hip& g, int argc, char** argv) { g.GenerateDoG_mpi(argc, argv); }
static void call_mpi(GaussPyramid_a512omp_hip&, int, char**) { std::fprintf(stderr, "no GenerateDoG_mpi\n"); std::exit(2); }
static void call_mpi(GaussPyramid_a512xp_hip&, int, char**) { std::fprintf(stderr, "no GenerateDoG_mpi\n"); std::exit(2); }
template <class G>
static void call_nomp(G&) {
    std::fprintf(stderr, "no GenerateDoG_nomp_dynamic\n");
    std::exit(2);
}
static void call_nomp(GaussPyramid_a512omp_hip& g) { g.GenerateDoG_nomp_dynamic(); }

template <class G>
static int run(G& g, int n, int S, const char* path, int nops, char** ops, int argc, char** argv) {
    std::vector<float*> reseated;
    for (int i = 0; i < nops; ++i) {
        const std::vector<std::string> f = split(ops[i]);
        const std::string& op = f[0];
        auto num = [&](size_t k) { return std::atoi(f.at(k).c_str()); };
        if (op == "init") g.GaussPyInit();
        else if (op == "dog") g.GenerateDoG();
        else if (op == "mpi") call_mpi(g, argc, argv);
        else if (op == "nomp") call_nomp(g);
        else if (op == "filter") g.GaussFilter(num(1));
        else if (op == "mirror") g.mirror_host = num(1) != 0;
        else if (op == "dirty") g.host_dirty = true;
        else if (op == "syncdev") g.SyncDevice();
        else if (op == "synchost") g.SyncHost();
        else if (op == "track") g.TrackWrites(num(1) != 0);
        else if (op == "written") std::fprintf(stderr, "written=%lld\n", g.written_bytes());
        else if (op == "defer") std::fprintf(stderr, "deferring=%d\n", (int)g.DeferDownload(num(1) != 0));
        else if (op == "stale") std::fprintf(stderr, "stale=%lld\n", g.stale_bytes());
        else if (op == "readmt" || op == "negmt") {
            const int T = num(op == "readmt" ? 1 : 3);
            std::vector<std::thread> th;
            std::vector<double> sums(T, 0.0);
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    int len = n;
                    for (int o = 0; o < gdp_octaves_for(n); ++o, len /= 2)
                        for (int sc = 0; sc < S + 3; ++sc) {
                            if (op == "negmt" && (o != num(1) || sc != num(2))) continue;
                            for (int r = t; r < len; r += T)
                                for (int c = 0; c < len; ++c) {
                                    if (op == "negmt") g.GaussPy[o][sc][r][c] = -g.GaussPy[o][sc][r][c];
                                    else sums[t] += g.GaussPy[o][sc][r][c];
                                }
                        }
                });
            for (auto& x : th) x.join();
        } else if (op == "read") {
            auto t0 = std::chrono::high_resolution_clock::now();
            double sum = 0;
            int len = n;
            for (int o = 0; o < gdp_octaves_for(n); ++o, len /= 2)
                for (int sc = 0; sc < S + 3; ++sc)
                    for (int r = 0; r < len; ++r)
                        for (int c = 0; c < len; ++c) sum += g.GaussPy[o][sc][r][c];
            auto t1 = std::chrono::high_resolution_clock::now();
            std::fprintf(stderr, "read_ms=%.3f sum=%g\n", std::chrono::duration<double, std::milli>(t1 - t0).count(), sum);
        }
        else if (op == "zero" || op == "neg" || op == "scale" || op == "set" || op == "reseat") {
            const int o = num(1), s = num(2), len = n >> o;
            if (op == "zero" || op == "neg") {
                for (int r = 0; r < len; ++r)
                    for (int c = 0; c < len; ++c) g.GaussPy[o][s][r][c] = op == "zero" ? 0.0f : -g.GaussPy[o][s][r][c];
            } else if (op == "scale") {
                const float k = std::strtof(f.at(4).c_str(), nullptr);
                for (int c = 0; c < len; ++c) g.GaussPy[o][s][num(3)][c] *= k;
            } else if (op == "set") {
                g.GaussPy[o][s][num(3)][num(4)] = std::strtof(f.at(5).c_str(), nullptr);
            } else {  // the reference's rows are separate new[] arrays: a caller may swap one
                float* row = new float[len];
                std::memcpy(row, g.GaussPy[o][s][num(3)], sizeof(float) * len);
                g.GaussPy[o][s][num(3)] = row;
                reseated.push_back(row);
            }
        } else if (op == "data") {
            g.data[num(1)][num(2)] = num(3);
        } else if (op == "time") {
            const int calls = num(1);
            auto t0 = std::chrono::high_resolution_clock::now();
            for (int c = 0; c < calls; ++c) g.GenerateDoG();
            auto t1 = std::chrono::high_resolution_clock::now();
            std::fprintf(stderr, "%s n=%d mirror_host=%d: %.3f ms per GenerateDoG\n", "state_hip", n, (int)g.mirror_host,
                         std::chrono::duration<double, std::milli>(t1 - t0).count() / calls);
        } else {
            std::fprintf(stderr, "unknown op %s\n", ops[i]);
            return 2;
        }
    }
    if (std::string(path) == "-") return 0;  // timing runs: no dump
    FILE* out = std::fopen(path, "wb");
    if (!out) return 3;
    // each row through a local copy: fwrite may hand a long buffer straight to write(2), which a
    // deferred GaussPy page would fail with EFAULT (the copy's CPU reads fetch it)
    std::vector<float> row(n);
    int len = n;
    for (int o = 0; o < gdp_octaves_for(n); ++o, len /= 2)
        for (int sc = 0; sc < S + 3; ++sc)
            for (int r = 0; r < len; ++r) {
                std::memcpy(row.data(), g.GaussPy[o][sc][r], sizeof(float) * len);
                if (std::fwrite(row.data(), sizeof(float), len, out) != (size_t)len) return 3;
            }
    if (std::fclose(out) != 0) return 3;
    return 0;  // (reseated rows are leaked like the reference leaks `data`; the process ends here)
}

int main(int argc, char* argv[]) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: see the header of examples/state_hip.cpp\n");
        return 2;
    }
    const std::string cls = argv[1];
    const int n = std::atoi(argv[2]), S = std::atoi(argv[3]);
    const std::string input = argv[4];
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
    if (cls == "hip") {
        GaussPyramid_hip g(p, n, S);
        return run(g, n, S, argv[5], argc - 6, argv + 6, argc, argv);
    }
    if (cls == "a512omp") {
        GaussPyramid_a512omp_hip g(p, n, S);
        return run(g, n, S, argv[5], argc - 6, argv + 6, argc, argv);
    }
    if (cls == "a512xp") {
        GaussPyramid_a512xp_hip g(p, n, S);
        return run(g, n, S, argv[5], argc - 6, argv + 6, argc, argv);
    }
    std::fprintf(stderr, "unknown class %s\n", cls.c_str());
    return 2;
}
