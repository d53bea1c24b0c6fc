// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// Driver that compiles the reference's own headers IN PLACE (-I /root/reference, see
// oracle/Makefile) and exposes them as a command-line tool, so the golden vectors in
// tests/golden/ and the "reference" CPU baseline in bench.py come from the reference code itself.
// No reference source is copied into this repository; the binary lands in oracle/_ref/
// (git-ignored, shipped to the GPU box with the snapshot like any other built artefact).
//
//   ref_harness hash   <n> <S> <input>                     per-level FNV hashes of GenerateDoG()
//   ref_harness dump   <n> <S> <input> <out.f32>           all levels, packed [o][s][r][c] float32
//   ref_harness taps   <n> <S> <out.f32>                   reference `filter` taps for every (o, s)
//   ref_harness regen  <n> <S> <input> <calls> <out.f32>   GenerateDoG() called <calls> times
//   ref_harness regen-hash <n> <S> <input> <calls>         per-level FNV hashes of the same
//   ref_harness gauss  <n> <S> <input> <calls> <out.f32>   GaussFilter(o) of every octave, <calls>
//                                                          rounds, on the constructor's GaussPyInit
//   ref_harness dump-a512omp <n> <S> <input> <out.f32>     GenerateDoG_nomp_dynamic() output
//   ref_harness dump-a512xp  <n> <S> <input> <out.f32>     GaussPyramid_a512xp::GenerateDoG() output
//   ref_harness hash-a512omp <n> <S> <input> <calls> <method> [threads]  per-level FNV hashes after
//               <calls> calls of GaussPyramid_a512omp::<method>, method "nomp_dynamic" or
//               "GenerateDoG" (or of GaussPyramid_a512xp::GenerateDoG: "xp.GenerateDoG"), with `counnt` = threads (default 1: its DoG loop, an `omp for` over
//               i < S-1 doing level i -= level i+1 in place, races between threads once S >= 3)
//   ref_harness time-serial  <n> <S> <input> <reps>
//   ref_harness time-a512omp <n> <S> <input> <reps> <threads>
//   ref_harness time-a512xp  <n> <S> <input> <reps>
// <input> is "lcg:SEED" (SURVEY.md Appendix A), "ones" (main.cpp:31-35), "synth:SEED:INDEX"
// (bench counter hash) or "file:PATH" (raw int32 n*n).
//
// Timing follows the reference's own convention: GaussPyInit() (refill) is outside the timed
// region, GenerateDoG*() inside it (main.cpp:62-74, commented sweep main.cpp:36-59).
#include "GuassDePyramid.h"
#ifdef WITH_AVX512
#include "GaussDePyramid-AVX512xOpenMP.h"
#include "GaussDePyramid-AVX512xPTHREAD.h"
#endif

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdlib.h>
#include <cstring>
#include <new>
#include <string>
#include <vector>

// The AVX/AVX-512 headers store with _mm512_store_ps into rows from `new float[]`
// (GaussDePyramid-AVX512xOpenMP.h:295, -AVX512xPTHREAD.h:232); they fault unless rows are 64-byte
// aligned.  This executable's array new therefore returns 64-byte-aligned blocks.
void* operator new[](std::size_t sz) {
    void* p = aligned_alloc(64, (sz + 63) / 64 * 64);
    if (!p) throw std::bad_alloc();
    return p;
}
void operator delete[](void* p) noexcept { std::free(p); }
void operator delete[](void* p, std::size_t) noexcept { std::free(p); }

#include "ref_common.h"

using namespace refh;

namespace {

// Reads the protected `filter` member after GaussFilter(o).  GaussFilter overwrites `filter`
// for every scale i in [0, S+3) (GuassDePyramid.h:117-121), so after the call it holds the taps
// of the LAST scale, S+2.  A probe constructed with S' = s - 2 therefore exposes scale s.
struct TapProbe : GaussPyramid {
    TapProbe(int** img, int len, int Sp) : GaussPyramid(img, len, Sp) {}
    const float* taps() const { return filter; }
};

template <class F>
double time_ms(F&& f) {
    auto t0 = std::chrono::high_resolution_clock::now();
    f();
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

void report(const char* kind, int n, int S, int reps, int threads, const std::vector<double>& ms) {
    // The first call pays first-touch page faults of the pyramid; it is a warm-up, not a sample.
    std::vector<double> v(ms.begin() + (ms.size() > 1 ? 1 : 0), ms.end());
    std::sort(v.begin(), v.end());
    double sum = 0;
    for (double x : v) sum += x;
    std::printf("{\"kind\": \"%s\", \"n\": %d, \"S\": %d, \"octaves\": %d, \"reps\": %d, \"threads\": %d, "
                "\"ms_median\": %.6f, \"ms_min\": %.6f, \"ms_mean\": %.6f}\n",
                kind, n, S, octaves_of(n), (int)v.size(), threads, v[v.size() / 2], v[0], sum / v.size());
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: see header of oracle/ref_harness.cpp\n");
        return 2;
    }
    const std::string mode = argv[1];
    const int n = std::atoi(argv[2]);
    const int S = std::atoi(argv[3]);
    if (mode == "taps") {
        if (argc < 5) return 2;
        FILE* f = std::fopen(argv[4], "wb");
        int** img = make_input(n, "ones");
        for (int s = 0; s < S + 3; ++s) {
            TapProbe probe(img, n, s - 2);
            int len = n;
            for (int o = 0; o < octaves_of(n); ++o, len /= 2) {
                probe.GaussFilter(o);
                std::fwrite(probe.taps(), sizeof(float), len, f);  // layout [s][o][len_o]
            }
        }
        std::fclose(f);
        return 0;
    }
    if (argc < 5) return 2;
    int** img = make_input(n, argv[4]);
    if (mode == "hash" || mode == "dump") {
        GaussPyramid g(img, n, S);
        g.GenerateDoG();
        if (mode == "hash")
            hash(g.GaussPy, n, S);
        else
            dump(g.GaussPy, n, S, argv[5]);
    } else if (mode == "regen-hash") {
        GaussPyramid g(img, n, S);
        const int calls = std::atoi(argv[5]);
        for (int c = 0; c < calls; ++c) g.GenerateDoG();
        hash(g.GaussPy, n, S);
    } else if (mode == "regen") {
        GaussPyramid g(img, n, S);
        const int calls = std::atoi(argv[5]);
        for (int c = 0; c < calls; ++c) g.GenerateDoG();
        dump(g.GaussPy, n, S, argv[6]);
    } else if (mode == "gauss") {
        GaussPyramid g(img, n, S);
        const int calls = std::atoi(argv[5]);
        for (int c = 0; c < calls; ++c)
            for (int o = 0; o < octaves_of(n); ++o) g.GaussFilter(o);
        dump(g.GaussPy, n, S, argv[6]);
#ifdef WITH_AVX512
    } else if (mode == "dump-a512omp") {
        GaussPyramid_a512omp g(img, n, S);
        g.GenerateDoG_nomp_dynamic();
        dump(g.GaussPy, n, S, argv[5]);
    } else if (mode == "hash-a512omp") {
        if (argc < 7) return 2;
        counnt = argc > 7 ? std::atoi(argv[7]) : 1;  // GaussDePyramid-AVX512xOpenMP.h:18
        const int calls = std::atoi(argv[5]);
        const std::string method = argv[6];
        if (method == "xp.GenerateDoG") {
            GaussPyramid_a512xp g(img, n, S);
            for (int c = 0; c < calls; ++c) g.GenerateDoG();
            hash(g.GaussPy, n, S);
            return 0;
        }
        GaussPyramid_a512omp g(img, n, S);
        for (int c = 0; c < calls; ++c) {
            if (method == "nomp_dynamic")
                g.GenerateDoG_nomp_dynamic();
            else if (method == "GenerateDoG")
                g.GenerateDoG();
            else
                return 2;
        }
        hash(g.GaussPy, n, S);
    } else if (mode == "dump-a512xp") {
        GaussPyramid_a512xp g(img, n, S);
        g.GenerateDoG();
        dump(g.GaussPy, n, S, argv[5]);
    } else if (mode == "time-a512omp" || mode == "time-a512xp") {
        const int reps = (argc > 5 ? std::atoi(argv[5]) : 3) + 1;  // + 1 warm-up call
        std::vector<double> ms;
        if (mode == "time-a512omp") {
            counnt = argc > 6 ? std::atoi(argv[6]) : 2;  // GaussDePyramid-AVX512xOpenMP.h:18
            GaussPyramid_a512omp g(img, n, S);
            for (int r = 0; r < reps; ++r) {
                g.GaussPyInit();
                ms.push_back(time_ms([&] { g.GenerateDoG_nomp_dynamic(); }));
            }
            report("GaussDePyramid-AVX512xOpenMP.h GenerateDoG_nomp_dynamic", n, S, reps, counnt, ms);
        } else {
            GaussPyramid_a512xp g(img, n, S);
            for (int r = 0; r < reps; ++r) {
                g.GaussPyInit();
                ms.push_back(time_ms([&] { g.GenerateDoG(); }));
            }
            report("GaussDePyramid-AVX512xPTHREAD.h GenerateDoG", n, S, reps, THREAD_COUNT_a512t, ms);
        }
#endif
    } else if (mode == "time-serial") {
        const int reps = (argc > 5 ? std::atoi(argv[5]) : 3) + 1;  // + 1 warm-up call
        std::vector<double> ms;
        GaussPyramid g(img, n, S);
        for (int r = 0; r < reps; ++r) {
            g.GaussPyInit();
            ms.push_back(time_ms([&] { g.GenerateDoG(); }));
        }
        report("serial GuassDePyramid.h GenerateDoG", n, S, reps, 1, ms);
    } else {
        std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
        return 2;
    }
    return 0;
}
