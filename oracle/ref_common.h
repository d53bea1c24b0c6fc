// ORACLE — TEST INFRASTRUCTURE ONLY.
// Helpers shared by the reference harnesses (ref_harness.cpp, ref_mpi_harness.cpp): the input
// generators of SURVEY.md Appendix A / §8d, the FNV level hash of tests/golden/meta.json, and the
// packed float32 dump.  Include after the reference header (needs <cstdio>, <cstring>, <string>).
#ifndef GDP_ORACLE_REF_COMMON_H
#define GDP_ORACLE_REF_COMMON_H

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace refh {

inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

inline int** make_input(int n, const std::string& spec) {
    int** p = new int*[n];
    for (int i = 0; i < n; ++i) p[i] = new int[n];
    if (spec == "ones") {
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) p[i][j] = 1;
    } else if (spec.rfind("lcg:", 0) == 0) {
        uint32_t s = (uint32_t)std::strtoul(spec.c_str() + 4, nullptr, 0);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                s = s * 1664525u + 1013904223u;
                p[i][j] = (int)(s >> 24);
            }
    } else if (spec.rfind("synth:", 0) == 0) {
        char* end = nullptr;
        uint32_t seed = (uint32_t)std::strtoul(spec.c_str() + 6, &end, 0);
        long index = (end && *end == ':') ? std::strtol(end + 1, nullptr, 0) : 0;
        for (long r = 0; r < n; ++r)
            for (long c = 0; c < n; ++c) {
                uint64_t idx = ((uint64_t)index * (uint64_t)n + (uint64_t)r) * (uint64_t)n + (uint64_t)c;
                p[r][c] = (int)(mix32(seed ^ (uint32_t)(idx ^ (idx >> 32))) >> 24);
            }
    } else if (spec.rfind("file:", 0) == 0) {
        FILE* f = std::fopen(spec.c_str() + 5, "rb");
        if (!f) {
            std::perror("input file");
            std::exit(2);
        }
        for (int i = 0; i < n; ++i)
            if (std::fread(p[i], sizeof(int), n, f) != (size_t)n) {
                std::fprintf(stderr, "short input file\n");
                std::exit(2);
            }
        std::fclose(f);
    } else {
        std::fprintf(stderr, "unknown input spec %s\n", spec.c_str());
        std::exit(2);
    }
    return p;
}

inline int octaves_of(int n) {
    int x = 0;
    while (n) {
        x++;
        n /= 2;
    }
    return x;
}

inline uint64_t fnv(const float* row, int len, uint64_t h) {
    for (int i = 0; i < len; ++i) {
        uint32_t b;
        std::memcpy(&b, row + i, 4);
        h = (h ^ b) * 0x100000001b3ull;
    }
    return h;
}

inline void dump(float**** G, int n, int S, const char* path) {
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        std::perror("dump");
        std::exit(2);
    }
    int len = n;
    for (int o = 0; o < octaves_of(n); ++o, len /= 2)
        for (int s = 0; s < S + 3; ++s)
            for (int r = 0; r < len; ++r) std::fwrite(G[o][s][r], sizeof(float), len, f);
    std::fclose(f);
}

inline void hash(float**** G, int n, int S) {
    int len = n;
    std::printf("{\"n\": %d, \"S\": %d, \"octaves\": [", n, S);
    for (int o = 0; o < octaves_of(n); ++o, len /= 2) {
        std::printf("%s[", o ? ", " : "");
        for (int s = 0; s < S + 3; ++s) {
            uint64_t h = 0xcbf29ce484222325ull;
            for (int r = 0; r < len; ++r) h = fnv(G[o][s][r], len, h);
            std::printf("%s\"%016llx\"", s ? ", " : "", (unsigned long long)h);
        }
        std::printf("]");
    }
    std::printf("]}\n");
}

}  // namespace refh

#endif  // GDP_ORACLE_REF_COMMON_H
