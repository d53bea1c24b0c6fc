/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's Gaussian / Difference-of-Gaussians pyramid
 * (ZhangShuui/SIFT-parallel-optimization, GuassDePyramid.h).  It is the CHECKER for the HIP
 * product path: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  Nothing in sift-parallel-optimization_amd/ links, loads or falls back to it.
 *
 * Parity is pinned: tests/test_oracle.py checks every function here against the golden
 * vectors in tests/golden/, which tests/golden/gen_golden.py produced from the reference's
 * own GuassDePyramid.h compiled in place (oracle/ref_harness.cpp, oracle/Makefile).
 *
 * Build: gcc -O2 -fPIC -shared -ffp-contract=off (no -ffast-math: denormals and the exact
 * rounding order are part of the contract, see DESIGN.md "bit-exactness").
 *
 * Pyramid layout used by every function here ("packed" layout):
 *   level (o, s), o in [0, O), s in [0, S+3), is an H_o x W_o row-major float32 array,
 *   H_o = H >> o, W_o = W >> o, levels stored back to back in (o, s) order.
 * After a full build level (o, s) holds DoG_s = G_s - G_{s+1} for s <= S+1 and
 * level (o, S+2) still holds G_{S+2}  (GuassDePyramid.h:136-149).
 *
 * The reference is square-only (the width argument is commented out, GuassDePyramid.h:15).  The non-square
 * extension used here applies the W-derived window along columns and the H-derived window along
 * rows; for H == W it is the reference's algorithm exactly.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* GuassDePyramid.h:7-8 — note PI is intentionally 3.1414926f in the reference. */
static const float kSigma = 2.0f;
static const float kPI = 3.1414926f;

/* GuassDePyramid.h:48-53: layer = number of halvings until len reaches 0. */
int gdo_octaves(int n) {
    int x = 0;
    while (n) {
        x++;
        n /= 2;
    }
    return x;
}

/* Level geometry of the packed layout. */
size_t gdo_level_offset(int H, int W, int S, int o, int s) {
    size_t off = 0;
    for (int q = 0; q < o; ++q) off += (size_t)(S + 3) * (size_t)(H >> q) * (size_t)(W >> q);
    return off + (size_t)s * (size_t)(H >> o) * (size_t)(W >> o);
}

size_t gdo_pyramid_floats(int H, int W, int S, int O) { return gdo_level_offset(H, W, S, O, 0); }

/*
 * Window taps of octave `octave`, scale `scale` for an axis of `length` input pixels.
 * GuassDePyramid.h:107-121:
 *   float len = length; halve it `octave` times in float; MyLen = (int)len; len = (len-1)/2;
 *   sig = sigma/(i+1); filter[k] = exp(-(k-len)*(k-len)/(2*sig*sig)) / (sig*sqrt(2*PI))
 * In C++ `exp(float)`/`sqrt(float)` are the float overloads, i.e. glibc expf/sqrtf; the
 * expression below has the same operand types and evaluation order.  Returns MyLen.
 */
int gdo_taps_centre(int length, int octave, int scale, float* out, int centre_mode) {
    float len = (float)length;
    for (int t = octave; t != 0; --t) len /= 2; /* :109-112 */
    int my_len = (int)len;                      /* :114 */
    if (centre_mode == 1)
        /* The multi-process variants centre on the INTEGER length: `len /= 2` on an int
         * (GaussDePyramid-MPI.h:289, mpitest.cpp:62,139) and `l = float(len - 1) / 2.0`
         * (GaussDePyramid-MPI.h:273, mpitest.cpp:44,123); the tap expression is the same
         * (GaussDePyramid-MPI.h:278,283; mpitest.cpp:50,56). */
        len = (float)((double)(float)(my_len - 1) / 2.0);
    else
        len = (len - 1) / 2;                    /* :115 */
    float sig = kSigma / (scale + 1);           /* :118 */
    for (int i = 0; i < my_len; ++i) {          /* :119-121 */
        out[i] = expf(-(i - len) * (i - len) / (2 * sig * sig)) / (sig * sqrtf(2 * kPI));
    }
    return my_len;
}

int gdo_taps(int length, int octave, int scale, float* out) { return gdo_taps_centre(length, octave, scale, out, 0); }

/*
 * Closed form of GaussPyInit + GenerateDoG (GuassDePyramid.h:60-87, 106-149) for the first O
 * octaves.  Octaves are independent because every octave decimates the ORIGINAL image
 * (:80 `data[k*step][l*step]`), so the first O octaves of a full build equal this.
 *   G_s[r][c] = ((float)img[r<<o][c<<o] * fc_s[c]) * fr_s[r]   (row pass :122-126 first,
 *                                                              then column pass :127-131)
 *   out_s = G_s - G_{s+1} (s ascending, :140-146),  out_{S+2} = G_{S+2}.
 * img has a row pitch of `pitch` int32 elements.  `taps` is scratch of >= 2*(S+3)*max(H,W)
 * floats.
 */
void gdo_build_centre(const int32_t* img, int H, int W, long pitch, int S, int O, float* out, float* taps,
                      int centre_mode) {
    const int L = S + 3;
    const int mx = H > W ? H : W;
    float* fc = taps;                  /* [L][mx] column-index taps (from W) */
    float* fr = taps + (size_t)L * mx; /* [L][mx] row-index taps (from H)    */
    for (int o = 0; o < O; ++o) {
        const int Ho = H >> o, Wo = W >> o;
        for (int s = 0; s < L; ++s) {
            gdo_taps_centre(W, o, s, fc + (size_t)s * mx, centre_mode);
            gdo_taps_centre(H, o, s, fr + (size_t)s * mx, centre_mode);
        }
        float* lev[64];
        for (int s = 0; s < L; ++s) lev[s] = out + gdo_level_offset(H, W, S, o, s);
#pragma omp parallel for schedule(static)
        for (int r = 0; r < Ho; ++r) {
            const int32_t* src = img + (size_t)(r << o) * (size_t)pitch;
            for (int c = 0; c < Wo; ++c) {
                const float x = (float)src[(size_t)c << o];
                float g_prev = (x * fc[c]) * fr[r];
                for (int s = 0; s + 1 < L; ++s) {
                    const float g_next = (x * fc[(size_t)(s + 1) * mx + c]) * fr[(size_t)(s + 1) * mx + r];
                    lev[s][(size_t)r * Wo + c] = g_prev - g_next;
                    g_prev = g_next;
                }
                lev[L - 1][(size_t)r * Wo + c] = g_prev;
            }
        }
    }
}

/* GuassDePyramid.h's closed form (serial window centre). */
void gdo_build(const int32_t* img, int H, int W, long pitch, int S, int O, float* out, float* taps) {
    gdo_build_centre(img, H, W, pitch, S, O, out, taps, 0);
}

/*
 * One row of every level of octave o — the closed form above (GuassDePyramid.h:76-86 refill,
 * :122-131 row then column window, :140-146 DoG) restricted to level row r, for checking sampled
 * rows of images too large to restate whole (65536^2: 114 GB of pyramid).
 * in_row = input row r << o (W int32); out = [S+3][W >> o]; taps scratch >= 2*(S+3)*max(H,W).
 */
void gdo_level_row(const int32_t* in_row, int H, int W, int S, int o, int r, float* out, float* taps) {
    const int L = S + 3, Wo = W >> o;
    float* fc = taps;
    float* fr = taps + (size_t)L * Wo;
    float* hwin = fr + L; /* row-index taps: only entry r of each scale's H-axis window is used */
    for (int s = 0; s < L; ++s) {
        gdo_taps(W, o, s, fc + (size_t)s * Wo);
        gdo_taps(H, o, s, hwin);
        fr[s] = hwin[r];
    }
    for (int c = 0; c < Wo; ++c) {
        const float x = (float)in_row[(size_t)c << o];
        float g_prev = (x * fc[c]) * fr[0];
        for (int s = 0; s + 1 < L; ++s) {
            const float g_next = (x * fc[(size_t)(s + 1) * Wo + c]) * fr[s + 1];
            out[(size_t)s * Wo + c] = g_prev - g_next;
            g_prev = g_next;
        }
        out[(size_t)(L - 1) * Wo + c] = g_prev;
    }
}

/* GaussPyInit refill (GuassDePyramid.h:74-86): every scale of octave o is (float)img[k<<o][l<<o]. */
void gdo_init(const int32_t* img, int H, int W, long pitch, int S, int O, float* pyr) {
    for (int o = 0; o < O; ++o) {
        const int Ho = H >> o, Wo = W >> o;
        for (int s = 0; s < S + 3; ++s) {
            float* lev = pyr + gdo_level_offset(H, W, S, o, s);
            for (int k = 0; k < Ho; ++k)
                for (int l = 0; l < Wo; ++l)
                    lev[(size_t)k * Wo + l] = (float)img[(size_t)(k << o) * (size_t)pitch + ((size_t)l << o)];
        }
    }
}

/* GaussFilter(o) in place (GuassDePyramid.h:106-134): row pass then column pass, per scale. */
void gdo_gauss_octave_centre(float* pyr, int H, int W, int S, int o, float* taps, int centre_mode) {
    const int Ho = H >> o, Wo = W >> o;
    const int mx = H > W ? H : W;
    float* fc = taps;
    float* fr = taps + mx;
    for (int s = 0; s < S + 3; ++s) {
        gdo_taps_centre(W, o, s, fc, centre_mode);
        gdo_taps_centre(H, o, s, fr, centre_mode);
        float* lev = pyr + gdo_level_offset(H, W, S, o, s);
        for (int j = 0; j < Ho; ++j) /* :122-126 row pass, column-index tap */
            for (int k = 0; k < Wo; ++k) lev[(size_t)j * Wo + k] *= fc[k];
        for (int j = 0; j < Wo; ++j) /* :127-131 column pass, row-index tap (column-major walk) */
            for (int k = 0; k < Ho; ++k) lev[(size_t)k * Wo + j] *= fr[k];
    }
}

void gdo_gauss_octave(float* pyr, int H, int W, int S, int o, float* taps) {
    gdo_gauss_octave_centre(pyr, H, W, S, o, taps, 0);
}

/* DoG subtraction of one octave in place (GuassDePyramid.h:140-146), s ascending. */
void gdo_dog_octave(float* pyr, int H, int W, int S, int o) {
    const size_t n = (size_t)(H >> o) * (size_t)(W >> o);
    for (int j = 0; j < S + 2; ++j) {
        float* a = pyr + gdo_level_offset(H, W, S, o, j);
        const float* b = pyr + gdo_level_offset(H, W, S, o, j + 1);
        for (size_t i = 0; i < n; ++i) a[i] -= b[i];
    }
}

/* GenerateDoG (GuassDePyramid.h:136-149) in place on the current pyramid contents, in the
 * reference's operation order.  Called on a fresh GaussPyInit it equals gdo_build; called again
 * it re-filters the DoG levels, which is what the reference's repeated-call timing loop does
 * (main.cpp:66-73). */
void gdo_generate_dog_centre(float* pyr, int H, int W, int S, int O, float* taps, int centre_mode) {
    for (int o = 0; o < O; ++o) {
        gdo_gauss_octave_centre(pyr, H, W, S, o, taps, centre_mode);
        gdo_dog_octave(pyr, H, W, S, o);
    }
}

void gdo_generate_dog(float* pyr, int H, int W, int S, int O, float* taps) {
    gdo_generate_dog_centre(pyr, H, W, S, O, taps, 0);
}

/* GaussPyramid_a512omp::GenerateDoG_nomp_dynamic (GaussDePyramid-AVX512xOpenMP.h:240-364)
 * output semantics restated (scalar): scales 0..S-1 of every octave are filtered with the
 * integer-length window centre float(len-1)/2 (:251,:279), then for i < S-1 level i -= level i+1
 * (:337-343).  Levels S..S+2 keep the GaussPyInit values.  Used only as a "port" CPU baseline
 * when the reference build (oracle/_ref) is absent. */
static void subset_taps(int len, float sig, float* f) {
    const float l = (float)(len - 1) / 2.0f; /* :251, :279 integer-length centre */
    for (int k = 0; k < len; ++k) f[k] = expf(-(k - l) * (k - l) / (2 * sig * sig)) / (sig * sqrtf(2 * kPI));
}

void gdo_subset_a512omp(float* pyr, int H, int W, int S, int O, float* taps) {
    const int mx = H > W ? H : W;
    float* fc = taps;
    float* fr = taps + mx;
    for (int i = 0; i < S; ++i) {
        const float sig = kSigma / (i + 1);
        for (int o = 0; o < O; ++o) {
            const int Ho = H >> o, Wo = W >> o;
            float* lev = pyr + gdo_level_offset(H, W, S, o, i);
            subset_taps(Wo, sig, fc);
            subset_taps(Ho, sig, fr);
#pragma omp parallel for schedule(static)
            for (int m = 0; m < Ho; ++m) /* :289-309 row pass then column pass, fused per row */
                for (int n = 0; n < Wo; ++n) lev[(size_t)m * Wo + n] = (lev[(size_t)m * Wo + n] * fc[n]) * fr[m];
        }
    }
    for (int o = 0; o < O; ++o)
        for (int i = 0; i < S - 1; ++i) { /* :337-357 */
            const long n = (long)(H >> o) * (long)(W >> o);
            float* a = pyr + gdo_level_offset(H, W, S, o, i);
            const float* b = pyr + gdo_level_offset(H, W, S, o, i + 1);
#pragma omp parallel for schedule(static)
            for (long k = 0; k < n; ++k) a[k] -= b[k];
        }
}

/* FNV-style level hash of SURVEY.md Appendix A: h = (h ^ bits32) * 0x100000001b3 over the
 * float32 bit patterns in row-major order, h0 = 0xcbf29ce484222325. */
uint64_t gdo_fnv(const float* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) {
        uint32_t b;
        memcpy(&b, p + i, 4);
        h = (h ^ b) * 0x100000001b3ull;
    }
    return h;
}

/* Parity input: s = s*1664525 + 1013904223 (mod 2^32), px = s >> 24,
 * row-major over an H x W image. */
void gdo_lcg_image(int32_t* img, int H, int W, uint32_t seed) {
    uint32_t s = seed;
    for (long i = 0; i < (long)H * W; ++i) {
        s = s * 1664525u + 1013904223u;
        img[i] = (int32_t)(s >> 24);
    }
}

/* Benchmark input: counter hash, so every GPU can generate its own shard.
 * idx = (b*H + r)*W + c (64-bit), x = seed ^ (uint32)(idx ^ (idx >> 32)), lowbias32 mix,
 * px = x >> 24 in [0, 255]. */
static uint32_t gdo_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

/* Row r of gdo_synthetic_image (W int32): the same counter hash. */
void gdo_synthetic_row(int32_t* row, int H, int W, uint32_t seed, long image_index, long r) {
    for (long c = 0; c < W; ++c) {
        const uint64_t idx = ((uint64_t)image_index * (uint64_t)H + (uint64_t)r) * (uint64_t)W + (uint64_t)c;
        row[c] = (int32_t)(gdo_mix32(seed ^ (uint32_t)(idx ^ (idx >> 32))) >> 24);
    }
}

void gdo_synthetic_image(int32_t* img, int H, int W, uint32_t seed, long image_index) {
    for (long r = 0; r < H; ++r)
        for (long c = 0; c < W; ++c) {
            const uint64_t idx = ((uint64_t)image_index * (uint64_t)H + (uint64_t)r) * (uint64_t)W + (uint64_t)c;
            img[r * W + c] = (int32_t)(gdo_mix32(seed ^ (uint32_t)(idx ^ (idx >> 32))) >> 24);
        }
}
