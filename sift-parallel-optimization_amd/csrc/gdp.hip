// libgdp.so — MI355X (gfx950) Gaussian / Difference-of-Gaussians pyramid: HIP kernels + C ABI.
//
// Hot path replaced: GuassDePyramid.h GaussPyInit (:60-87) + GaussFilter (:106-134) +
// GenerateDoG (:136-149) of ZhangShuui/SIFT-parallel-optimization.  The reference's "Gaussian"
// is a rank-1 WINDOW, not a convolution: level (o, s) pixel (r, c) is
//     G_s = ((float)img[r<<o][c<<o] * fc_{o,s}[c]) * fr_{o,s}[r]
// (row pass with the column-index tap first, :122-126, then the column pass with the row-index
// tap, :127-131), and the DoG is DoG_s = G_s - G_{s+1}, s ascending, level S+2 keeping G_{S+2}
// (:140-146).  No neighbourhood, so no halo and no LDS staging: the op is a pure HBM stream —
// read 4 B per input pixel, write 4*(S+3) B per pyramid pixel — and the kernels below are built
// for that roofline.
//
// Bit-exactness contract: taps are computed on the HOST with glibc expf/sqrtf exactly
// as GuassDePyramid.h:119-121 does and uploaded; every product/difference is a single IEEE
// binary32 operation in the reference's order — FP contraction is disabled for this file
// (pragma below + -ffp-contract=off in the Makefile) and f32 denormals are kept (gfx950 default
// .amdhsa_float_denorm_mode_32 = 3; never built with -ffast-math / FTZ).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "gdp.h"

#pragma clang fp contract(off)

namespace {

// ------------------------------------------------------------------------------------------
// geometry
// ------------------------------------------------------------------------------------------
constexpr int kMaxOct = 32;
constexpr int kBlock = 256;     // 4 waves (in-place / synthetic kernels)
constexpr int kTailGroups = 256; // groups of 4 pixels per tail work unit
constexpr int kLevBlock = 1024;  // threads (= 4-pixel groups) per block of the in-place passes
constexpr int kFused = 5;       // octaves 0..4 share one 16 x 256 input tile
constexpr int kTileRows = 16;   // 2^(kFused-1): every fused octave has whole rows in a tile
constexpr int kTileCols = 256;  // tile width of the register octave-0 path (64 lanes x 4 pixels)
constexpr int kLevelAlign = 64; // floats (256 B) — every level starts 16-B (and 256-B) aligned
constexpr size_t kStageFloats = size_t(16) << 20;  // pinned D2H staging chunk (64 MiB)

struct OctGeom {
    int rows;             // output rows of this octave held by the context (band-local)
    int row0;             // global output row of band-local row 0
    int cols;             // W >> o
    int gpr;              // groups of 4 columns per row, ceil(cols / 4)
    long long lev_off;    // floats from an image's pyramid base to level (o, 0)
    long long lev_stride; // floats from level (o, s) to (o, s+1)
    int ctap;             // float offset of column taps (o, 0) in the tap table
    int ctap_stride;      // floats between scales (multiple of 4, zero padded)
    int rtap;             // float offset of row taps (o, 0), indexed by GLOBAL output row
    int rtap_stride;
    long long grp_begin;  // prefix (over octaves 0..o-1) of rows*gpr per image
    unsigned long long gpr_magic; // fast k / gpr for k < 2^31: (k * magic) >> gpr_shift
    int gpr_shift;
    int pad_;
};

// Granlund-Montgomery division by an invariant d >= 1 for numerators n < 2^31:
// magic = ceil(2^(31+l) / d), l = ceil(log2 d); n / d == (n * magic) >> (31 + l).
inline void make_magic(unsigned d, unsigned long long* magic, int* shift) {
    int l = 0;
    while ((1ull << l) < d) ++l;
    *shift = 31 + l;
    *magic = ((1ull << *shift) + d - 1) / d;
}

__device__ __forceinline__ unsigned fast_div(unsigned n, unsigned long long magic, int shift) {
    return (unsigned)(((unsigned long long)n * magic) >> shift);
}

struct Geom {
    int H, W, S, L, O, F, batch;
    int in_rows, in_row0; // input rows held (band) and their first global row
    int vec_in;           // one vector load per 4 pixels legal (pitch % 4 == 0, base aligned)
    int tile_order;       // GDP_TUNE_TILE_ORDER
    int in_fmt;           // GDP_INPUT_I32 / GDP_INPUT_U8
    int pad2_;
    long long in_pitch, in_img_stride;
    long long pyr_stride; // floats between image pyramids
    int tiles_r, tiles_c;
    unsigned tiles_per_img, tiles_total;       // host checks the unit count fits 31 bits
    unsigned tail_groups_per_img, tail_units;  // octaves >= F, 256 groups per unit
    OctGeom oct[kMaxOct];
    unsigned lv_blk[kMaxOct + 1]; // prefix over octaves of ceil(rows*gpr / kLevBlock) per image
    unsigned lx_blk[kMaxOct + 1]; // prefix over octaves of ceil(rows*gpr / 64) per image (k_levels_x)
    unsigned cv_blk[kMaxOct + 1]; // convolution mode: prefix over octaves of 16x256 output tiles
    int cv_tiles_c[kMaxOct];      // convolution mode: tile columns per octave
    unsigned sw_blk[kMaxOct + 1]; // convolution sweep: prefix over octaves of blocks (4 strips of T rows);
                                  // octaves whose width is not a multiple of 4 count 0 (tiles do them)
    int sw_strips_c[kMaxOct];     // convolution sweep: 240-column strips per octave
    unsigned cvx_blk[kMaxOct + 1]; // convolution tiles for the octaves the sweep skips
};

typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ f4 ld_f4(const float* p) { return *reinterpret_cast<const f4*>(p); }

// Streaming load of pyramid data that is read once per pass (in-place passes): non-temporal.
template <bool NT>
__device__ __forceinline__ f4 ld_stream(const float* p) {
    if constexpr (NT)
        return __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
    else
        return *reinterpret_cast<const f4*>(p);
}

template <bool NT>
__device__ __forceinline__ void st_f4(float* p, f4 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p));
    else
        *reinterpret_cast<f4*>(p) = v;
}

// Stores the first `n` lanes of v (n in 1..4) — ragged right edge or unaligned rows.
__device__ __forceinline__ void st_part(float* p, f4 v, int n, bool aligned_full) {
    if (aligned_full) {
        *reinterpret_cast<f4*>(p) = v;
        return;
    }
    p[0] = v.x;
    if (n > 1) p[1] = v.y;
    if (n > 2) p[2] = v.z;
    if (n > 3) p[3] = v.w;
}

// Input pixels (R, C..C+3) of octave o for image b as float (zero beyond the row end).  The
// input is int32 (the reference's `int** img`) or uint8 (GDP_INPUT_U8: 4x fewer input bytes);
// the format is a wave-uniform scalar branch.  (float) of an int32 or uint8 value is the same
// single rounding the reference's `GaussPy[..] = data[..]` assignment performs (:80).
__device__ __forceinline__ f4 load_px(const Geom* __restrict__ g, const void* __restrict__ in, int b, int o,
                                      int Rg, int C, int n) {
    const long long in_row = ((long long)Rg << o) - g->in_row0;
    const long long row_off = (long long)b * g->in_img_stride + in_row * g->in_pitch;
    f4 x = {0.f, 0.f, 0.f, 0.f};
    if (g->in_fmt == GDP_INPUT_U8) {
        const unsigned char* row = static_cast<const unsigned char*>(in) + row_off;
        if (o == 0 && n == 4 && g->vec_in) {
            const unsigned w = *reinterpret_cast<const unsigned*>(row + C);
            x.x = (float)(w & 0xffu);
            x.y = (float)((w >> 8) & 0xffu);
            x.z = (float)((w >> 16) & 0xffu);
            x.w = (float)(w >> 24);
            return x;
        }
        x.x = (float)row[(long long)C << o];
        if (n > 1) x.y = (float)row[(long long)(C + 1) << o];
        if (n > 2) x.z = (float)row[(long long)(C + 2) << o];
        if (n > 3) x.w = (float)row[(long long)(C + 3) << o];
        return x;
    }
    const int* row = static_cast<const int*>(in) + row_off;
    if (o == 0 && n == 4 && g->vec_in) {
        const i4 v = *reinterpret_cast<const i4*>(row + C);
        return __builtin_convertvector(v, f4);
    }
    x.x = (float)row[(long long)C << o];
    if (n > 1) x.y = (float)row[(long long)(C + 1) << o];
    if (n > 2) x.z = (float)row[(long long)(C + 2) << o];
    if (n > 3) x.w = (float)row[(long long)(C + 3) << o];
    return x;
}

// One group = 4 consecutive output pixels (Rl, C..C+3) of octave o, all S+3 scales.
// G_s = (x * fc_s) * fr_s ; out_s = G_s - G_{s+1} ; out_{L-1} = G_{L-1}.
template <int LT, bool NT>
__device__ __forceinline__ void build_group(const Geom* __restrict__ g, const void* __restrict__ in,
                                            float* __restrict__ out, const float* __restrict__ taps, int b,
                                            int o, const OctGeom& og, int Rl, int C) {
    const int L = LT > 0 ? LT : g->L;
    const int n = min(4, og.cols - C);
    const int Rg = og.row0 + Rl;
    const f4 x = load_px(g, in, b, o, Rg, C, n);
    const float* ct = taps + og.ctap + C;
    const float* rt = taps + og.rtap + Rg;
    float* dst = out + (long long)b * g->pyr_stride + og.lev_off + (long long)Rl * og.cols + C;
    const bool full = (n == 4) && ((og.cols & 3) == 0);
    f4 gp = (x * ld_f4(ct)) * rt[0];
#pragma unroll
    for (int s = 0; s + 1 < L; ++s) {
        const f4 gn = (x * ld_f4(ct + (s + 1) * og.ctap_stride)) * rt[(s + 1) * og.rtap_stride];
        const f4 d = gp - gn;
        if (full)
            st_f4<NT>(dst + s * og.lev_stride, d);
        else
            st_part(dst + s * og.lev_stride, d, n, false);
        gp = gn;
    }
    if (full)
        st_f4<NT>(dst + (L - 1) * og.lev_stride, gp);
    else
        st_part(dst + (L - 1) * og.lev_stride, gp, n, false);
}

// Octave 0 of one 16 x 256 tile, S+3 = LT known at compile time: wave w owns tile rows w, w+4,
// w+8, w+12 and lane l owns columns 4l..4l+3 of each.  The LT column windows of the lane are
// loaded once into registers and reused for the 4 rows; the row windows are wave-uniform
// (scalar loads); the 4 int4 input loads are issued before any arithmetic.  Every wave store is
// 64 lanes x 16 B = 1 KiB contiguous of one level row.
template <int LT, bool NT>
__device__ __forceinline__ void tile_octave0(const Geom* __restrict__ g, const void* __restrict__ in,
                                             float* __restrict__ out, const float* __restrict__ taps, int b,
                                             int in_r0, int in_c0) {
    const OctGeom og = g->oct[0];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int C = in_c0 + 4 * lane;
    if (C >= og.cols) return;
    const int n = min(4, og.cols - C);
    const bool full = (n == 4) && ((og.cols & 3) == 0);
    constexpr int kRows = kTileRows / 4;
    f4 fc[LT];
#pragma unroll
    for (int s = 0; s < LT; ++s) fc[s] = ld_f4(taps + og.ctap + s * og.ctap_stride + C);
    f4 x[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
        const int Rl = in_r0 + wave + 4 * k;
        x[k] = Rl < og.rows ? load_px(g, in, b, 0, og.row0 + Rl, C, n) : f4{0.f, 0.f, 0.f, 0.f};
    }
    float* base = out + (long long)b * g->pyr_stride + og.lev_off + C;
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
        const int Rl = in_r0 + wave + 4 * k; // wave-uniform
        if (Rl >= og.rows) break;
        const float* rt = taps + og.rtap + og.row0 + Rl;
        float* dst = base + (long long)Rl * og.cols;
        f4 gp = (x[k] * fc[0]) * rt[0];
#pragma unroll
        for (int s = 0; s + 1 < LT; ++s) {
            const f4 gn = (x[k] * fc[s + 1]) * rt[(s + 1) * og.rtap_stride];
            if (full)
                st_f4<NT>(dst + s * og.lev_stride, gp - gn);
            else
                st_part(dst + s * og.lev_stride, gp - gn, n, false);
            gp = gn;
        }
        if (full)
            st_f4<NT>(dst + (LT - 1) * og.lev_stride, gp);
        else
            st_part(dst + (LT - 1) * og.lev_stride, gp, n, false);
    }
}

// Fused build.  Work units: [0, tiles_total) are 16 x 256 input tiles (octaves 0..F-1 of the
// tile: octave o covers (16>>o) rows x (256>>o) columns, reading lines the o = 0 pass of the
// same block just brought on chip); [tiles_total, +tail_units) are 256-group slices of the tiny
// octaves >= F.  Default launch: one unit per block (the dispatcher back-fills CUs as blocks
// retire, which measured faster than a persistent grid); the grid-stride loop serves capped grids.
// BLK = threads per block; O0REG selects the register-resident octave-0 path (BLK = 256 only).
template <int LT, bool NT, int BLK, int TC, bool O0REG, int TR>
__device__ __forceinline__ void build_body(const Geom* __restrict__ g, const void* __restrict__ in,
                                           float* __restrict__ out, const float* __restrict__ taps) {
    const unsigned tiles_total = g->tiles_total;
    const unsigned units = tiles_total + g->tail_units;
    const int F = g->F;
    for (unsigned u = blockIdx.x; u < units; u += gridDim.x) {
        if (u < tiles_total) {
            // tile order: 0 = linear; 1 = XCD-chunked (blocks b and b+8 share an XCD under the
            // observed round-robin dispatch, so XCD x walks the contiguous tile range x/8 of the
            // grid) — a speed knob only, any order gives the same bits
            unsigned t = u;
            if (g->tile_order == 1 && (tiles_total & 7u) == 0) {
                t = (u & 7u) * (tiles_total >> 3) + (u >> 3);
            } else if (g->tile_order == 2 && ((tiles_total / (unsigned)g->tiles_c) & 7u) == 0) {
                // XCD row-interleave: XCD x sweeps whole tile rows x, x+8, ... left to right
                const unsigned k = u >> 3, tcs = (unsigned)g->tiles_c;
                const unsigned q = k / tcs;
                t = (q * 8u + (u & 7u)) * tcs + (k - q * tcs);
            }
            const unsigned b = t / g->tiles_per_img;
            const unsigned rem = t - b * g->tiles_per_img;
            const unsigned tr = rem / (unsigned)g->tiles_c;
            const unsigned tc = rem - tr * (unsigned)g->tiles_c;
            const int in_r0 = (int)tr * TR; // band-local input row of the tile
            const int in_c0 = (int)tc * TC;
            constexpr int kFusedT = TR == 16 ? 5 : TR == 8 ? 4 : TR == 4 ? 3 : TR == 2 ? 2 : 1; // log2(TR)+1
#pragma unroll
            for (int o = 0; o < kFusedT; ++o) {
                if (o >= F) break;
                if constexpr (LT > 0 && O0REG && BLK == 256 && TC == kTileCols && TR == kTileRows) {
                    if (o == 0) {
                        tile_octave0<LT, NT>(g, in, out, taps, (int)b, in_r0, in_c0);
                        continue;
                    }
                }
                const OctGeom og = g->oct[o];
                const int gpr_t = (TC / 4) >> o; // groups per tile row (TC = 256: 64, 32, 16, 8, 4)
                const int groups = (TR >> o) * gpr_t;
#pragma unroll
                for (int q0 = 0; q0 < groups; q0 += BLK) {
                    const int q = q0 + (int)threadIdx.x;
                    if (q >= groups) break;
                    const int r = q / gpr_t;
                    const int cg = q - r * gpr_t;
                    // band-local output row: in_row0 is a multiple of 16, so local input row
                    // in_r0 + (r << o) maps to local output row (in_r0 >> o) + r.
                    const int Rl = (in_r0 >> o) + r;
                    const int C = (in_c0 >> o) + 4 * cg;
                    if (Rl < og.rows && C < og.cols) build_group<LT, NT>(g, in, out, taps, (int)b, o, og, Rl, C);
                }
            }
        } else {
            for (int q = threadIdx.x; q < kTailGroups; q += BLK) {
                const unsigned t = (u - tiles_total) * kTailGroups + q;
                const unsigned per = g->tail_groups_per_img;
                if (t >= per * (unsigned)g->batch) break;
                const unsigned b = t / per;
                const long long rem = (long long)(t - b * per) + g->oct[F].grp_begin;
                int o = F;
                while (o + 1 < g->O && rem >= g->oct[o + 1].grp_begin) ++o;
                const OctGeom og = g->oct[o];
                const int k = (int)(rem - og.grp_begin);
                const int Rl = k / og.gpr;
                const int C = 4 * (k - Rl * og.gpr);
                build_group<LT, NT>(g, in, out, taps, (int)b, o, og, Rl, C);
            }
        }
    }
}

template <int LT, bool NT, int BLK, int TC, bool O0REG, int TR>
__global__ void __launch_bounds__(BLK) k_build(const Geom* __restrict__ g, const void* __restrict__ in,
                                               float* __restrict__ out, const float* __restrict__ taps) {
    build_body<LT, NT, BLK, TC, O0REG, TR>(g, in, out, taps);
}

// Build-kernel code variants (GDP_TUNE_VARIANT); all bit-identical, A/B'd by tools/tune.py.
struct BuildVariant {
    int block, tile_cols, tile_rows;
    void (*k[2][2])(const Geom*, const void*, float*, const float*); // [LT==5][NT]
};
#define GDP_VARIANT(BLK, TC, REG, TR)                                                             \
    BuildVariant {                                                                                \
        BLK, TC, TR, {{k_build<0, false, BLK, TC, REG, TR>, k_build<0, true, BLK, TC, REG, TR>},   \
                      {k_build<5, false, BLK, TC, REG, TR>, k_build<5, true, BLK, TC, REG, TR>}}   \
    }
const BuildVariant kVariants[] = {
    GDP_VARIANT(1024, 256, false, 16), // 0 (default): 16 waves, one octave-0 group per thread
    GDP_VARIANT(256, 256, true, 16),   // 1: 4 waves, register-resident octave 0 (4 groups per thread)
    GDP_VARIANT(512, 256, false, 16),  // 2: 8 waves, 2 groups per thread
    GDP_VARIANT(256, 256, false, 16),  // 3: 4 waves, generic loop
    GDP_VARIANT(512, 128, false, 16),  // 4: 8 waves, 16 x 128 tile, one group per thread
    GDP_VARIANT(1024, 512, false, 16), // 5: 16 waves, 16 x 512 tile, 2 groups per thread
    GDP_VARIANT(256, 64, false, 16),   // 6: 4 waves, 16 x 64 tile, one group per thread
    GDP_VARIANT(256, 256, false, 4),   // 7: 4 waves, 4 x 256 tile (octaves 0-2 fused, 3+ as tail units)
    GDP_VARIANT(512, 256, false, 8),   // 8: 8 waves, 8 x 256 tile (octaves 0-3 fused)
};

// Default variant for a width (tools/tune.py, MI355X): 1024 threads on 16 x 256 tiles (v0) is the
// fastest everywhere the width fills its tiles; when a 256-wide tile grid would leave more lanes
// idle than a 128-wide one (e.g. W = 1920: 7.5 tiles), 512 threads on 16 x 128 tiles (v4).
// A single image of <= 16 Mpix (e.g. the 4096^2 headline) is fastest on 8 x 256 tiles with 512
// threads (v8: 0.067 vs 0.073 ms at 4096^2); batches stream best with v0.  gdp_autotune measures.
int default_variant(int W, long long pixels, int batch) {
    const long long waste256 = (long long)((W + 255) / 256) * 256 - W;
    const long long waste128 = (long long)((W + 127) / 128) * 128 - W;
    if (waste256 * 128 > waste128 * 256) return 4;
    return (batch == 1 && pixels <= (1ll << 24)) ? 8 : 0;
}
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

// In-place passes over octaves [o_begin, o_end) of every image (GaussPyInit refill, GaussFilter,
// DoG, GenerateDoG re-entry).  MODE bits: 1 = window multiply (GaussFilter), 2 = DoG subtract,
// 4 = refill from the input (GaussPyInit; exclusive).  One block = kLevBlock consecutive groups
// (4 pixels each) of one octave's level rows; every thread owns one group across all S+3 levels:
// the S+3 float4 loads are issued together (LT known), then the rolling window/DoG and the stores.
// SUB splits each 1024-group chunk over SUB blocks of 1024/SUB threads (GDP_TUNE_INPLACE_SUB).
template <int LT, int MODE, bool NT, int SUB>
__global__ void __launch_bounds__(kLevBlock / SUB) k_levels(const Geom* __restrict__ g, const void* __restrict__ in,
                                                            float* __restrict__ out, const float* __restrict__ taps,
                                                            int o_begin, int o_end) {
    const unsigned first = g->lv_blk[o_begin];
    const unsigned per = g->lv_blk[o_end] - first;
    const unsigned chunk = blockIdx.x / SUB;
    const unsigned b = chunk / per;
    const unsigned v = chunk - b * per + first;
    int o = o_begin;
    while (o + 1 < o_end && v >= g->lv_blk[o + 1]) ++o;
    const OctGeom og = g->oct[o];
    const unsigned k = (v - g->lv_blk[o]) * kLevBlock + (blockIdx.x % SUB) * (kLevBlock / SUB) + threadIdx.x;
    if (k >= (unsigned)og.rows * (unsigned)og.gpr) return;
    const int Rl = (int)fast_div(k, og.gpr_magic, og.gpr_shift);
    const int C = 4 * (int)(k - (unsigned)Rl * (unsigned)og.gpr);
    const int n = min(4, og.cols - C);
    const bool full = (n == 4) && ((og.cols & 3) == 0);
    float* p = out + (long long)b * g->pyr_stride + og.lev_off + (long long)Rl * og.cols + C;
    const int L = LT > 0 ? LT : g->L;
    auto ld = [&](int s) -> f4 {
        const float* q = p + s * og.lev_stride;
        if (full) return ld_stream<NT>(q);
        f4 r = {q[0], 0.f, 0.f, 0.f};
        if (n > 1) r.y = q[1];
        if (n > 2) r.z = q[2];
        if (n > 3) r.w = q[3];
        return r;
    };
    auto st = [&](int s, f4 val) {
        if (full)
            st_f4<NT>(p + s * og.lev_stride, val);
        else
            st_part(p + s * og.lev_stride, val, n, false);
    };
    if constexpr (MODE == 4) {
        const f4 x = load_px(g, in, (int)b, o, og.row0 + Rl, C, n);
        for (int s = 0; s < L; ++s) st(s, x);
    } else {
        const int Rg = og.row0 + Rl;
        const float* ct = taps + og.ctap + C;
        const float* rt = taps + og.rtap + Rg;
        auto win = [&](int s, f4 val) -> f4 {
            if constexpr ((MODE & 1) != 0) return (val * ld_f4(ct + s * og.ctap_stride)) * rt[s * og.rtap_stride];
            return val;
        };
        if constexpr (LT > 0) {
            f4 x[LT];
#pragma unroll
            for (int s = 0; s < LT; ++s) x[s] = ld(s);
            if constexpr (MODE == 1) {
#pragma unroll
                for (int s = 0; s < LT; ++s) st(s, win(s, x[s]));
            } else {
                f4 gp = win(0, x[0]);
#pragma unroll
                for (int s = 0; s + 1 < LT; ++s) {
                    const f4 gn = win(s + 1, x[s + 1]);
                    st(s, gp - gn);
                    gp = gn;
                }
                if constexpr ((MODE & 1) != 0) st(LT - 1, gp);
            }
        } else if constexpr (MODE == 1) {
            for (int s = 0; s < L; ++s) st(s, win(s, ld(s)));
        } else {
            f4 gp = win(0, ld(0));
            for (int s = 0; s + 1 < L; ++s) {
                const f4 gn = win(s + 1, ld(s + 1));
                st(s, gp - gn);
                gp = gn;
            }
            if constexpr ((MODE & 1) != 0) st(L - 1, gp);
        }
    }
}

// GaussFilter pass (MODE 1 of the in-place passes) with one LEVEL per block slice: the levels of
// an octave are independent under the window, so every thread moves exactly one float4 (load,
// two multiplies, store) — the shape that streams best in place on MI355X (tools/membench:
// 1 float4 per lane with non-temporal load+store ≈ 6.5 TB/s vs ≈ 6.1 at 4 per lane).
template <bool NT, int SUB>
__global__ void __launch_bounds__(kLevBlock / SUB) k_window(const Geom* __restrict__ g, float* __restrict__ out,
                                                            const float* __restrict__ taps, int o_begin, int o_end) {
    const unsigned L = (unsigned)g->L;
    const unsigned first = g->lv_blk[o_begin] * L;
    const unsigned per = g->lv_blk[o_end] * L - first;
    const unsigned chunk = blockIdx.x / SUB;
    const unsigned b = chunk / per;
    const unsigned v = chunk - b * per + first;
    int o = o_begin;
    while (o + 1 < o_end && v >= g->lv_blk[o + 1] * L) ++o;
    const OctGeom og = g->oct[o];
    const unsigned nb = g->lv_blk[o + 1] - g->lv_blk[o]; // blocks per level of octave o
    const unsigned w = v - g->lv_blk[o] * L;
    const int s = (int)(w / nb);
    const unsigned k = (w - (unsigned)s * nb) * kLevBlock + (blockIdx.x % SUB) * (kLevBlock / SUB) + threadIdx.x;
    if (k >= (unsigned)og.rows * (unsigned)og.gpr) return;
    const int Rl = (int)fast_div(k, og.gpr_magic, og.gpr_shift);
    const int C = 4 * (int)(k - (unsigned)Rl * (unsigned)og.gpr);
    const int n = min(4, og.cols - C);
    const bool full = (n == 4) && ((og.cols & 3) == 0);
    float* p = out + (long long)b * g->pyr_stride + og.lev_off + (long long)s * og.lev_stride + (long long)Rl * og.cols + C;
    const f4 fc = ld_f4(taps + og.ctap + s * og.ctap_stride + C);
    const float fr = taps[og.rtap + s * og.rtap_stride + og.row0 + Rl];
    if (full) {
        st_f4<NT>(p, (ld_stream<NT>(p) * fc) * fr);
    } else {
        f4 r = {p[0], 0.f, 0.f, 0.f};
        if (n > 1) r.y = p[1];
        if (n > 2) r.z = p[2];
        if (n > 3) r.w = p[3];
        st_part(p, (r * fc) * fr, n, false);
    }
}

// DoG / GenerateDoG re-entry (MODE 2 / 3) with one LEVEL per wave: a block of 64 x L threads
// takes 64 four-pixel groups; wave s loads level s (one float4 per lane, like k_window), applies
// the window of scale s (MODE 3), parks the result in LDS, and after one barrier forms
// out_s = G_s - G_{s+1} from its own value and wave s+1's; level L-1 keeps G (MODE 3) or is left
// untouched (MODE 2).  In place is safe: every value a wave needs from another level is read
// (into LDS) before the barrier, every store happens after it, and blocks own disjoint pixels.
template <int MODE, bool NT>
__global__ void __launch_bounds__(1024) k_levels_x(const Geom* __restrict__ g, float* __restrict__ out,
                                                   const float* __restrict__ taps, int o_begin, int o_end) {
    __shared__ f4 xs[16][64];
    const unsigned first = g->lx_blk[o_begin];
    const unsigned per = g->lx_blk[o_end] - first;
    const unsigned b = blockIdx.x / per;
    const unsigned v = blockIdx.x - b * per + first;
    int o = o_begin;
    while (o + 1 < o_end && v >= g->lx_blk[o + 1]) ++o;
    const OctGeom og = g->oct[o];
    const int L = g->L;
    const int s = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const unsigned k = (v - g->lx_blk[o]) * 64u + (unsigned)lane;
    const bool valid = k < (unsigned)og.rows * (unsigned)og.gpr;
    int Rl = 0, C = 0, n = 0;
    float* p = nullptr;
    f4 gs = {0.f, 0.f, 0.f, 0.f};
    bool full = false;
    if (valid) {
        Rl = (int)fast_div(k, og.gpr_magic, og.gpr_shift);
        C = 4 * (int)(k - (unsigned)Rl * (unsigned)og.gpr);
        n = min(4, og.cols - C);
        full = (n == 4) && ((og.cols & 3) == 0);
        p = out + (long long)b * g->pyr_stride + og.lev_off + (long long)s * og.lev_stride + (long long)Rl * og.cols + C;
        if (full) {
            gs = ld_stream<NT>(p);
        } else {
            gs.x = p[0];
            if (n > 1) gs.y = p[1];
            if (n > 2) gs.z = p[2];
            if (n > 3) gs.w = p[3];
        }
        if constexpr ((MODE & 1) != 0)
            gs = (gs * ld_f4(taps + og.ctap + s * og.ctap_stride + C)) * taps[og.rtap + s * og.rtap_stride + og.row0 + Rl];
    }
    xs[s][lane] = gs;
    __syncthreads();
    if (!valid) return;
    if (s + 1 < L) {
        const f4 d = gs - xs[s + 1][lane];
        if (full)
            st_f4<NT>(p, d);
        else
            st_part(p, d, n, false);
    } else if constexpr ((MODE & 1) != 0) {
        if (full)
            st_f4<NT>(p, gs);
        else
            st_part(p, gs, n, false);
    }
}

// ------------------------------------------------------------------------------------------
// Extension (no reference counterpart, no parity claim): a TRUE separable
// Gaussian convolution pyramid.  Same octave bases (decimated input) and σ schedule
// (σ_s = sigma/(s+1)) and the same DoG layout as the reference, but G_s = base ⊛ k_s with
// normalised taps over radius R_s = ceil(3σ_s) and clamp-to-edge borders.  This is the stencil the
// north star's "LDS halo" design is for: each block stages its 16 x 256 output tile plus a 6-pixel
// halo of the base image in LDS once, then for every scale runs the horizontal pass LDS -> LDS
// and the vertical pass LDS -> registers, forms the DoG against the previous scale in registers
// and streams the S+3 levels out with 1-KiB wave stores.
// ------------------------------------------------------------------------------------------
constexpr int kCvTH = 16, kCvTW = 256;  // output tile
constexpr int kCvR = 6;                 // max radius: ceil(3 * sigma_0) with sigma_0 = 2
constexpr int kCvPadL = 8;              // left halo (16-B aligned rows)
constexpr int kCvInW = kCvTW + 2 * kCvPadL;
constexpr int kCvInH = kCvTH + 2 * kCvR;
constexpr int kCvMaxTaps = 2 * kCvR + 1;

// No bit-exactness contract in this mode, so the stencil uses fused multiply-adds explicitly
// (the file-wide contract(off) keeps the reference path unfused).
__device__ __forceinline__ f4 fma4(float k, f4 x, f4 acc) {
    const f4 kk = {k, k, k, k};
    return __builtin_elementwise_fma(kk, x, acc);
}

// Vertical pass first (rows of the staged tile carry the vertical halo): h_s[r][j] for the 16 output
// rows and all kCvInW staged columns (the horizontal halo included), one float4 column group and
// four rows per work item, the 4 + 2R input rows read once per item.
template <int R>
__device__ __forceinline__ void conv_v_pass(const float* __restrict__ in_s, float* __restrict__ h_s, const float* k,
                                            int tid) {
    // 2 x 68 items of 8 rows x 4 columns: one iteration for threads 0..135 (the 272-column staged
    // width is not a multiple of 256 lanes, so 4-row items would give one wave two iterations)
    constexpr int kG = kCvInW / 4; // float4 column groups per staged row
    constexpr int kRows = kCvTH / 2;
    if (tid >= 2 * kG) return;
    const int rq = tid / kG, j4 = tid - (tid / kG) * kG;
    f4 w[kRows + 2 * R];
#pragma unroll
    for (int j = 0; j < kRows + 2 * R; ++j)
        w[j] = *reinterpret_cast<const f4*>(in_s + (kCvR - R + kRows * rq + j) * kCvInW + 4 * j4);
#pragma unroll
    for (int q = 0; q < kRows; ++q) {
        f4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int d = 0; d <= 2 * R; ++d) o = fma4(k[d], w[q + d], o);
        *reinterpret_cast<f4*>(h_s + (kRows * rq + q) * kCvInW + 4 * j4) = o;
    }
}

// Horizontal pass: thread (rg, cg) produces output rows 4rg..4rg+3, columns 4cg..4cg+3, reading
// the aligned float4s that cover staged columns kCvPadL + 4cg - R .. kCvPadL + 4cg + 3 + R.
template <int R>
__device__ __forceinline__ void conv_h_pass(const float* __restrict__ h_s, const float* k, int tid, f4 (&g)[4]) {
    constexpr int kLo = (kCvPadL - R) / 4 * 4;
    constexpr int kN = (kCvPadL + 4 + R - kLo + 3) / 4;
    const int cg = tid & 63, rg = tid >> 6;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        float a[4 * kN];
        const float* src = h_s + (4 * rg + q) * kCvInW + 4 * cg + kLo;
#pragma unroll
        for (int j = 0; j < kN; ++j) {
            const f4 v = *reinterpret_cast<const f4*>(src + 4 * j);
            a[4 * j] = v.x;
            a[4 * j + 1] = v.y;
            a[4 * j + 2] = v.z;
            a[4 * j + 3] = v.w;
        }
        const float* w = a + (kCvPadL - R - kLo);
        f4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int d = 0; d <= 2 * R; ++d) {
            const f4 x = {w[d], w[d + 1], w[d + 2], w[d + 3]};
            o = fma4(k[d], x, o);
        }
        g[q] = o;
    }
}

template <int R>
__device__ __forceinline__ void conv_pass(const float* __restrict__ in_s, float* __restrict__ h_s, const float* k,
                                          int tid, f4 (&g)[4]) {
    conv_v_pass<R>(in_s, h_s, k, tid);
    __syncthreads();
    conv_h_pass<R>(h_s, k, tid, g);
    __syncthreads(); // h_s is rewritten by the next scale
}

template <bool NT>
__global__ void __launch_bounds__(256, 3) k_conv(const Geom* __restrict__ g, const void* __restrict__ in,
                                                 float* __restrict__ out, const float* __restrict__ ctaps,
                                                 const int* __restrict__ cradius, int rest) {
    __shared__ __attribute__((aligned(16))) float in_s[kCvInH * kCvInW];
    __shared__ __attribute__((aligned(16))) float h_s[kCvTH * kCvInW];
    const unsigned* pre = rest ? g->cvx_blk : g->cv_blk; // rest: only the octaves the sweep skips
    const unsigned per = pre[g->O];
    const unsigned b = blockIdx.x / per;
    const unsigned v = blockIdx.x - b * per;
    int o = 0;
    while (o + 1 < g->O && v >= pre[o + 1]) ++o;
    const OctGeom og = g->oct[o];
    const unsigned t = v - pre[o];
    const int tr = (int)(t / (unsigned)g->cv_tiles_c[o]);
    const int tc = (int)(t - (unsigned)tr * (unsigned)g->cv_tiles_c[o]);
    const int r0 = tr * kCvTH, c0 = tc * kCvTW; // octave-o output coordinates of the tile
    const int tid = threadIdx.x;
    const int rows = og.rows, cols = og.cols;
    // stage the base-image tile + halo (clamp-to-edge), decimated from the input, as float
    const long long img_off = (long long)b * g->in_img_stride;
    const bool interior = o == 0 && g->vec_in && g->in_fmt == GDP_INPUT_I32 && r0 - kCvR >= 0 &&
                          r0 + kCvTH + kCvR <= rows && c0 - kCvPadL >= 0 && c0 + kCvTW + kCvPadL <= cols;
    if (interior) {  // no clamping: 16-B int4 loads (all issued first), 16-B LDS stores
        const int* src = static_cast<const int*>(in) + img_off + (long long)(r0 - kCvR) * g->in_pitch + (c0 - kCvPadL);
        constexpr int kItems = kCvInH * (kCvInW / 4);
        constexpr int kIter = (kItems + 255) / 256;
        i4 v[kIter];
#pragma unroll
        for (int u = 0; u < kIter; ++u) {
            const int e = tid + 256 * u;
            const int i = e / (kCvInW / 4), j4 = e - i * (kCvInW / 4);
            if (e < kItems) v[u] = *reinterpret_cast<const i4*>(src + (long long)i * g->in_pitch + 4 * j4);
        }
#pragma unroll
        for (int u = 0; u < kIter; ++u) {
            const int e = tid + 256 * u;
            if (e < kItems) *reinterpret_cast<f4*>(in_s + 4 * e) = __builtin_convertvector(v[u], f4);
        }
    } else
    for (int e = tid; e < kCvInH * kCvInW; e += 256) {
        const int i = e / kCvInW, j = e - (e / kCvInW) * kCvInW;
        const int r = min(max(r0 - kCvR + i, 0), rows - 1);
        const int c = min(max(c0 - kCvPadL + j, 0), cols - 1);
        const long long idx = img_off + ((long long)r << o) * g->in_pitch + ((long long)c << o);
        in_s[e] = g->in_fmt == GDP_INPUT_U8 ? (float)static_cast<const unsigned char*>(in)[idx]
                                            : (float)static_cast<const int*>(in)[idx];
    }
    __syncthreads();
    const int cg = tid & 63, rg = tid >> 6;
    const int C = c0 + 4 * cg;
    const int n = min(4, cols - C);
    const bool full = (n == 4) && ((cols & 3) == 0);
    float* base = out + (long long)b * g->pyr_stride + og.lev_off + C;
    auto store = [&](int s, int q, f4 val) {
        const int R = r0 + 4 * rg + q;
        if (R >= rows || n <= 0) return;
        float* p = base + (long long)s * og.lev_stride + (long long)R * cols;
        if (full)
            st_f4<NT>(p, val);
        else
            st_part(p, val, n, false);
    };
    f4 prev[4], cur[4];
    for (int s = 0; s < g->L; ++s) {
        const float* k = ctaps + s * kCvMaxTaps;
        switch (cradius[s]) {
            case 1: conv_pass<1>(in_s, h_s, k, tid, cur); break;
            case 2: conv_pass<2>(in_s, h_s, k, tid, cur); break;
            case 3: conv_pass<3>(in_s, h_s, k, tid, cur); break;
            case 4: conv_pass<4>(in_s, h_s, k, tid, cur); break;
            case 5: conv_pass<5>(in_s, h_s, k, tid, cur); break;
            default: conv_pass<6>(in_s, h_s, k, tid, cur); break;
        }
        if (s > 0) {
#pragma unroll
            for (int q = 0; q < 4; ++q) store(s - 1, q, prev[q] - cur[q]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) prev[q] = cur[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) store(g->L - 1, q, prev[q]);
}

// ------------------------------------------------------------------------------------------
// Convolution extension, register-sweep form (default; k_conv above is the LDS-tile form kept for
// A/B).  One wave owns a strip of output columns x T output rows of one octave; each lane holds V
// (2 or 4) consecutive columns, and the ceil(6/V) lanes at each end of the wave carry the left /
// right halo and store nothing.  No LDS and no barriers:
//  * vertical pass in registers: the wave walks down its T + 2*6 input rows once (a 16-row ring
//    of registers, 3 rows of prefetch), and every scale's vertical sum reuses the same symmetric
//    pair sums x[i+d] + x[i-d] (taps are symmetric), so all S+3 scales cost sum(R_s + 1) FMAs;
//  * horizontal pass across lanes: the neighbouring columns come from lanes l +- 1.. through DPP
//    wave shifts (v_mov_b32_dpp wave_shr:1 / wave_shl:1);
//  * DoG against the previous scale in registers, contiguous wave stores per level row.
// Four waves per block take four vertically adjacent strips, so their shared halo rows are read
// from L2 at the same time.  Radii and taps are compile-time constants of the scale
// (R_s = ceil(3 sigma_s), sigma_s = 2/(s+1)); gdp_conv_taps returns the same values.
// ------------------------------------------------------------------------------------------
constexpr int kSwWaves = 4; // vertically adjacent strips per block
// Columns per lane.  The code is generic in V; V = 2 (116-column strips, 464-B wave stores) measured
// 1.6x slower than V = 4 (240 columns, 960-B stores) and is not instantiated.
constexpr int kSwV = 4;

template <int V>
struct SwGeom {                                            // strip geometry for V columns per lane
    static constexpr int kHaloLanes = (kCvR + V - 1) / V;  // lanes at each end that only load
    static constexpr int kLanesOut = 64 - 2 * kHaloLanes;  // lanes that store
    static constexpr int kCols = V * kLanesOut;            // output columns per strip (240 / 116)
    static constexpr int kHalo = V * kHaloLanes;           // input columns left of the first one
};
template <int V>
struct VecT;
template <>
struct VecT<2> {
    typedef float f __attribute__((ext_vector_type(2)));
    typedef int i __attribute__((ext_vector_type(2)));
    typedef unsigned u __attribute__((ext_vector_type(2)));
};
template <>
struct VecT<4> {
    typedef float f __attribute__((ext_vector_type(4)));
    typedef int i __attribute__((ext_vector_type(4)));
    typedef unsigned u __attribute__((ext_vector_type(4)));
};

__host__ __device__ constexpr int conv_radius_of(int s) {
    return (6 + s) / (s + 1) > kCvR ? kCvR : ((6 + s) / (s + 1) < 1 ? 1 : (6 + s) / (s + 1));
}

// Normalised Gaussian taps of scale s as compile-time constants (the kernel's FMA operands) and
// for gdp_conv_taps on the host — one definition, so host and device agree bit for bit.
// e^x for 0 <= x <= 13 by its (positive, non-cancelling) Taylor series in double.
__host__ __device__ constexpr double conv_exp_pos(double x) {
    double term = 1.0, sum = 1.0;
    for (int n = 1; n < 100; ++n) {
        term *= x / n;
        sum += term;
    }
    return sum;
}
__host__ __device__ constexpr double conv_weight(int s, int d) { // exp(-d^2 / (2 sigma_s^2))
    return 1.0 / conv_exp_pos((double)d * d * (s + 1) * (s + 1) / 8.0); // sigma_s = 2 / (s + 1)
}
struct ConvTaps {
    float k[kCvR + 1]; // k[|d|], d = -R..R
};
__host__ __device__ constexpr ConvTaps conv_taps_of(int s) {
    const int R = conv_radius_of(s);
    double sum = 0.0;
    for (int d = -R; d <= R; ++d) sum += conv_weight(s, d);
    ConvTaps t{};
    for (int d = 0; d <= R; ++d) t.k[d] = (float)(conv_weight(s, d) / sum);
    return t;
}

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// lane l receives lane l-1's (prev) / lane l+1's (next) value; the wave's end lanes receive 0.
// (Measured: the exchanges cost ~1 % of the sweep — ds_bpermute instead of DPP, or no exchange
// at all, time the same.)
__device__ __forceinline__ float lane_prev(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x138, 0xf, 0xf, true)); // wave_shr:1
}
__device__ __forceinline__ float lane_next(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x130, 0xf, 0xf, true)); // wave_shl:1
}

// Horizontal symmetric filter of scale s over the wave-distributed row v (V columns per lane):
// out_j = k[0] a_j + sum_{d=1..R} k[d] (a_{j+d} + a_{j-d}), a_m = column V*l + m, taken from lane
// l - k / l + k (k = 1..ceil(R/V)) by chains of one-lane DPP shifts.
template <int s, int V>
__device__ __forceinline__ typename VecT<V>::f conv_h_lanes(typename VecT<V>::f v) {
    constexpr int R = conv_radius_of(s);
    constexpr ConvTaps K = conv_taps_of(s);
    constexpr int KL = (R + V - 1) / V; // lanes of reach
    float P[KL + 1][V], N[KL + 1][V];  // P[k][j] / N[k][j]: column j of lane l - k / l + k
#pragma unroll
    for (int j = 0; j < V; ++j) P[0][j] = N[0][j] = v[j];
#pragma unroll
    for (int k = 1; k <= KL; ++k)
#pragma unroll
        for (int j = 0; j < V; ++j) {
            P[k][j] = j >= V * k - R ? lane_prev(P[k - 1][j]) : 0.f;         // column V(l-k) + j
            N[k][j] = j <= V - 1 + R - V * k ? lane_next(N[k - 1][j]) : 0.f; // column V(l+k) + j
        }
    auto a = [&](int m) -> float {
        if (m < 0) {
            const int k = (-m + V - 1) / V;
            return P[k][m + k * V];
        }
        return m < V ? P[0][m] : N[m / V][m % V];
    };
    typename VecT<V>::f out;
#pragma unroll
    for (int j = 0; j < V; ++j) {
        float acc = K.k[0] * a(j);
#pragma unroll
        for (int d = 1; d <= R; ++d) acc = __builtin_fmaf(K.k[d], a(j + d) + a(j - d), acc);
        out[j] = acc;
    }
    return out;
}

// Buffer resources for the sweep: with raw buffer loads/stores every memory instruction is issued
// unconditionally (disabled lanes get an offset past num_records: the store is dropped), so the
// compiler can count outstanding loads exactly (s_waitcnt vmcnt(N), not vmcnt(0) after every
// skip-branch around a store), and all row addressing is scalar (SGPR base per row / level).
constexpr int kOOB = 0x7FFFFFF0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, kOOB, 0x00020000);
}
enum { kLdVecI32 = 0, kLdVecU8 = 1, kLdScalarI32 = 2, kLdScalarU8 = 3 };

template <int L, int T, int V, int LD>
__device__ __forceinline__ void conv_sweep_body(const Geom* __restrict__ g, const OctGeom& og, const void* __restrict__ in,
                                                float* __restrict__ out, int b, int o, int R0, int cin, int lane, int dir) {
    typedef typename VecT<V>::f fv;
    typedef typename VecT<V>::u uv;
    constexpr int kWin = 2 * kCvR + 1; // input rows one output row needs
    constexpr int kRing = kWin + 3;    // + 3 rows of prefetch: a 16-row register ring
    static_assert(T % kRing == 0, "strip rows must be a multiple of the ring");
    constexpr int esz = (LD == kLdVecU8 || LD == kLdScalarU8) ? 1 : 4;
    const int rows = og.rows, cols = og.cols;
    // per-lane column offsets (bytes within an input row).  Vector loads: cin and cols are
    // multiples of V, so a halo group is inside the row, wholly left of it (every column clamps to
    // column 0: broadcast [0] of the group at 0) or wholly right of it (broadcast [V-1] of the last)
    int voff[V];
    const int cl = min(max(cin, 0), max(cols - V, 0));
    const bool left = cin < 0, right = cin >= cols;
#pragma unroll
    for (int j = 0; j < V; ++j)
        voff[j] = (LD == kLdVecI32 || LD == kLdVecU8) ? cl * esz : (min(max(cin + j, 0), cols - 1) << o) * esz;
    auto clamp_group = [&](fv w) -> fv {
        fv r;
#pragma unroll
        for (int j = 0; j < V; ++j) r[j] = left ? w[0] : (right ? w[V - 1] : w[j]);
        return r;
    };
    const char* img = static_cast<const char*>(in) + (long long)b * g->in_img_stride * esz;
    const long long row_bytes = ((long long)g->in_pitch << o) * esz; // input bytes between octave-o rows
    // the strip is swept top-down (dir = 1) or bottom-up (dir = -1) from output row Rb
    const int Rb = dir > 0 ? R0 : R0 + T - 1;
    auto load = [&](int q) -> fv {                                    // input row Rb + dir (q - kCvR), clamped
        const int r = min(max(Rb + dir * (q - kCvR), 0), rows - 1);   // wave-uniform
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(img + (long long)r * row_bytes);
        fv x;
        if constexpr (LD == kLdVecI32) {
            typename VecT<V>::i w;
            if constexpr (V == 4)
                w = __builtin_bit_cast(typename VecT<V>::i, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[0], 0, 0));
            else
                w = __builtin_bit_cast(typename VecT<V>::i, __builtin_amdgcn_raw_buffer_load_b64(rs, voff[0], 0, 0));
            return clamp_group(__builtin_convertvector(w, fv));
        } else if constexpr (LD == kLdVecU8) {
            const unsigned w = V == 4 ? __builtin_amdgcn_raw_buffer_load_b32(rs, voff[0], 0, 0)
                                      : (unsigned)__builtin_amdgcn_raw_buffer_load_b16(rs, voff[0], 0, 0);
#pragma unroll
            for (int j = 0; j < V; ++j) x[j] = (float)((w >> (8 * j)) & 0xffu);
            return clamp_group(x);
        } else {
#pragma unroll
            for (int j = 0; j < V; ++j) {
                if constexpr (LD == kLdScalarI32)
                    x[j] = (float)(int)__builtin_amdgcn_raw_buffer_load_b32(rs, voff[j], 0, 0);
                else
                    x[j] = (float)__builtin_amdgcn_raw_buffer_load_b8(rs, voff[j], 0, 0);
            }
            return x;
        }
    };
    // one store resource per level, based at this wave's first row; halo lanes and columns past the
    // row end store out of range
    const bool active = lane >= SwGeom<V>::kHaloLanes && lane < 64 - SwGeom<V>::kHaloLanes && cin < cols;
    const int soff_lane = active ? cin * 4 : kOOB;
    float* lev0 = out + (long long)b * g->pyr_stride + og.lev_off + (long long)R0 * cols;
    __amdgpu_buffer_rsrc_t rs_out[L];
#pragma unroll
    for (int s = 0; s < L; ++s) rs_out[s] = make_rsrc(lev0 + (long long)s * og.lev_stride);
    // soffset stays the constant 0: with an SGPR soffset the compiler omits the wait state that a
    // VALU overwrite of a >8-byte store's data VGPRs needs right after the store, and gfx950 then
    // stores the overwritten values (measured); the row offset goes into voffset instead.  Stores
    // are non-temporal (nt).
    auto store = [&](fv val, __amdgpu_buffer_rsrc_t rs, int vo) {
        if constexpr (V == 4)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uv, val), rs, vo, 0, 2);
        else
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uv, val), rs, vo, 0, 2);
    };
    // ring of input rows: slot q % kRing holds input row Rb + dir (q - kCvR)
    fv x[kRing];
#pragma unroll
    for (int q = 0; q < kRing; ++q) x[q] = load(q);
#pragma unroll 1
    for (int i0 = 0; i0 < T && (dir < 0 || R0 + i0 < rows); i0 += kRing) {
#pragma unroll
        for (int u = 0; u < kRing; ++u) {
            const int i = i0 + u; // output row Rb + dir i needs ring slots (u + 0..12) % kRing
            const int Ri = Rb + dir * i;
            fv pr[kCvR + 1];      // symmetric pair sums, shared by every scale
            pr[0] = x[(u + kCvR) % kRing];
#pragma unroll
            for (int d = 1; d <= kCvR; ++d) pr[d] = x[(u + kCvR + d) % kRing] + x[(u + kCvR - d) % kRing];
            if (i + kRing < T + 2 * kCvR) x[u] = load(i + kRing); // refill the slot just used (uniform)
            const int vo = (Ri < rows ? soff_lane : kOOB) + (Ri - R0) * cols * 4; // OOB stays OOB (< 2^32)
            fv hprev = {};
            static_for<L>([&](auto si) {
                constexpr int s = decltype(si)::value;
                constexpr int R = conv_radius_of(s);
                constexpr ConvTaps K = conv_taps_of(s);
                fv vs = pr[0] * K.k[0];
#pragma unroll
                for (int d = 1; d <= R; ++d) vs = __builtin_elementwise_fma((fv)K.k[d], pr[d], vs);
                const fv h = conv_h_lanes<s, V>(vs);
                if constexpr (s > 0) store(hprev - h, rs_out[s - 1], vo);
                hprev = h;
            });
            store(hprev, rs_out[L - 1], vo);
            __builtin_amdgcn_sched_barrier(0); // keep each row's loads in its own row: no hoisting into spills
        }
    }
}

template <int L, int T, int V>
__global__ void __launch_bounds__(64 * kSwWaves, V == 4 ? 4 : 6) k_conv_sweep(const Geom* __restrict__ g,
                                                                              const void* __restrict__ in,
                                                                              float* __restrict__ out, unsigned units,
                                                                              int order) {
    // order 1 (XCD-chunked): blocks u and u+8 share an XCD under round-robin dispatch, so XCD x
    // takes the contiguous work range x/8 — horizontally adjacent strips of a row band then run
    // on one XCD at the same time and their shared boundary lines meet in one L2 (the grid is
    // padded to a multiple of 8; the padding blocks exit)
    unsigned w = blockIdx.x;
    if (order & 1) w = (w & 7u) * (gridDim.x >> 3) + (w >> 3);
    if (w >= units) return;
    const unsigned per = g->sw_blk[g->O];
    const unsigned b = w / per;
    const unsigned v = w - b * per;
    int o = 0;
    while (o + 1 < g->O && v >= g->sw_blk[o + 1]) ++o;
    const OctGeom og = g->oct[o];
    const unsigned t = v - g->sw_blk[o];
    const unsigned sc = (unsigned)g->sw_strips_c[o];
    const int tr = (int)(t / sc), tc = (int)(t - (unsigned)tr * sc);
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const int R0 = (tr * kSwWaves + wave) * T; // first output row of this wave
    if (R0 >= og.rows) return;                 // whole waves only; no barriers in this kernel
    const int cin = tc * SwGeom<V>::kCols - SwGeom<V>::kHalo + V * lane;
    // order bit 1: odd waves sweep bottom-up, so every halo shared by two waves of the block is
    // loaded by both at the same time (ends meet ends, starts meet starts) and hits in cache
    const int dir = (order & 2) && (wave & 1) ? -1 : 1;
    if (o == 0 && g->vec_in && og.cols >= 4) {
        if (g->in_fmt == GDP_INPUT_U8)
            conv_sweep_body<L, T, V, kLdVecU8>(g, og, in, out, (int)b, o, R0, cin, lane, dir);
        else
            conv_sweep_body<L, T, V, kLdVecI32>(g, og, in, out, (int)b, o, R0, cin, lane, dir);
    } else if (g->in_fmt == GDP_INPUT_U8) {
        conv_sweep_body<L, T, V, kLdScalarU8>(g, og, in, out, (int)b, o, R0, cin, lane, dir);
    } else {
        conv_sweep_body<L, T, V, kLdScalarI32>(g, og, in, out, (int)b, o, R0, cin, lane, dir);
    }
}

// Order-independent pyramid checksum (verification of multi-GPU runs without moving pyramids):
// sum over every word of every level of splitmix64(global element index * phi + level id * c
// + float bits), mod 2^64.  Global rows make row-band checksums add up to the whole image's.
// Restated in numpy by the test suite (tests/test_gpu_parity.py::_checksum).
__device__ __forceinline__ unsigned long long splitmix_fin(unsigned long long x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    x ^= x >> 31;
    return x;
}

__global__ void __launch_bounds__(kBlock) k_checksum(const Geom* __restrict__ g, const float* __restrict__ out, int b,
                                                     unsigned long long* __restrict__ sum) {
    const long long total = g->oct[g->O - 1].grp_begin + (long long)g->oct[g->O - 1].rows * g->oct[g->O - 1].gpr;
    unsigned long long acc = 0;
    for (long long t = (long long)blockIdx.x * kBlock + threadIdx.x; t < total; t += (long long)gridDim.x * kBlock) {
        int o = 0;
        while (o + 1 < g->O && t >= g->oct[o + 1].grp_begin) ++o;
        const OctGeom& og = g->oct[o];
        const long long k = t - og.grp_begin;
        const int Rl = (int)(k / og.gpr);
        const int C = 4 * (int)(k - (long long)Rl * og.gpr);
        const int n = min(4, og.cols - C);
        const unsigned long long idx0 = (unsigned long long)(og.row0 + Rl) * og.cols + C;
        const float* p = out + (long long)b * g->pyr_stride + og.lev_off + (long long)Rl * og.cols + C;
        for (int s = 0; s < g->L; ++s) {
            const unsigned long long lid = (unsigned long long)(o * 64 + s) * 0xD1B54A32D192ED03ull;
            for (int j = 0; j < n; ++j) {
                const unsigned bits = __float_as_uint(p[s * og.lev_stride + j]);
                acc += splitmix_fin((idx0 + j) * 0x9E3779B97F4A7C15ull + lid + bits);
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(sum, acc);
}

__device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// Counter-hash synthetic images, generated in place on each GPU.
__global__ void __launch_bounds__(kBlock) k_synth(const Geom* __restrict__ g, void* __restrict__ in, unsigned seed,
                                                  long long first_image) {
    const long long W = g->W;
    const long long per = (long long)g->in_rows * W;
    const long long total = per * g->batch;
    for (long long t = (long long)blockIdx.x * kBlock + threadIdx.x; t < total; t += (long long)gridDim.x * kBlock) {
        const long long b = t / per;
        const long long rem = t - b * per;
        const long long r = rem / W;
        const long long c = rem - r * W;
        const unsigned long long idx =
            ((unsigned long long)(first_image + b) * (unsigned long long)g->H + (unsigned long long)(g->in_row0 + r)) *
                (unsigned long long)W +
            (unsigned long long)c;
        const unsigned px = mix32(seed ^ (unsigned)(idx ^ (idx >> 32))) >> 24;
        const long long off = b * g->in_img_stride + r * g->in_pitch + c;
        if (g->in_fmt == GDP_INPUT_U8)
            static_cast<unsigned char*>(in)[off] = (unsigned char)px;
        else
            static_cast<int*>(in)[off] = (int)px;
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// GuassDePyramid.h:7-8 (PI is 3.1414926f in the reference, reproduced on purpose).
const float kSigma = 2.0f;
const float kPI = 3.1414926f;

// GuassDePyramid.h:107-121, evaluated on the host in the reference's float expression order:
// the window centre is the FLOAT length halved o times, minus 1, over 2 (:107-115).
int host_taps(int length, int octave, int scale, float* out) {
    float len = (float)length;
    for (int t = octave; t != 0; --t) len /= 2;
    const int my_len = (int)len;
    len = (len - 1) / 2;
    const float sig = kSigma / (scale + 1);
    for (int i = 0; i < my_len; ++i) out[i] = expf(-(i - len) * (i - len) / (2 * sig * sig)) / (sig * sqrtf(2 * kPI));
    return my_len;
}

int octaves_for(int n) {
    int x = 0;
    while (n > 0) {
        ++x;
        n /= 2;
    }
    return x;
}

long long round_up(long long v, long long a) { return (v + a - 1) / a * a; }

thread_local std::string g_create_error;

}  // namespace

struct gdp_ctx {
    int device = 0;
    Geom geom{};
    Geom* d_geom = nullptr;
    void* d_in_own = nullptr;     // context-owned input buffer (int32 or uint8 per geom.in_fmt)
    const void* d_in = nullptr;   // buffer the kernels read (own or caller's)
    float* d_out = nullptr;
    float* d_taps = nullptr;
    int conv_kernel = 0;          // GDP_TUNE_CONV_KERNEL: 0 register sweep (default), 1 LDS tiles
    int conv_rows = 16;           // GDP_TUNE_CONV_ROWS: output rows per wave strip of the sweep
    int conv_order = 0;           // GDP_TUNE_CONV_ORDER: bit 0 XCD-chunked blocks, bit 1 alternate sweep directions
    float* d_ctaps = nullptr;     // convolution-mode taps [L][13] (extension)
    int* d_cradius = nullptr;     // convolution-mode radius per scale
    float* d_out_own = nullptr;   // context-owned pyramid (d_out may point at caller memory)
    float* h_stage = nullptr;     // pinned staging for row-pointer downloads (largest level)
    size_t h_stage_floats = 0;
    unsigned long long* d_sum = nullptr;
    std::vector<float> h_taps;
    long long in_pitch_own = 0, in_img_stride_own = 0;
    hipStream_t stream = nullptr;
    int cus = 256;
    int blocks_max = 2048;        // 256 CUs x 8 blocks of 256 threads
    int nontemporal = 1;          // GDP_TUNE_NONTEMPORAL
    int grid_override = 0;        // GDP_TUNE_GRID (0 = automatic)
    int persistent = 0;           // set by GDP_TUNE_BLOCKS_PER_CU: grid = CUs x blocks per CU
    int variant = 0;              // GDP_TUNE_VARIANT: index into kVariants (default_variant(W))
    int inplace_sub = 1;          // GDP_TUNE_INPLACE_SUB: k_levels blocks per 1024-group chunk (1, 2, 4)
    int window_sub = 4;           // GDP_TUNE_WINDOW_SUB: k_window blocks per chunk (4 = 256-thread blocks:
                                  // 6.7 vs 5.9 TB/s at 4096^2, tools/tune.py)
    std::string err;
    int status(int code, const char* fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
    // NULL = the context's own stream; GDP_STREAM_NULL ((void*)1) = HIP's default (null) stream
    hipStream_t pick(void* s) const {
        if (s == GDP_STREAM_NULL) return (hipStream_t)0;
        return s ? (hipStream_t)s : stream;
    }
};

namespace {

#define GDP_HIP(ctx, call)                                                                                   \
    do {                                                                                                     \
        hipError_t e_ = (call);                                                                              \
        if (e_ != hipSuccess) return (ctx)->status(GDP_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_));    \
    } while (0)

// Tile grid of the selected build variant (tile width differs per variant).
int retile(gdp_ctx* c, int tile_cols, int tile_rows) {
    Geom& g = c->geom;
    // octaves fused into a tile: those with whole rows in it (tile_rows = 2^(F-1)); the rest are
    // flattened tail units
    int fused = 1;
    while ((1 << fused) <= tile_rows) ++fused;
    g.F = std::min(g.O, std::min(fused, kFused));
    const long long total_groups = g.oct[g.O - 1].grp_begin + (long long)g.oct[g.O - 1].rows * g.oct[g.O - 1].gpr;
    const long long tail_per_img = (g.F < g.O) ? total_groups - g.oct[g.F].grp_begin : 0;
    const long long tail_units = (tail_per_img * g.batch + kTailGroups - 1) / kTailGroups;
    if (tail_per_img * g.batch >= (1ll << 31)) return c->status(GDP_ERR_ARG, "image/batch too large for one context");
    g.tail_groups_per_img = (unsigned)tail_per_img;
    g.tail_units = (unsigned)tail_units;
    g.tiles_r = (g.in_rows + tile_rows - 1) / tile_rows;
    g.tiles_c = (g.W + tile_cols - 1) / tile_cols;
    const long long tiles_per_img = (long long)g.tiles_r * g.tiles_c;
    if (tiles_per_img * g.batch + g.tail_units >= (1ll << 31))
        return c->status(GDP_ERR_ARG, "image/batch too large for one context (split the batch)");
    g.tiles_per_img = (unsigned)tiles_per_img;
    g.tiles_total = (unsigned)(tiles_per_img * g.batch);
    return GDP_OK;
}

// Geometry changes are configuration-time events: drain the device first so no in-flight launch
// (on any stream) reads a half-updated Geom.
int upload_geom(gdp_ctx* c) {
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_HIP(c, hipDeviceSynchronize());
    GDP_HIP(c, hipMemcpy(c->d_geom, &c->geom, sizeof(Geom), hipMemcpyHostToDevice));
    return GDP_OK;
}

int launch_build(gdp_ctx* c, hipStream_t st) {
    const Geom& g = c->geom;
    const long long units = (long long)g.tiles_total + g.tail_units;
    if (units == 0) return GDP_OK;
    // default: one unit per block; GDP_TUNE_GRID / GDP_TUNE_BLOCKS_PER_CU cap it (persistent loop)
    const long long cap = c->grid_override > 0 ? c->grid_override : (c->persistent ? c->blocks_max : units);
    const int grid = (int)std::min<long long>(units, cap);
    const BuildVariant& v = kVariants[c->variant];
    hipLaunchKernelGGL(v.k[g.L == 5][c->nontemporal ? 1 : 0], dim3(grid), dim3(v.block), 0, st, c->d_geom, c->d_in,
                       c->d_out, c->d_taps);
    GDP_HIP(c, hipGetLastError());
    return GDP_OK;
}

template <int MODE, int SUB>
int launch_inplace_sub(gdp_ctx* c, int ob, int oe, hipStream_t st) {
    const Geom& g = c->geom;
    if constexpr (MODE == 1) {
        const long long grid = ((long long)g.lv_blk[oe] - g.lv_blk[ob]) * g.L * g.batch * SUB;
        if (grid <= 0) return GDP_OK;
        if (grid >= (1ll << 31) || (long long)g.lv_blk[g.O] * g.L >= (1ll << 32))
            return c->status(GDP_ERR_ARG, "window pass too large for one launch");
        auto wkern = c->nontemporal ? k_window<true, SUB> : k_window<false, SUB>;
        hipLaunchKernelGGL(wkern, dim3((unsigned)grid), dim3(kLevBlock / SUB), 0, st, c->d_geom, c->d_out, c->d_taps, ob,
                           oe);
        GDP_HIP(c, hipGetLastError());
        return GDP_OK;
    }
    const long long per = (long long)g.lv_blk[oe] - g.lv_blk[ob];
    const long long grid = per * g.batch * SUB;
    if (grid <= 0) return GDP_OK;
    if (grid >= (1ll << 31)) return c->status(GDP_ERR_ARG, "in-place pass too large for one launch");
    auto kern = g.L == 5 ? (c->nontemporal ? k_levels<5, MODE, true, SUB> : k_levels<5, MODE, false, SUB>)
                         : (c->nontemporal ? k_levels<0, MODE, true, SUB> : k_levels<0, MODE, false, SUB>);
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kLevBlock / SUB), 0, st, c->d_geom, c->d_in, c->d_out, c->d_taps,
                       ob, oe);
    GDP_HIP(c, hipGetLastError());
    return GDP_OK;
}

template <int MODE>
int launch_inplace(gdp_ctx* c, int ob, int oe, hipStream_t st) {
    const Geom& g = c->geom;
    if ((MODE == 2 || MODE == 3) && c->inplace_sub == 0 && g.L <= 16) {
        const long long grid = ((long long)g.lx_blk[oe] - g.lx_blk[ob]) * g.batch;
        if (grid <= 0) return GDP_OK;
        if (grid >= (1ll << 31)) return c->status(GDP_ERR_ARG, "in-place pass too large for one launch");
        auto kern = c->nontemporal ? k_levels_x<MODE == 3 ? 3 : 2, true> : k_levels_x<MODE == 3 ? 3 : 2, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * g.L), 0, st, c->d_geom, c->d_out, c->d_taps, ob, oe);
        GDP_HIP(c, hipGetLastError());
        return GDP_OK;
    }
    switch (MODE == 1 ? c->window_sub : c->inplace_sub) {
        case 2: return launch_inplace_sub<MODE, 2>(c, ob, oe, st);
        case 4: return launch_inplace_sub<MODE, 4>(c, ob, oe, st);
        default: return launch_inplace_sub<MODE, 1>(c, ob, oe, st);
    }
}

bool valid_level(const gdp_ctx* c, int b, int o, int s) {
    return c && b >= 0 && b < c->geom.batch && o >= 0 && o < c->geom.O && s >= 0 && s < c->geom.L;
}

}  // namespace

// ==========================================================================================
// C ABI
// ==========================================================================================
// Block prefix of the convolution sweep (kSwWaves strips of conv_rows rows x kSwCols columns).
static void conv_sweep_geom(gdp_ctx* c) {
    Geom& g = c->geom;
    const int strip_cols = SwGeom<kSwV>::kCols;
    g.sw_blk[0] = 0;
    g.cvx_blk[0] = 0;
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        const bool sweep = og.cols >= 4 && og.cols % 4 == 0; // full-vector stores on every row
        g.sw_strips_c[o] = (og.cols + strip_cols - 1) / strip_cols;
        const long long rows_per_blk = (long long)kSwWaves * c->conv_rows;
        g.sw_blk[o + 1] = g.sw_blk[o] + (sweep ? (unsigned)((og.rows + rows_per_blk - 1) / rows_per_blk * g.sw_strips_c[o]) : 0u);
        g.cvx_blk[o + 1] = g.cvx_blk[o] + (sweep ? 0u : g.cv_blk[o + 1] - g.cv_blk[o]);
    }
}

template <int L, int T>
hipError_t launch_conv_sweep_t(gdp_ctx* c, unsigned units, hipStream_t st) {
    auto k = k_conv_sweep<L, T, kSwV>;
    const unsigned grid = (c->conv_order & 1) ? (units + 7u) / 8u * 8u : units;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * kSwWaves), 0, st, c->d_geom, c->d_in, c->d_out, units, c->conv_order);
    return hipGetLastError();
}

template <int L>
hipError_t launch_conv_sweep_l(gdp_ctx* c, unsigned grid, hipStream_t st) {
    return c->conv_rows == 32 ? launch_conv_sweep_t<L, 32>(c, grid, st) : launch_conv_sweep_t<L, 16>(c, grid, st);
}

extern "C" {

int gdp_abi_version(void) { return GDP_ABI_VERSION; }

int gdp_octaves_for(int n) { return octaves_for(n); }

int gdp_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

const char* gdp_status_string(int s) {
    switch (s) {
        case GDP_OK: return "ok";
        case GDP_ERR_ARG: return "invalid argument";
        case GDP_ERR_HIP: return "HIP runtime error";
        case GDP_ERR_STATE: return "invalid state";
        case GDP_ERR_NOMEM: return "out of memory";
        case GDP_ERR_NODEV: return "no gfx950 device";
        default: return "unknown status";
    }
}

const char* gdp_last_error(const gdp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

int gdp_create_band(gdp_ctx** out, int H, int W, int S, int O, int batch, int row_begin, int row_end, int device) {
    if (!out) return GDP_ERR_ARG;
    *out = nullptr;
    auto fail = [](int code, const std::string& m) {
        g_create_error = m;
        return code;
    };
    if (H <= 0 || W <= 0 || S < 0 || S > 60 || batch <= 0 || O < 0)
        return fail(GDP_ERR_ARG, "gdp_create: need H, W, batch > 0, 0 <= S <= 60, octaves >= 0");
    const int Omax = octaves_for(std::min(H, W));
    if (O == 0) O = Omax;
    if (O > Omax || O > kMaxOct - 1)
        return fail(GDP_ERR_ARG, "gdp_create: octaves " + std::to_string(O) + " > floor(log2(min(H,W)))+1 = " +
                                     std::to_string(Omax));
    const int align = 1 << (std::max(O, kFused) - 1);
    if (row_begin < 0 || row_end > H || row_begin >= row_end || row_begin % align != 0 ||
        (row_end != H && row_end % align != 0))
        return fail(GDP_ERR_ARG, "gdp_create_band: rows [" + std::to_string(row_begin) + ", " +
                                     std::to_string(row_end) + ") must be multiples of " + std::to_string(align));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(GDP_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(GDP_ERR_ARG, "device index out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail(GDP_ERR_NODEV, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(GDP_ERR_NODEV, std::string("libgdp is built for gfx950, device is ") + prop.gcnArchName);

    gdp_ctx* c = new (std::nothrow) gdp_ctx();
    if (!c) return fail(GDP_ERR_NOMEM, "host allocation failed");
    c->device = device;
    c->variant = default_variant(W, (long long)(row_end - row_begin) * W, batch);
    c->cus = std::max(1, prop.multiProcessorCount);
    c->blocks_max = c->cus * 8;
    Geom& g = c->geom;
    g.H = H;
    g.W = W;
    g.S = S;
    g.L = S + 3;
    g.O = O;
    g.F = std::min(O, kFused);
    g.batch = batch;
    g.in_row0 = row_begin;
    g.in_rows = row_end - row_begin;
    g.in_pitch = round_up(W, 4);
    g.in_img_stride = (long long)g.in_rows * g.in_pitch;
    g.vec_in = 1;
    c->in_pitch_own = g.in_pitch;
    c->in_img_stride_own = g.in_img_stride;

    // optional padding between levels (floats, multiple of 64) — layout experiment knob
    const char* pad_env = std::getenv("GDP_LEVEL_PAD");
    const long long level_pad = pad_env ? round_up(std::max(0ll, std::atoll(pad_env)), kLevelAlign) : 0;
    // tap table: per octave, column taps [L][round4(W_o)] then row taps [L][round4(H_o)] (global rows)
    long long tap_off = 0, lev_off = 0, grp = 0;
    for (int o = 0; o < O; ++o) {
        OctGeom& og = g.oct[o];
        const int Hg = H >> o;
        og.row0 = (row_begin + (1 << o) - 1) >> o;
        const int row_hi = (row_end == H) ? Hg : std::min(Hg, (row_end + (1 << o) - 1) >> o);
        og.rows = std::max(0, row_hi - og.row0);
        og.cols = W >> o;
        og.gpr = (og.cols + 3) / 4;
        og.lev_stride = round_up((long long)og.rows * og.cols, kLevelAlign) + level_pad;
        og.lev_off = lev_off;
        lev_off += og.lev_stride * g.L;
        og.ctap_stride = (int)round_up(og.cols, 4);
        og.ctap = (int)tap_off;
        tap_off += (long long)og.ctap_stride * g.L;
        og.rtap_stride = (int)round_up(Hg, 4);
        og.rtap = (int)tap_off;
        tap_off += (long long)og.rtap_stride * g.L;
        og.grp_begin = grp;
        make_magic((unsigned)std::max(1, og.gpr), &og.gpr_magic, &og.gpr_shift);
        grp += (long long)og.rows * og.gpr;
        g.lv_blk[o + 1] = g.lv_blk[o] + (unsigned)(((long long)og.rows * og.gpr + kLevBlock - 1) / kLevBlock);
        g.lx_blk[o + 1] = g.lx_blk[o] + (unsigned)(((long long)og.rows * og.gpr + 63) / 64);
        g.cv_tiles_c[o] = (og.cols + kCvTW - 1) / kCvTW;
        g.cv_blk[o + 1] = g.cv_blk[o] + (unsigned)(((long long)og.rows + kCvTH - 1) / kCvTH * g.cv_tiles_c[o]);
    }
    g.pyr_stride = round_up(lev_off, kLevelAlign);
    const long long tail_per_img = (g.F < O) ? grp - g.oct[g.F].grp_begin : 0;
    const long long tail_units = (tail_per_img * batch + kTailGroups - 1) / kTailGroups;
    const long long min_tiles = (long long)((g.in_rows + kTileRows - 1) / kTileRows) * ((W + 63) / 64) * batch;
    if (tap_off > (1ll << 31) || min_tiles + tail_units >= (1ll << 31) || tail_per_img * batch >= (1ll << 31) ||
        grp >= (1ll << 31)) {
        delete c;
        return fail(GDP_ERR_ARG, "image/batch too large for one context (split the batch)");
    }
    g.tail_groups_per_img = (unsigned)tail_per_img;
    g.tail_units = (unsigned)tail_units;
    // Tile order default (tools/tune.py, MI355X): a single very large image (>= 64 Mpix, e.g. the
    // 16384^2 config) streams 7-8 % faster when each XCD sweeps its own contiguous eighth of the
    // tiles; batches and <= 4096^2 images are fastest in linear order.
    g.tile_order = (batch == 1 && (long long)g.in_rows * W >= (1ll << 26)) ? 1 : 0;
    retile(c, kVariants[c->variant].tile_cols, kVariants[c->variant].tile_rows);
    conv_sweep_geom(c);
    c->h_taps.assign((size_t)tap_off, 0.0f);
    for (int o = 0; o < O; ++o) {
        const OctGeom& og = g.oct[o];
        for (int s = 0; s < g.L; ++s) {
            host_taps(W, o, s, c->h_taps.data() + og.ctap + (long long)s * og.ctap_stride);
            host_taps(H, o, s, c->h_taps.data() + og.rtap + (long long)s * og.rtap_stride);
        }
    }

    auto hip_fail = [&](hipError_t e, const char* what) {
        std::string m = std::string(what) + ": " + hipGetErrorString(e);
        gdp_destroy(c);
        return fail(e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP, m);
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "hipStreamCreate");
    if ((e = hipMalloc(&c->d_geom, sizeof(Geom))) != hipSuccess) return hip_fail(e, "hipMalloc(geom)");
    if ((e = hipMalloc(&c->d_taps, std::max<size_t>(4, c->h_taps.size() * 4))) != hipSuccess)
        return hip_fail(e, "hipMalloc(taps)");
    if ((e = hipMalloc(&c->d_in_own, std::max<size_t>(16, (size_t)g.in_img_stride * batch * 4))) != hipSuccess)  // int32
        return hip_fail(e, "hipMalloc(input)");
    if ((e = hipMalloc(&c->d_out_own, std::max<size_t>(16, (size_t)g.pyr_stride * batch * 4))) != hipSuccess)
        return hip_fail(e, "hipMalloc(pyramid)");
    c->d_out = c->d_out_own;
    if ((e = hipMalloc(&c->d_sum, sizeof(unsigned long long))) != hipSuccess) return hip_fail(e, "hipMalloc(sum)");
    c->d_in = c->d_in_own;
    if ((e = hipMemcpy(c->d_taps, c->h_taps.data(), c->h_taps.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy(taps)");
    if ((e = hipMemset(c->d_in_own, 0, (size_t)g.in_img_stride * batch * 4)) != hipSuccess) return hip_fail(e, "hipMemset");
    if (upload_geom(c) != GDP_OK) {
        std::string m = c->err;
        gdp_destroy(c);
        return fail(GDP_ERR_HIP, m);
    }
    *out = c;
    return GDP_OK;
}

int gdp_create(gdp_ctx** out, int H, int W, int S, int O, int batch, int device) {
    return gdp_create_band(out, H, W, S, O, batch, 0, H, device);
}

void gdp_destroy(gdp_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->d_geom) (void)hipFree(c->d_geom);
    if (c->d_taps) (void)hipFree(c->d_taps);
    if (c->d_in_own) (void)hipFree(c->d_in_own);
    if (c->d_out_own) (void)hipFree(c->d_out_own);
    if (c->d_ctaps) (void)hipFree(c->d_ctaps);
    if (c->d_cradius) (void)hipFree(c->d_cradius);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->d_sum) (void)hipFree(c->d_sum);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int gdp_get_geometry(const gdp_ctx* c, int* H, int* W, int* S, int* O, int* batch) {
    if (!c) return GDP_ERR_ARG;
    if (H) *H = c->geom.H;
    if (W) *W = c->geom.W;
    if (S) *S = c->geom.S;
    if (O) *O = c->geom.O;
    if (batch) *batch = c->geom.batch;
    return GDP_OK;
}

int gdp_level_dims(const gdp_ctx* c, int o, int* rows, int* cols, int* first_row) {
    if (!c || o < 0 || o >= c->geom.O) return GDP_ERR_ARG;
    if (rows) *rows = c->geom.oct[o].rows;
    if (cols) *cols = c->geom.oct[o].cols;
    if (first_row) *first_row = c->geom.oct[o].row0;
    return GDP_OK;
}

size_t gdp_pyramid_bytes(const gdp_ctx* c) { return c ? (size_t)c->geom.pyr_stride * c->geom.batch * 4 : 0; }

size_t gdp_packed_floats(const gdp_ctx* c) {
    if (!c) return 0;
    size_t n = 0;
    for (int o = 0; o < c->geom.O; ++o) n += (size_t)c->geom.L * c->geom.oct[o].rows * c->geom.oct[o].cols;
    return n;
}

namespace {
size_t in_elem_size(const gdp_ctx* c) { return c->geom.in_fmt == GDP_INPUT_U8 ? 1 : 4; }

int upload_input(gdp_ctx* c, int b, const void* base, size_t pitch, int fmt, void* stream, const char* who) {
    if (!c || !base || b < 0 || b >= c->geom.batch || pitch < (size_t)c->geom.W)
        return c ? c->status(GDP_ERR_ARG, "%s: bad argument", who) : GDP_ERR_ARG;
    if (c->geom.in_fmt != fmt) return c->status(GDP_ERR_STATE, "%s: context input format differs (gdp_set_input_format)", who);
    if (c->d_in != c->d_in_own) return c->status(GDP_ERR_STATE, "%s: input is bound to caller device memory", who);
    const size_t esz = in_elem_size(c);
    GDP_HIP(c, hipSetDevice(c->device));
    hipStream_t st = c->pick(stream);
    GDP_HIP(c, hipMemcpy2DAsync(static_cast<char*>(c->d_in_own) + (size_t)b * c->geom.in_img_stride * esz,
                                (size_t)c->geom.in_pitch * esz, base, pitch * esz, (size_t)c->geom.W * esz,
                                (size_t)c->geom.in_rows, hipMemcpyHostToDevice, st));
    GDP_HIP(c, hipStreamSynchronize(st));
    return GDP_OK;
}

int bind_input(gdp_ctx* c, const void* base, size_t pitch, size_t image_stride, int fmt, const char* who) {
    if (!c) return GDP_ERR_ARG;
    Geom& g = c->geom;
    if (!base) {
        c->d_in = c->d_in_own;
        g.in_pitch = c->in_pitch_own;
        g.in_img_stride = c->in_img_stride_own;
        g.vec_in = 1;
        return upload_geom(c);
    }
    if (g.in_fmt != fmt) return c->status(GDP_ERR_STATE, "%s: context input format differs (gdp_set_input_format)", who);
    if (pitch < (size_t)g.W || (g.batch > 1 && image_stride < pitch * (size_t)g.in_rows))
        return c->status(GDP_ERR_ARG, "%s: pitch/image_stride too small", who);
    const uintptr_t align = fmt == GDP_INPUT_U8 ? 3 : 15; // one uchar4 / int4 load per 4 pixels
    c->d_in = base;
    g.in_pitch = (long long)pitch;
    g.in_img_stride = (long long)image_stride;
    g.vec_in = ((reinterpret_cast<uintptr_t>(base) & align) == 0 && pitch % 4 == 0 && image_stride % 4 == 0) ? 1 : 0;
    return upload_geom(c);
}
}  // namespace

int gdp_set_input_host(gdp_ctx* c, int b, const int32_t* base, size_t pitch, void* stream) {
    return upload_input(c, b, base, pitch, GDP_INPUT_I32, stream, "gdp_set_input_host");
}

int gdp_set_input_host_u8(gdp_ctx* c, int b, const uint8_t* base, size_t pitch, void* stream) {
    return upload_input(c, b, base, pitch, GDP_INPUT_U8, stream, "gdp_set_input_host_u8");
}

int gdp_set_input_rows(gdp_ctx* c, int b, const int32_t* const* rows, void* stream) {
    if (!c || !rows || b < 0 || b >= c->geom.batch) return c ? c->status(GDP_ERR_ARG, "gdp_set_input_rows: bad argument") : GDP_ERR_ARG;
    if (c->d_in != c->d_in_own) return c->status(GDP_ERR_STATE, "input is bound to caller device memory");
    // Gather the row pointers into one staging image, then one 2-D copy.
    const size_t W = (size_t)c->geom.W, R = (size_t)c->geom.in_rows;
    std::vector<int32_t> stage(W * R);
    for (size_t r = 0; r < R; ++r) {
        if (!rows[r]) return c->status(GDP_ERR_ARG, "gdp_set_input_rows: null row %zu", r);
        std::memcpy(stage.data() + r * W, rows[r], W * 4);
    }
    return gdp_set_input_host(c, b, stage.data(), W, stream);
}

int gdp_set_input_device(gdp_ctx* c, const int32_t* base, size_t pitch, size_t image_stride) {
    return bind_input(c, base, pitch, image_stride, GDP_INPUT_I32, "gdp_set_input_device");
}

int gdp_set_input_device_u8(gdp_ctx* c, const uint8_t* base, size_t pitch, size_t image_stride) {
    return bind_input(c, base, pitch, image_stride, GDP_INPUT_U8, "gdp_set_input_device_u8");
}

int gdp_set_input_format(gdp_ctx* c, int fmt) {
    if (!c || (fmt != GDP_INPUT_I32 && fmt != GDP_INPUT_U8)) return c ? c->status(GDP_ERR_ARG, "unknown input format") : GDP_ERR_ARG;
    if (fmt == c->geom.in_fmt) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_HIP(c, hipDeviceSynchronize());
    const size_t bytes = (size_t)c->in_img_stride_own * c->geom.batch * (fmt == GDP_INPUT_U8 ? 1 : 4);
    void* fresh = nullptr;
    hipError_t e = hipMalloc(&fresh, std::max<size_t>(16, bytes));
    if (e != hipSuccess) return c->status(e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP, "hipMalloc(input)");
    GDP_HIP(c, hipMemset(fresh, 0, std::max<size_t>(16, bytes)));
    GDP_HIP(c, hipFree(c->d_in_own));
    c->d_in_own = fresh;
    c->geom.in_fmt = fmt;
    return bind_input(c, nullptr, 0, 0, fmt, "gdp_set_input_format");
}

int gdp_get_input_format(const gdp_ctx* c) { return c ? c->geom.in_fmt : -1; }

int gdp_fill_synthetic(gdp_ctx* c, uint32_t seed, long first_image, void* stream) {
    if (!c) return GDP_ERR_ARG;
    if (c->d_in != c->d_in_own) return c->status(GDP_ERR_STATE, "input is bound to caller device memory");
    GDP_HIP(c, hipSetDevice(c->device));
    const long long total = (long long)c->geom.in_rows * c->geom.W * c->geom.batch;
    const int grid = (int)std::min<long long>((total + kBlock - 1) / kBlock, c->blocks_max);
    hipLaunchKernelGGL(k_synth, dim3(grid), dim3(kBlock), 0, c->pick(stream), c->d_geom, c->d_in_own, seed,
                       (long long)first_image);
    GDP_HIP(c, hipGetLastError());
    return GDP_OK;
}

int gdp_build(gdp_ctx* c, void* stream) {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_build(c, c->pick(stream));
}

int gdp_conv_taps(int S, int scale, float* taps, int* radius) {
    if (S < 0 || scale < 0 || scale >= S + 3 || !taps || !radius) return GDP_ERR_ARG;
    const int R = conv_radius_of(scale); // ceil(3 sigma), sigma = 2 / (scale + 1), at most kCvR
    const ConvTaps k = conv_taps_of(scale);
    for (int j = 0; j < kCvMaxTaps; ++j) taps[j] = j <= 2 * R ? k.k[j < R ? R - j : j - R] : 0.0f;
    *radius = R;
    return GDP_OK;
}

int gdp_build_gaussian(gdp_ctx* c, void* stream) {
    if (!c) return GDP_ERR_ARG;
    const Geom& g = c->geom;
    if (g.in_row0 != 0 || g.in_rows != g.H)
        return c->status(GDP_ERR_STATE, "gdp_build_gaussian: row-band contexts are not supported (needs halo rows)");
    GDP_HIP(c, hipSetDevice(c->device));
    if (!c->d_ctaps) {
        std::vector<float> t((size_t)g.L * kCvMaxTaps);
        std::vector<int> r(g.L);
        for (int s = 0; s < g.L; ++s) gdp_conv_taps(g.S, s, t.data() + (size_t)s * kCvMaxTaps, &r[s]);
        GDP_HIP(c, hipMalloc(&c->d_ctaps, t.size() * 4));
        GDP_HIP(c, hipMalloc(&c->d_cradius, r.size() * 4));
        GDP_HIP(c, hipMemcpy(c->d_ctaps, t.data(), t.size() * 4, hipMemcpyHostToDevice));
        GDP_HIP(c, hipMemcpy(c->d_cradius, r.data(), r.size() * 4, hipMemcpyHostToDevice));
    }
    const hipStream_t st = c->pick(stream);
    // the register sweep is compiled for S = 0..3 (L = 3..6) and takes the octaves whose width is a
    // multiple of 4; the LDS tiles take the rest (and everything for other S or conv_kernel = 1)
    const bool sweep = c->conv_kernel == 0 && g.L >= 3 && g.L <= 6;
    if (sweep) {
        const long long grid = (long long)g.sw_blk[g.O] * g.batch;
        if (grid >= (1ll << 31) - 8) return c->status(GDP_ERR_ARG, "convolution build too large for one launch");
        if (grid > 0) {
            switch (g.L) {
                case 3: GDP_HIP(c, launch_conv_sweep_l<3>(c, (unsigned)grid, st)); break;
                case 4: GDP_HIP(c, launch_conv_sweep_l<4>(c, (unsigned)grid, st)); break;
                case 5: GDP_HIP(c, launch_conv_sweep_l<5>(c, (unsigned)grid, st)); break;
                default: GDP_HIP(c, launch_conv_sweep_l<6>(c, (unsigned)grid, st)); break;
            }
        }
    }
    const long long grid = (long long)(sweep ? g.cvx_blk[g.O] : g.cv_blk[g.O]) * g.batch;
    if (grid <= 0) return GDP_OK;
    if (grid >= (1ll << 31)) return c->status(GDP_ERR_ARG, "convolution build too large for one launch");
    hipLaunchKernelGGL(c->nontemporal ? k_conv<true> : k_conv<false>, dim3((unsigned)grid), dim3(256), 0, st,
                       c->d_geom, c->d_in, c->d_out, c->d_ctaps, c->d_cradius, sweep ? 1 : 0);
    GDP_HIP(c, hipGetLastError());
    return GDP_OK;
}

int gdp_init(gdp_ctx* c, void* stream) {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<4>(c, 0, c->geom.O, c->pick(stream));
}

int gdp_gauss_octave(gdp_ctx* c, int o, void* stream) {
    if (!c || o < 0 || o >= c->geom.O) return c ? c->status(GDP_ERR_ARG, "octave out of range") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<1>(c, o, o + 1, c->pick(stream));
}

int gdp_gauss_range(gdp_ctx* c, int ob, int oe, void* stream) {
    if (!c || ob < 0 || oe > c->geom.O || ob >= oe) return c ? c->status(GDP_ERR_ARG, "octave range invalid") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<1>(c, ob, oe, c->pick(stream));
}

int gdp_dog_octave(gdp_ctx* c, int o, void* stream) {
    if (!c || o < 0 || o >= c->geom.O) return c ? c->status(GDP_ERR_ARG, "octave out of range") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<2>(c, o, o + 1, c->pick(stream));
}

int gdp_generate_dog(gdp_ctx* c, void* stream) {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<3>(c, 0, c->geom.O, c->pick(stream));
}

const float* gdp_device_level(const gdp_ctx* c, int b, int o, int s) {
    if (!valid_level(c, b, o, s)) return nullptr;
    const OctGeom& og = c->geom.oct[o];
    return c->d_out + (size_t)b * c->geom.pyr_stride + og.lev_off + (size_t)s * og.lev_stride;
}

int gdp_download_level(gdp_ctx* c, int b, int o, int s, float* host) {
    if (!valid_level(c, b, o, s) || !host) return c ? c->status(GDP_ERR_ARG, "gdp_download_level: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    const OctGeom& og = c->geom.oct[o];
    GDP_HIP(c, hipMemcpyAsync(host, gdp_device_level(c, b, o, s), (size_t)og.rows * og.cols * 4, hipMemcpyDeviceToHost,
                              c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
}

int gdp_download_level_rows(gdp_ctx* c, int b, int o, int s, float* const* rows) {
    if (!valid_level(c, b, o, s) || !rows) return c ? c->status(GDP_ERR_ARG, "gdp_download_level_rows: bad argument") : GDP_ERR_ARG;
    const OctGeom& og = c->geom.oct[o];
    if ((size_t)og.rows * og.cols == 0) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    // one pinned staging buffer of at most kStageFloats (or one row), reused chunk by chunk
    const size_t chunk_rows = std::max<size_t>(1, std::min<size_t>(og.rows, kStageFloats / (size_t)og.cols));
    const size_t nfl = chunk_rows * og.cols;
    if (c->h_stage_floats < nfl) {
        if (c->h_stage) GDP_HIP(c, hipHostFree(c->h_stage));
        c->h_stage = nullptr;
        c->h_stage_floats = 0;
        GDP_HIP(c, hipHostMalloc((void**)&c->h_stage, nfl * 4, hipHostMallocDefault));
        c->h_stage_floats = nfl;
    }
    const float* src = gdp_device_level(c, b, o, s);
    for (size_t r0 = 0; r0 < (size_t)og.rows; r0 += chunk_rows) {
        const size_t nr = std::min(chunk_rows, (size_t)og.rows - r0);
        GDP_HIP(c, hipMemcpyAsync(c->h_stage, src + r0 * og.cols, nr * og.cols * 4, hipMemcpyDeviceToHost, c->stream));
        GDP_HIP(c, hipStreamSynchronize(c->stream));
        for (size_t r = 0; r < nr; ++r) std::memcpy(rows[r0 + r], c->h_stage + r * og.cols, (size_t)og.cols * 4);
    }
    return GDP_OK;
}

int gdp_download_pyramid_rows(gdp_ctx* c, int b, float* const* const* const* py) {
    if (!c || !py || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_download_pyramid_rows: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    const Geom& g = c->geom;
    // levels are gathered into one pinned staging buffer (<= kStageFloats, or one level) with one
    // stream sync per fill, then scattered into the caller's rows; a level larger than the
    // staging buffer goes through the row-chunked gdp_download_level_rows
    size_t cap = 0;
    for (int o = 0; o < g.O; ++o) cap += (size_t)g.oct[o].rows * g.oct[o].cols * g.L;
    cap = std::min(cap, kStageFloats);
    if (cap == 0) return GDP_OK;
    if (c->h_stage_floats < cap) {
        if (c->h_stage) GDP_HIP(c, hipHostFree(c->h_stage));
        c->h_stage = nullptr;
        c->h_stage_floats = 0;
        GDP_HIP(c, hipHostMalloc((void**)&c->h_stage, cap * 4, hipHostMallocDefault));
        c->h_stage_floats = cap;
    }
    struct Pending { int o, s; size_t off; };
    std::vector<Pending> pend;
    size_t used = 0;
    auto flush = [&]() -> int {
        if (pend.empty()) return GDP_OK;
        GDP_HIP(c, hipStreamSynchronize(c->stream));
        for (const Pending& q : pend) {
            const OctGeom& og = g.oct[q.o];
            for (int r = 0; r < og.rows; ++r)
                std::memcpy(py[q.o][q.s][r], c->h_stage + q.off + (size_t)r * og.cols, (size_t)og.cols * 4);
        }
        pend.clear();
        used = 0;
        return GDP_OK;
    };
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        const size_t n = (size_t)og.rows * og.cols;
        for (int s = 0; s < g.L && n; ++s) {
            if (n > c->h_stage_floats) {  // does not fit: row-chunked path
                int rc = flush();
                if (rc == GDP_OK) rc = gdp_download_level_rows(c, b, o, s, py[o][s]);
                if (rc != GDP_OK) return rc;
                continue;
            }
            if (used + n > c->h_stage_floats) {
                const int rc = flush();
                if (rc != GDP_OK) return rc;
            }
            GDP_HIP(c, hipMemcpyAsync(c->h_stage + used, gdp_device_level(c, b, o, s), n * 4, hipMemcpyDeviceToHost,
                                      c->stream));
            pend.push_back({o, s, used});
            used += n;
        }
    }
    return flush();
}

int gdp_download_level_range(gdp_ctx* c, int b, int o, int s, int first_row, int nrows, float* host) {
    if (!valid_level(c, b, o, s) || !host || first_row < 0 || nrows < 0 || first_row > c->geom.oct[o].rows ||
        nrows > c->geom.oct[o].rows - first_row)
        return c ? c->status(GDP_ERR_ARG, "gdp_download_level_range: bad argument") : GDP_ERR_ARG;
    if (nrows == 0) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    const OctGeom& og = c->geom.oct[o];
    GDP_HIP(c, hipMemcpyAsync(host, gdp_device_level(c, b, o, s) + (size_t)first_row * og.cols,
                              (size_t)nrows * og.cols * 4, hipMemcpyDeviceToHost, c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
}

int gdp_download_pyramid(gdp_ctx* c, int b, float* host) {
    if (!c || !host || b < 0 || b >= c->geom.batch) return c ? c->status(GDP_ERR_ARG, "gdp_download_pyramid: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    size_t off = 0;
    for (int o = 0; o < c->geom.O; ++o) {
        const OctGeom& og = c->geom.oct[o];
        const size_t n = (size_t)og.rows * og.cols;
        for (int s = 0; s < c->geom.L; ++s, off += n)
            if (n) GDP_HIP(c, hipMemcpyAsync(host + off, gdp_device_level(c, b, o, s), n * 4, hipMemcpyDeviceToHost, c->stream));
    }
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
}

int gdp_upload_pyramid(gdp_ctx* c, int b, const float* host) {
    if (!c || !host || b < 0 || b >= c->geom.batch) return c ? c->status(GDP_ERR_ARG, "gdp_upload_pyramid: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    size_t off = 0;
    for (int o = 0; o < c->geom.O; ++o) {
        const OctGeom& og = c->geom.oct[o];
        const size_t n = (size_t)og.rows * og.cols;
        for (int s = 0; s < c->geom.L; ++s, off += n)
            if (n)
                GDP_HIP(c, hipMemcpyAsync(const_cast<float*>(gdp_device_level(c, b, o, s)), host + off, n * 4,
                                          hipMemcpyHostToDevice, c->stream));
    }
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
}

int gdp_get_taps(gdp_ctx* c, int axis, int o, int s, float* host) {
    if (!c || !host || o < 0 || o >= c->geom.O || s < 0 || s >= c->geom.L || (axis != 0 && axis != 1))
        return c ? c->status(GDP_ERR_ARG, "gdp_get_taps: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    const OctGeom& og = c->geom.oct[o];
    const int n = axis == 0 ? og.cols : (c->geom.H >> o);
    const long long off = axis == 0 ? og.ctap + (long long)s * og.ctap_stride : og.rtap + (long long)s * og.rtap_stride;
    // read back what the device holds, not the host copy: this is what the kernels use
    GDP_HIP(c, hipMemcpy(host, c->d_taps + off, (size_t)n * 4, hipMemcpyDeviceToHost));
    return GDP_OK;
}

int gdp_set_output_device(gdp_ctx* c, float* base, size_t bytes) {
    if (!c) return GDP_ERR_ARG;
    if (!base) {
        c->d_out = c->d_out_own;
        return GDP_OK;
    }
    if (bytes < gdp_pyramid_bytes(c) || (reinterpret_cast<uintptr_t>(base) & 255) != 0)
        return c->status(GDP_ERR_ARG, "gdp_set_output_device: need >= %zu bytes, 256-B aligned", gdp_pyramid_bytes(c));
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_HIP(c, hipDeviceSynchronize());
    c->d_out = base;
    return GDP_OK;
}

size_t gdp_level_offset(const gdp_ctx* c, int b, int o, int s) {
    if (!valid_level(c, b, o, s)) return (size_t)-1;
    const OctGeom& og = c->geom.oct[o];
    return (size_t)b * c->geom.pyr_stride + og.lev_off + (size_t)s * og.lev_stride;
}

int gdp_checksum(gdp_ctx* c, int b, uint64_t* out) {
    if (!c || !out || b < 0 || b >= c->geom.batch) return c ? c->status(GDP_ERR_ARG, "gdp_checksum: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_HIP(c, hipMemsetAsync(c->d_sum, 0, sizeof(unsigned long long), c->stream));
    const Geom& g = c->geom;
    const long long total = g.oct[g.O - 1].grp_begin + (long long)g.oct[g.O - 1].rows * g.oct[g.O - 1].gpr;
    const int grid = (int)std::max<long long>(1, std::min<long long>((total + kBlock - 1) / kBlock, c->blocks_max));
    hipLaunchKernelGGL(k_checksum, dim3(grid), dim3(kBlock), 0, c->stream, c->d_geom, c->d_out, b, c->d_sum);
    GDP_HIP(c, hipGetLastError());
    unsigned long long v = 0;
    GDP_HIP(c, hipMemcpyAsync(&v, c->d_sum, sizeof v, hipMemcpyDeviceToHost, c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    *out = v;
    return GDP_OK;
}

int gdp_sync(gdp_ctx* c) {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
}

void* gdp_stream(const gdp_ctx* c) { return c ? (void*)c->stream : nullptr; }

int gdp_autotune(gdp_ctx* c, int iters, void* stream, int* best_variant, int* best_order, float* best_ms) {
    // Times every build-kernel variant x tile order on the context's current input (HIP events on
    // `stream`, median of 3 repeats of `iters` launches) and keeps the fastest.  All candidates
    // produce identical bits, so this only ever changes speed.
    if (!c || iters <= 0) return c ? c->status(GDP_ERR_ARG, "gdp_autotune: iters must be > 0") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    const int old_variant = c->variant, old_order = c->geom.tile_order;
    int bv = old_variant, bo = old_order;
    float bt = 3.4e38f;
    for (int v = 0; v < kNumVariants; ++v) {
        for (int ord = 0; ord <= 1; ++ord) {
            int rc = gdp_set_tuning(c, GDP_TUNE_VARIANT, v);
            if (rc == GDP_OK) rc = gdp_set_tuning(c, GDP_TUNE_TILE_ORDER, ord);
            if (rc != GDP_OK) return rc;
            float t[3];
            rc = gdp_time_builds(c, 1, stream, &t[0]);  // warm-up
            for (int r = 0; r < 3 && rc == GDP_OK; ++r) rc = gdp_time_builds(c, iters, stream, &t[r]);
            if (rc != GDP_OK) return rc;
            std::sort(t, t + 3);
            if (t[1] < bt) {
                bt = t[1];
                bv = v;
                bo = ord;
            }
        }
    }
    int rc = gdp_set_tuning(c, GDP_TUNE_VARIANT, bv);
    if (rc == GDP_OK) rc = gdp_set_tuning(c, GDP_TUNE_TILE_ORDER, bo);
    if (rc != GDP_OK) return rc;
    if (best_variant) *best_variant = bv;
    if (best_order) *best_order = bo;
    if (best_ms) *best_ms = bt / iters;
    return GDP_OK;
}

int gdp_get_tuning(const gdp_ctx* c, int key, int* value) {
    if (!c || !value) return GDP_ERR_ARG;
    switch (key) {
        case GDP_TUNE_NONTEMPORAL: *value = c->nontemporal; return GDP_OK;
        case GDP_TUNE_BLOCKS_PER_CU: *value = c->persistent ? c->blocks_max / c->cus : 0; return GDP_OK;
        case GDP_TUNE_GRID: *value = c->grid_override; return GDP_OK;
        case GDP_TUNE_VARIANT: *value = c->variant; return GDP_OK;
        case GDP_TUNE_TILE_ORDER: *value = c->geom.tile_order; return GDP_OK;
        case GDP_TUNE_INPLACE_SUB: *value = c->inplace_sub; return GDP_OK;
        case GDP_TUNE_WINDOW_SUB: *value = c->window_sub; return GDP_OK;
        case GDP_TUNE_CONV_KERNEL: *value = c->conv_kernel; return GDP_OK;
        case GDP_TUNE_CONV_ROWS: *value = c->conv_rows; return GDP_OK;
        case GDP_TUNE_CONV_ORDER: *value = c->conv_order; return GDP_OK;
        default: return GDP_ERR_ARG;
    }
}

int gdp_set_tuning(gdp_ctx* c, int key, int value) {
    if (!c) return GDP_ERR_ARG;
    switch (key) {
        case GDP_TUNE_NONTEMPORAL:
            c->nontemporal = value ? 1 : 0;
            return GDP_OK;
        case GDP_TUNE_BLOCKS_PER_CU:
            if (value < 0 || value > 64) return c->status(GDP_ERR_ARG, "blocks per CU must be in [0, 64]");
            c->persistent = value > 0;
            c->blocks_max = c->cus * (value > 0 ? value : 8);
            return GDP_OK;
        case GDP_TUNE_GRID:
            if (value < 0) return c->status(GDP_ERR_ARG, "grid must be >= 0");
            c->grid_override = value;
            return GDP_OK;
        case GDP_TUNE_INPLACE_SUB:
        case GDP_TUNE_WINDOW_SUB:
            if ((value != 1 && value != 2 && value != 4) && !(key == GDP_TUNE_INPLACE_SUB && value == 0))
                return c->status(GDP_ERR_ARG, "sub-blocks must be 1, 2 or 4 (in-place DoG also 0: one level per wave)");
            (key == GDP_TUNE_INPLACE_SUB ? c->inplace_sub : c->window_sub) = value;
            return GDP_OK;
        case GDP_TUNE_CONV_KERNEL:
            if (value != 0 && value != 1) return c->status(GDP_ERR_ARG, "conv kernel must be 0 (sweep) or 1 (tiles)");
            c->conv_kernel = value;
            return GDP_OK;
        case GDP_TUNE_CONV_ROWS: {
            if (value != 16 && value != 32) return c->status(GDP_ERR_ARG, "conv rows must be 16 or 32");
            const int old = c->conv_rows;
            c->conv_rows = value;
            conv_sweep_geom(c);
            const int rc = upload_geom(c);
            if (rc != GDP_OK) {
                c->conv_rows = old;
                conv_sweep_geom(c);
            }
            return rc;
        }
        case GDP_TUNE_CONV_ORDER:
            if (value < 0 || value > 3) return c->status(GDP_ERR_ARG, "conv order must be 0..3");
            c->conv_order = value;
            return GDP_OK;
        case GDP_TUNE_TILE_ORDER:
            if (value < 0 || value > 2) return c->status(GDP_ERR_ARG, "tile order must be 0, 1 or 2");
            c->geom.tile_order = value;
            return upload_geom(c);
        case GDP_TUNE_VARIANT: {
            if (value < 0 || value >= kNumVariants) return c->status(GDP_ERR_ARG, "variant out of range");
            const int old = c->variant;
            c->variant = value;
            int rc = retile(c, kVariants[value].tile_cols, kVariants[value].tile_rows);
            if (rc == GDP_OK) rc = upload_geom(c);
            if (rc != GDP_OK) {
                c->variant = old;
                retile(c, kVariants[old].tile_cols, kVariants[old].tile_rows);
            }
            return rc;
        }
        default:
            return c->status(GDP_ERR_ARG, "unknown tuning key %d", key);
    }
}

int gdp_time_builds(gdp_ctx* c, int iters, void* stream, float* total_ms) {
    if (!c || iters <= 0 || !total_ms) return c ? c->status(GDP_ERR_ARG, "gdp_time_builds: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    hipStream_t st = c->pick(stream);
    hipEvent_t e0, e1;
    GDP_HIP(c, hipEventCreate(&e0));
    GDP_HIP(c, hipEventCreate(&e1));
    int rc = GDP_OK;
    if (hipEventRecord(e0, st) != hipSuccess) rc = c->status(GDP_ERR_HIP, "hipEventRecord");
    for (int i = 0; i < iters && rc == GDP_OK; ++i) rc = launch_build(c, st);
    if (rc == GDP_OK && hipEventRecord(e1, st) != hipSuccess) rc = c->status(GDP_ERR_HIP, "hipEventRecord");
    if (rc == GDP_OK && hipEventSynchronize(e1) != hipSuccess) rc = c->status(GDP_ERR_HIP, "hipEventSynchronize");
    if (rc == GDP_OK && hipEventElapsedTime(total_ms, e0, e1) != hipSuccess) rc = c->status(GDP_ERR_HIP, "hipEventElapsedTime");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

}  // extern "C"
