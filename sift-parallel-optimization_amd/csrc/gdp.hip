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
#include <functional>
#include <new>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <array>
#include <atomic>
#include <mutex>
#include <vector>

#include <linux/futex.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "gdp.h"

#pragma clang fp contract(off)

namespace {

#include "gdp_geom.inc"
#include "gdp_build.inc"
#include "gdp_inplace.inc"
#include "gdp_conv.inc"
#include "gdp_util.inc"
#include "gdp_track.inc"

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// GuassDePyramid.h:7-8 (PI is 3.1414926f in the reference, reproduced on purpose).
const float kSigma = 2.0f;
const float kPI = 3.1414926f;

// GuassDePyramid.h:107-121, evaluated on the host in the reference's float expression order:
// the window centre is the FLOAT length halved o times, minus 1, over 2 (:107-115).  With
// GDP_CENTRE_INTLEN the centre is float(len_o - 1) / 2 of the INTEGER length len_o = length >> o,
// as the multi-process variants compute it (GaussDePyramid-MPI.h:273, mpitest.cpp:44,123); their
// tap expression is otherwise the same (GaussDePyramid-MPI.h:278,283).
int host_taps(int length, int octave, int scale, float* out, int centre_mode) {
    float len = (float)length;
    for (int t = octave; t != 0; --t) len /= 2;
    const int my_len = (int)len;
    if (centre_mode == GDP_CENTRE_INTLEN)
        len = (float)((double)(my_len - 1) / 2.0);  // l = float(len - 1) / 2.0
    else
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

// Layout / allocation experiment knobs (GDP_SPREAD_CHUNK_MB / _KB, GDP_SPREAD_PHYS_MB,
// GDP_SPREAD_PERM, GDP_IMAGE_STRIDE_MB, GDP_LEVEL_PAD, GDP_ROWTAP_LAYOUT, GDP_INPUT_VMM: the
// measurements of DESIGN §4 / §5.1) are read only by a library built with -DGDP_EXPERIMENTS
// (`make -C csrc exp`, a separate research build); the product library ignores them and runs the
// measured defaults.  The one product environment switch is GDP_SPREAD_VMM=0 (one hipMalloc).
#ifdef GDP_EXPERIMENTS
const char* exp_env(const char* name) { return std::getenv(name); }
#else
const char* exp_env(const char*) { return nullptr; }
#endif

thread_local std::string g_create_error;

}  // namespace

struct gdp_ctx {
    int device = 0;
    Geom geom{};
    Geom* d_geom = nullptr;
    void* d_in_own = nullptr;     // context-owned input buffer (int32 or uint8 per geom.in_fmt)
    // GDP_INPUT_VMM=1 (experiment): the input in 2 MiB physical pieces like the pyramid (in_vmm_*)
    struct VmmBuf {
        std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks;  // handle, offset
        size_t span = 0;  // 0: the buffer is one hipMalloc
    } in_vmm;
    void* d_halo_own[2] = {nullptr, nullptr}; // context-owned halo rows above / below a band (conv extension)
    const void* d_in = nullptr;   // buffer the kernels read (own or caller's)
    float* d_out = nullptr;
    float* d_taps = nullptr;      // the table the next launch reads: d_taps_mode[centre_mode]
    float* d_taps_mode[2] = {nullptr, nullptr}; // one device tap table per window-centre mode, built on
                                  // first use, so switching centres is a pointer swap (no drain)
    int conv_kernel = 2;          // GDP_TUNE_CONV_KERNEL: 0 register sweep, 1 LDS tiles, 2 block tiles (default)
    int conv_rows = 48;           // GDP_TUNE_CONV_ROWS: output rows per wave strip of the sweep / per block tile
    int conv_waves = 16;          // GDP_TUNE_CONV_WAVES: waves per block of the block tiles
    bool conv_rows_set = false;   // GDP_TUNE_CONV_ROWS set by the caller; until then the rows follow
                                  // the selected kernel / waves (conv_default_rows)
    std::vector<std::array<int, 5>> support; // per octave: nz_r0, nz_r1, nz_c0, nz_c1, rows exact in place
    int zero_window = 0;          // GDP_TUNE_ZERO_WINDOW: build groups outside the windows' support store
                                  // their input-independent levels without waiting for the input
    int conv_order = 4;           // GDP_TUNE_CONV_ORDER: bit 0 XCD-chunked blocks, bit 1 alternate sweep directions,
                                  // bit 2 input-row-interleaved octaves (conv_sweep_perm; default 4)
    int build_lds = 0;            // GDP_TUNE_BUILD_LDS: dynamic LDS bytes per build block (caps blocks per CU)
    int centre_mode = GDP_CENTRE_SERIAL; // gdp_set_window_centre
    float* d_ctaps = nullptr;     // convolution-mode taps [L][13] (extension)
    int* d_cradius = nullptr;     // convolution-mode radius per scale
    unsigned* d_conv_perm = nullptr; // conv sweep block order for GDP_TUNE_CONV_ORDER bit 2 (per image)
    bool conv_perm_dirty = true;
    int conv_perm_kernel = -1;       // the conv kernel d_conv_perm was built for (its block prefix)
    float* d_out_own = nullptr;   // context-owned pyramid (d_out may point at caller memory)
    long long img_floats = 0;     // one image's dense extent (pyr_stride may be larger: GDP_IMAGE_STRIDE_MB)
    // GDP_SPREAD_VMM: the pyramid as one reserved address range with separately created physical
    // chunks mapped into it (alloc_spread); each entry: handle, byte offset, bytes
    struct VmmChunk {
        hipMemGenericAllocationHandle_t h;
        size_t off, bytes;
    };
    std::vector<VmmChunk> vmm_chunks;
    size_t vmm_span = 0;
    int pyr_chunk_kb = 0;         // GDP_TUNE_PYRAMID_CHUNK_KB: 0 one hipMalloc, -1 one chunk per image
    float* h_stage = nullptr;     // pinned staging for row-pointer downloads (two halves)
    size_t h_stage_floats = 0;
    size_t stage_half_floats = kStageFloats / 2; // GDP_TUNE_STAGE_KB
    int stage_threads = 8;        // GDP_TUNE_STAGE_THREADS: host threads scattering a staged batch (8: 4096^2
                                  // pyramid download 8.77 vs 9.99 ms with 4, tools/mirror_bench.py; capped by
                                  // the host's hardware threads at context creation)
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    // gdp_generate_dog_mirrored: copy streams (host -> device, device -> host) and per-chunk events
    hipStream_t st_up = nullptr, st_down = nullptr;
    std::vector<hipEvent_t> ev_mirror;
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
    if (tile_rows == 0) {
        // Contiguous-span variants (PATH 4): every octave's groups, in row-major
        // order (the levels are dense row-major, GuassDePyramid.h:63-72), are cut into the same
        // number of contiguous chunks, one per work unit — octave 0 into chunks of at most
        // `tile_cols` groups, octave o into proportional ones, which read the same input rows.
        // A unit's stores are then one contiguous span of each level, crossing row boundaries,
        // instead of tile rows a row pitch apart.  No tail units: every octave lives in the units.
        const long long total0 = (long long)g.oct[0].rows * g.oct[0].gpr;
        const long long nblk = std::max(1ll, (total0 + tile_cols - 1) / tile_cols);
        long long rest = 0;
        for (int o = 0; o < g.O; ++o) {
            OctGeom& og = g.oct[o];
            og.span = (int)(((long long)og.rows * og.gpr + nblk - 1) / nblk);
            if (o > 0) rest += og.span;
        }
        if (nblk * g.batch >= (1ll << 31) || rest >= (1ll << 31))
            return c->status(GDP_ERR_ARG, "image/batch too large for one context (split the batch)");
        g.span_rest = (int)rest;
        g.F = g.O;
        g.tail_groups_per_img = 0;
        g.tail_units = 0;
        g.tiles_r = (int)nblk;
        g.tiles_c = 1;
        g.tiles_per_img = (unsigned)nblk;
        g.tiles_total = (unsigned)(nblk * g.batch);
        return GDP_OK;
    }
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

int launch_build(gdp_ctx* c, hipStream_t st, bool subset = false) {
    const Geom& g = c->geom;
    const long long units = (long long)g.tiles_total + g.tail_units;
    if (units == 0) return GDP_OK;
    // default: one unit per block; GDP_TUNE_GRID / GDP_TUNE_BLOCKS_PER_CU cap it (persistent loop)
    const long long cap = c->grid_override > 0 ? c->grid_override : (c->persistent ? c->blocks_max : units);
    const int grid = (int)std::min<long long>(units, cap);
    const BuildVariant& v = kVariants[variant_index(c->variant)];
    auto kern = (subset ? v.ksub : v.k)[g.L == 5][c->nontemporal ? 1 : 0];
    hipLaunchKernelGGL(kern, dim3(grid), dim3(v.block), (unsigned)c->build_lds, st, c->d_geom, c->d_in, c->d_out,
                       c->d_taps);
    GDP_HIP(c, hipGetLastError());
    return GDP_OK;
}

template <int MODE, int SUB>
int launch_inplace_sub(gdp_ctx* c, int ob, int oe, hipStream_t st, int sb = 0, int se = -1) {
    const Geom& g = c->geom;
    if constexpr (MODE == 1) {
        const int Ls = (se < 0 ? g.L : se) - sb;  // scales [sb, sb + Ls) (gdp_gauss_scales), all by default
        const long long grid = ((long long)g.lv_blk[oe] - g.lv_blk[ob]) * Ls * g.batch * SUB;
        if (grid <= 0) return GDP_OK;
        if (grid >= (1ll << 31) || (long long)g.lv_blk[g.O] * g.L >= (1ll << 32))
            return c->status(GDP_ERR_ARG, "window pass too large for one launch");
        auto wkern = c->nontemporal ? k_window<true, SUB> : k_window<false, SUB>;
        hipLaunchKernelGGL(wkern, dim3((unsigned)grid), dim3(kLevBlock / SUB), 0, st, c->d_geom, c->d_out, c->d_taps, ob,
                           oe, sb, Ls);
        GDP_HIP(c, hipGetLastError());
        return GDP_OK;
    }
    const long long per = (long long)g.lv_blk[oe] - g.lv_blk[ob];
    const long long grid = per * g.batch * SUB;
    if (grid <= 0) return GDP_OK;
    if (grid >= (1ll << 31)) return c->status(GDP_ERR_ARG, "in-place pass too large for one launch");
    auto kern = c->nontemporal ? k_levels<0, MODE, true, SUB> : k_levels<0, MODE, false, SUB>;
    if constexpr (MODE != 9) {
        if (g.L == 5) kern = c->nontemporal ? k_levels<5, MODE, true, SUB> : k_levels<5, MODE, false, SUB>;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kLevBlock / SUB), 0, st, c->d_geom, c->d_in, c->d_out, c->d_taps,
                       ob, oe);
    GDP_HIP(c, hipGetLastError());
    return GDP_OK;
}

template <int MODE>
int launch_inplace(gdp_ctx* c, int ob, int oe, hipStream_t st, int sb = 0, int se = -1) {
    const Geom& g = c->geom;
    if ((MODE == 2 || MODE == 3) && c->inplace_sub == -kLtRows) {  // k_build-shaped block tiles
        const long long grid = ((long long)g.lt_blk[oe] - g.lt_blk[ob]) * g.batch;
        if (grid <= 0) return GDP_OK;
        if (grid >= (1ll << 31)) return c->status(GDP_ERR_ARG, "in-place pass too large for one launch");
        auto kern = c->nontemporal ? k_levels_tile<0, MODE, true> : k_levels_tile<0, MODE, false>;
        if (g.L == 5) kern = c->nontemporal ? k_levels_tile<5, MODE, true> : k_levels_tile<5, MODE, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * kLtRows), 0, st, c->d_geom, c->d_in, c->d_out, c->d_taps,
                           ob, oe);
        GDP_HIP(c, hipGetLastError());
        return GDP_OK;
    }
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
        case 2: return launch_inplace_sub<MODE, 2>(c, ob, oe, st, sb, se);
        case 4: return launch_inplace_sub<MODE, 4>(c, ob, oe, st, sb, se);
        case 8: return launch_inplace_sub<MODE, 8>(c, ob, oe, st, sb, se);
        case 16: return launch_inplace_sub<MODE, 16>(c, ob, oe, st, sb, se);
        default: return launch_inplace_sub<MODE, 1>(c, ob, oe, st, sb, se);
    }
}

// Column taps of every (o, s) from W, row taps from H (aliased for square images), in window-
// centre mode `mode` (host memory only).
void fill_host_taps(gdp_ctx* c, int mode) {
    const Geom& g = c->geom;
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        // host_taps writes (int) of the float-halved axis length, which above 2^24 can round to one
        // more (or fewer) than len >> o: compute into scratch sized with slack and copy exactly the
        // len >> o taps the octave has (taps the float length did not reach stay +0)
        const int Hg = g.H >> o, Wg = og.cols;
        std::vector<float> t((size_t)std::max(1, std::max(Hg, Wg)) + 8);
        auto taps_of = [&](int length, int n_axis, int s) {
            std::fill(t.begin(), t.end(), 0.0f);
            host_taps(length, o, s, t.data(), mode);
            return n_axis;
        };
        for (int s = 0; s < g.L; ++s) {
            const int nc = taps_of(g.W, Wg, s);
            std::copy(t.begin(), t.begin() + nc, c->h_taps.begin() + og.ctap + (long long)s * og.ctap_stride);
            if (og.rtap_row == 1) {  // contiguous per scale (a square image's: the column taps again)
                const int nr = taps_of(g.H, Hg, s);
                std::copy(t.begin(), t.begin() + nr, c->h_taps.begin() + og.rtap + (long long)s * og.rtap_stride);
                continue;
            }
            const int nr = taps_of(g.H, Hg, s);  // [row][scale] interleaved
            for (int r = 0; r < nr; ++r) c->h_taps[og.rtap + (size_t)r * og.rtap_row + s] = t[r];
        }
    }
}

// Window support of every octave (OctGeom::nz_*): the smallest global row / column ranges that
// hold every non-zero tap of any scale under EITHER window centre (so switching centres, a tap-
// table pointer swap, needs no geometry change).  The reference's windows underflow to +0 a few
// σ from the centre (expf(-d²/(2σ²)) = 0 for d >= 29 at σ = 2), so on a large image almost every
// pixel lies outside them.  `on` = 0: the ranges cover the whole octave (every group computed).
// The ranges are computed once per context (host expf over every row and column of every octave)
// and only copied in and out of the Geom when the knob changes.
void set_window_support(gdp_ctx* c, bool on) {
    Geom& g = c->geom;
    if (on && c->support.size() != (size_t)g.O) {
        c->support.assign((size_t)g.O, {0, 0, 0, 0, 0});
        for (int o = 0; o < g.O; ++o) {
            auto support = [&](int length, int& lo, int& hi, float& peak) {
                // host_taps writes (int) of the float-halved length: above 2^24 that can round up
                std::vector<float> t((size_t)std::max(1, length >> o) + 8);
                lo = INT32_MAX;
                hi = 0;
                peak = 0.0f;
                for (int mode : {GDP_CENTRE_SERIAL, GDP_CENTRE_INTLEN})
                    for (int s = 0; s < g.L; ++s) {
                        const int n = std::min(host_taps(length, o, s, t.data(), mode), std::max(0, length >> o));
                        for (int i = 0; i < n; ++i) {
                            peak = std::max(peak, t[i]);
                            if (t[i] != 0.0f) {
                                lo = std::min(lo, i);
                                hi = std::max(hi, i + 1);
                            }
                        }
                    }
                if (lo > hi) lo = hi = 0; // no non-zero tap at all: every pixel is outside
            };
            auto& r = c->support[(size_t)o];
            float col_peak = 0.0f, row_peak = 0.0f;
            support(g.W, r[2], r[3], col_peak);
            support(g.H, r[0], r[1], row_peak);
            r[4] = col_peak <= 1.0f ? 1 : 0;  // rows outside the support exact for the in-place passes
        }
    }
    for (int o = 0; o < g.O; ++o) {
        OctGeom& og = g.oct[o];
        if (on) {
            const auto& r = c->support[(size_t)o];
            og.nz_r0 = r[0], og.nz_r1 = r[1], og.nz_c0 = r[2], og.nz_c1 = r[3];
            og.nzi_r0 = r[4] ? r[0] : 0;
            og.nzi_r1 = r[4] ? r[1] : g.H >> o;
        } else {
            og.nz_r0 = og.nzi_r0 = 0, og.nz_r1 = og.nzi_r1 = g.H >> o, og.nz_c0 = 0, og.nz_c1 = og.cols;
        }
    }
}

bool valid_level(const gdp_ctx* c, int b, int o, int s) {
    return c && b >= 0 && b < c->geom.batch && o >= 0 && o < c->geom.O && s >= 0 && s < c->geom.L;
}

}  // namespace

// ==========================================================================================
// C ABI
// ==========================================================================================
// Block prefixes of the convolution sweep (kSwWaves strips of conv_rows rows x kSwCols columns)
// and of the block tiles (conv_rows rows x kSwCols columns).
static int conv_sweep_rows(const gdp_ctx* c) { return c->conv_rows == 32 ? 32 : 16; }
// The block tiles are instantiated for these (rows per block, waves per block) pairs only: each
// wave owns whole output rows, so 16 waves take 16/32/48-row tiles and 8 waves 8/16/24/32.
// (Measured and dropped, round 3: 64-row tiles on 16 waves — 80 staged rows, 80 KB of LDS, two
// blocks per CU — cut the staged-row overhead from 44/32 to 76/64 but ran slower on every config:
// 4096^2 0.110 vs 0.099 ms, 64 x 1080 x 1920 0.767 vs 0.714, 64 x 4096^2 5.95 vs 5.71, 16384^2
// 1.48 vs 1.45; profiles/conv_ab_r03c.log.  Re-measured with the stores paced, still behind the
// 48-row default: 4096^2 0.1088 vs 0.1021 ms, 64 x 4096^2 5.84 vs 5.69, 16384^2 1.483 vs 1.453;
// profiles/cpy_conv_c*_r03ay.log.)
static bool conv_blk_pair_ok(int rows, int waves) {
    return waves == 16 ? (rows == 16 || rows == 32 || rows == 48)
                       : waves == 8 && (rows == 8 || rows == 16 || rows == 24 || rows == 32);
}
// Rows per tile / strip when the caller has not chosen them: the sweep's 16-row strips, the block
// tiles' 48 rows on 16 waves (the default) and 32 on 8 waves — so selecting only the kernel or only
// the waves never leaves an uninstantiated pair.  The LDS tiles take no row count.
static int conv_default_rows(const gdp_ctx* c) {
    if (c->conv_kernel == 0) return 16;
    if (c->conv_kernel == 2) return c->conv_waves == 8 ? 32 : 48;
    return c->conv_rows;
}
static void conv_sweep_geom(gdp_ctx* c) {
    Geom& g = c->geom;
    const int strip_cols = SwGeom<kSwV>::kCols;
    g.sw_blk[0] = 0;
    g.cvx_blk[0] = 0;
    g.bk_blk[0] = 0;
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        const bool sweep = og.cols >= 4 && og.cols % 4 == 0; // full-vector stores on every row
        g.sw_strips_c[o] = (og.cols + strip_cols - 1) / strip_cols;
        const long long rows_per_blk = (long long)kSwWaves * conv_sweep_rows(c);
        g.sw_blk[o + 1] = g.sw_blk[o] + (sweep ? (unsigned)((og.rows + rows_per_blk - 1) / rows_per_blk * g.sw_strips_c[o]) : 0u);
        const long long bk_rows = c->conv_rows;
        const int bk_cols = 4 * (64 - 2 * kBkHaloLanes);  // block-tile output columns (240)
        g.bk_strips_c[o] = (og.cols + bk_cols - 1) / bk_cols;
        g.bk_blk[o + 1] = g.bk_blk[o] + (sweep ? (unsigned)((og.rows + bk_rows - 1) / bk_rows * g.bk_strips_c[o]) : 0u);
        g.cvx_blk[o + 1] = g.cvx_blk[o] + (sweep ? 0u : g.cv_blk[o + 1] - g.cv_blk[o]);
    }
    c->conv_perm_dirty = true;
}

static int conv_set_rows(gdp_ctx* c, int rows) {
    if (rows == c->conv_rows) return GDP_OK;
    const int old = c->conv_rows;
    c->conv_rows = rows;
    conv_sweep_geom(c);
    const int rc = upload_geom(c);
    if (rc != GDP_OK) {
        c->conv_rows = old;
        conv_sweep_geom(c);
    }
    return rc;
}
// after a kernel / waves change: rows the caller never set follow the selection
static int conv_follow_rows(gdp_ctx* c) { return c->conv_rows_set ? GDP_OK : conv_set_rows(c, conv_default_rows(c)); }

// Input-row-interleaved block order of the convolution sweep / block tiles (GDP_TUNE_CONV_ORDER
// bit 2): each octave-o block row (2^o times as many input rows as an octave-0 block row) is
// issued right after the octave-0 block row that covers the last of its input rows, so the
// decimated rows it reads were just brought on chip by octave 0 instead of being fetched again.
// `blk` is the block prefix of the kernel that will run (sw_blk or bk_blk).
static int conv_sweep_perm(gdp_ctx* c, const unsigned* blk, const int* strips) {
    const Geom& g = c->geom;
    std::vector<unsigned> perm;
    perm.reserve(blk[g.O]);
    auto emit_row = [&](int o, unsigned tr) {
        const unsigned sc = (unsigned)strips[o];
        for (unsigned tc = 0; tc < sc; ++tc) perm.push_back(blk[o] + tr * sc + tc);
    };
    const unsigned rows0 = g.oct[0].cols ? (blk[1] - blk[0]) / std::max(1u, (unsigned)strips[0]) : 0;
    std::vector<unsigned> next(g.O, 0); // next block row of each octave
    for (unsigned k = 0; k < rows0; ++k) {
        emit_row(0, k);
        for (int o = 1; o < g.O; ++o) {
            const unsigned sc = (unsigned)std::max(1, strips[o]);
            const unsigned nrows = (blk[o + 1] - blk[o]) / sc;
            // octave-o block row tr covers octave-0 block rows [2^o tr, 2^o (tr + 1))
            while (next[o] < nrows && ((unsigned long long)(next[o] + 1) << o) <= (unsigned long long)k + 1)
                emit_row(o, next[o]++);
        }
    }
    for (int o = 1; o < g.O; ++o) { // leftovers (octave 0 swept nothing, or rounding at the bottom)
        const unsigned sc = (unsigned)std::max(1, strips[o]);
        const unsigned nrows = (blk[o + 1] - blk[o]) / sc;
        while (next[o] < nrows) emit_row(o, next[o]++);
    }
    if (perm.size() != blk[g.O]) return c->status(GDP_ERR_STATE, "conv block order: %zu of %u blocks", perm.size(), blk[g.O]);
    if (c->d_conv_perm) GDP_HIP(c, hipFree(c->d_conv_perm));
    c->d_conv_perm = nullptr;
    if (!perm.empty()) {
        GDP_HIP(c, hipMalloc(&c->d_conv_perm, perm.size() * sizeof(unsigned)));
        GDP_HIP(c, hipMemcpy(c->d_conv_perm, perm.data(), perm.size() * sizeof(unsigned), hipMemcpyHostToDevice));
    }
    c->conv_perm_dirty = false;
    return GDP_OK;
}

template <int L, int T>
hipError_t launch_conv_sweep_t(gdp_ctx* c, unsigned units, hipStream_t st) {
    auto k = k_conv_sweep<L, T, kSwV>;
    const unsigned grid = (c->conv_order & 1) ? (units + 7u) / 8u * 8u : units;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * kSwWaves), 0, st, c->d_geom, c->d_in, c->d_out, units, c->conv_order,
                       c->d_conv_perm);
    return hipGetLastError();
}

template <int L, int T, int W>
hipError_t launch_conv_blk_t(gdp_ctx* c, unsigned units, hipStream_t st) {
    // the default pacing (vmcnt(2)) compiled in for the 16-wave tiles; any other pace, and the
    // 8-wave tiles, read it at run time.  (Round 6, every pace compiled in for S = 2 and measured
    // alternated twice on c2 / c4 / c5: all within 0.7 % — conv_pace_ab_r06m.log.)
    auto k = (W == 16 && c->geom.conv_pace == 2) ? k_conv_blk<L, T, W, kBkHaloLanes, 2>
                                                 : k_conv_blk<L, T, W, kBkHaloLanes, kPaceRuntime>;
    const unsigned grid = (c->conv_order & 1) ? (units + 7u) / 8u * 8u : units;
    hipLaunchKernelGGL(k, dim3(grid), dim3(64 * W), 0, st, c->d_geom, c->d_in, c->d_out, units, c->conv_order,
                       c->d_conv_perm);
    return hipGetLastError();
}

// block tiles: the instantiated (rows per block, waves per block) pairs (conv_blk_pair_ok); the
// tile grid (bk_blk) was planned for conv_rows, so any other pair is refused, never run with a
// different tile height
template <int L>
hipError_t launch_conv_blk(gdp_ctx* c, unsigned units, hipStream_t st) {
    const int T = c->conv_rows, W = c->conv_waves;
    if (W == 8) {
        switch (T) {
            case 8: return launch_conv_blk_t<L, 8, 8>(c, units, st);
            case 16: return launch_conv_blk_t<L, 16, 8>(c, units, st);
            case 24: return launch_conv_blk_t<L, 24, 8>(c, units, st);
            case 32: return launch_conv_blk_t<L, 32, 8>(c, units, st);
            default: return hipErrorInvalidConfiguration;
        }
    }
    if (W != 16) return hipErrorInvalidConfiguration;
    switch (T) {
        case 16: return launch_conv_blk_t<L, 16, 16>(c, units, st);
        case 32: return launch_conv_blk_t<L, 32, 16>(c, units, st);
        case 48: return launch_conv_blk_t<L, 48, 16>(c, units, st);
        default: return hipErrorInvalidConfiguration;
    }
}

template <int L>
hipError_t launch_conv_sweep_l(gdp_ctx* c, unsigned grid, hipStream_t st) {
    if (c->conv_kernel == 2) return launch_conv_blk<L>(c, grid, st);
    return conv_sweep_rows(c) == 32 ? launch_conv_sweep_t<L, 32>(c, grid, st) : launch_conv_sweep_t<L, 16>(c, grid, st);
}

// ---- no C++ exception crosses the C ABI --------------------------------------------------------
// Every int-returning export is a function-try-block ending in GDP_ABI_CATCH(ctx): std::bad_alloc
// becomes GDP_ERR_NOMEM, anything else GDP_ERR_INTERNAL, with the text in gdp_last_error(ctx)
// (ctx NULL: the thread's create error).  The exports that return pointers / sizes / void do not
// allocate.
static int abi_exception(const gdp_ctx* c, int code, const char* what) noexcept {
    try {
        if (c)
            const_cast<gdp_ctx*>(c)->err = what;
        else
            g_create_error = what;
    } catch (...) {
    }
    return code;
}
#define GDP_ABI_CATCH(ctx)                                                                                   \
    catch (const std::bad_alloc&) { return abi_exception((ctx), GDP_ERR_NOMEM, "host allocation failed (std::bad_alloc)"); } \
    catch (const std::exception& e_) { return abi_exception((ctx), GDP_ERR_INTERNAL, e_.what()); }         \
    catch (...) { return abi_exception((ctx), GDP_ERR_INTERNAL, "unknown C++ exception"); }

// Deferred mirrors overlapping the caller host memory an entry is given are completed first: no
// libgdp copy may fault on a stale page (gdp_track.inc).  `ranges(f)` calls f(ptr, bytes) for
// each host range the entry touches; a registry lock and one walk over its slots when nothing is
// deferred.
static size_t packed_pyramid_bytes(const gdp_ctx* c) {  // gdp_download_pyramid's layout
    size_t n = 0;
    for (int o = 0; o < c->geom.O; ++o) n += (size_t)c->geom.oct[o].rows * c->geom.oct[o].cols * c->geom.L;
    return n * 4;
}
template <class F>
static int settle_deferred(gdp_ctx* c, const char* what, F&& ranges) {
    std::lock_guard<std::mutex> lk(g_track_mu);
    if (!track_any_deferred()) return GDP_OK;
    int rc = GDP_OK;
    ranges([&](const void* p, size_t n) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        if (p && n && track_settle_overlap(a, a + n) != GDP_OK) rc = GDP_ERR_HIP;
    });
    return rc == GDP_OK ? GDP_OK : c->status(rc, "%s: completing a deferred host mirror failed", what);
}
#define GDP_SETTLE(c, what, ...)                                          \
    do {                                                                  \
        const int settle_rc_ = settle_deferred((c), (what), __VA_ARGS__); \
        if (settle_rc_ != GDP_OK) return settle_rc_;                      \
    } while (0)

extern "C" {

int gdp_abi_version(void) { return GDP_ABI_VERSION; }

int gdp_octaves_for(int n) { return octaves_for(n); }

int gdp_device_count(void) try {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
} GDP_ABI_CATCH(nullptr)

const char* gdp_status_string(int s) {
    switch (s) {
        case GDP_OK: return "ok";
        case GDP_ERR_ARG: return "invalid argument";
        case GDP_ERR_HIP: return "HIP runtime error";
        case GDP_ERR_STATE: return "invalid state";
        case GDP_ERR_NOMEM: return "out of memory";
        case GDP_ERR_NODEV: return "no gfx950 device";
        case GDP_ERR_INTERNAL: return "internal error";
        default: return "unknown status";
    }
}

const char* gdp_last_error(const gdp_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_error.c_str(); }

// The input buffer: one hipMalloc, or (GDP_INPUT_VMM=1) 2 MiB physical pieces in one 2 MiB-aligned
// range; `vb` records which (free_input releases either form).
static hipError_t alloc_input(gdp_ctx* c, size_t bytes, void** out, gdp_ctx::VmmBuf& vb) {
    bytes = std::max<size_t>(16, bytes);
    *out = nullptr;
    const char* iv = exp_env("GDP_INPUT_VMM");
    if (!iv || std::atoi(iv) == 0) return hipMalloc(out, bytes);
    const size_t two = (size_t)2 << 20, span = (bytes + two - 1) / two * two;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = c->device;
    void* base = nullptr;
    hipError_t e = hipMemAddressReserve(&base, span, two, nullptr, 0);
    if (e != hipSuccess) return e;
    vb.span = span;
    *out = base;
    for (size_t off = 0; off < span && e == hipSuccess; off += two) {
        hipMemGenericAllocationHandle_t h;
        if ((e = hipMemCreate(&h, two, &prop, 0)) != hipSuccess) break;
        if ((e = hipMemMap(static_cast<char*>(base) + off, two, 0, h, 0)) != hipSuccess) {
            (void)hipMemRelease(h);
            break;
        }
        vb.chunks.push_back({h, off});
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (e == hipSuccess) e = hipMemSetAccess(base, span, &acc, 1);
    return e;
}

static void free_input(void* p, gdp_ctx::VmmBuf& vb) {
    if (vb.span && p) {
        for (const auto& k : vb.chunks) {
            (void)hipMemUnmap(static_cast<char*>(p) + k.second, (size_t)2 << 20);
            (void)hipMemRelease(k.first);
        }
        (void)hipMemAddressFree(p, vb.span);
    } else if (p) {
        (void)hipFree(p);
    }
    vb = gdp_ctx::VmmBuf{};
}

// Release the context-owned pyramid (one hipMalloc, or alloc_spread's chunks and range).
static void free_pyramid(gdp_ctx* c) {
    if (c->vmm_span) {
        for (const gdp_ctx::VmmChunk& k : c->vmm_chunks) {
            (void)hipMemUnmap(reinterpret_cast<char*>(c->d_out_own) + k.off, k.bytes);
            (void)hipMemRelease(k.h);
        }
        if (c->d_out_own) (void)hipMemAddressFree(c->d_out_own, c->vmm_span);
    } else if (c->d_out_own) {
        (void)hipFree(c->d_out_own);
    }
    c->vmm_chunks.clear();
    c->vmm_span = 0;
    c->d_out_own = nullptr;
    c->pyr_chunk_kb = 0;
}

// The pyramid's default backing (GDP_SPREAD_VMM=0 opts out): reserve its address range
// and back it with separately created 2 MiB physical pieces (larger past 4,096 pieces), created in
// a fixed pseudo-random order.  Research builds (GDP_EXPERIMENTS) also take GDP_SPREAD_CHUNK_MB/_KB
// (piece size; 0 = one piece per image), GDP_IMAGE_STRIDE_MB (images that far apart, the gaps left
// unmapped), GDP_SPREAD_PHYS_MB (a physical spacer after each piece, released once all are mapped)
// and GDP_SPREAD_PERM (creation order).  Nothing but placement changes: same offsets, same bits.
static hipError_t alloc_spread(gdp_ctx* c, std::string& where) {
    Geom& g = c->geom;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = c->device;
    size_t gran = 0;
    hipError_t e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended);
    if (e != hipSuccess) {
        where = "hipMemGetAllocationGranularity";
        return e;
    }
    gran = std::max<size_t>(gran, 256);
    auto up = [gran](size_t v) { return (v + gran - 1) / gran * gran; };
    const char* ck = exp_env("GDP_SPREAD_CHUNK_MB");
    const char* ckk = exp_env("GDP_SPREAD_CHUNK_KB");
    // Image starts: each image of the batch starts on an allocation granule (the layout every
    // round-4 measurement of this backing ran with) only where that wastes at most 1/16 of an
    // image — 1080x1920 (55 MB) and 4096^2 (447 MB) images; smaller images stay dense, so a batch
    // of small images costs at most one granule extra (64x64 images were rounded from
    // 27 KB to 2 MiB each).  GDP_IMAGE_ALIGN (GDP_EXPERIMENTS builds) forces 1 / 0 for A/B runs.
    // An experiment that spaces the images (GDP_IMAGE_STRIDE_MB) or asks for one piece per image
    // (GDP_SPREAD_CHUNK_MB=0) always aligns.
    const bool per_image = (ckk && std::atoll(ckk) <= 0) || (!ckk && ck && std::atoll(ck) <= 0);
    const size_t dense = (size_t)c->img_floats * 4;
    const char* al = exp_env("GDP_IMAGE_ALIGN");
    const bool align_images = per_image || (al ? std::atoi(al) != 0 : (up(dense) - dense) * 16 <= dense);
    const size_t img = align_images ? up(dense) : dense;
    // an experiment's wider stride (GDP_IMAGE_STRIDE_MB set pyr_stride) is rounded to the granule
    const size_t stride = (size_t)g.pyr_stride * 4 > dense ? up(std::max((size_t)g.pyr_stride * 4, img)) : img;
    g.pyr_stride = (long long)(stride / 4);
    const size_t span = up(stride * (size_t)g.batch);
    const char* ph = exp_env("GDP_SPREAD_PHYS_MB");
    const size_t spacer = ph ? up((size_t)std::max(0ll, std::atoll(ph)) << 20) : 0;
    // default piece: 2 MiB (at most 4096 pieces: larger pyramids take larger pieces).  Measured
    // against one hipMalloc (tools/tune.py A/B, profiles/chunk_*_r04z.log, vmm_*_r04y.log): 4096^2
    // 0.0789 vs 0.0860 ms, 64 x 1080x1920 0.606 vs 0.684, 16384^2 1.175 vs 1.218-1.261 on one box
    // and equal on another, 64 x 4096^2 within 1 %; 512 MiB+ pieces behave like one allocation.
    // GDP_SPREAD_CHUNK_MB = n MiB pieces, 0 = one piece per image.
    // (GDP_SPREAD_CHUNK_KB: the same in KiB — below 2 MiB only for measurement: 37-62 % of 8 TB/s)
    const size_t two = (size_t)2 << 20;
    const size_t fixed = ckk ? (std::atoll(ckk) > 0 ? up((size_t)std::atoll(ckk) << 10) : 0)
                       : ck  ? (std::atoll(ck) > 0 ? up((size_t)std::atoll(ck) << 20) : 0)
                             : up(std::max(two, (span / 4096 + two - 1) / two * two));
    // the pieces to map: [off, off + bytes)
    std::vector<std::pair<size_t, size_t>> pieces;
    if (fixed && stride == img) {  // dense images: fixed pieces tiling the (granule-rounded) span
        for (size_t off = 0; off < span; off += fixed) pieces.push_back({off, std::min(fixed, span - off)});
        c->pyr_chunk_kb = (int)(fixed >> 10);
    } else {
        for (int b = 0; b < g.batch; ++b) pieces.push_back({(size_t)b * stride, img});
        c->pyr_chunk_kb = -1;
    }
    const bool contiguous = stride == img;  // the pieces tile [0, span) with no unmapped gap
    for (size_t k = 0; k < pieces.size(); ++k)  // host-side invariant: disjoint, granule-sized, in the span
        if (pieces[k].second == 0 || pieces[k].first % gran || pieces[k].second % gran ||
            pieces[k].first + pieces[k].second > span || (k && pieces[k].first < pieces[k - 1].first + pieces[k - 1].second)) {
            where = "piece plan " + std::to_string(k) + " [" + std::to_string(pieces[k].first) + ", +" +
                    std::to_string(pieces[k].second) + ") of span " + std::to_string(span);
            return hipErrorInvalidValue;
        }
    void* base = nullptr;
    where = "granularity " + std::to_string(gran) + ", span " + std::to_string(span) + ", pieces " +
            std::to_string(pieces.size()) + ": ";
    // 2 MiB-aligned range: a 2 MiB piece then covers exactly one large page (pieces below 2 MiB
    // ran 2-2.5x slower, 256 KiB-1 MiB: profiles/kb_*_r04ad.log)
    if ((e = hipMemAddressReserve(&base, span, std::max(gran, two), nullptr, 0)) != hipSuccess) {
        where += "hipMemAddressReserve";
        return e;
    }
    c->d_out_own = static_cast<float*>(base);
    c->vmm_span = span;
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    std::vector<hipMemGenericAllocationHandle_t> spacers;
    // GDP_SPREAD_PERM: the order the physical pieces are created in — 3 (default) a fixed
    // pseudo-random order, 0 address order, 1 residue classes mod 8 (pieces 0, 8, 16, .., then 1,
    // 9, ..), 2 last piece first.  The random order makes the rate insensitive to the tile order:
    // 64 x 4096^2 v16 linear 4.78 vs 5.17 ms (best 4.733 vs 4.770), 64 x 1080x1920 v17 linear
    // 0.601 vs 0.689 (best equal), 4096^2 equal, 16384^2 -0.1..-0.7 % (rperm_*_r04a{h,i}.log)
    const char* pm = exp_env("GDP_SPREAD_PERM");
    const int perm = pm ? std::atoi(pm) : 3;
    const size_t np = pieces.size();
    std::vector<size_t> shuffled;
    if (perm == 3) {  // a fixed pseudo-random order (Fisher-Yates over a 64-bit LCG)
        shuffled.resize(np);
        for (size_t k = 0; k < np; ++k) shuffled[k] = k;
        unsigned long long x = 0x9E3779B97F4A7C15ull;
        for (size_t k = np; k > 1; --k) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            std::swap(shuffled[k - 1], shuffled[(size_t)((x >> 33) % k)]);
        }
    }
    auto piece_at = [&](size_t k) -> size_t {
        if (perm == 3) return shuffled[k];
        if (perm == 1) {
            auto count = [np](size_t r) { return r < np ? (np - r + 7) / 8 : 0; };  // pieces r, r + 8, ...
            size_t r = 0, kk = k;
            while (r < 7 && kk >= count(r)) kk -= count(r++);
            return r + 8 * kk;
        }
        return perm == 2 ? np - 1 - k : k;
    };
    for (size_t k = 0; k < np && e == hipSuccess; ++k) {
        const size_t i = piece_at(k);
        hipMemGenericAllocationHandle_t h;
        if ((e = hipMemCreate(&h, pieces[i].second, &prop, 0)) != hipSuccess) {
            where += "hipMemCreate(piece " + std::to_string(i) + ", " + std::to_string(pieces[i].second) + " B)";
            break;
        }
        char* at = static_cast<char*>(base) + pieces[i].first;
        if ((e = hipMemMap(at, pieces[i].second, 0, h, 0)) != hipSuccess) {
            where += "hipMemMap(piece " + std::to_string(i) + " at " + std::to_string(pieces[i].first) + ")";
            (void)hipMemRelease(h);
            break;
        }
        c->vmm_chunks.push_back({h, pieces[i].first, pieces[i].second});  // gdp_destroy unmaps it
        // access: per piece where gaps stay unmapped, else once over the whole range below (a piece
        // that is not a multiple of 2 MiB was refused on its own: hipMemSetAccess, r04x)
        if (!contiguous && (e = hipMemSetAccess(at, pieces[i].second, &acc, 1)) != hipSuccess) {
            where += "hipMemSetAccess(piece " + std::to_string(i) + ")";
            break;
        }
        if (spacer && k + 1 < np) {
            hipMemGenericAllocationHandle_t sp;
            if ((e = hipMemCreate(&sp, spacer, &prop, 0)) != hipSuccess) {
                where += "hipMemCreate(spacer)";
                break;
            }
            spacers.push_back(sp);
        }
    }
    for (hipMemGenericAllocationHandle_t sp : spacers) (void)hipMemRelease(sp);
    if (e == hipSuccess && contiguous && (e = hipMemSetAccess(base, span, &acc, 1)) != hipSuccess)
        where += "hipMemSetAccess(whole range)";
    return e;
}

int gdp_create_band(gdp_ctx** out, int H, int W, int S, int O, int batch, int row_begin, int row_end, int device) try {
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
    // Host planning first (geometry, tap tables: pure host work, no device needed), then the
    // device probe and the allocations.  Anything that throws past this point (std::bad_alloc of
    // the tap table, ...) frees the half-built context and is turned into a status by the
    // function-try-block below: no exception crosses the C ABI.
    gdp_ctx* c = new (std::nothrow) gdp_ctx();
    if (!c) return fail(GDP_ERR_NOMEM, "host allocation failed");
    auto drop = [&c]() {  // free the half-built context exactly once
        gdp_destroy(c);
        c = nullptr;
    };
    try {
    c->device = device;
    const char* vm = std::getenv("GDP_SPREAD_VMM");  // "0": the pyramid in one hipMalloc
    const bool want_vmm = !vm || std::atoi(vm) != 0;
    c->variant = default_variant(W, want_vmm);  // revised below if the chunked backing is refused
    // in-place re-entry pass (GenerateDoG on the current contents): 64-thread blocks stream best on
    // single images (4096^2 0.148 vs 0.152 ms for 256 threads, 16384^2 2.37 vs 2.49;
    // profiles/ab_sub_c*_r03m.log), 256-thread blocks on small batches, 1024-thread above
    c->inplace_sub = batch == 1 ? 16 : (long long)(row_end - row_begin) * W * batch <= (32ll << 20) ? 4 : 1;
    // Convolution extension default: block tiles (16 waves) in block order 5 (below; octave-o block
    // rows right after the octave-0 rows that hold their input rows, XCD-chunked) — the fastest form
    // on every config (tools/conv_ab.sh, cold buffers: 4096^2 0.111 ms vs 0.119 for the sweep,
    // 64 x 1080x1920 0.795 vs 0.809, 64 x 4096^2 6.34 vs 6.79, 16384^2 1.62 vs 1.72).  48 rows per
    // block since round 3: unpaced, 48 and 32 rows ran equal; with the stores paced at vmcnt(2)
    // (GDP_TUNE_CONV_PACE) 48 rows is 2-3 % ahead of 32 on every config (4096^2 0.1031 vs 0.1056 ms,
    // 64 x 4096^2 5.72 vs 5.92, 16384^2 1.461 vs 1.509; profiles/cpw_conv_c*_r03aw.log).
    c->conv_kernel = 2;
    c->conv_rows = 48;
    // Block order 5 (round 5): order 4's sequence XCD-chunked, so an octave-o block row runs on
    // the XCD whose L2 has just staged its input rows — DRAM-bound reads halve (4096^2 162.4 ->
    // 81.4 MB per launch, traffic 1.186 -> 1.036 x; 64 x 4096^2 1.185 -> 1.022 x) at the same
    // speed (4096^2 0.1055-0.1060 vs 0.1058 ms, 64 x 4096^2 5.656-5.663 vs 5.631-5.674, 64 x
    // 1080x1920 0.814-0.822 vs 0.808-0.811; profiles/conv_o{4,5}_c*_r05{v,w}.log).  A single image
    // of >= 2^27 pixels keeps order 4: 16384^2 1.594-1.607 vs 1.623-1.633 ms in order 5.
    c->conv_order = (batch == 1 && (long long)(row_end - row_begin) * W >= (1ll << 27)) ? 4 : 5;
    {
        const unsigned hw = std::thread::hardware_concurrency();
        if (hw > 0) c->stage_threads = std::max(1, std::min<int>(c->stage_threads, (int)hw));
    }
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
    g.store_pace = -1;
    g.inplace_pace = -1;
    // the convolution block tiles' five stores per output row go out back to back; vmcnt(2) after
    // each measured 0.5-1.3 % faster on 4096^2 / 64 x 4096^2 / 16384^2 (profiles/sp_conv_c*_r03ap.log)
    g.conv_pace = 2;
    c->in_pitch_own = g.in_pitch;
    c->in_img_stride_own = g.in_img_stride;

    // optional padding between levels (floats, multiple of 64) — layout experiment knob
    const char* pad_env = exp_env("GDP_LEVEL_PAD");
    const long long level_pad = pad_env ? round_up(std::max(0ll, std::atoll(pad_env)), kLevelAlign) : 0;
    // Row-window layout of a non-square image: [row][scale] (default) or, with GDP_ROWTAP_LAYOUT=0,
    // [scale][row].  A tile's rows then read their S+3 windows from ~L/32 lines per row instead of
    // one cold line per scale: 65536 x 4096 builds in 1.227 vs 1.43-1.46 ms (v15), 16384 x 4096 in
    // 0.315 vs 0.363 ms — the speed of row windows that are always hot (timing-only build, 1.25
    // ms); config 3 and the in-place passes unchanged (profiles/ab_rowtap_r03c.log, bit-exact)
    const char* rl_env = exp_env("GDP_ROWTAP_LAYOUT");
    const bool rowtap_interleave = rl_env ? std::atoi(rl_env) != 0 : true;
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
        // Row taps.  A square image's row and column windows are the same array (host_taps of
        // the same length), so its row taps alias the column taps: those stay hot in L2 (every
        // tile row re-reads them), while a separate row-tap array is touched once per tile row and
        // misses cold on every octave of every tile of a large image (measured: 16384^2 1.41 ->
        // 1.28 ms).  Bit-identical either way.
        if (H == W) {
            og.rtap_stride = og.ctap_stride;
            og.rtap_row = 1;
            og.rtap = og.ctap;
        } else if (!rowtap_interleave) {
            og.rtap_stride = (int)round_up(Hg, 4);
            og.rtap_row = 1;
            og.rtap = (int)tap_off;
            tap_off += (long long)og.rtap_stride * g.L;
        } else {
            // [row][scale]: the S+3 windows of a row are adjacent, so a tile's rows of one octave
            // touch ~L/32 lines per row instead of one line per scale
            og.rtap_stride = 1;
            og.rtap_row = g.L;
            og.rtap = (int)tap_off;
            tap_off += round_up((long long)Hg * g.L, 4);
        }
        og.grp_begin = grp;
        make_magic((unsigned)std::max(1, og.gpr), &og.gpr_magic, &og.gpr_shift);
        grp += (long long)og.rows * og.gpr;
        g.lv_blk[o + 1] = g.lv_blk[o] + (unsigned)(((long long)og.rows * og.gpr + kLevBlock - 1) / kLevBlock);
        g.lx_blk[o + 1] = g.lx_blk[o] + (unsigned)(((long long)og.rows * og.gpr + 63) / 64);
        g.lt_blk[o + 1] = g.lt_blk[o] + (unsigned)(((long long)og.rows + kLtRows - 1) / kLtRows * ((og.gpr + 63) / 64));
        g.cv_tiles_c[o] = (og.cols + kCvTW - 1) / kCvTW;
        g.cv_blk[o + 1] = g.cv_blk[o] + (unsigned)(((long long)og.rows + kCvTH - 1) / kCvTH * g.cv_tiles_c[o]);
    }
    g.pyr_stride = round_up(lev_off, kLevelAlign);
    c->img_floats = g.pyr_stride;
    // optional image stride (MiB) — layout experiment knob, like GDP_LEVEL_PAD: images that far
    // apart, so tile order 1's eight XCD ranges (batch / 8 images each) start 8 x stride apart
    if (const char* is_env = exp_env("GDP_IMAGE_STRIDE_MB"))
        g.pyr_stride = std::max(g.pyr_stride, round_up(std::max(0ll, std::atoll(is_env)) << 18, kLevelAlign));
    const long long tail_per_img = (g.F < O) ? grp - g.oct[g.F].grp_begin : 0;
    const long long tail_units = (tail_per_img * batch + kTailGroups - 1) / kTailGroups;
    const long long min_tiles = (long long)((g.in_rows + kTileRows - 1) / kTileRows) * ((W + 63) / 64) * batch;
    if (tap_off > (1ll << 31) || min_tiles + tail_units >= (1ll << 31) || tail_per_img * batch >= (1ll << 31) ||
        grp >= (1ll << 31)) {
        drop();
        return fail(GDP_ERR_ARG, "image/batch too large for one context (split the batch)");
    }
    g.tail_groups_per_img = (unsigned)tail_per_img;
    g.tail_units = (unsigned)tail_units;
    // Tile order default: linear.  (With v0 a single >= 64 Mpix image streamed 7-8 % faster in
    // the XCD-chunked order; with the default v15 the linear order is the faster one on 16384^2,
    // 1.344 vs 1.375 ms, and batches differ box to box — gdp_autotune measures both.)
    g.tile_order = 0;
    if (retile(c, kVariants[variant_index(c->variant)].tile_cols, kVariants[variant_index(c->variant)].tile_rows) != GDP_OK) {
        const std::string m = c->err;
        drop();
        return fail(GDP_ERR_ARG, m);
    }
    conv_sweep_geom(c);
    c->h_taps.assign((size_t)tap_off, 0.0f);
    fill_host_taps(c, c->centre_mode);
    set_window_support(c, c->zero_window != 0);

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        drop();
        return fail(GDP_ERR_NODEV, "no HIP device visible");
    }
    hipDeviceProp_t prop;
    if (device < 0 || device >= ndev) {
        drop();
        return fail(GDP_ERR_ARG, "device index out of range");
    }
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        drop();
        return fail(GDP_ERR_NODEV, "hipGetDeviceProperties failed");
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        drop();
        return fail(GDP_ERR_NODEV, std::string("libgdp is built for gfx950, device is ") + prop.gcnArchName);
    }
    c->cus = std::max(1, prop.multiProcessorCount);
    c->blocks_max = c->cus * 8;

    auto hip_fail = [&](hipError_t e, const char* what) {
        std::string m = std::string(what) + ": " + hipGetErrorString(e);
        drop();
        return fail(e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP, m);
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return hip_fail(e, "hipSetDevice");
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "hipStreamCreate");
    if ((e = hipMalloc(&c->d_geom, sizeof(Geom))) != hipSuccess) return hip_fail(e, "hipMalloc(geom)");
    if ((e = hipMalloc(&c->d_taps, std::max<size_t>(4, c->h_taps.size() * 4))) != hipSuccess)
        return hip_fail(e, "hipMalloc(taps)");
    c->d_taps_mode[c->centre_mode] = c->d_taps;
    if ((e = alloc_input(c, (size_t)g.in_img_stride * batch * 4, &c->d_in_own, c->in_vmm)) != hipSuccess)  // int32
        return hip_fail(e, "hipMalloc(input)");
    // The pyramid: separately created physical pieces mapped into one address range (alloc_spread;
    // default), or one hipMalloc (GDP_SPREAD_VMM=0, or when the VMM calls are refused).
    bool pyr_done = false;
    if (want_vmm) {
        std::string where;
        const long long stride0 = g.pyr_stride;
        if ((e = alloc_spread(c, where)) == hipSuccess) {
            pyr_done = true;
        } else if (vm) {
            return hip_fail(e, ("spread pyramid (GDP_SPREAD_VMM, " + where + ")").c_str());
        } else {
            free_pyramid(c);  // not asked for explicitly: one hipMalloc instead
            g.pyr_stride = stride0;  // alloc_spread may have rounded it
            (void)hipGetLastError();
        }
    }
    if (!pyr_done) {
        if ((e = hipMalloc(&c->d_out_own, std::max<size_t>(16, (size_t)g.pyr_stride * batch * 4))) != hipSuccess)
            return hip_fail(e, "hipMalloc(pyramid)");
        if (want_vmm) {  // the chunked backing was refused: the default for one allocation
            c->variant = default_variant(W, false);
            if (retile(c, kVariants[variant_index(c->variant)].tile_cols, kVariants[variant_index(c->variant)].tile_rows) != GDP_OK) {
                const std::string m = c->err;
                drop();
                return fail(GDP_ERR_ARG, m);
            }
        }
    }
    c->d_out = c->d_out_own;
    if ((e = hipMalloc(&c->d_sum, sizeof(unsigned long long))) != hipSuccess) return hip_fail(e, "hipMalloc(sum)");
    c->d_in = c->d_in_own;
    if ((e = hipMemcpy(c->d_taps, c->h_taps.data(), c->h_taps.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy(taps)");
    if ((e = hipMemset(c->d_in_own, 0, (size_t)g.in_img_stride * batch * 4)) != hipSuccess) return hip_fail(e, "hipMemset");
    if (upload_geom(c) != GDP_OK) {
        std::string m = c->err;
        drop();
        return fail(GDP_ERR_HIP, m);
    }
    *out = c;
    return GDP_OK;
    } catch (...) {
        drop();  // safe on a half-built context (null members are skipped)
        throw;
    }
} GDP_ABI_CATCH(nullptr)

int gdp_create(gdp_ctx** out, int H, int W, int S, int O, int batch, int device) try {
    return gdp_create_band(out, H, W, S, O, batch, 0, H, device);
} GDP_ABI_CATCH(nullptr)

void gdp_destroy(gdp_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    {
        // host mirrors deferred to this context keep their contents: fetched now
        std::lock_guard<std::mutex> lk(g_track_mu);
        (void)track_settle_all(c);
    }
    if (c->d_geom) (void)hipFree(c->d_geom);
    for (float* t : c->d_taps_mode)
        if (t) (void)hipFree(t);
    free_input(c->d_in_own, c->in_vmm);
    for (void* h : c->d_halo_own)
        if (h) (void)hipFree(h);
    free_pyramid(c);
    if (c->d_ctaps) (void)hipFree(c->d_ctaps);
    if (c->d_cradius) (void)hipFree(c->d_cradius);
    if (c->d_conv_perm) (void)hipFree(c->d_conv_perm);
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    for (hipEvent_t e : c->ev_stage)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->ev_mirror)
        if (e) (void)hipEventDestroy(e);
    if (c->st_up) (void)hipStreamDestroy(c->st_up);
    if (c->st_down) (void)hipStreamDestroy(c->st_down);
    if (c->d_sum) (void)hipFree(c->d_sum);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int gdp_get_geometry(const gdp_ctx* c, int* H, int* W, int* S, int* O, int* batch) try {
    if (!c) return GDP_ERR_ARG;
    if (H) *H = c->geom.H;
    if (W) *W = c->geom.W;
    if (S) *S = c->geom.S;
    if (O) *O = c->geom.O;
    if (batch) *batch = c->geom.batch;
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_level_dims(const gdp_ctx* c, int o, int* rows, int* cols, int* first_row) try {
    if (!c || o < 0 || o >= c->geom.O) return GDP_ERR_ARG;
    if (rows) *rows = c->geom.oct[o].rows;
    if (cols) *cols = c->geom.oct[o].cols;
    if (first_row) *first_row = c->geom.oct[o].row0;
    return GDP_OK;
} GDP_ABI_CATCH(c)

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

int gdp_set_input_host(gdp_ctx* c, int b, const int32_t* base, size_t pitch, void* stream) try {
    if (c) GDP_SETTLE(c, "gdp_set_input_host", [&](auto&& f) { f(base, pitch * 4 * (size_t)c->geom.in_rows); });
    return upload_input(c, b, base, pitch, GDP_INPUT_I32, stream, "gdp_set_input_host");
} GDP_ABI_CATCH(c)

int gdp_set_input_host_u8(gdp_ctx* c, int b, const uint8_t* base, size_t pitch, void* stream) try {
    if (c) GDP_SETTLE(c, "gdp_set_input_host_u8", [&](auto&& f) { f(base, pitch * (size_t)c->geom.in_rows); });
    return upload_input(c, b, base, pitch, GDP_INPUT_U8, stream, "gdp_set_input_host_u8");
} GDP_ABI_CATCH(c)

static int ensure_stage(gdp_ctx* c, size_t floats);
static void parallel_rows(size_t nrows, size_t floats, int threads, const std::function<void(size_t, size_t)>& fn);

int gdp_set_input_rows(gdp_ctx* c, int b, const int32_t* const* rows, void* stream) try {
    if (!c || !rows || b < 0 || b >= c->geom.batch) return c ? c->status(GDP_ERR_ARG, "gdp_set_input_rows: bad argument") : GDP_ERR_ARG;
    if (c->d_in != c->d_in_own) return c->status(GDP_ERR_STATE, "input is bound to caller device memory");
    if (c->geom.in_fmt != GDP_INPUT_I32)
        return c->status(GDP_ERR_STATE, "gdp_set_input_rows: context input format differs (gdp_set_input_format)");
    const size_t W = (size_t)c->geom.W, R = (size_t)c->geom.in_rows, pitch = (size_t)c->geom.in_pitch;
    for (size_t r = 0; r < R; ++r)
        if (!rows[r]) return c->status(GDP_ERR_ARG, "gdp_set_input_rows: null row %zu", r);
    if (W * R == 0) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_set_input_rows", [&](auto&& f) { for (size_t r = 0; r < R; ++r) f(rows[r], W * 4); });
    hipStream_t st = c->pick(stream);
    // The rows are gathered into the double-buffered pinned staging (the mirror of
    // stage_download): the host gathers batch k into one half while batch k-1's 2-D copy runs.
    const size_t per = std::max<size_t>(1, std::min(R, c->stage_half_floats / W)), half = per * W;
    const size_t nb = (R + per - 1) / per;
    const int rc = ensure_stage(c, nb > 1 ? 2 * half : half);
    if (rc != GDP_OK) return rc;
    int32_t* dst = static_cast<int32_t*>(c->d_in_own) + (size_t)b * c->geom.in_img_stride;
    for (size_t k = 0; k < nb; ++k) {
        int32_t* h = reinterpret_cast<int32_t*>(c->h_stage) + (k & 1) * half;
        if (k >= 2) GDP_HIP(c, hipEventSynchronize(c->ev_stage[k & 1]));  // batch k-2 has left this half
        const size_t r0 = k * per, nr = std::min(per, R - r0);
        parallel_rows(nr, nr * W, c->stage_threads, [&](size_t a, size_t e) {
            for (size_t r = a; r < e; ++r) std::memcpy(h + r * W, rows[r0 + r], W * 4);
        });
        GDP_HIP(c, hipMemcpy2DAsync(dst + r0 * pitch, pitch * 4, h, W * 4, W * 4, nr, hipMemcpyHostToDevice, st));
        GDP_HIP(c, hipEventRecord(c->ev_stage[k & 1], st));
    }
    GDP_HIP(c, hipStreamSynchronize(st));
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_set_input_device(gdp_ctx* c, const int32_t* base, size_t pitch, size_t image_stride) try {
    return bind_input(c, base, pitch, image_stride, GDP_INPUT_I32, "gdp_set_input_device");
} GDP_ABI_CATCH(c)

int gdp_set_input_device_u8(gdp_ctx* c, const uint8_t* base, size_t pitch, size_t image_stride) try {
    return bind_input(c, base, pitch, image_stride, GDP_INPUT_U8, "gdp_set_input_device_u8");
} GDP_ABI_CATCH(c)

int gdp_set_input_format(gdp_ctx* c, int fmt) try {
    if (!c || (fmt != GDP_INPUT_I32 && fmt != GDP_INPUT_U8)) return c ? c->status(GDP_ERR_ARG, "unknown input format") : GDP_ERR_ARG;
    if (fmt == c->geom.in_fmt) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_HIP(c, hipDeviceSynchronize());
    const size_t bytes = (size_t)c->in_img_stride_own * c->geom.batch * (fmt == GDP_INPUT_U8 ? 1 : 4);
    void* fresh = nullptr;
    gdp_ctx::VmmBuf vb;
    hipError_t e = alloc_input(c, bytes, &fresh, vb);
    if (e == hipSuccess) e = hipMemset(fresh, 0, std::max<size_t>(16, bytes));
    if (e != hipSuccess) {  // the context keeps its current input buffer
        free_input(fresh, vb);
        return c->status(e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP, "allocating the input: %s",
                         hipGetErrorString(e));
    }
    free_input(c->d_in_own, c->in_vmm);
    c->d_in_own = fresh;
    c->in_vmm = std::move(vb);
    c->geom.in_fmt = fmt;
    for (int side = 0; side < 2; ++side) { // halo rows follow the input format: re-created on next use
        if (c->d_halo_own[side]) GDP_HIP(c, hipFree(c->d_halo_own[side]));
        c->geom.halo_ptr[side] = nullptr;
        c->d_halo_own[side] = nullptr;
    }
    return bind_input(c, nullptr, 0, 0, fmt, "gdp_set_input_format");
} GDP_ABI_CATCH(c)

int gdp_get_input_format(const gdp_ctx* c) { return c ? c->geom.in_fmt : -1; }

int gdp_fill_synthetic(gdp_ctx* c, uint32_t seed, long first_image, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    const long long total = (long long)c->geom.in_rows * c->geom.W * c->geom.batch;
    const int grid = (int)std::min<long long>((total + kBlock - 1) / kBlock, c->blocks_max);
    // the images land in whatever input the builds read: the context's own buffer, or the caller's
    // device buffer bound by gdp_set_input_device* (its pitch / image stride)
    hipLaunchKernelGGL(k_synth, dim3(grid), dim3(kBlock), 0, c->pick(stream), c->d_geom, const_cast<void*>(c->d_in),
                       seed, (long long)first_image);
    GDP_HIP(c, hipGetLastError());
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_build(gdp_ctx* c, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_build(c, c->pick(stream));
} GDP_ABI_CATCH(c)

int gdp_conv_taps(int S, int scale, float* taps, int* radius) try {
    if (S < 0 || scale < 0 || scale >= S + 3 || !taps || !radius) return GDP_ERR_ARG;
    const int R = conv_radius_of(scale); // ceil(3 sigma), sigma = 2 / (scale + 1), at most kCvR
    const ConvTaps k = conv_taps_of(scale);
    for (int j = 0; j < kCvMaxTaps; ++j) taps[j] = j <= 2 * R ? k.k[j < R ? R - j : j - R] : 0.0f;
    *radius = R;
    return GDP_OK;
} GDP_ABI_CATCH(nullptr)

// ---- convolution extension on row bands: halo rows --------------------------------------------
// A band's convolution reads 6 octave-o rows beyond its octave-o rows; with band edges multiples of
// 2^(O-1) that is at most 6 * 2^(O-1) input rows above and below (clipped to the image).
static void conv_halo_counts(const Geom& g, int* above, int* below) {
    const int hh = kCvR << (g.O - 1);
    *above = std::min(hh, g.in_row0);
    *below = std::min(hh, g.H - (g.in_row0 + g.in_rows));
}

int gdp_conv_halo_rows(const gdp_ctx* c, int* above, int* below) try {
    if (!c || !above || !below) return GDP_ERR_ARG;
    conv_halo_counts(c->geom, above, below);
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_input_halo(gdp_ctx* c, int side, void** rows, size_t* pitch) try {
    if (!c || side < 0 || side > 1 || !rows || !pitch) return c ? c->status(GDP_ERR_ARG, "gdp_input_halo: bad argument") : GDP_ERR_ARG;
    Geom& g = c->geom;
    int n[2];
    conv_halo_counts(g, &n[0], &n[1]);
    *pitch = (size_t)c->in_pitch_own;
    if (n[side] == 0) {  // nothing beyond the image edge
        *rows = nullptr;
        return GDP_OK;
    }
    GDP_HIP(c, hipSetDevice(c->device));
    if (!c->d_halo_own[side]) {
        const size_t bytes = (size_t)n[side] * (size_t)c->in_pitch_own * g.batch * in_elem_size(c);
        hipError_t e = hipMalloc(&c->d_halo_own[side], bytes);
        if (e != hipSuccess) {
            c->d_halo_own[side] = nullptr;
            return c->status(e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP, "hipMalloc(halo rows)");
        }
        GDP_HIP(c, hipMemset(c->d_halo_own[side], 0, bytes));
    }
    *rows = c->d_halo_own[side];
    if (g.halo_ptr[side] == c->d_halo_own[side] && g.halo_rows[side] == n[side] &&
        g.halo_pitch[side] == c->in_pitch_own && g.halo_img_stride[side] == (long long)n[side] * c->in_pitch_own)
        return GDP_OK;  // already bound (every exchange asks again): no geometry upload, no drain
    g.halo_ptr[side] = c->d_halo_own[side];
    g.halo_rows[side] = n[side];
    g.halo_pitch[side] = c->in_pitch_own;
    g.halo_img_stride[side] = (long long)n[side] * c->in_pitch_own;
    return upload_geom(c);
} GDP_ABI_CATCH(c)

int gdp_bind_input_halo(gdp_ctx* c, const void* above, const void* below, size_t pitch, size_t image_stride) try {
    if (!c) return GDP_ERR_ARG;
    Geom& g = c->geom;
    int n[2];
    conv_halo_counts(g, &n[0], &n[1]);
    const void* p[2] = {above, below};
    for (int side = 0; side < 2; ++side) {
        if (!p[side] || n[side] == 0) continue;
        if (pitch < (size_t)g.W || pitch % 4 || (g.batch > 1 && image_stride < pitch * (size_t)n[side]) ||
            image_stride % 4 || (reinterpret_cast<uintptr_t>(p[side]) & (g.in_fmt == GDP_INPUT_U8 ? 3 : 15)))
            return c->status(GDP_ERR_ARG, "gdp_bind_input_halo: pitch / image stride must be multiples of 4 "
                                          "(>= width, >= rows x pitch) and the rows 16-B (uint8: 4-B) aligned");
    }
    for (int side = 0; side < 2; ++side) {
        g.halo_ptr[side] = n[side] ? p[side] : nullptr;
        g.halo_rows[side] = n[side];
        g.halo_pitch[side] = (long long)pitch;
        g.halo_img_stride[side] = (long long)(g.batch > 1 ? image_stride : pitch * (size_t)n[side]);
    }
    return upload_geom(c);
} GDP_ABI_CATCH(c)

int gdp_device_input(const gdp_ctx* c, int b, const void** rows, size_t* pitch) try {
    if (!c || b < 0 || b >= c->geom.batch || !rows || !pitch) return GDP_ERR_ARG;
    *rows = static_cast<const char*>(c->d_in) + (size_t)b * (size_t)c->geom.in_img_stride * in_elem_size(c);
    *pitch = (size_t)c->geom.in_pitch;
    return GDP_OK;
} GDP_ABI_CATCH(c)

// Every input row a band convolution launch can read lies in the band or its held halo rows.
static int conv_band_check(gdp_ctx* c) {
    const Geom& g = c->geom;
    int n[2];
    conv_halo_counts(g, &n[0], &n[1]);
    for (int side = 0; side < 2; ++side)
        if (n[side] > 0 && (!g.halo_ptr[side] || g.halo_rows[side] != n[side]))
            return c->status(GDP_ERR_STATE, "gdp_build_gaussian: this row band needs its %d halo rows %s "
                                            "(gdp_input_halo / gdp_bind_input_halo / gdp_comm_exchange_halo)",
                             n[side], side ? "below" : "above");
    const long long lo = (long long)g.in_row0 - n[0], hi = (long long)g.in_row0 + g.in_rows + n[1]; // held rows
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        if (og.rows == 0) continue;
        if (og.cols < 4 || og.cols % 4)
            return c->status(GDP_ERR_ARG, "gdp_build_gaussian on a row band needs every octave width a multiple "
                                          "of 4 (width a multiple of 2^(octaves+1))");
        const long long Hg = g.H >> o;
        const long long first = std::max(0ll, (long long)og.row0 - kCvR) << o;
        const long long last = std::min(Hg - 1, (long long)og.row0 + og.rows - 1 + kCvR) << o;
        if (first < lo || last >= hi)
            return c->status(GDP_ERR_STATE, "gdp_build_gaussian: octave %d reads input rows [%lld, %lld] beyond the "
                                            "held rows [%lld, %lld)", o, first, last, lo, hi);
    }
    return GDP_OK;
}

int gdp_build_gaussian(gdp_ctx* c, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    const Geom& g = c->geom;
    const bool band = g.in_row0 != 0 || g.in_rows != g.H;
    if (band) {  // row band: only the block tiles read halo rows (every octave through them)
        if (c->conv_kernel != 2 || g.L < 3 || g.L > 8)
            return c->status(GDP_ERR_STATE, "gdp_build_gaussian on a row band runs the block tiles only "
                                            "(GDP_TUNE_CONV_KERNEL 2, S <= 5)");
        const int rc = conv_band_check(c);
        if (rc != GDP_OK) return rc;
    }
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
    // the block tiles (kernel 2) are compiled for S = 0..5 (L = 3..8), the register sweep (kernel
    // 0) for S = 0..3; both take the octaves whose width is a multiple of 4, the LDS tiles the rest
    // (and everything for other S or conv_kernel = 1)
    const bool sweep = c->conv_kernel != 1 && g.L >= 3 && g.L <= (c->conv_kernel == 2 ? 8 : 6);
    // the block tiles address a wave's rows as byte offsets from its first row (k_conv_blk)
    if (sweep && c->conv_kernel == 2 && 65ll * 4 * g.W >= kOOB)
        return c->status(GDP_ERR_ARG, "gdp_build_gaussian: width %d too large for the block tiles", g.W);
    {  // rows per tile / strip (and waves per block) the selected kernel is instantiated for
        const int r = c->conv_rows, k = c->conv_kernel, w = c->conv_waves;
        if (sweep && k == 0 && r != 16 && r != 32)
            return c->status(GDP_ERR_STATE, "conv rows %d not available for the register sweep (16 or 32)", r);
        if (sweep && k == 2 && !conv_blk_pair_ok(r, w))
            return c->status(GDP_ERR_STATE, "conv block tiles: %d rows with %d waves is not an instantiated pair "
                                            "(16 waves: 16 / 32 / 48 rows; 8 waves: 8 / 16 / 24 / 32 rows)", r, w);
    }
    const unsigned* blk = c->conv_kernel == 2 ? g.bk_blk : g.sw_blk;
    if (sweep && (c->conv_order & 4) && (c->conv_perm_dirty || c->conv_perm_kernel != c->conv_kernel)) {
        const int rc = conv_sweep_perm(c, blk, c->conv_kernel == 2 ? g.bk_strips_c : g.sw_strips_c);
        if (rc != GDP_OK) return rc;
        c->conv_perm_kernel = c->conv_kernel;
    }
    if (sweep) {
        const long long grid = (long long)blk[g.O] * g.batch;
        if (grid >= (1ll << 31) - 8) return c->status(GDP_ERR_ARG, "convolution build too large for one launch");
        if (grid > 0) {
            switch (g.L) {
                case 3: GDP_HIP(c, launch_conv_sweep_l<3>(c, (unsigned)grid, st)); break;
                case 4: GDP_HIP(c, launch_conv_sweep_l<4>(c, (unsigned)grid, st)); break;
                case 5: GDP_HIP(c, launch_conv_sweep_l<5>(c, (unsigned)grid, st)); break;
                case 6: GDP_HIP(c, launch_conv_sweep_l<6>(c, (unsigned)grid, st)); break;
                case 7: GDP_HIP(c, launch_conv_blk<7>(c, (unsigned)grid, st)); break;
                default: GDP_HIP(c, launch_conv_blk<8>(c, (unsigned)grid, st)); break;
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
} GDP_ABI_CATCH(c)

int gdp_init(gdp_ctx* c, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<4>(c, 0, c->geom.O, c->pick(stream));
} GDP_ABI_CATCH(c)

int gdp_gauss_octave(gdp_ctx* c, int o, void* stream) try {
    if (!c || o < 0 || o >= c->geom.O) return c ? c->status(GDP_ERR_ARG, "octave out of range") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<1>(c, o, o + 1, c->pick(stream));
} GDP_ABI_CATCH(c)

int gdp_gauss_range(gdp_ctx* c, int ob, int oe, void* stream) try {
    if (!c || ob < 0 || oe > c->geom.O || ob >= oe) return c ? c->status(GDP_ERR_ARG, "octave range invalid") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<1>(c, ob, oe, c->pick(stream));
} GDP_ABI_CATCH(c)

int gdp_gauss_scales(gdp_ctx* c, int sb, int se, int ob, int oe, void* stream) try {
    if (!c || ob < 0 || oe > c->geom.O || ob >= oe || sb < 0 || se > c->geom.L || sb >= se)
        return c ? c->status(GDP_ERR_ARG, "gdp_gauss_scales: scale / octave range invalid") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<1>(c, ob, oe, c->pick(stream), sb, se);
} GDP_ABI_CATCH(c)

int gdp_dog_octave(gdp_ctx* c, int o, void* stream) try {
    if (!c || o < 0 || o >= c->geom.O) return c ? c->status(GDP_ERR_ARG, "octave out of range") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<2>(c, o, o + 1, c->pick(stream));
} GDP_ABI_CATCH(c)

int gdp_dog_range(gdp_ctx* c, int ob, int oe, void* stream) try {
    if (!c || ob < 0 || oe > c->geom.O || ob >= oe) return c ? c->status(GDP_ERR_ARG, "octave range invalid") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<2>(c, ob, oe, c->pick(stream));
} GDP_ABI_CATCH(c)

int gdp_generate_dog(gdp_ctx* c, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace<3>(c, 0, c->geom.O, c->pick(stream));
} GDP_ABI_CATCH(c)

int gdp_build_subset(gdp_ctx* c, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_build(c, c->pick(stream), true);
} GDP_ABI_CATCH(c)

int gdp_generate_dog_subset(gdp_ctx* c, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    return launch_inplace_sub<9, 1>(c, 0, c->geom.O, c->pick(stream));
} GDP_ABI_CATCH(c)

const float* gdp_device_level(const gdp_ctx* c, int b, int o, int s) {
    if (!valid_level(c, b, o, s)) return nullptr;
    const OctGeom& og = c->geom.oct[o];
    return c->d_out + (size_t)b * c->geom.pyr_stride + og.lev_off + (size_t)s * og.lev_stride;
}

int gdp_download_level(gdp_ctx* c, int b, int o, int s, float* host) try {
    if (!valid_level(c, b, o, s) || !host) return c ? c->status(GDP_ERR_ARG, "gdp_download_level: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_download_level", [&](auto&& f) { f(host, (size_t)c->geom.oct[o].rows * c->geom.oct[o].cols * 4); });
    const OctGeom& og = c->geom.oct[o];
    GDP_HIP(c, hipMemcpyAsync(track_dma_ptr(host), gdp_device_level(c, b, o, s), (size_t)og.rows * og.cols * 4, hipMemcpyDeviceToHost,
                              c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
} GDP_ABI_CATCH(c)

// Row-pointer downloads (the drop-in class's float**** mirror): device levels -> pinned staging ->
// the caller's rows.  The pinned buffer is split in two halves: batch k's D2H copies go into half
// k % 2 while the host scatters batch k-1 out of the other half, so the PCIe copy and the host
// memcpy overlap; a large batch is scattered by `stage_threads` host threads.
struct StagePiece {
    const float* src;      // device rows [0, nrows) of a level slice, `cols` floats each
    size_t cols, nrows;
    float* const* rows;    // the caller's destination row pointers for those rows
    size_t off;            // float offset in the staging half
};

// Runs fn(r0, r1) over [0, nrows) on `threads` host threads (one thread below 1 M floats: the
// spawn cost, ~20-50 us a thread, only pays off for batches of several MiB).
static void parallel_rows(size_t nrows, size_t floats, int threads, const std::function<void(size_t, size_t)>& fn) {
    const size_t nt = floats >= (size_t(1) << 20) ? std::min<size_t>(std::max(1, threads), nrows) : 1;
    if (nt <= 1) return fn(0, nrows);
    std::vector<std::thread> pool;
    size_t t = 1;
    try {  // no exception may cross the C ABI: parts whose thread could not start run here
        pool.reserve(nt - 1);
        for (; t < nt; ++t) pool.emplace_back(fn, nrows * t / nt, nrows * (t + 1) / nt);
    } catch (...) {
    }
    for (; t < nt; ++t) fn(nrows * t / nt, nrows * (t + 1) / nt);
    fn(0, nrows / nt);
    for (std::thread& th : pool) th.join();
}

static void scatter_batch(const float* half, const std::vector<StagePiece>& batch, size_t floats, int threads) {
    size_t rows = 0;
    for (const StagePiece& q : batch) rows = std::max(rows, q.nrows);
    // thread t takes the same fraction of every piece's rows
    parallel_rows(rows, floats, threads, [&](size_t a, size_t e) {
        for (const StagePiece& q : batch) {
            const size_t r0 = q.nrows * a / rows, r1 = q.nrows * e / rows;
            for (size_t r = r0; r < r1; ++r) std::memcpy(q.rows[r], half + q.off + r * q.cols, q.cols * 4);
        }
    });
}

// The pinned staging buffer (floats) and its two half-events, grown on demand.
static int ensure_stage(gdp_ctx* c, size_t need) {
    if (c->h_stage_floats < need) {
        if (c->h_stage) GDP_HIP(c, hipHostFree(c->h_stage));
        c->h_stage = nullptr;
        c->h_stage_floats = 0;
        GDP_HIP(c, hipHostMalloc((void**)&c->h_stage, need * 4, hipHostMallocDefault));
        c->h_stage_floats = need;
    }
    for (hipEvent_t& e : c->ev_stage)
        if (!e) GDP_HIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return GDP_OK;
}

static int stage_download(gdp_ctx* c, const std::vector<StagePiece>& pieces) {
    size_t total = 0, max_cols = 1;
    for (const StagePiece& q : pieces) {
        total += q.cols * q.nrows;
        max_cols = std::max(max_cols, q.cols);
    }
    if (total == 0) return GDP_OK;
    // one half holds at least one row; a download that fits one half uses a single buffer
    size_t half = std::max(c->stage_half_floats, max_cols);
    const bool dbl = total > half;
    if (!dbl) half = total;
    const int rc = ensure_stage(c, dbl ? 2 * half : half);
    if (rc != GDP_OK) return rc;
    // cut the pieces into batches of at most `half` floats (whole rows)
    std::vector<std::vector<StagePiece>> batches(1);
    std::vector<size_t> used(1, 0);
    for (const StagePiece& q : pieces) {
        for (size_t r = 0; r < q.nrows;) {
            size_t fit = (half - used.back()) / q.cols;
            if (fit == 0) {
                batches.emplace_back();
                used.push_back(0);
                fit = half / q.cols;
            }
            const size_t nr = std::min(fit, q.nrows - r);
            batches.back().push_back({q.src + r * q.cols, q.cols, nr, q.rows + r, used.back()});
            used.back() += nr * q.cols;
            r += nr;
        }
    }
    const size_t nb = batches.size();
    for (size_t k = 0; k <= nb; ++k) {
        if (k < nb) {  // half k % 2 was scattered (batch k-2) before this iteration started
            // pieces adjacent both on the device and in the half (the levels of one image are packed
            // [o][s][r][c]) go as one copy: a small pyramid is one DMA, not one per level
            float* dst = c->h_stage + (k & 1) * half;
            const std::vector<StagePiece>& bk = batches[k];
            for (size_t i = 0; i < bk.size();) {
                size_t n = bk[i].cols * bk[i].nrows, j = i + 1;
                for (; j < bk.size() && bk[j].src == bk[i].src + n && bk[j].off == bk[i].off + n; ++j)
                    n += bk[j].cols * bk[j].nrows;
                GDP_HIP(c, hipMemcpyAsync(dst + bk[i].off, bk[i].src, n * 4, hipMemcpyDeviceToHost, c->stream));
                i = j;
            }
            GDP_HIP(c, hipEventRecord(c->ev_stage[k & 1], c->stream));
        }
        if (k > 0) {  // batch k-1 lands while batch k is in flight
            const size_t j = k - 1;
            GDP_HIP(c, hipEventSynchronize(c->ev_stage[j & 1]));
            scatter_batch(c->h_stage + (j & 1) * half, batches[j], used[j], c->stage_threads);
        }
    }
    return GDP_OK;
}

int gdp_download_level_rows(gdp_ctx* c, int b, int o, int s, float* const* rows) try {
    if (!valid_level(c, b, o, s) || !rows) return c ? c->status(GDP_ERR_ARG, "gdp_download_level_rows: bad argument") : GDP_ERR_ARG;
    const OctGeom& og = c->geom.oct[o];
    if ((size_t)og.rows * og.cols == 0) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_download_level_rows", [&](auto&& f) { for (int r = 0; r < og.rows; ++r) f(rows[r], (size_t)og.cols * 4); });
    return stage_download(c, {{gdp_device_level(c, b, o, s), (size_t)og.cols, (size_t)og.rows, rows, 0}});
} GDP_ABI_CATCH(c)

int gdp_download_pyramid_rows(gdp_ctx* c, int b, float* const* const* const* py) try {
    if (!c || !py || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_download_pyramid_rows: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_download_pyramid_rows", [&](auto&& f) {
        for (int o = 0; o < c->geom.O; ++o)
            for (int s = 0; s < c->geom.L && py[o]; ++s)
                for (int r = 0; r < c->geom.oct[o].rows && py[o][s]; ++r) f(py[o][s][r], (size_t)c->geom.oct[o].cols * 4);
    });
    const Geom& g = c->geom;
    std::vector<StagePiece> pieces;
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        if ((size_t)og.rows * og.cols == 0) continue;
        for (int s = 0; s < g.L; ++s)
            pieces.push_back({gdp_device_level(c, b, o, s), (size_t)og.cols, (size_t)og.rows, py[o][s], 0});
    }
    return stage_download(c, pieces);
} GDP_ABI_CATCH(c)

int gdp_download_level_range(gdp_ctx* c, int b, int o, int s, int first_row, int nrows, float* host) try {
    if (!valid_level(c, b, o, s) || !host || first_row < 0 || nrows < 0 || first_row > c->geom.oct[o].rows ||
        nrows > c->geom.oct[o].rows - first_row)
        return c ? c->status(GDP_ERR_ARG, "gdp_download_level_range: bad argument") : GDP_ERR_ARG;
    if (nrows == 0) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_download_level_range", [&](auto&& f) { f(host, (size_t)nrows * c->geom.oct[o].cols * 4); });
    const OctGeom& og = c->geom.oct[o];
    GDP_HIP(c, hipMemcpyAsync(track_dma_ptr(host), gdp_device_level(c, b, o, s) + (size_t)first_row * og.cols,
                              (size_t)nrows * og.cols * 4, hipMemcpyDeviceToHost, c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_download_pyramid(gdp_ctx* c, int b, float* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch) return c ? c->status(GDP_ERR_ARG, "gdp_download_pyramid: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_download_pyramid", [&](auto&& f) { f(host, packed_pyramid_bytes(c)); });
    size_t off = 0;
    for (int o = 0; o < c->geom.O; ++o) {
        const OctGeom& og = c->geom.oct[o];
        const size_t n = (size_t)og.rows * og.cols;
        for (int s = 0; s < c->geom.L; ++s, off += n)
            if (n) GDP_HIP(c, hipMemcpyAsync(track_dma_ptr(host + off), gdp_device_level(c, b, o, s), n * 4, hipMemcpyDeviceToHost, c->stream));
    }
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_upload_pyramid(gdp_ctx* c, int b, const float* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch) return c ? c->status(GDP_ERR_ARG, "gdp_upload_pyramid: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_upload_pyramid", [&](auto&& f) { f(host, packed_pyramid_bytes(c)); });
    size_t off = 0;
    for (int o = 0; o < c->geom.O; ++o) {
        const OctGeom& og = c->geom.oct[o];
        const size_t n = (size_t)og.rows * og.cols;
        for (int s = 0; s < c->geom.L; ++s, off += n)
            if (n)
                GDP_HIP(c, hipMemcpyAsync(const_cast<float*>(gdp_device_level(c, b, o, s)), track_dma_ptr(host + off), n * 4,
                                          hipMemcpyHostToDevice, c->stream));
    }
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
} GDP_ABI_CATCH(c)

// ---- host -> device state (the drop-in classes' two-way GaussPy, GuassDePyramid.h:16) ----------
// The reference's float**** IS the pyramid: GaussFilter / GenerateDoG work on whatever the caller
// left in it (:122-131, :140-146).  These copy a host-side pyramid back into the device levels.
// Staged row uploads are the mirror of stage_download: the host threads gather batch k into one
// pinned half while batch k-1's H2D copy runs out of the other.
struct UpPiece {
    float* dst;                 // device rows [0, nrows) of a level slice, `cols` floats each
    size_t cols, nrows;
    const float* const* rows;   // the caller's source row pointers for those rows
};

static int stage_upload(gdp_ctx* c, const std::vector<UpPiece>& pieces) {
    size_t total = 0, max_cols = 1;
    for (const UpPiece& q : pieces) {
        total += q.cols * q.nrows;
        max_cols = std::max(max_cols, q.cols);
        for (size_t r = 0; r < q.nrows; ++r)
            if (!q.rows[r]) return c->status(GDP_ERR_ARG, "pyramid row upload: null row pointer");
    }
    if (total == 0) return GDP_OK;
    size_t half = std::max(c->stage_half_floats, max_cols);
    const bool dbl = total > half;
    if (!dbl) half = total;
    const int rc = ensure_stage(c, dbl ? 2 * half : half);
    if (rc != GDP_OK) return rc;
    struct Cut { const UpPiece* q; size_t r0, nr, off; };
    std::vector<std::vector<Cut>> batches(1);
    std::vector<size_t> used(1, 0);
    for (const UpPiece& q : pieces)
        for (size_t r = 0; r < q.nrows;) {
            size_t fit = (half - used.back()) / q.cols;
            if (fit == 0) {
                batches.emplace_back();
                used.push_back(0);
                fit = half / q.cols;
            }
            const size_t nr = std::min(fit, q.nrows - r);
            batches.back().push_back({&q, r, nr, used.back()});
            used.back() += nr * q.cols;
            r += nr;
        }
    for (size_t k = 0; k < batches.size(); ++k) {
        float* h = c->h_stage + (k & 1) * half;
        if (k >= 2) GDP_HIP(c, hipEventSynchronize(c->ev_stage[k & 1]));  // batch k-2 has left this half
        const std::vector<Cut>& bk = batches[k];
        size_t rows = 0;
        for (const Cut& t : bk) rows = std::max(rows, t.nr);
        parallel_rows(rows, used[k], c->stage_threads, [&](size_t a, size_t e) {
            for (const Cut& t : bk) {
                const size_t r0 = t.nr * a / rows, r1 = t.nr * e / rows;
                for (size_t r = r0; r < r1; ++r)
                    std::memcpy(h + t.off + r * t.q->cols, t.q->rows[t.r0 + r], t.q->cols * 4);
            }
        });
        for (size_t i = 0; i < bk.size();) {  // device-adjacent slices go as one copy
            size_t n = bk[i].nr * bk[i].q->cols, j = i + 1;
            float* dst = bk[i].q->dst + bk[i].r0 * bk[i].q->cols;
            for (; j < bk.size() && bk[j].q->dst + bk[j].r0 * bk[j].q->cols == dst + n && bk[j].off == bk[i].off + n; ++j)
                n += bk[j].nr * bk[j].q->cols;
            GDP_HIP(c, hipMemcpyAsync(dst, h + bk[i].off, n * 4, hipMemcpyHostToDevice, c->stream));
            i = j;
        }
        GDP_HIP(c, hipEventRecord(c->ev_stage[k & 1], c->stream));
    }
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
}

int gdp_upload_level(gdp_ctx* c, int b, int o, int s, const float* host) try {
    if (!valid_level(c, b, o, s) || !host) return c ? c->status(GDP_ERR_ARG, "gdp_upload_level: bad argument") : GDP_ERR_ARG;
    const OctGeom& og = c->geom.oct[o];
    if ((size_t)og.rows * og.cols == 0) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_upload_level", [&](auto&& f) { f(host, (size_t)og.rows * og.cols * 4); });
    GDP_HIP(c, hipMemcpyAsync(const_cast<float*>(gdp_device_level(c, b, o, s)), track_dma_ptr(host), (size_t)og.rows * og.cols * 4,
                              hipMemcpyHostToDevice, c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_upload_level_rows(gdp_ctx* c, int b, int o, int s, const float* const* rows) try {
    if (!valid_level(c, b, o, s) || !rows) return c ? c->status(GDP_ERR_ARG, "gdp_upload_level_rows: bad argument") : GDP_ERR_ARG;
    const OctGeom& og = c->geom.oct[o];
    if ((size_t)og.rows * og.cols == 0) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_upload_level_rows", [&](auto&& f) { for (int r = 0; r < og.rows; ++r) f(rows[r], (size_t)og.cols * 4); });
    return stage_upload(c, {{const_cast<float*>(gdp_device_level(c, b, o, s)), (size_t)og.cols, (size_t)og.rows, rows}});
} GDP_ABI_CATCH(c)

int gdp_upload_pyramid_rows(gdp_ctx* c, int b, const float* const* const* const* py) try {
    if (!c || !py || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_upload_pyramid_rows: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_upload_pyramid_rows", [&](auto&& f) {
        for (int o = 0; o < c->geom.O; ++o)
            for (int s = 0; s < c->geom.L && py[o]; ++s)
                for (int r = 0; r < c->geom.oct[o].rows && py[o][s]; ++r) f(py[o][s][r], (size_t)c->geom.oct[o].cols * 4);
    });
    const Geom& g = c->geom;
    std::vector<UpPiece> pieces;
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        if ((size_t)og.rows * og.cols == 0) continue;
        if (!py[o]) return c->status(GDP_ERR_ARG, "gdp_upload_pyramid_rows: null octave %d", o);
        for (int s = 0; s < g.L; ++s) {
            if (!py[o][s]) return c->status(GDP_ERR_ARG, "gdp_upload_pyramid_rows: null level (%d, %d)", o, s);
            pieces.push_back({const_cast<float*>(gdp_device_level(c, b, o, s)), (size_t)og.cols, (size_t)og.rows, py[o][s]});
        }
    }
    return stage_upload(c, pieces);
} GDP_ABI_CATCH(c)

int gdp_upload_image_raw(gdp_ctx* c, int b, const float* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_upload_image_raw: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_upload_image_raw", [&](auto&& f) { f(host, (size_t)c->img_floats * 4); });
    GDP_HIP(c, hipMemcpyAsync(c->d_out + (size_t)b * c->geom.pyr_stride, track_dma_ptr(host), (size_t)c->img_floats * 4,
                              hipMemcpyHostToDevice, c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_get_taps(gdp_ctx* c, int axis, int o, int s, float* host) try {
    if (!c || !host || o < 0 || o >= c->geom.O || s < 0 || s >= c->geom.L || (axis != 0 && axis != 1))
        return c ? c->status(GDP_ERR_ARG, "gdp_get_taps: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_SETTLE(c, "gdp_get_taps", [&](auto&& f) { f(host, (size_t)(axis == 0 ? c->geom.oct[o].cols : (c->geom.H >> o)) * 4); });
    const OctGeom& og = c->geom.oct[o];
    const int n = axis == 0 ? og.cols : (c->geom.H >> o);
    const long long off = axis == 0 ? og.ctap + (long long)s * og.ctap_stride : og.rtap + (long long)s * og.rtap_stride;
    // read back what the device holds, not the host copy: this is what the kernels use
    if (axis == 0 || og.rtap_row == 1) {
        GDP_HIP(c, hipMemcpy(host, c->d_taps + off, (size_t)n * 4, hipMemcpyDeviceToHost));
        return GDP_OK;
    }
    std::vector<float> rows((size_t)n * og.rtap_row);  // [row][scale]: pick scale s of each row
    if (n > 0) GDP_HIP(c, hipMemcpy(rows.data(), c->d_taps + og.rtap, rows.size() * 4, hipMemcpyDeviceToHost));
    for (int r = 0; r < n; ++r) host[r] = rows[(size_t)r * og.rtap_row + s];
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_set_output_device(gdp_ctx* c, float* base, size_t bytes) try {
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
} GDP_ABI_CATCH(c)

size_t gdp_level_offset(const gdp_ctx* c, int b, int o, int s) {
    if (!valid_level(c, b, o, s)) return (size_t)-1;
    const OctGeom& og = c->geom.oct[o];
    return (size_t)b * c->geom.pyr_stride + og.lev_off + (size_t)s * og.lev_stride;
}

int gdp_host_alloc(size_t bytes, void** host) try {
    if (!host || bytes == 0) return GDP_ERR_ARG;
    *host = nullptr;
    const hipError_t e = hipHostMalloc(host, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        *host = nullptr;
        return e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP;
    }
    return GDP_OK;
} GDP_ABI_CATCH(nullptr)

void gdp_host_free(void* host) {
    if (!host) return;
    {
        std::lock_guard<std::mutex> lk(g_track_mu);
        if (track_free_alias(host)) return;
        if (TrackedMirror* t = track_find(host)) {  // a tracked plain buffer: forget it first
            (void)mprotect(reinterpret_cast<void*>(t->base.load(std::memory_order_relaxed)),
                           t->bytes.load(std::memory_order_relaxed), PROT_READ | PROT_WRITE);
            track_retire(t);
        }
    }
    (void)hipHostFree(host);
}

size_t gdp_image_floats(const gdp_ctx* c) { return c ? (size_t)c->img_floats : 0; }

// A whole-image download into `host` is about to replace a deferred mirror's contents: true when
// it covers the mirror exactly (its stale pages then end as clean — track_undefer after the copy);
// any other deferred mirror is completed first.
static bool download_covers_deferred(gdp_ctx* c, const void* host, int* rc) {
    std::lock_guard<std::mutex> lk(g_track_mu);
    const TrackedMirror* t = track_find(host);
    const uintptr_t a = reinterpret_cast<uintptr_t>(host);
    const size_t n = (size_t)c->img_floats * 4;
    if (t && t->stale && t->user_bytes <= n) {
        *rc = GDP_OK;
        for (TrackedMirror& u : g_tracked) {
            const uintptr_t b = u.base.load(std::memory_order_relaxed);
            if (&u != t && b && u.stale && a < b + u.bytes.load(std::memory_order_relaxed) && a + n > b &&
                track_settle(u) != GDP_OK)
                *rc = GDP_ERR_HIP;
        }
        return true;
    }
    *rc = track_settle_overlap(a, a + n);
    return false;
}
static int finish_download(gdp_ctx* c, const void* host, bool covers) {
    if (!covers) return GDP_OK;
    std::lock_guard<std::mutex> lk(g_track_mu);
    TrackedMirror* t = track_find(host);
    return t && track_undefer(*t) != GDP_OK ? c->status(GDP_ERR_STATE, "mprotect refused arming a downloaded mirror") : GDP_OK;
}

int gdp_download_image_raw(gdp_ctx* c, int b, float* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_download_image_raw: bad argument") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    int rc = GDP_OK;
    const bool covers = download_covers_deferred(c, host, &rc);
    if (rc != GDP_OK) return c->status(rc, "gdp_download_image_raw: completing a deferred host mirror failed");
    GDP_HIP(c, hipMemcpyAsync(track_dma_ptr(host), c->d_out + (size_t)b * c->geom.pyr_stride, (size_t)c->img_floats * 4,
                              hipMemcpyDeviceToHost, c->stream));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return finish_download(c, host, covers);
} GDP_ABI_CATCH(c)

// GenerateDoG on a HOST pyramid (the drop-in classes' mirrored GaussPy, GuassDePyramid.h:16,
// :136-149): = gdp_upload_image_raw(b, host) + the in-place GenerateDoG of image b +
// gdp_download_image_raw(b, host), bit for bit, but pipelined over row chunks so the PCIe copies in
// both directions and the kernel overlap: chunk j's upload (copy stream 1) runs beside chunk j-1's
// pass (the context's stream) and chunk j-2's download (copy stream 2).  The op is pointwise in
// (octave, row, column) across the S+3 levels, so any row split is exact.
// `runs` (write-tracked mirrors): instead of every chunk, upload only these byte ranges of the
// image (the pages written since the mirror was armed), all before the first chunk's pass.
constexpr size_t kMirrorSerialBytes = 32u << 20;  // generate_dog_mirrored: unpipelined up to this image size
static int generate_dog_mirrored(gdp_ctx* c, int b, float* host, const std::vector<std::pair<size_t, size_t>>* runs) {
    const Geom& g = c->geom;
    GDP_HIP(c, hipSetDevice(c->device));
    auto pass = [&](int o, unsigned k0, unsigned k1, hipStream_t st) {  // octave o's groups [k0, k1) in place
        auto kern = c->nontemporal ? k_levels_range<0, 3, true> : k_levels_range<0, 3, false>;
        if (g.L == 5) kern = c->nontemporal ? k_levels_range<5, 3, true> : k_levels_range<5, 3, false>;
        hipLaunchKernelGGL(kern, dim3((k1 - k0 + 255) / 256), dim3(256), 0, st, c->d_geom, c->d_out, c->d_taps,
                           (unsigned)b, o, k0, k1);
        return hipGetLastError();
    };
    // Small images (main.cpp's 512^2: 7 MB each way): the row-chunk pipeline's ~20 chunks of per-level
    // copies and events cost more than the copies themselves, so one contiguous copy each way around
    // one pass per octave, all on the context's stream.  Same bits (the op is pointwise).
    const size_t img_bytes = (size_t)c->img_floats * 4;
    if (img_bytes <= kMirrorSerialBytes) {
        struct DrainOnError {  // (as below: no return while a copy of `host` is in flight)
            gdp_ctx* c;
            bool armed = true;
            ~DrainOnError() {
                if (armed) (void)hipStreamSynchronize(c->stream);
            }
        } drain{c};
        char* dev = reinterpret_cast<char*>(c->d_out + (size_t)b * g.pyr_stride);
        if (runs) {
            for (const auto& r : *runs)
                GDP_HIP(c, hipMemcpyAsync(dev + r.first, reinterpret_cast<const char*>(host) + r.first, r.second - r.first,
                                          hipMemcpyHostToDevice, c->stream));
        } else {
            GDP_HIP(c, hipMemcpyAsync(dev, host, img_bytes, hipMemcpyHostToDevice, c->stream));
        }
        for (int o = 0; o < g.O; ++o) {
            const unsigned k1 = (unsigned)g.oct[o].rows * (unsigned)g.oct[o].gpr;
            if (k1) GDP_HIP(c, pass(o, 0u, k1, c->stream));
        }
        GDP_HIP(c, hipMemcpyAsync(host, dev, img_bytes, hipMemcpyDeviceToHost, c->stream));
        GDP_HIP(c, hipStreamSynchronize(c->stream));
        drain.armed = false;
        return GDP_OK;
    }
    if (!c->st_up) GDP_HIP(c, hipStreamCreateWithFlags(&c->st_up, hipStreamNonBlocking));
    if (!c->st_down) GDP_HIP(c, hipStreamCreateWithFlags(&c->st_down, hipStreamNonBlocking));
    // chunks of about 1/16 of the image's bytes: octave 0 in ~12 row ranges, each smaller octave in
    // proportionally fewer (one for the tiny ones)
    struct Chunk { int o, r0, r1; };
    std::vector<Chunk> chunks;
    long long total = 0;
    for (int o = 0; o < g.O; ++o) total += (long long)g.oct[o].rows * g.oct[o].cols;
    const long long target = std::max(1ll, total / 16);
    for (int o = 0; o < g.O; ++o) {
        const OctGeom& og = g.oct[o];
        if ((long long)og.rows * og.cols == 0) continue;
        const long long px = (long long)og.rows * og.cols;
        const int n = (int)std::max(1ll, std::min<long long>(og.rows, (px + target / 2) / target));
        for (int k = 0; k < n; ++k) {
            const int r0 = (int)((long long)og.rows * k / n), r1 = (int)((long long)og.rows * (k + 1) / n);
            if (r1 > r0) chunks.push_back({o, r0, r1});
        }
    }
    const size_t need = 2 * chunks.size() + 1;
    while (c->ev_mirror.size() < need) {
        hipEvent_t e;
        GDP_HIP(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->ev_mirror.push_back(e);
    }
    hipEvent_t* ev = c->ev_mirror.data();
    // an error after the first copy was queued returns only once every queued copy and pass has
    // finished, so the caller never frees or reuses `host` under a DMA still in flight
    struct DrainOnError {
        gdp_ctx* c;
        bool armed = true;
        ~DrainOnError() {
            if (!armed) return;
            (void)hipStreamSynchronize(c->st_up);
            (void)hipStreamSynchronize(c->stream);
            (void)hipStreamSynchronize(c->st_down);
        }
    } drain{c};
    // the uploads overwrite levels earlier work on the context's stream may still use
    GDP_HIP(c, hipEventRecord(ev[2 * chunks.size()], c->stream));
    GDP_HIP(c, hipStreamWaitEvent(c->st_up, ev[2 * chunks.size()], 0));
    auto image_level = [&](int o, int s) { return g.oct[o].lev_off + (long long)s * g.oct[o].lev_stride; };
    if (runs) {
        char* dev = reinterpret_cast<char*>(c->d_out + (size_t)b * g.pyr_stride);
        for (const auto& r : *runs)
            GDP_HIP(c, hipMemcpyAsync(dev + r.first, reinterpret_cast<const char*>(host) + r.first, r.second - r.first,
                                      hipMemcpyHostToDevice, c->st_up));
    }
    for (size_t j = 0; j < chunks.size(); ++j) {
        const Chunk& ch = chunks[j];
        const OctGeom& og = g.oct[ch.o];
        const size_t off = (size_t)ch.r0 * og.cols, n = (size_t)(ch.r1 - ch.r0) * og.cols;
        for (int s = 0; s < g.L && !runs; ++s)
            GDP_HIP(c, hipMemcpyAsync(const_cast<float*>(gdp_device_level(c, b, ch.o, s)) + off,
                                      host + image_level(ch.o, s) + off, n * 4, hipMemcpyHostToDevice, c->st_up));
        GDP_HIP(c, hipEventRecord(ev[2 * j], c->st_up));
        GDP_HIP(c, hipStreamWaitEvent(c->stream, ev[2 * j], 0));
        const unsigned k0 = (unsigned)ch.r0 * (unsigned)og.gpr, k1 = (unsigned)ch.r1 * (unsigned)og.gpr;
        GDP_HIP(c, pass(ch.o, k0, k1, c->stream));
        GDP_HIP(c, hipEventRecord(ev[2 * j + 1], c->stream));
        GDP_HIP(c, hipStreamWaitEvent(c->st_down, ev[2 * j + 1], 0));
        for (int s = 0; s < g.L; ++s)
            GDP_HIP(c, hipMemcpyAsync(host + image_level(ch.o, s) + off, gdp_device_level(c, b, ch.o, s) + off, n * 4,
                                      hipMemcpyDeviceToHost, c->st_down));
    }
    GDP_HIP(c, hipStreamSynchronize(c->st_down));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    drain.armed = false;
    return GDP_OK;
}

int gdp_generate_dog_mirrored(gdp_ctx* c, int b, float* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_generate_dog_mirrored: bad argument") : GDP_ERR_ARG;
    GDP_SETTLE(c, "gdp_generate_dog_mirrored", [&](auto&& f) { f(host, (size_t)c->img_floats * 4); });  // the whole host image is the input
    return generate_dog_mirrored(c, b, track_dma_ptr(host), nullptr);
} GDP_ABI_CATCH(c)

// ---- write-tracked host mirrors (gdp_track.inc) ----
// the SIGSEGV handler (once per process) and a free registry slot; caller holds g_track_mu
static TrackedMirror* track_slot() {
    if (!g_segv_installed) {
        const long pg = sysconf(_SC_PAGESIZE);
        if (pg > 0) g_page_bytes = (size_t)pg;
        struct sigaction sa;
        std::memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = track_on_segv;
        sa.sa_flags = SA_SIGINFO | SA_RESTART | SA_ONSTACK;
        sigemptyset(&sa.sa_mask);
        if (sigaction(SIGSEGV, &sa, &g_prev_segv) != 0) return nullptr;
        g_segv_installed = true;
    }
    for (TrackedMirror& s : g_tracked)
        if (!s.base.load(std::memory_order_relaxed)) return &s;
    return nullptr;
}

// publish a registry entry for the CPU range [host, host + bytes) (caller holds g_track_mu)
static void track_publish(TrackedMirror* t, void* host, size_t bytes, void* dma, size_t map_bytes) {
    const uintptr_t u = reinterpret_cast<uintptr_t>(host);
    const uintptr_t base = u / g_page_bytes * g_page_bytes;
    const uintptr_t end = (u + bytes + g_page_bytes - 1) / g_page_bytes * g_page_bytes;
    t->pages = (end - base) / g_page_bytes;
    // a larger flag array when needed; the old one stays allocated and referenced (a handler on
    // another thread may still read it): a slot keeps at most one array per size it has grown to
    if (t->written_cap < t->pages) {
        if (t->written) g_track_retired->push_back(t->written);
        t->written = new std::atomic<unsigned char>[t->pages];
        t->written_cap = t->pages;
    }
    for (size_t p = 0; p < t->pages; ++p) t->written[p].store(0, std::memory_order_relaxed);
    t->maybe_written.store(false, std::memory_order_relaxed);
    t->user = host;
    t->user_bytes = bytes;
    t->armed = false;
    t->tracking = true;
    t->dma = dma;
    t->map_bytes = map_bytes;
    t->bytes.store(end - base, std::memory_order_relaxed);
    t->base.store(base, std::memory_order_release);
}

int gdp_host_alloc_tracked(size_t bytes, void** host) try {
    if (!host || bytes == 0) return GDP_ERR_ARG;
    *host = nullptr;
    std::lock_guard<std::mutex> lk(g_track_mu);
    TrackedMirror* t = track_slot();
    if (!t) return GDP_ERR_STATE;
    const size_t map = (bytes + g_page_bytes - 1) / g_page_bytes * g_page_bytes;
    // one shared-memory object, two mappings: `dma` registered with HIP (never protected),
    // `cpu` the caller's view (the one write-protected)
    const int fd = (int)memfd_create("gdp_mirror", MFD_CLOEXEC);
    if (fd < 0) return GDP_ERR_STATE;
    void* dma = MAP_FAILED;
    void* cpu = MAP_FAILED;
    if (ftruncate(fd, (off_t)map) == 0) {
        dma = mmap(nullptr, map, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        cpu = mmap(nullptr, map, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    }
    close(fd);
    if (dma != MAP_FAILED && cpu != MAP_FAILED) {
        // huge pages where the kernel gives them to shared memory (fewer IOMMU translations for the
        // DMA engines), then the pages faulted in through the DMA view before it is registered
        (void)madvise(dma, map, MADV_HUGEPAGE);
        (void)madvise(cpu, map, MADV_HUGEPAGE);
        for (size_t off = 0; off < map; off += g_page_bytes) static_cast<volatile char*>(dma)[off] = 0;
    }
    auto unmap = [&] {
        if (dma != MAP_FAILED) munmap(dma, map);
        if (cpu != MAP_FAILED) munmap(cpu, map);
    };
    if (dma == MAP_FAILED || cpu == MAP_FAILED) {
        unmap();
        return GDP_ERR_NOMEM;
    }
    // like pinned memory, not inherited by fork()ed children (a shared mapping would otherwise let
    // a child's writes reach this process's mirror)
    (void)madvise(dma, map, MADV_DONTFORK);
    (void)madvise(cpu, map, MADV_DONTFORK);
    const hipError_t e = hipHostRegister(dma, map, hipHostRegisterDefault);
    if (e != hipSuccess) {
        unmap();
        return e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP;
    }
    track_publish(t, cpu, bytes, dma, map);
    *host = cpu;
    return GDP_OK;
} GDP_ABI_CATCH(nullptr)

int gdp_host_track(void* host, size_t bytes) try {
    if (!host || bytes == 0) return GDP_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_track_mu);
    if (TrackedMirror* t = track_find(host)) {  // registered before (an alias whose tracking was off)
        t->tracking = true;
        return GDP_OK;
    }
    // memory the GPU driver registered must not be protected (gdp_track.inc): refuse it
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, host) == hipSuccess && attr.type != hipMemoryTypeUnregistered) {
        (void)hipGetLastError();
        return GDP_ERR_STATE;
    }
    (void)hipGetLastError();
    TrackedMirror* t = track_slot();
    if (!t) return GDP_ERR_STATE;
    const uintptr_t base = reinterpret_cast<uintptr_t>(host) / g_page_bytes * g_page_bytes;
    // protection must be available on this memory (a probe of its first page)
    if (mprotect(reinterpret_cast<void*>(base), g_page_bytes, PROT_READ) != 0) return GDP_ERR_STATE;
    if (mprotect(reinterpret_cast<void*>(base), g_page_bytes, PROT_READ | PROT_WRITE) != 0) return GDP_ERR_STATE;
    track_publish(t, host, bytes, nullptr, 0);
    return GDP_OK;
} GDP_ABI_CATCH(nullptr)

int gdp_host_untrack(void* host) try {
    std::lock_guard<std::mutex> lk(g_track_mu);
    TrackedMirror* t = host ? track_find(host) : nullptr;
    if (!t || !t->tracking) return GDP_ERR_ARG;
    if (track_settle(*t) != GDP_OK) return GDP_ERR_HIP;  // a deferred mirror is completed first
    const uintptr_t base = t->base.load(std::memory_order_relaxed);
    const int rc = mprotect(reinterpret_cast<void*>(base), t->bytes.load(std::memory_order_relaxed), PROT_READ | PROT_WRITE) == 0
                       ? GDP_OK
                       : GDP_ERR_STATE;
    t->armed = t->tracking = false;
    for (size_t p = 0; p < t->pages; ++p) t->written[p].store(0, std::memory_order_relaxed);
    t->maybe_written.store(false, std::memory_order_relaxed);
    if (!t->dma) track_retire(t);  // an alias stays registered for its DMA view until gdp_host_free
    return rc;
} GDP_ABI_CATCH(nullptr)

int gdp_host_arm(void* host) try {
    std::lock_guard<std::mutex> lk(g_track_mu);
    TrackedMirror* t = host ? track_find(host) : nullptr;
    if (!t) return GDP_ERR_ARG;
    if (!t->tracking) return GDP_ERR_STATE;
    // already armed: every page not written since is still protected, so only the written ones
    // are protected again (no walk over the whole range)
    if (t->armed) return track_rearm(*t, track_written_runs(*t), false);
    if (track_settle(*t) != GDP_OK) return GDP_ERR_HIP;  // (arming all: stale pages fetched first)
    return track_rearm(*t, {}, true);
} GDP_ABI_CATCH(nullptr)

int gdp_host_written_bytes(const void* host, size_t* bytes) try {
    if (!bytes) return GDP_ERR_ARG;
    std::lock_guard<std::mutex> lk(g_track_mu);
    const TrackedMirror* t = host ? track_find(host) : nullptr;
    if (!t) return GDP_ERR_ARG;
    if (!t->armed) return GDP_ERR_STATE;
    const uintptr_t b = t->base.load(std::memory_order_relaxed);
    const uintptr_t u0 = reinterpret_cast<uintptr_t>(t->user), u1 = u0 + t->user_bytes;
    size_t n = 0;
    for (size_t p = t->maybe_written.load(std::memory_order_acquire) ? 0 : t->pages; p < t->pages; ++p)
        if (t->written[p].load(std::memory_order_relaxed) == kPageWritten) {
            const uintptr_t lo = std::max<uintptr_t>(u0, b + p * g_page_bytes);
            const uintptr_t hi = std::min<uintptr_t>(u1, b + (p + 1) * g_page_bytes);
            n += hi > lo ? hi - lo : 0;
        }
    *bytes = n;
    return GDP_OK;
} GDP_ABI_CATCH(nullptr)

// The written pages of an armed mirror covering image b.  Returns the entry (nullptr: not
// tracked); *partial: only `runs` need uploading (armed, large enough, not too fragmented).
// Caller holds g_track_mu.
static TrackedMirror* track_for_image(const gdp_ctx* c, const void* host, std::vector<std::pair<size_t, size_t>>* runs,
                                      bool* partial) {
    *partial = false;
    TrackedMirror* t = track_find(host);
    if (!t || !t->tracking) return nullptr;
    const size_t img_bytes = (size_t)c->img_floats * 4;
    if (!t->armed || t->user_bytes < img_bytes) return t;
    *runs = track_written_runs(*t);
    for (auto& r : *runs) r.second = std::min(r.second, img_bytes);
    runs->erase(std::remove_if(runs->begin(), runs->end(), [](const std::pair<size_t, size_t>& r) { return r.second <= r.first; }),
                runs->end());
    *partial = runs->size() <= 4096;
    return t;
}

// (The registry lock is held while the written runs are collected and while the mirror is
// re-armed, not across the copies and kernels between, so drop-in objects on other threads keep
// their GPU work concurrent.  A buffer must not be freed or untracked by another thread during a
// call on it — the caller's contract for any buffer it passes in.)
int gdp_upload_image_written(gdp_ctx* c, int b, const float* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_upload_image_written: bad argument") : GDP_ERR_ARG;
    std::vector<std::pair<size_t, size_t>> runs;
    bool partial = false;
    TrackedMirror* t;
    {
        std::lock_guard<std::mutex> lk(g_track_mu);
        t = track_for_image(c, host, &runs, &partial);
        // the written runs never cover a stale page; a whole upload needs every page current
        if (!partial && track_settle_overlap(reinterpret_cast<uintptr_t>(host), reinterpret_cast<uintptr_t>(host) + (size_t)c->img_floats * 4) != GDP_OK) {
            if (t) t->armed = false;
            return c->status(GDP_ERR_HIP, "gdp_upload_image_written: completing a deferred host mirror failed");
        }
    }
    // an error from here on leaves the collected runs un-uploaded: the next call uploads all
    struct DisarmOnError {
        TrackedMirror* t;
        bool on = true;
        ~DisarmOnError() {
            if (!on || !t) return;
            std::lock_guard<std::mutex> lk(g_track_mu);
            t->armed = false;
        }
    } disarm{t};
    const char* src = static_cast<const char*>(track_dma_ptr(static_cast<const void*>(host)));
    GDP_HIP(c, hipSetDevice(c->device));
    char* dev = reinterpret_cast<char*>(c->d_out + (size_t)b * c->geom.pyr_stride);
    if (partial) {
        for (const auto& r : runs)
            GDP_HIP(c, hipMemcpyAsync(dev + r.first, src + r.first, r.second - r.first, hipMemcpyHostToDevice, c->stream));
    } else {
        GDP_HIP(c, hipMemcpyAsync(dev, src, (size_t)c->img_floats * 4, hipMemcpyHostToDevice, c->stream));
    }
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    disarm.on = false;
    std::lock_guard<std::mutex> lk(g_track_mu);
    if (t && track_rearm(*t, runs, !partial) != GDP_OK)
        return c->status(GDP_ERR_STATE, "gdp_upload_image_written: mprotect refused re-arming the mirror");
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_generate_dog_mirrored_written(gdp_ctx* c, int b, float* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_generate_dog_mirrored_written: bad argument") : GDP_ERR_ARG;
    std::vector<std::pair<size_t, size_t>> runs;
    bool partial = false;
    TrackedMirror* t;
    {
        std::lock_guard<std::mutex> lk(g_track_mu);
        t = track_for_image(c, host, &runs, &partial);
        // (as gdp_upload_image_written; the download at the end replaces every page)
        if (!partial && track_settle_overlap(reinterpret_cast<uintptr_t>(host), reinterpret_cast<uintptr_t>(host) + (size_t)c->img_floats * 4) != GDP_OK) {
            if (t) t->armed = false;
            return c->status(GDP_ERR_HIP, "gdp_generate_dog_mirrored_written: completing a deferred host mirror failed");
        }
    }
    const int rc = generate_dog_mirrored(c, b, track_dma_ptr(host), partial ? &runs : nullptr);
    std::lock_guard<std::mutex> lk(g_track_mu);
    if (rc != GDP_OK) {
        if (t) t->armed = false;  // the device may hold a partial result: the next call uploads all
        return rc;
    }
    if (t && track_undefer(*t) != GDP_OK)
        return c->status(GDP_ERR_STATE, "gdp_generate_dog_mirrored_written: mprotect refused arming the mirror");
    if (t && track_rearm(*t, runs, !partial) != GDP_OK)
        return c->status(GDP_ERR_STATE, "gdp_generate_dog_mirrored_written: mprotect refused re-arming the mirror");
    return GDP_OK;
} GDP_ABI_CATCH(c)

// ---- deferred download (gdp_track.inc) ----
int gdp_host_defer(gdp_ctx* c, int b, void* host) try {
    if (!c || !host || b < 0 || b >= c->geom.batch)
        return c ? c->status(GDP_ERR_ARG, "gdp_host_defer: bad argument") : GDP_ERR_ARG;
    const size_t img_bytes = (size_t)c->img_floats * 4;
    std::lock_guard<std::mutex> lk(g_track_mu);
    TrackedMirror* t = track_find(host);
    if (!t || !t->tracking || !t->dma)
        return c->status(GDP_ERR_STATE, "gdp_host_defer: not a write-tracked gdp_host_alloc_tracked buffer");
    if (t->user_bytes > img_bytes)
        return c->status(GDP_ERR_ARG, "gdp_host_defer: the buffer (%zu bytes) is larger than the image (%zu)", t->user_bytes,
                         img_bytes);
    const char* src = reinterpret_cast<const char*>(c->d_out + (size_t)b * c->geom.pyr_stride);
    // stale pages of ANOTHER source are fetched first (they are older than this image only if the
    // caller says so for every page — it does not: only for the image it names)
    if ((t->stale || t->trips) && (t->src_ctx != c || t->src != src) && track_settle(*t) != GDP_OK)
        return c->status(GDP_ERR_HIP, "gdp_host_defer: completing the previous deferral failed");
    if (!g_fetch_worker.exchange(true)) {
        static bool atfork = false;  // a fork()ed child has no copy thread (and no mirrors: DONTFORK)
        if (!atfork) atfork = pthread_atfork(nullptr, nullptr, [] { g_fetch_worker.store(false); }) == 0;
        try {
            std::thread(track_fetch_worker).detach();
        } catch (...) {  // no copy thread: a fault could never be served, so refuse to defer
            g_fetch_worker.store(false);
            return c->status(GDP_ERR_STATE, "gdp_host_defer: the fetch thread could not be started");
        }
    }
    state_lock_quiesced();  // no copy of an older deferral still landing
    const uintptr_t base = t->base.load(std::memory_order_relaxed);
    int rc = GDP_OK;
    // every page not stale yet: no access (tripwires are inaccessible already)
    auto open = [&](size_t p) {
        const unsigned char st = t->written[p].load(std::memory_order_relaxed);
        return st == kPageClean || st == kPageWritten;
    };
    for (size_t p = t->stale == t->pages ? t->pages : 0; p < t->pages;) {
        const unsigned char st = t->written[p].load(std::memory_order_relaxed);
        if (st == kPageTrip) {
            t->written[p].store(kPageStale, std::memory_order_relaxed);
            --t->trips;
            ++t->stale;
        }
        if (!open(p)) {
            ++p;
            continue;
        }
        size_t q = p + 1;
        while (q < t->pages && open(q)) ++q;
        if (mprotect(reinterpret_cast<void*>(base + p * g_page_bytes), (q - p) * g_page_bytes, PROT_NONE) != 0) {
            rc = GDP_ERR_STATE;
            break;
        }
        for (size_t k = p; k < q; ++k) t->written[k].store(kPageStale, std::memory_order_relaxed);
        t->stale += q - p;
        p = q;
    }
    t->src_ctx = c;
    t->src = src;
    t->src_bytes = img_bytes;
    t->src_device = c->device;
    t->src_stream = c->stream;
    t->ra_next = t->ra_len = 0;
    t->fetched_bytes = 0;
    t->fetches = 0;
    if (rc == GDP_OK) t->maybe_written.store(false, std::memory_order_relaxed);  // every page stale
    t->armed = rc == GDP_OK;  // no written page is pending: a record exists (nothing written yet)
    state_unlock();
    if (rc != GDP_OK) {
        // the mirror is in a mixed state: complete it and give up tracking
        (void)track_settle(*t);
        return c->status(GDP_ERR_STATE, "gdp_host_defer: mprotect refused");
    }
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_host_fetch(void* host) try {
    std::lock_guard<std::mutex> lk(g_track_mu);
    TrackedMirror* t = host ? track_find(host) : nullptr;
    if (!t) return GDP_ERR_ARG;
    return track_settle(*t);
} GDP_ABI_CATCH(nullptr)

int gdp_host_deferred_stats(const void* host, size_t* stale_bytes, size_t* fetched_bytes, uint64_t* fetches) try {
    std::lock_guard<std::mutex> lk(g_track_mu);
    const TrackedMirror* t = host ? track_find(host) : nullptr;
    if (!t) return GDP_ERR_ARG;
    state_lock();
    if (stale_bytes) *stale_bytes = t->stale * g_page_bytes;
    if (fetched_bytes) *fetched_bytes = t->fetched_bytes;
    if (fetches) *fetches = t->fetches;
    state_unlock();
    return GDP_OK;
} GDP_ABI_CATCH(nullptr)

int gdp_checksum(gdp_ctx* c, int b, uint64_t* out) try {
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
} GDP_ABI_CATCH(c)

int gdp_set_window_centre(gdp_ctx* c, int mode) try {
    if (!c || (mode != GDP_CENTRE_SERIAL && mode != GDP_CENTRE_INTLEN))
        return c ? c->status(GDP_ERR_ARG, "gdp_set_window_centre: mode must be GDP_CENTRE_SERIAL or GDP_CENTRE_INTLEN") : GDP_ERR_ARG;
    if (mode == c->centre_mode) return GDP_OK;
    GDP_HIP(c, hipSetDevice(c->device));
    if (!c->d_taps_mode[mode]) {
        // first use of this centre: its own table (the other one stays intact for launches already
        // queued, which captured its pointer), uploaded once; later switches are a pointer swap
        fill_host_taps(c, mode);
        float* t = nullptr;
        hipError_t e = hipMalloc(&t, std::max<size_t>(4, c->h_taps.size() * 4));
        if (e != hipSuccess) return c->status(e == hipErrorOutOfMemory ? GDP_ERR_NOMEM : GDP_ERR_HIP, "hipMalloc(taps)");
        e = hipMemcpy(t, c->h_taps.data(), c->h_taps.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(t);
            return c->status(GDP_ERR_HIP, "hipMemcpy(taps): %s", hipGetErrorString(e));
        }
        c->d_taps_mode[mode] = t;
    }
    c->centre_mode = mode;
    c->d_taps = c->d_taps_mode[mode];
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_get_window_centre(const gdp_ctx* c) { return c ? c->centre_mode : -1; }

int gdp_copy_band(gdp_ctx* band, int bi, const gdp_ctx* full, int fi, void* stream) try {
    if (!band || !full || bi < 0 || bi >= band->geom.batch || fi < 0 || fi >= full->geom.batch)
        return band ? band->status(GDP_ERR_ARG, "gdp_copy_band: bad argument") : GDP_ERR_ARG;
    const Geom &gb = band->geom, &gf = full->geom;
    if (gb.H != gf.H || gb.W != gf.W || gb.S != gf.S || gb.O != gf.O || gf.in_row0 != 0 || gf.in_rows != gf.H)
        return band->status(GDP_ERR_ARG, "gdp_copy_band: `full` must be a whole-image context of the same geometry");
    if (band->device != full->device) return band->status(GDP_ERR_ARG, "gdp_copy_band: contexts on different devices");
    GDP_HIP(band, hipSetDevice(band->device));
    GDP_HIP(band, hipStreamSynchronize(full->stream));  // full's own work has landed
    const hipStream_t st = band->pick(stream);
    for (int o = 0; o < gb.O; ++o) {
        const OctGeom& og = gb.oct[o];
        if ((size_t)og.rows * og.cols == 0) continue;
        for (int s = 0; s < gb.L; ++s)
            GDP_HIP(band, hipMemcpyAsync(const_cast<float*>(gdp_device_level(band, bi, o, s)),
                                         gdp_device_level(full, fi, o, s) + (size_t)og.row0 * og.cols,
                                         (size_t)og.rows * og.cols * 4, hipMemcpyDeviceToDevice, st));
    }
    GDP_HIP(band, hipStreamSynchronize(st));
    return GDP_OK;
} GDP_ABI_CATCH(band)

int gdp_sync(gdp_ctx* c) try {
    if (!c) return GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    GDP_HIP(c, hipStreamSynchronize(c->stream));
    return GDP_OK;
} GDP_ABI_CATCH(c)

void* gdp_stream(const gdp_ctx* c) { return c ? (void*)c->stream : nullptr; }

int gdp_autotune(gdp_ctx* c, int iters, void* stream, int* best_variant, int* best_order, float* best_ms) try {
    // Times every build-kernel variant x tile order x store mode on the context's current input
    // (HIP events on `stream`, median of 3 repeats of `iters` launches) and keeps the fastest.
    // Store modes (zero window, store pace): (0, off), (0, 1), (1, off), (1, 0) — the pairs that won
    // somewhere in profiles/sp*_r03a{p,q}.log.  All candidates produce identical bits, so this only
    // ever changes speed.
    if (!c || iters <= 0) return c ? c->status(GDP_ERR_ARG, "gdp_autotune: iters must be > 0") : GDP_ERR_ARG;
    GDP_HIP(c, hipSetDevice(c->device));
    const int old_variant = c->variant, old_order = c->geom.tile_order;
    int bv = old_variant, bo = old_order, bz = c->zero_window, bp = c->geom.store_pace;
    float bt = 3.4e38f;
    static const int kModes[4][2] = {{0, -1}, {0, 1}, {1, -1}, {1, 0}};
    for (const auto& mode : kModes) {
        const int zw = mode[0], sp = mode[1];
        int rc = gdp_set_tuning(c, GDP_TUNE_ZERO_WINDOW, zw);
        if (rc == GDP_OK) rc = gdp_set_tuning(c, GDP_TUNE_STORE_PACE, sp);
        if (rc != GDP_OK) return rc;
        for (const BuildVariant& bvar : kVariants) {
            const int v = bvar.id;
            for (int ord = 0; ord <= 1; ++ord) {
                rc = gdp_set_tuning(c, GDP_TUNE_VARIANT, v);
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
                    bz = zw;
                    bp = sp;
                }
            }
        }
    }
    int rc = gdp_set_tuning(c, GDP_TUNE_VARIANT, bv);
    if (rc == GDP_OK) rc = gdp_set_tuning(c, GDP_TUNE_TILE_ORDER, bo);
    if (rc == GDP_OK) rc = gdp_set_tuning(c, GDP_TUNE_ZERO_WINDOW, bz);
    if (rc == GDP_OK) rc = gdp_set_tuning(c, GDP_TUNE_STORE_PACE, bp);
    if (rc != GDP_OK) return rc;
    if (best_variant) *best_variant = bv;
    if (best_order) *best_order = bo;
    if (best_ms) *best_ms = bt / iters;
    return GDP_OK;
} GDP_ABI_CATCH(c)

int gdp_build_variants(int* ids, int capacity) {
    for (int i = 0; i < kNumVariants && i < capacity && ids; ++i) ids[i] = kVariants[i].id;
    return kNumVariants;
}

int gdp_get_tuning(const gdp_ctx* c, int key, int* value) try {
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
        case GDP_TUNE_CONV_WAVES: *value = c->conv_waves; return GDP_OK;
        case GDP_TUNE_ZERO_WINDOW: *value = c->zero_window; return GDP_OK;
        case GDP_TUNE_STORE_PACE: *value = c->geom.store_pace; return GDP_OK;
        case GDP_TUNE_INPLACE_PACE: *value = c->geom.inplace_pace; return GDP_OK;
        case GDP_TUNE_CONV_PACE: *value = c->geom.conv_pace; return GDP_OK;
        case GDP_TUNE_BUILD_LDS: *value = c->build_lds; return GDP_OK;
        case GDP_TUNE_STAGE_KB: *value = (int)(c->stage_half_floats / 256); return GDP_OK;
        case GDP_TUNE_STAGE_THREADS: *value = c->stage_threads; return GDP_OK;
        case GDP_TUNE_PYRAMID_CHUNK_KB: *value = c->pyr_chunk_kb; return GDP_OK;
        default: return GDP_ERR_ARG;
    }
} GDP_ABI_CATCH(c)

int gdp_set_tuning(gdp_ctx* c, int key, int value) try {
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
            if ((value != 1 && value != 2 && value != 4 && value != 8 && value != 16) &&
                !(key == GDP_TUNE_INPLACE_SUB && (value == 0 || value == -kLtRows)))
                return c->status(GDP_ERR_ARG, "sub-blocks must be 1, 2, 4, 8 or 16 (1024 / sub threads per block; "
                                              "in-place DoG also 0: one level per wave, -16: 16 x 256 block tiles)");
            (key == GDP_TUNE_INPLACE_SUB ? c->inplace_sub : c->window_sub) = value;
            return GDP_OK;
        case GDP_TUNE_CONV_KERNEL:
            if (value < 0 || value > 2)
                return c->status(GDP_ERR_ARG, "conv kernel must be 0 (sweep), 1 (LDS tiles) or 2 (block tiles)");
            c->conv_kernel = value;
            return conv_follow_rows(c);
        case GDP_TUNE_CONV_ROWS: {
            if (value != 8 && value != 16 && value != 24 && value != 32 && value != 48)
                return c->status(GDP_ERR_ARG, "conv rows must be 8, 16, 24, 32 or 48 (sweep: 16 / 32; block tiles: "
                                              "16 / 32 / 48 with 16 waves, 8 / 16 / 24 / 32 with 8)");
            const int rc = conv_set_rows(c, value);
            if (rc == GDP_OK) c->conv_rows_set = true;
            return rc;
        }
        case GDP_TUNE_CONV_WAVES:
            if (value != 8 && value != 16) return c->status(GDP_ERR_ARG, "conv waves must be 8 or 16");
            c->conv_waves = value;
            return conv_follow_rows(c);
        case GDP_TUNE_STORE_PACE:
        case GDP_TUNE_CONV_PACE:
        case GDP_TUNE_INPLACE_PACE: {
            if (value < -1 || value > 3) return c->status(GDP_ERR_ARG, "store pace must be -1 (off) or 0..3");
            int& field = key == GDP_TUNE_STORE_PACE ? c->geom.store_pace
                         : key == GDP_TUNE_CONV_PACE ? c->geom.conv_pace : c->geom.inplace_pace;
            const int old = field;
            field = value;
            const int rc = upload_geom(c);
            if (rc != GDP_OK) field = old;
            return rc;
        }
        case GDP_TUNE_ZERO_WINDOW: {
            const int old = c->zero_window;
            if (value != 0 && value != 1) return c->status(GDP_ERR_ARG, "zero window must be 0 or 1");
            c->zero_window = value;
            set_window_support(c, c->zero_window != 0);
            const int rc = upload_geom(c);
            if (rc != GDP_OK) {
                c->zero_window = old;
                set_window_support(c, old != 0);
            }
            return rc;
        }
        case GDP_TUNE_CONV_ORDER:
            if (value < 0 || value > 7) return c->status(GDP_ERR_ARG, "conv order must be 0..7");
            c->conv_order = value;
            return GDP_OK;
        case GDP_TUNE_BUILD_LDS:
            if (value < 0 || value > 160 * 1024) return c->status(GDP_ERR_ARG, "build LDS bytes must be in [0, 163840]");
            c->build_lds = value;
            return GDP_OK;
        case GDP_TUNE_STAGE_KB:
            if (value < 1 || value > 1024 * 1024) return c->status(GDP_ERR_ARG, "staging KiB must be in [1, 1048576]");
            c->stage_half_floats = (size_t)value * 256;
            return GDP_OK;
        case GDP_TUNE_STAGE_THREADS:
            if (value < 1 || value > 64) return c->status(GDP_ERR_ARG, "staging threads must be in [1, 64]");
            c->stage_threads = value;
            return GDP_OK;
        case GDP_TUNE_TILE_ORDER:
            if (value < 0 || value > 2) return c->status(GDP_ERR_ARG, "tile order must be 0, 1 or 2");
            c->geom.tile_order = value;
            return upload_geom(c);
        case GDP_TUNE_VARIANT: {
            const int vi = variant_index(value);
            if (vi < 0) return c->status(GDP_ERR_ARG, "build variant %d is not built (gdp_build_variants lists them)", value);
            const int old = c->variant;
            c->variant = value;
            int rc = retile(c, kVariants[vi].tile_cols, kVariants[vi].tile_rows);
            if (rc == GDP_OK) rc = upload_geom(c);
            if (rc != GDP_OK) {
                c->variant = old;
                retile(c, kVariants[variant_index(old)].tile_cols, kVariants[variant_index(old)].tile_rows);
            }
            return rc;
        }
        default:
            return c->status(GDP_ERR_ARG, "unknown tuning key %d", key);
    }
} GDP_ABI_CATCH(c)

int gdp_time_builds(gdp_ctx* c, int iters, void* stream, float* total_ms) try {
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
} GDP_ABI_CATCH(c)

#ifdef GDP_TRACE_BLOCKS
// Diagnostic build only: device buffer of 3 x u64 per block for the next build launches (NULL off).
int gdp_debug_set_block_trace(void* dev_buf) try {
    unsigned long long* p = static_cast<unsigned long long*>(dev_buf);
    return hipMemcpyToSymbol(HIP_SYMBOL(g_block_trace), &p, sizeof p) == hipSuccess ? GDP_OK : GDP_ERR_HIP;
} GDP_ABI_CATCH(nullptr)
#endif
}  // extern "C"
