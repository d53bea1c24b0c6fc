// GaussDePyramid-HIP-mpitest.h — drop-in for the free-function / global-state API of the
// reference's mpitest.cpp (GaussPyInit(int* data[MAX]) :438-473, GenerateDoG_mpi :114-189,
// GenerateDoG_mpi_omp :35-113, delete_mpi :474-493, globals :26-34), running on one MI355X through
// libgdp (gdp.h).  Like mpitest.cpp itself, it DEFINES the globals and functions, so include it in
// exactly one translation unit, in place of those definitions; link -lgdp.
//
// Semantics kept: GaussPy[layer][S+3][len_o][len_o] host arrays, n/length/layer/S globals,
// GaussPyInit refills from data[k<<o][l<<o], GenerateDoG_* leave the finished pyramid (DoG levels
// 0..S+1, Gaussian S+2) in GaussPy and print the elapsed seconds like the collector rank does
// (mpitest.cpp:95-96, :171-172).  The reference's MPI fan-out over S+3 worker ranks is replaced by
// the GPU; the functions can be called repeatedly (no MPI_Init/MPI_Finalize inside).
// GaussPy is two-way state, as in mpitest.cpp, whose GenerateDoG_* multiply and subtract the
// GLOBAL GaussPy in place (:50-56, :89, :128-133, :165): a caller that writes GaussPy between
// GaussPyInit(p) and GenerateDoG_mpi has that edit processed.  With `gdp_mpitest_mirror_host`
// (default true) every GenerateDoG_* uploads what the caller wrote into GaussPy first — the mirror
// is write-tracked like GaussPyramid_hip's (gdp_host_alloc_tracked, round 6): only the pages
// written since the last call, none when nothing was written; the whole mirror when tracking is
// unavailable or `gdp_mpitest_track_writes` is false; staged row gathers when a caller re-seated a
// row pointer — and runs the in-place re-entry pass on it; after the call the result is copied
// back into GaussPy.  With it false the device pyramid is
// the state: GaussPy is refreshed only after GaussPyInit / GenerateDoG_* / gdp_mpitest_SyncHost(),
// and edits reach the device only with `gdp_mpitest_host_dirty = true` (the next call uploads first)
// or gdp_mpitest_SyncDevice().  Only in that mode may a GenerateDoG_* right after GaussPyInit use
// the fused build (GaussPyInit + GenerateDoG in one pass, bit-identical on unedited contents).
// `gdp_mpitest_defer_download = true` (opt-in) replaces the copy back by the deferred download
// (pages fetched from the device when first touched).
// Window centre: mpitest.cpp centres on the INTEGER octave length, `l = float(len - 1) / 2.0`
// (:44, :123), not on GuassDePyramid.h's float-halved length (:107-115); the context uses the same
// (GDP_CENTRE_INTLEN), so the result equals mpitest.cpp's collector for every n — the two centres
// agree for power-of-two n (mpitest.cpp runs n = 256, :548) and differ e.g. for n = 100 (pinned
// against the reference's own runs under mpiexec, tests/golden/mpi_hashes.json).
#ifndef SIFT_GAUSSDEPYRAMID_HIP_MPITEST_H
#define SIFT_GAUSSDEPYRAMID_HIP_MPITEST_H

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "gdp.h"

#ifndef GDP_MPITEST_MAX
#define GDP_MPITEST_MAX 4096  // mpitest.cpp:28
#endif

int thread_count = 4;  // mpitest.cpp:26 (unused on the GPU)
int chunk_size = 5;    // :27 (unused)
const int MAX = GDP_MPITEST_MAX;
int n = 128;  // :29
int S = 2;    // :30
float**** GaussPy;
int length = n;
int layer = 0;
bool is_initialized = false;
static gdp_ctx* gdp_mpitest_ctx = nullptr;
static bool gdp_mpitest_fresh = false;
static float* gdp_mpitest_host = nullptr;  // pinned device-layout mirror the GaussPy rows point into
bool gdp_mpitest_mirror_host = true;  // GaussPy two-way: upload before / download after every GenerateDoG_*
bool gdp_mpitest_host_dirty = false;  // mirror off: the caller edited GaussPy, the next call uploads first
// write tracking of the mirror; set false before GaussPyInit(p) to keep plain
// pinned memory (e.g. when GaussPy is filled by read(2), which fails on a protected page)
bool gdp_mpitest_track_writes = true;
static bool gdp_mpitest_tracked = false;  // gdp_mpitest_host is gdp_host_alloc_tracked memory
static bool gdp_mpitest_armed = false;    // ... protected since it last equalled the device copy
// deferred download (opt-in; needs the tracked mirror): GaussPyInit / GenerateDoG_*
// leave GaussPy's pages to be fetched from the device when first touched instead of copying the
// pyramid back (gdp_host_defer).  Read at every call; a caller that hands GaussPy to system calls
// reading it (write(2) of a row) calls gdp_mpitest_SyncHost() first.
bool gdp_mpitest_defer_download = [] {  // GDP_DEFER_DOWNLOAD=1 in the environment: on from the start
    const char* e = std::getenv("GDP_DEFER_DOWNLOAD");
    return e && e[0] == '1';
}();

static inline void gdp_mpitest_check(int status, const char* what) {
    if (status != GDP_OK) {
        std::fprintf(stderr, "%s failed: %s (%s)\n", what, gdp_status_string(status), gdp_last_error(gdp_mpitest_ctx));
        std::abort();
    }
}

// every GaussPy row still where GaussPyInit put it (a caller may re-seat one: the reference's rows
// are separate new[] arrays, :451-453)
static int gdp_mpitest_rows_memo = -1;  // the walk below, taken once per public call (gdp_mpitest_scope)
static inline bool gdp_mpitest_rows_scan();
static inline bool gdp_mpitest_rows_in_mirror() {
    return gdp_mpitest_rows_memo >= 0 ? gdp_mpitest_rows_memo != 0 : gdp_mpitest_rows_scan();
}
struct gdp_mpitest_scope {  // the caller cannot re-seat a row while one of these functions runs
    bool outer;
    gdp_mpitest_scope() : outer(gdp_mpitest_rows_memo < 0) {
        if (outer) gdp_mpitest_rows_memo = gdp_mpitest_rows_scan() ? 1 : 0;
    }
    ~gdp_mpitest_scope() {
        if (outer) gdp_mpitest_rows_memo = -1;
    }
};
static inline bool gdp_mpitest_rows_scan() {
    if (!gdp_mpitest_host) return false;
    for (int o = 0; o < layer; ++o)
        for (int s = 0; s < S + 3; ++s) {
            const float* lev = gdp_mpitest_host + gdp_level_offset(gdp_mpitest_ctx, 0, o, s);
            const int len = length >> o;
            for (int r = 0; r < len; ++r)
                if (GaussPy[o][s][r] != lev + (size_t)r * len) return false;
        }
    return true;
}

// GaussPy == the device copy now: write-protect the tracked mirror again
static inline void gdp_mpitest_arm() {
    gdp_mpitest_armed = gdp_mpitest_tracked && gdp_mpitest_rows_in_mirror() && gdp_host_arm(gdp_mpitest_host) == GDP_OK;
}

static inline int gdp_mpitest_download() {
    const int rc = gdp_mpitest_rows_in_mirror() ? gdp_download_image_raw(gdp_mpitest_ctx, 0, gdp_mpitest_host)
                                                : gdp_download_pyramid_rows(gdp_mpitest_ctx, 0, GaussPy);
    if (rc == GDP_OK) gdp_mpitest_arm();
    return rc;
}

static inline bool gdp_mpitest_deferring() {
    return gdp_mpitest_defer_download && gdp_mpitest_tracked && gdp_mpitest_rows_in_mirror();
}

// after a call: GaussPy shows the device pyramid — deferred, or copied now
static inline int gdp_mpitest_publish() {
    if (gdp_mpitest_deferring() && gdp_host_defer(gdp_mpitest_ctx, 0, gdp_mpitest_host) == GDP_OK) {
        gdp_mpitest_armed = true;  // pages fetched and then written are recorded from here on
        return GDP_OK;
    }
    return gdp_mpitest_download();
}

// bytes of GaussPy still to be fetched (-1: nothing deferred / not tracked)
inline long long gdp_mpitest_stale_bytes() {
    size_t b = 0;
    return gdp_mpitest_tracked && gdp_host_deferred_stats(gdp_mpitest_host, &b, nullptr, nullptr) == GDP_OK ? (long long)b
                                                                                                          : -1;
}

// GaussPy (the host pyramid, possibly edited) -> the device pyramid now
inline void gdp_mpitest_SyncDevice() {
    gdp_mpitest_scope scope;
    if (!is_initialized) return;
    gdp_mpitest_check(gdp_mpitest_rows_in_mirror()
                          ? gdp_upload_image_raw(gdp_mpitest_ctx, 0, gdp_mpitest_host)
                          : gdp_upload_pyramid_rows(gdp_mpitest_ctx, 0, (const float* const* const* const*)GaussPy),
                      "SyncDevice");
    gdp_mpitest_host_dirty = false;
    gdp_mpitest_fresh = false;  // the caller's contents now, not necessarily GaussPyInit's
    gdp_mpitest_arm();
}

// the device pyramid -> GaussPy now
inline void gdp_mpitest_SyncHost() {
    gdp_mpitest_scope scope;
    if (is_initialized) gdp_mpitest_check(gdp_mpitest_download(), "SyncHost");
}

// :438-473 — first call allocates GaussPy (and the device context); every call refills.
void GaussPyInit(int* data[MAX]) {
    length = n;
    if (!is_initialized) {
        layer = gdp_octaves_for(length);
        gdp_mpitest_check(gdp_create(&gdp_mpitest_ctx, length, length, S, layer, 1, 0), "GaussPyInit");
        gdp_mpitest_check(gdp_set_window_centre(gdp_mpitest_ctx, GDP_CENTRE_INTLEN), "GaussPyInit");
        // the rows (one new float[] each in the reference) point into one pinned buffer in the
        // device layout: every download is a single DMA copy (separate rows if pinning is refused)
        void* h = nullptr;
        const size_t bytes = gdp_image_floats(gdp_mpitest_ctx) * sizeof(float);
        gdp_mpitest_tracked = gdp_mpitest_track_writes && gdp_host_alloc_tracked(bytes, &h) == GDP_OK;
        if (!gdp_mpitest_tracked && gdp_host_alloc(bytes, &h) != GDP_OK) h = nullptr;
        gdp_mpitest_host = static_cast<float*>(h);
        GaussPy = new float***[layer];
        for (int o = 0; o < layer; ++o) {
            GaussPy[o] = new float**[S + 3];
            for (int s = 0; s < S + 3; ++s) {
                GaussPy[o][s] = new float*[length >> o];
                float* lev = gdp_mpitest_host ? gdp_mpitest_host + gdp_level_offset(gdp_mpitest_ctx, 0, o, s) : nullptr;
                for (int r = 0; r < (length >> o); ++r)
                    GaussPy[o][s][r] = lev ? lev + (size_t)r * (length >> o) : new float[length >> o];
            }
        }
    }
    is_initialized = true;
    gdp_mpitest_scope scope;
    gdp_mpitest_armed = false;  // every level is refilled on the device
    gdp_mpitest_check(gdp_set_input_rows(gdp_mpitest_ctx, 0, (const int32_t* const*)data, nullptr), "GaussPyInit");
    gdp_mpitest_check(gdp_init(gdp_mpitest_ctx, nullptr), "GaussPyInit");
    gdp_mpitest_host_dirty = false;  // every level refilled: host edits are overwritten, as in :462-472
    gdp_mpitest_fresh = true;
    gdp_mpitest_check(gdp_mpitest_publish(), "GaussPyInit");
}

static inline void gdp_mpitest_generate() {
    gdp_mpitest_scope scope;
    auto begin = std::chrono::steady_clock::now();
    // the GLOBAL GaussPy is what the reference's workers multiply and its collector subtracts
    // (:128-133, :165): upload it first, then the in-place pass on exactly those contents
    if (gdp_mpitest_mirror_host && gdp_mpitest_rows_in_mirror() && !gdp_mpitest_deferring()) {
        // upload (the written pages only, when armed) + in-place pass + download in one call,
        // pipelined over row chunks
        const bool clean = gdp_mpitest_armed;
        gdp_mpitest_armed = false;
        gdp_mpitest_check(clean ? gdp_generate_dog_mirrored_written(gdp_mpitest_ctx, 0, gdp_mpitest_host)
                                : gdp_generate_dog_mirrored(gdp_mpitest_ctx, 0, gdp_mpitest_host),
                          "GenerateDoG_mpi");
        gdp_mpitest_arm();
        gdp_mpitest_host_dirty = false;
    } else {
        const bool clean = gdp_mpitest_armed;
        gdp_mpitest_armed = false;  // the device changes below; the download / deferral re-arms
        if (gdp_mpitest_mirror_host || gdp_mpitest_host_dirty) {
            if (clean && gdp_mpitest_rows_in_mirror())  // the written pages only (deferred mirrors)
                gdp_mpitest_check(gdp_upload_image_written(gdp_mpitest_ctx, 0, gdp_mpitest_host), "GenerateDoG_mpi");
            else
                gdp_mpitest_SyncDevice();
            gdp_mpitest_host_dirty = false;
            gdp_mpitest_fresh = false;
        }
        gdp_mpitest_check(gdp_mpitest_fresh ? gdp_build(gdp_mpitest_ctx, nullptr) : gdp_generate_dog(gdp_mpitest_ctx, nullptr),
                          "GenerateDoG_mpi");
        gdp_mpitest_check(gdp_sync(gdp_mpitest_ctx), "GenerateDoG_mpi");
        gdp_mpitest_check(gdp_mpitest_publish(), "GenerateDoG_mpi");
    }
    gdp_mpitest_fresh = false;
    auto end = std::chrono::steady_clock::now();
    std::cout << std::chrono::duration<double>(end - begin).count() << std::endl;
}

void GenerateDoG_mpi(int, char**) { gdp_mpitest_generate(); }      // :114-189
void GenerateDoG_mpi_omp(int, char**) { gdp_mpitest_generate(); }  // :35-113

// :474-493
void delete_mpi() {
    if (!is_initialized) return;
    for (int o = 0; o < layer; ++o) {
        for (int s = 0; s < S + 3; ++s) {
            if (!gdp_mpitest_host)
                for (int r = 0; r < (length >> o); ++r) delete[] GaussPy[o][s][r];
            delete[] GaussPy[o][s];
        }
        delete[] GaussPy[o];
    }
    delete[] GaussPy;
    gdp_host_free(gdp_mpitest_host);
    gdp_mpitest_host = nullptr;
    gdp_mpitest_tracked = gdp_mpitest_armed = false;
    gdp_destroy(gdp_mpitest_ctx);
    gdp_mpitest_ctx = nullptr;
    is_initialized = false;
    layer = 0;
}

#endif  // SIFT_GAUSSDEPYRAMID_HIP_MPITEST_H
