// GaussDePyramid-HIP-mpi.h — drop-in for `class GaussPyramid_mpi` (GaussDePyramid-MPI.h:16-53):
// the multi-process variant, with MPI kept only as the launcher/bootstrap and the pyramid built on
// one MI355X per rank and collected over RCCL (xGMI) by libgdp_comm (gdp_comm.h).
//
//     #include "GaussDePyramid-HIP-mpi.h"         // was "GaussDePyramid-MPI.h"
//     GaussPyramid_hip_mpi g(p, n, 2);           // was GaussPyramid_mpi
//     g.GenerateDoG_mpi(argc, argv);             // main.cpp:68, under mpiexec -n <ranks>
//
// Build: g++ -I<repo>/include -I/opt/conda/include main.cpp -L<lib> -lgdp_comm -lgdp
//        -L/opt/conda/lib -lmpi   (any MPI; it only launches ranks and broadcasts 128 bytes)
//
// Semantics.  The reference's GenerateDoG_mpi needs >= S+4 ranks: ranks i < S+3 filter scale i
// of every octave and send each row to rank S+3, the collector, which forms all DoG levels
// (:265-335); the collector's GaussPy ends as the full pyramid.  Two role maps are provided:
//  - ROLES_BANDS (default, `roles`): ANY number of ranks; rank r builds row band
//    gdp_band_rows(n, size, r, layer) of every level on GPU r % devices, and rank 0 — the
//    collector (collector() == 0) — receives every band into its whole-image context
//    (gdp_comm_gather_bands) and mirrors it into GaussPy.  A worker's GaussPy keeps what it held
//    before the call (its band's rows live only in its device band context), where the
//    reference's worker i < S+3 ends holding scale i windowed; no caller in the reference reads a
//    worker's GaussPy (main.cpp:61-74 only times the call).
//  - ROLES_REFERENCE (opt-in; needs >= S+4 ranks, aborts below): the reference's own roles —
//    rank i < S+3 windows scale i of every octave of its own state (gdp_gauss_scales, integer-
//    length centre) and sends it to rank S+3 (gdp_comm_collect_scales), which forms every DoG level
//    (gdp_dog_range); ranks > S+3 take no part.  Every rank's GaussPy then ends where the reference
//    leaves it: worker i with scale i windowed (the other scales untouched), the collector
//    (collector() == S+3) with the pyramid.  Opt-in because each worker builds a whole pyramid
//    (no speed-up over one GPU) and its RCCL transport has not yet run on >= S+4 GPUs; ROLES_AUTO
//    picks it whenever the world has >= S+4 ranks.
// The collector's pyramid is bit-identical to the reference's collector for EVERY n under either
// map: GenerateDoG_mpi centres its windows on the integer octave length (`l = float(len-1)/2`,
// :273 — GDP_CENTRE_INTLEN), while GaussFilter/GenerateDoG use the float-halved centre of
// :134-143 like GuassDePyramid.h (the two differ only when n is not a multiple of 2^(layer-1),
// e.g. n = 100; pinned against the reference's own MPI runs, tests/golden/mpi_hashes.json).
// Repeated calls continue from the current contents, like the reference's in-place methods:
// every call is collective.  With the band map a rank's band starts from the fused build right
// after GaussPyInit, from its own rows of the last GenerateDoG_mpi result (re-entry: the op is
// pointwise, so this equals the collector's whole-pyramid re-entry), or — after single-process
// calls (GaussFilter / GenerateDoG) or host edits — from its own rows of its whole-image state
// (gdp_copy_band).  GaussPy is two-way state, as in the reference (GaussDePyramid-MPI.h:18, the
// float**** every method works on): with `mirror_host` (default) a rank whose GaussPy mirrors its
// device state (every rank after GaussPyInit and the single-process calls, the collector after
// GenerateDoG_mpi) uploads what the caller wrote into it before each mutating call, so edits are
// processed — write-tracked like GaussPyramid_hip's mirror: only the pages
// written since it last equalled the device state, none when nothing was written (which also keeps
// the fused build and the live band rows); a worker's GaussPy is not refreshed by a band
// GenerateDoG_mpi, so it uploads only when the caller sets `host_dirty`.
// In the reference the collector's output depends only on the workers' states (scale i from rank
// i); with the band map on every rank's own rows — the same whenever the ranks hold the same
// GaussPy (SPMD callers).
// Differences: MPI is initialised once (if the caller has not) and finalised by the
// destructor, so GenerateDoG_mpi may be called repeatedly (the reference calls
// MPI_Init/MPI_Finalize inside and cannot); errors abort with a message instead of continuing.
#ifndef SIFT_GAUSSDEPYRAMID_HIP_MPI_H
#define SIFT_GAUSSDEPYRAMID_HIP_MPI_H

#include <mpi.h>

// What a caller of the replaced header gets transitively: GaussDePyramid-MPI.h:8-13 pulls in
// <iostream>, <chrono>, <math.h> and <sys/time.h>, and main.cpp:62-69 relies on <chrono>.
#include <math.h>
#include <sys/time.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "gdp.h"
#include "gdp_comm.h"

class GaussPyramid_hip_mpi {
public:
    int** data;
    GaussPyramid_hip_mpi();
    GaussPyramid_hip_mpi(int** img, int len, int S);
    float**** GaussPy;
    void GaussPyInit();
    void output();
    void GaussFilter(int theLayer);
    void GenerateDoG();
    void GenerateDoG_mpi_normal() {}  // empty in the reference (:337-339)
    void GenerateDoG_mpi(int argc, char** argv);
    // SURVEY.md §8(b)/(f2)'s name for the same entry point: the RCCL counterpart of
    // GenerateDoG_mpi (GaussDePyramid-MPI.h:265), same signature and collector semantics.
    void GenerateDoG_mgpu(int argc, char** argv) { GenerateDoG_mpi(argc, argv); }
    ~GaussPyramid_hip_mpi();
    int thread_count;  // kept for source compatibility (:39-43); unused on the GPU
    int chunk_size;
    int all_time;
    int rank() const { return rank_; }
    enum { ROLES_AUTO = 0, ROLES_BANDS = 1, ROLES_REFERENCE = 2 };
    int roles = ROLES_BANDS;  // see the header comment; decided at the first GenerateDoG_mpi
    int collector() const { return ref_roles_ ? S + 3 : 0; }  // the rank holding the pyramid
    // The role map a world of `world` ranks runs under `roles` (ROLES_AUTO: the reference's from
    // S+4 ranks on) — what the first GenerateDoG_mpi decides; read the pyramid on collector().
    static bool reference_roles(int roles_, int world, int S_) {
        return roles_ == ROLES_REFERENCE || (roles_ == ROLES_AUTO && world >= S_ + 4);
    }
    bool mirror_host = true;  // two-way GaussPy (see the header comment)
    bool host_dirty = false;  // the caller edited GaussPy / data: upload before the next call
    void SyncHost() {
        CallScope scope(this);
        sync_host_();
        host_current_ = true;
    }
    void SyncDevice();        // upload GaussPy into this rank's whole-image state now
    // Deferred download (opt-in, as GaussPyramid_hip::DeferDownload): where GaussPy would be
    // refreshed after a call, its pages are left to be fetched from this rank's whole-image state
    // when first touched.  Returns whether it is on (needs the write-tracked mirror).
    bool DeferDownload(bool on) {
        if (!on && defer_) check_(gdp_host_fetch(host_), "DeferDownload", full_);
        defer_ = on && track_ && host_;
        return defer_;
    }
    long long stale_bytes() const {  // bytes of GaussPy still to be fetched, -1 when not deferring
        size_t b = 0;
        return defer_ && gdp_host_deferred_stats(host_, &b, nullptr, nullptr) == GDP_OK ? (long long)b : -1;
    }

protected:
    int length;
    int S;
    int layer;
    float* filter;
    bool is_initialized;
    gdp_ctx* full_;  // whole-image context: single-process methods and the collector's target
    gdp_ctx* band_;
    gdp_comm* comm_;
    int rank_, size_;
    bool owns_mpi_;
    bool fresh_;      // contents == GaussPyInit() on every rank
    bool band_live_;  // band_ holds this rank's rows of the last GenerateDoG_mpi result
    bool host_current_ = true;  // GaussPy mirrors full_ (false on workers after GenerateDoG_mpi)
    bool ref_roles_ = false;    // the reference's role map is in use (>= S+4 ranks)
    bool band_tried_ = false;   // the band context was planned (band split only)
    // the row walk once per public call (as GaussPyramid_hip's CallScope)
    mutable int rows_memo_ = -1;
    struct CallScope {
        const GaussPyramid_hip_mpi* g;
        bool outer;
        explicit CallScope(const GaussPyramid_hip_mpi* g_) : g(g_), outer(g_->rows_memo_ < 0) {
            if (outer) g->rows_memo_ = g->rows_scan_() ? 1 : 0;
        }
        ~CallScope() {
            if (outer) g->rows_memo_ = -1;
        }
    };
    bool rows_in_mirror_() const { return rows_memo_ >= 0 ? rows_memo_ != 0 : rows_scan_(); }
    bool rows_scan_() const {
        if (!host_) return false;
        for (int o = 0; o < layer; ++o)
            for (int s = 0; s < S + 3; ++s) {
                const float* lev = host_ + gdp_level_offset(full_, 0, o, s);
                const int n = length >> o;
                for (int r = 0; r < n; ++r)
                    if (GaussPy[o][s][r] != lev + (size_t)r * n) return false;
            }
        return true;
    }
    void pull_host_() {  // before a mutating call (the written pages only, when the mirror is armed)
        const bool clean = armed_;
        armed_ = false;  // the call changes the device; SyncHost re-arms
        if (!((mirror_host && host_current_) || host_dirty)) return;
        if (clean && rows_in_mirror_()) {
            size_t w = 0;
            const bool any = gdp_host_written_bytes(host_, &w) != GDP_OK || w > 0;
            check_(gdp_upload_image_written(full_, 0, host_), "SyncDevice", full_);
            host_dirty = false;
            host_current_ = true;
            if (any) fresh_ = band_live_ = false;  // nothing written: the device state is unchanged
            return;
        }
        SyncDevice();
        armed_ = false;
    }
    bool track_ = false;  // host_ is write-tracked (gdp_host_alloc_tracked, GaussDePyramid-HIP.h)
    bool armed_ = false;  // ... and equals full_'s pyramid as of its arming
    bool defer_ = false;  // DeferDownload
    void arm_() {
        armed_ = track_ && rows_in_mirror_() && gdp_host_arm(host_) == GDP_OK;
    }
    // after a call that changed full_ with mirror_host: GaussPy shows it — deferred, or copied now
    void publish_() {
        if (defer_ && rows_in_mirror_() && gdp_host_defer(full_, 0, host_) == GDP_OK) {
            armed_ = true;
            host_current_ = true;
            return;
        }
        SyncHost();
    }
    // before a call that changes full_: a deferred GaussPy that the call will not defer again
    // (`republished` false: mirror off, rows re-seated) is fetched while full_ still holds it
    void keep_deferred_(bool republished) {
        if (defer_ && !(republished && rows_in_mirror_())) check_(gdp_host_fetch(host_), "DeferDownload", full_);
    }
    // the error text is read only after the failing call returned (never as a sibling argument,
    // whose evaluation order relative to the call is unspecified)
    static void check_(int status, const char* what, const gdp_ctx* c) {
        if (status != GDP_OK) {
            std::fprintf(stderr, "GaussPyramid_hip_mpi::%s failed: %s (%s)\n", what, gdp_status_string(status),
                         gdp_last_error(c));
            std::abort();
        }
    }
    static void check_comm_(int status, const char* what, const gdp_comm* c) {
        if (status != GDP_OK) {
            std::fprintf(stderr, "GaussPyramid_hip_mpi::%s failed: %s (%s)\n", what, gdp_status_string(status),
                         gdp_comm_last_error(c));
            std::abort();
        }
    }
    float* host_ = nullptr;  // pinned device-layout mirror the GaussPy rows point into (NULL: new[] rows)
    void sync_host_() {
        check_(rows_in_mirror_() ? gdp_download_image_raw(full_, 0, host_) : gdp_download_pyramid_rows(full_, 0, GaussPy),
               "download", full_);
        arm_();
    }
    void ensure_full_();
};

inline GaussPyramid_hip_mpi::GaussPyramid_hip_mpi()
    : data(nullptr), GaussPy(nullptr), thread_count(8), chunk_size(5), all_time(0), length(0), S(0), layer(0),
      filter(nullptr), is_initialized(false), full_(nullptr), band_(nullptr), comm_(nullptr), rank_(0), size_(1),
      owns_mpi_(false), fresh_(false), band_live_(false) {}

inline GaussPyramid_hip_mpi::GaussPyramid_hip_mpi(int** img, int len, int S_) : GaussPyramid_hip_mpi() {
    length = len;
    S = S_;
    data = new int*[len];
    for (int i = 0; i < len; ++i) {
        data[i] = new int[len];
        for (int j = 0; j < len; ++j) data[i][j] = img[i][j];
    }
    layer = gdp_octaves_for(len);
    filter = new float[len];
    ensure_full_();
    // the rows (one new float[] each in the reference) point into one pinned buffer laid out like
    // the device pyramid: the collector's mirror is a single DMA copy (new[] rows if refused)
    // (write-tracked like GaussPyramid_hip's mirror where available: a call uploads only the pages
    // the caller wrote since the last one)
    void* h = nullptr;
    const size_t mirror_bytes = gdp_image_floats(full_) * sizeof(float);
    if (gdp_host_alloc_tracked(mirror_bytes, &h) == GDP_OK) {
        host_ = static_cast<float*>(h);
        track_ = true;
    } else if (gdp_host_alloc(mirror_bytes, &h) == GDP_OK) {
        host_ = static_cast<float*>(h);
    }
    GaussPy = new float***[layer];
    for (int o = 0; o < layer; ++o) {
        GaussPy[o] = new float**[S + 3];
        for (int s = 0; s < S + 3; ++s) {
            GaussPy[o][s] = new float*[len >> o];
            float* lev = host_ ? host_ + gdp_level_offset(full_, 0, o, s) : nullptr;
            for (int r = 0; r < (len >> o); ++r) GaussPy[o][s][r] = lev ? lev + (size_t)r * (len >> o) : new float[len >> o];
        }
    }
    GaussPyInit();
    if (const char* e = std::getenv("GDP_DEFER_DOWNLOAD"))  // as GaussPyramid_hip
        if (e[0] == '1') DeferDownload(true);
}

// The rank this process will have, also before MPI_Init (main.cpp constructs the pyramid before
// its first GenerateDoG_mpi call): MPI_Comm_rank when MPI is up, else the launcher's environment.
inline int gdp_launcher_rank() {
    int on = 0;
    MPI_Initialized(&on);
    if (on) {
        int r = 0;
        MPI_Comm_rank(MPI_COMM_WORLD, &r);
        return r;
    }
    for (const char* v : {"PMI_RANK", "OMPI_COMM_WORLD_RANK", "PMIX_RANK", "SLURM_PROCID", "RANK"})
        if (const char* e = std::getenv(v)) return std::atoi(e);
    return 0;
}

inline void GaussPyramid_hip_mpi::ensure_full_() {  // the whole-image context on this rank's GPU
    if (full_) return;
    const int ndev = gdp_device_count();
    check_(gdp_create(&full_, length, length, S, layer, 1, ndev > 0 ? gdp_launcher_rank() % ndev : 0), "GaussPyInit",
           nullptr);
    check_(gdp_set_input_rows(full_, 0, (const int32_t* const*)data, nullptr), "GaussPyInit", full_);
}

inline void GaussPyramid_hip_mpi::SyncDevice() {
    CallScope scope(this);
    check_(rows_in_mirror_() ? gdp_upload_image_raw(full_, 0, host_)
                             : gdp_upload_pyramid_rows(full_, 0, (const float* const* const* const*)GaussPy),
           "SyncDevice", full_);
    host_dirty = false;
    host_current_ = true;
    fresh_ = band_live_ = false;  // the caller's contents: bands start from this rank's rows of them
    arm_();
}

inline void GaussPyramid_hip_mpi::GaussPyInit() {  // :87-114 (on this rank's GPU), from the CURRENT `data`
    CallScope scope(this);
    const bool constructing = !is_initialized;  // the constructor just uploaded `data`
    ensure_full_();
    if (!constructing && (mirror_host || host_dirty)) {
        check_(gdp_set_input_rows(full_, 0, (const int32_t* const*)data, nullptr), "GaussPyInit", full_);
        int r0 = 0;  // the band's first input row
        if (band_ && gdp_level_dims(band_, 0, nullptr, nullptr, &r0) == GDP_OK)
            check_(gdp_set_input_rows(band_, 0, (const int32_t* const*)(data + r0), nullptr), "GaussPyInit", band_);
    }
    host_dirty = false;
    keep_deferred_(mirror_host);
    armed_ = false;  // every level is refilled on the device
    check_(gdp_init(full_, nullptr), "GaussPyInit", full_);
    is_initialized = true;
    fresh_ = true;
    band_live_ = false;
    if (mirror_host) publish_();
    else host_current_ = false;
}

inline void GaussPyramid_hip_mpi::GaussFilter(int theLayer) {  // :133-167
    CallScope scope(this);
    keep_deferred_(mirror_host);
    pull_host_();
    check_(gdp_gauss_octave(full_, theLayer, nullptr), "GaussFilter", full_);
    fresh_ = band_live_ = false;
    if (mirror_host) publish_();
    else host_current_ = false;
}

inline void GaussPyramid_hip_mpi::GenerateDoG() {  // :169-183 (single process, current contents)
    CallScope scope(this);
    keep_deferred_(mirror_host);
    pull_host_();
    check_(gdp_generate_dog(full_, nullptr), "GenerateDoG", full_);
    fresh_ = band_live_ = false;
    if (mirror_host) publish_();
    else host_current_ = false;
}

inline void GaussPyramid_hip_mpi::GenerateDoG_mpi(int argc, char** argv) {  // :265-335
    CallScope scope(this);
    int inited = 0;
    MPI_Initialized(&inited);
    if (!inited) {
        MPI_Init(&argc, &argv);
        owns_mpi_ = true;
    }
    MPI_Comm_rank(MPI_COMM_WORLD, &rank_);
    MPI_Comm_size(MPI_COMM_WORLD, &size_);
    const int ndev = gdp_device_count();
    const int device = ndev > 0 ? rank_ % ndev : 0;
    if (!comm_) {
        unsigned char id[GDP_COMM_ID_BYTES] = {0};
        if (rank_ == 0) check_comm_(gdp_comm_unique_id(id), "GenerateDoG_mpi", nullptr);
        MPI_Bcast(id, GDP_COMM_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
        check_comm_(gdp_comm_init(&comm_, id, size_, rank_, device), "GenerateDoG_mpi", nullptr);
        if (roles == ROLES_REFERENCE && size_ < S + 4) {
            std::fprintf(stderr, "GaussPyramid_hip_mpi: the reference's role map needs >= S+4 = %d ranks, have %d\n",
                         S + 4, size_);
            std::abort();
        }
        ref_roles_ = reference_roles(roles, size_, S);
    }
    if (ref_roles_) {  // GaussDePyramid-MPI.h:265-335, role for role
        keep_deferred_(rank_ > S + 3 || mirror_host);  // ranks <= S+3 change full_ below
        pull_host_();
        const int L = S + 3;
        if (rank_ < L) {  // worker: window this rank's scale of every octave (:271-284)
            check_(gdp_set_window_centre(full_, GDP_CENTRE_INTLEN), "GenerateDoG_mpi", full_);
            const int rc = gdp_gauss_scales(full_, rank_, rank_ + 1, 0, layer, nullptr);
            check_(gdp_set_window_centre(full_, GDP_CENTRE_SERIAL), "GenerateDoG_mpi", full_);
            check_(rc, "GenerateDoG_mpi", full_);
        }
        // worker scale i -> collector level (o, i) (:285 / :295-303)
        check_comm_(gdp_comm_collect_scales(comm_, full_, 0, nullptr), "GenerateDoG_mpi", comm_);
        if (rank_ == L) check_(gdp_dog_range(full_, 0, layer, nullptr), "GenerateDoG_mpi", full_);  // :304-318
        check_(gdp_sync(full_), "GenerateDoG_mpi", full_);
        fresh_ = band_live_ = false;
        if (rank_ <= L) {
            if (mirror_host) publish_();
            else host_current_ = false;
        }
        return;
    }
    if (!band_ && !band_tried_) {
        band_tried_ = true;
        int r0, r1;
        check_comm_(gdp_band_rows(length, size_, rank_, layer, &r0, &r1), "GenerateDoG_mpi", nullptr);
        if (r1 > r0) {  // more ranks than aligned bands leaves the last ranks without rows
            check_(gdp_create_band(&band_, length, length, S, layer, 1, r0, r1, device), "GenerateDoG_mpi",
                   nullptr);
            // the variant's window centre (GaussDePyramid-MPI.h:273), see the header comment
            check_(gdp_set_window_centre(band_, GDP_CENTRE_INTLEN), "GenerateDoG_mpi", band_);
            check_(gdp_set_input_rows(band_, 0, (const int32_t* const*)(data + r0), nullptr), "GenerateDoG_mpi",
                   band_);
        }
    }
    keep_deferred_(rank_ != 0 || mirror_host);  // the gather changes rank 0's full_ only
    pull_host_();
    // every rank takes the same (collective) path; only where its band starts from differs
    if (band_) {
        if (fresh_) {
            check_(gdp_build(band_, nullptr), "GenerateDoG_mpi", band_);
        } else {
            if (!band_live_)  // single-process calls or host edits since: this rank's rows of full_
                check_(gdp_copy_band(band_, 0, full_, 0, nullptr), "GenerateDoG_mpi", band_);
            check_(gdp_generate_dog(band_, nullptr), "GenerateDoG_mpi", band_);
        }
    }
    check_comm_(gdp_comm_gather_bands(comm_, band_, 0, rank_ == 0 ? full_ : nullptr, 0, 0, nullptr), "GenerateDoG_mpi",
                comm_);
    fresh_ = false;
    band_live_ = true;
    if (rank_ == 0 && mirror_host) publish_();
    else host_current_ = false;  // workers: the result rows live in the band context
}

inline void GaussPyramid_hip_mpi::output() {  // :116-131
    int len = length;
    for (int i = 0; i < layer; ++i) {
        for (int j = 0; j < len; ++j) {
            for (int k = 0; k < len; ++k) std::cout << GaussPy[i][0][j][k] << " ";
            std::cout << std::endl;
        }
        for (int k = 0; k < len; ++k) std::cout << "==";
        std::cout << std::endl;
        len /= 2;
    }
}

inline GaussPyramid_hip_mpi::~GaussPyramid_hip_mpi() {
    if (GaussPy) {
        for (int o = 0; o < layer; ++o) {
            for (int s = 0; s < S + 3; ++s) {
                if (!host_)
                    for (int r = 0; r < (length >> o); ++r) delete[] GaussPy[o][s][r];
                delete[] GaussPy[o][s];
            }
            delete[] GaussPy[o];
        }
        delete[] GaussPy;
    }
    gdp_host_free(host_);
    if (data) {
        for (int i = 0; i < length; ++i) delete[] data[i];
        delete[] data;
    }
    delete[] filter;
    gdp_comm_destroy(comm_);
    gdp_destroy(band_);
    gdp_destroy(full_);
    if (owns_mpi_) {
        int fin = 0;
        MPI_Finalized(&fin);
        if (!fin) MPI_Finalize();
    }
}

#endif  // SIFT_GAUSSDEPYRAMID_HIP_MPI_H
