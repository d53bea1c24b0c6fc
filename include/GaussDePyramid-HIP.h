// GaussDePyramid-HIP.h — drop-in MI355X replacement for the reference's pyramid classes.
//
// Usage is the reference's own (main.cpp:2-13, 61-74): swap the #include line and the class name,
//     #include "GaussDePyramid-HIP.h"
//     GaussPyramid_hip g(p, n, 2);
//     g.GenerateDoG();            // GaussFilter + DoG of every octave on the GPU
//     g.GaussPy[o][s][r][c] ...   // host float**** mirror, as in GuassDePyramid.h:16
// and link with -lgdp (libgdp.so, sift-parallel-optimization_amd/lib).  The class mirrors
// `class GaussPyramid` (GuassDePyramid.h:11-29) member for member; every method is a thin
// caller of the C ABI in gdp.h.  Host code only: this header needs no HIP headers and compiles
// with plain g++.
//
// Semantics kept from the reference:
//  - the constructor deep-copies img[0:len][0:len] and calls GaussPyInit() (:36-58);
//  - GaussPyInit() refills every level with the decimated input (:60-87);
//  - GaussFilter(o) window-multiplies every scale of octave o in place (:106-134);
//  - GenerateDoG() = GaussFilter + DoG per octave on the CURRENT contents (:136-149), so calling
//    it twice without GaussPyInit() filters twice, like the timing loop of main.cpp:66-73;
//  - GaussPy holds [layer][S+3][len_o][len_o] floats allocated with new[] (:63-72), freed by the
//    destructor (:151-170).
// GaussPy is two-way state, as in the reference, where the float**** IS the pyramid and every
// method works on whatever the caller left in it (:16, :122-131, :140-146):
//  - mirror_host = true (default): before each mutating call (GaussFilter, GenerateDoG,
//    GenerateDoG_mpi) the host GaussPy is uploaded to the device, and after it the device pyramid
//    is copied back into GaussPy; GaussPyInit re-reads `data` (:80).  A caller may write
//    g.GaussPy[o][s][r][c] (or g.data[r][c]) at any time and the next call processes the edit.
//    Cost: the upload is only of what the caller wrote.  The mirror (gdp_host_alloc_tracked: the
//    pages GaussPy points into, DMA'd through a second, registered mapping of the same memory) is
//    write-protected whenever it equals the device copy (gdp_host_arm); a CPU write to a page
//    faults once and is recorded, and the next mutating call uploads only the written pages
//    (gdp_upload_image_written, gdp_generate_dog_mirrored_written) — none in main.cpp's loop
//    (:66-73), which never writes GaussPy.  The D2H copy back is one per call (447 MB at 4096^2,
//    INTEGRATION §2c); GenerateDoG / GenerateDoG_mpi overlap it with the kernel over row chunks
//    (best-effort: the copy streams share the process's hardware queues — 4 on the MI355X boxes —
//    with every other stream and context, so under concurrent work they may serialise; the result
//    is the same either way).
//    Writes that do not fault on the CPU (read(2) into GaussPy — EFAULT on a protected page —, or
//    DMA into it) are not seen: call TrackWrites(false) first, and every call uploads the whole
//    mirror as before (also the fallback when page protection is unavailable).
//    DeferDownload(true) (opt-in; or GDP_DEFER_DOWNLOAD=1 in the environment): the copy back is deferred too — after a mutating call GaussPy's
//    pages are inaccessible and the first access to one fetches its neighbourhood from the device
//    (gdp_host_defer); main.cpp's loop then moves nothing over PCIe.  Reads see the same values.
//  - mirror_host = false: the device pyramid is the state; GaussPy is refreshed only by
//    SyncHost(), and host edits reach the device only through SyncDevice() — or set
//    `host_dirty = true` after editing and the next mutating call uploads first (then clears it).
// Row pointers the caller re-seated (GaussPy[o][s][r] = other array) are honoured both ways: the
// single raw DMA copy is used only while every row still points into the pinned mirror.
// Errors: the reference never reports them; a failing libgdp call here prints gdp_last_error()
// and aborts rather than continuing on bad state.
#ifndef SIFT_GAUSSDEPYRAMID_HIP_H
#define SIFT_GAUSSDEPYRAMID_HIP_H

// What a caller of the replaced header gets transitively: GaussDePyramid-MPI.h:8-13 pulls in
// <iostream>, <chrono>, <math.h> and <sys/time.h>, and main.cpp:62-69 relies on <chrono>.
#include <math.h>
#include <sys/time.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include "gdp.h"

class GaussPyramid_hip {
public:
    int** data;  // copy of the input image (:13)
    GaussPyramid_hip();
    GaussPyramid_hip(int** img, int len, int S, int device = 0);
    float**** GaussPy;  // [layer][S+3][len_o][len_o] host mirror (:16)
    void GaussPyInit();
    void output();
    void GaussFilter(int theLayer);
    void GenerateDoG();
    // GaussPyramid_mpi::GenerateDoG_mpi (GaussDePyramid-MPI.h:265-335), the call main.cpp:68 makes.
    // The reference fans scales out over >= S+4 MPI ranks and collects on rank S+3; here one GPU
    // does the whole pyramid and GaussPy ends as that collector's GaussPy.  Like the method it
    // replaces, it centres every window on the INTEGER octave length (`l = float(len - 1) / 2.0`,
    // :273 — GDP_CENTRE_INTLEN), not on the float-halved length GaussFilter/GenerateDoG use
    // (:133-183, GuassDePyramid.h:107-115); the two differ when n is not a multiple of
    // 2^(layer-1) (n = 100, 1000, ...).  The context returns to the serial centre afterwards, so
    // GaussFilter/GenerateDoG keep theirs.  Unlike the reference (MPI_Init/MPI_Finalize inside)
    // it may be called any number of times; each call continues from the current contents.
    void GenerateDoG_mpi(int argc, char** argv);
    void GenerateDoG_mgpu(int argc, char** argv) { GenerateDoG_mpi(argc, argv); }  // SURVEY §8(f2) name
    ~GaussPyramid_hip();
    bool initialized;
    bool mirror_host;  // GaussPy two-way: upload before / download after every mutating call (default true)
    bool host_dirty;   // mirror_host == false: the caller edited GaussPy / data; the next call uploads first
    void SyncHost();   // copy the device pyramid into GaussPy now
    void SyncDevice(); // copy GaussPy (the host pyramid, possibly edited) into the device pyramid now
    // Write tracking of the mirror (default on when pinned memory and page protection are
    // available): off, every mutating call uploads the whole mirror (see the header comment).
    void TrackWrites(bool on);
    bool tracking_writes() const { return track_; }
    // Bytes of GaussPy in pages written since the mirror was last armed (the next call's upload),
    // or -1 when no such record exists (not tracked / not armed: the next call uploads everything).
    long long written_bytes() const {
        size_t b = 0;
        return track_ && armed_ && gdp_host_written_bytes(host_, &b) == GDP_OK ? (long long)b : -1;
    }
    // Deferred download (opt-in, needs the write-tracked mirror): with mirror_host, a mutating call
    // leaves GaussPy's pages inaccessible instead of copying the device pyramid back, and the first
    // access to one has its neighbourhood fetched (gdp_host_defer).  A caller that does not read
    // GaussPy between calls — main.cpp's timing loop (:66-73) — moves nothing over PCIe; one that
    // reads it gets the same values as with the eager copy.  Off (the default), or for a caller
    // that hands GaussPy to system calls (write(2) of a deferred page fails with EFAULT) or straight
    // to HIP copies: call SyncHost() / DeferDownload(false) before those.  Returns whether it is on.
    bool DeferDownload(bool on);
    bool deferring() const { return defer_; }
    // Bytes of GaussPy still to be fetched (inaccessible pages), or -1 when not deferring.
    long long stale_bytes() const {
        size_t b = 0;
        return defer_ && gdp_host_deferred_stats(host_, &b, nullptr, nullptr) == GDP_OK ? (long long)b : -1;
    }
    gdp_ctx* context() const { return ctx_; }

protected:
    int length;
    int S;
    int layer;
    float* filter;  // unused (taps live on the device); kept for layout parity with :28
    gdp_ctx* ctx_;
    bool fresh_;  // contents == GaussPyInit(): GenerateDoG may use the fused build kernel
    float* host_; // pinned host pyramid in the device layout that the GaussPy rows point into
                  // (gdp_host_alloc); NULL: rows are separate new[] arrays (pinned memory refused)
    bool track_;  // host_ is write-tracked (gdp_host_track)
    bool armed_;  // the device pyramid equals host_ as of its last arming and the pages written
                  // since are recorded: the next mutating call may upload only those
    bool defer_;  // DeferDownload: mutating calls end in gdp_host_defer instead of SyncHost
    // rows_in_mirror_() is a walk over every row pointer (41k at 4096^2, tens of microseconds):
    // each public call takes it once (CallScope) and its helpers reuse the answer — the caller
    // cannot re-seat a row while one of its calls runs
    mutable int rows_memo_ = -1;
    mutable int call_depth_ = 0;
    struct CallScope {
        const GaussPyramid_hip* g;
        explicit CallScope(const GaussPyramid_hip* g_) : g(g_) {
            if (g->call_depth_++ == 0) g->rows_memo_ = g->rows_scan_() ? 1 : 0;
        }
        ~CallScope() {
            if (--g->call_depth_ == 0) g->rows_memo_ = -1;
        }
    };
    bool rows_in_mirror_() const { return rows_memo_ >= 0 ? rows_memo_ != 0 : rows_scan_(); }
    bool rows_scan_() const {  // every GaussPy row still where the constructor put it
        if (!host_) return false;
        for (int o = 0; o < layer; ++o)
            for (int s = 0; s < S + 3; ++s) {
                const float* lev = host_ + gdp_level_offset(ctx_, 0, o, s);
                const int n = length >> o;
                for (int r = 0; r < n; ++r)
                    if (GaussPy[o][s][r] != lev + (size_t)r * n) return false;
            }
        return true;
    }
    void keep_deferred_() {  // before a mutating call: a deferred GaussPy that the call will not
        // defer again (mirror_host off, rows re-seated) is fetched now, while the device still
        // holds what it shows
        if (defer_ && !(mirror_host && rows_in_mirror_())) check_(ctx_, gdp_host_fetch(host_), "DeferDownload");
    }
    void pull_host_() {  // before a mutating call: the caller's GaussPy is the state
        keep_deferred_();
        const bool clean = armed_;
        armed_ = false;  // the call changes the device; SyncHost re-arms
        if (!(mirror_host || host_dirty)) return;
        if (clean && rows_in_mirror_())
            check_(ctx_, gdp_upload_image_written(ctx_, 0, host_), "SyncDevice");
        else
            upload_();
        host_dirty = false;
        fresh_ = false;  // the contents are the caller's now, not necessarily GaussPyInit's
    }
    void upload_() {  // the whole mirror: one H2D DMA copy, or staged row gathers
        check_(ctx_, rows_in_mirror_() ? gdp_upload_image_raw(ctx_, 0, host_)
                                       : gdp_upload_pyramid_rows(ctx_, 0, (const float* const* const* const*)GaussPy),
               "SyncDevice");
    }
    void arm_() {  // host_ == the device copy now: protect it again (or stop tracking if refused)
        armed_ = false;
        if (!track_ || !rows_in_mirror_()) return;
        if (gdp_host_arm(host_) == GDP_OK) {
            armed_ = true;
        } else {
            (void)gdp_host_untrack(host_);
            track_ = false;
        }
    }
    int mirrored_call_() {  // gdp_generate_dog_mirrored(_written) on host_, the status returned
        const bool clean = armed_;
        armed_ = false;
        return clean ? gdp_generate_dog_mirrored_written(ctx_, 0, host_) : gdp_generate_dog_mirrored(ctx_, 0, host_);
    }
    void mirrored_done_() {  // after a successful mirrored call: host_ == the device copy
        host_dirty = false;
        fresh_ = false;
        arm_();
    }
    void mirrored_(const char* what) {
        check_(ctx_, mirrored_call_(), what);
        mirrored_done_();
    }
    bool piped_() const { return mirror_host && !defer_ && rows_in_mirror_(); }  // the mirrored single call
    void publish_() {  // after a mutating call with mirror_host: GaussPy shows the device pyramid
        if (defer_ && rows_in_mirror_() && gdp_host_defer(ctx_, 0, host_) == GDP_OK) {
            armed_ = true;  // pages fetched and then written are recorded from here on
            return;
        }
        SyncHost();
    }
    static void check_(gdp_ctx* c, int status, const char* what) {
        if (status != GDP_OK) {
            std::fprintf(stderr, "GaussPyramid_hip::%s failed: %s (%s)\n", what, gdp_status_string(status),
                         gdp_last_error(c));
            std::abort();
        }
    }
};

inline GaussPyramid_hip::GaussPyramid_hip()
    : data(nullptr), GaussPy(nullptr), initialized(false), mirror_host(true), host_dirty(false), length(0), S(0),
      layer(0), filter(nullptr), ctx_(nullptr), fresh_(false), host_(nullptr), track_(false), armed_(false),
      defer_(false) {}

inline GaussPyramid_hip::GaussPyramid_hip(int** img, int len, int S_, int device)
    : data(nullptr), GaussPy(nullptr), initialized(false), mirror_host(true), host_dirty(false), length(len), S(S_),
      layer(0), filter(nullptr), ctx_(nullptr), fresh_(false), host_(nullptr), track_(false), armed_(false),
      defer_(false) {
    data = new int*[len];
    for (int i = 0; i < len; ++i) {
        data[i] = new int[len];
        for (int j = 0; j < len; ++j) data[i][j] = img[i][j];
    }
    layer = gdp_octaves_for(len);  // :48-53
    filter = new float[len];
    check_(nullptr, gdp_create(&ctx_, len, len, S, layer, 1, device), "GaussPyramid_hip");
    check_(ctx_, gdp_set_input_rows(ctx_, 0, (const int32_t* const*)data, nullptr), "GaussPyramid_hip");
    // The GaussPy rows (:16, one new float[] per row in the reference) point into ONE pinned host
    // buffer laid out like the device pyramid, so SyncHost is a single DMA copy at the full PCIe
    // rate; if pinned memory is refused, separate rows and the staged scatter are used instead.
    void* h = nullptr;
    // Write-tracked when the platform allows it (gdp_host_alloc_tracked: a registered DMA view and a
    // protectable CPU view of the same pages), else plain pinned memory and whole uploads.
    const size_t mirror_bytes = gdp_image_floats(ctx_) * sizeof(float);
    if (gdp_host_alloc_tracked(mirror_bytes, &h) == GDP_OK) {
        host_ = static_cast<float*>(h);
        track_ = true;
    } else if (gdp_host_alloc(mirror_bytes, &h) == GDP_OK) {
        host_ = static_cast<float*>(h);
    }
    GaussPy = new float***[layer];
    for (int o = 0; o < layer; ++o) {
        const int n = len >> o;
        GaussPy[o] = new float**[S + 3];
        for (int s = 0; s < S + 3; ++s) {
            GaussPy[o][s] = new float*[n];
            float* lev = host_ ? host_ + gdp_level_offset(ctx_, 0, o, s) : nullptr;
            for (int r = 0; r < n; ++r) GaussPy[o][s][r] = lev ? lev + (size_t)r * n : new float[n];
        }
    }
    check_(ctx_, gdp_init(ctx_, nullptr), "GaussPyramid_hip");  // GaussPyInit (:57); `data` just uploaded
    initialized = true;
    fresh_ = true;
    if (mirror_host) SyncHost();
    // GDP_DEFER_DOWNLOAD=1 in the environment turns the deferred download on for an unmodified
    // caller (main.cpp after the two-line switch)
    if (const char* e = std::getenv("GDP_DEFER_DOWNLOAD"))
        if (e[0] == '1') DeferDownload(true);
}

inline void GaussPyramid_hip::SyncHost() {  // one DMA copy (pinned mirror) or one staged copy per 64 MiB
    CallScope scope(this);
    check_(ctx_, rows_in_mirror_() ? gdp_download_image_raw(ctx_, 0, host_) : gdp_download_pyramid_rows(ctx_, 0, GaussPy),
           "SyncHost");
    arm_();
}

inline void GaussPyramid_hip::SyncDevice() {  // the inverse: the whole mirror, one H2D DMA copy or staged row gathers
    CallScope scope(this);
    upload_();
    host_dirty = false;
    fresh_ = false;  // the contents are the caller's now, not necessarily GaussPyInit's
    arm_();
}

inline void GaussPyramid_hip::TrackWrites(bool on) {
    CallScope scope(this);
    if (!on && track_) {
        check_(ctx_, gdp_host_untrack(host_), "TrackWrites");  // fetched if deferred; every page writable again
        track_ = armed_ = defer_ = false;
    } else if (on && !track_ && host_) {
        // armed by the next SyncHost (every mutating call with mirror_host ends in one)
        track_ = gdp_host_track(host_, gdp_image_floats(ctx_) * sizeof(float)) == GDP_OK;
    }
}

inline bool GaussPyramid_hip::DeferDownload(bool on) {
    CallScope scope(this);
    if (!on && defer_) check_(ctx_, gdp_host_fetch(host_), "DeferDownload");  // GaussPy complete again
    defer_ = on && track_ && host_;  // takes effect from the next mutating call
    return defer_;
}

inline void GaussPyramid_hip::GaussPyInit() {  // :60-87, from the CURRENT `data` (:80)
    CallScope scope(this);
    keep_deferred_();
    armed_ = false;  // every level is refilled on the device
    if (mirror_host || host_dirty)
        check_(ctx_, gdp_set_input_rows(ctx_, 0, (const int32_t* const*)data, nullptr), "GaussPyInit");
    host_dirty = false;  // every level is refilled: host edits of GaussPy are overwritten, as in :76-86
    check_(ctx_, gdp_init(ctx_, nullptr), "GaussPyInit");
    initialized = true;
    fresh_ = true;
    if (mirror_host) publish_();
}

inline void GaussPyramid_hip::GaussFilter(int theLayer) {
    CallScope scope(this);
    pull_host_();
    check_(ctx_, gdp_gauss_octave(ctx_, theLayer, nullptr), "GaussFilter");
    fresh_ = false;
    if (mirror_host) publish_();
}

inline void GaussPyramid_hip::GenerateDoG() {
    CallScope scope(this);
    if (piped_()) {
        // GaussPy mirrored in the pinned device-layout buffer: upload (only the pages written since
        // the last call when tracked), in-place pass and download in one call, pipelined over row
        // chunks
        mirrored_("GenerateDoG");
        return;
    }
    // on freshly initialised contents the fused single-pass build is bit-identical to
    // GaussFilter + DoG in place; otherwise run the in-place pass on what is there
    pull_host_();
    check_(ctx_, fresh_ ? gdp_build(ctx_, nullptr) : gdp_generate_dog(ctx_, nullptr), "GenerateDoG");
    fresh_ = false;
    check_(ctx_, gdp_sync(ctx_), "GenerateDoG");
    if (mirror_host) publish_();
}

inline void GaussPyramid_hip::GenerateDoG_mpi(int, char**) {
    CallScope scope(this);
    // switching centres selects the other device tap table (no drain, no re-upload after the
    // first call); both calls below are ordered on the context's stream
    const bool piped = piped_();  // see GenerateDoG
    if (!piped) pull_host_();
    check_(ctx_, gdp_set_window_centre(ctx_, GDP_CENTRE_INTLEN), "GenerateDoG_mpi");
    if (piped) {
        const int rc = mirrored_call_();
        check_(ctx_, gdp_set_window_centre(ctx_, GDP_CENTRE_SERIAL), "GenerateDoG_mpi");
        check_(ctx_, rc, "GenerateDoG_mpi");
        mirrored_done_();
        return;
    }
    const int rc = fresh_ ? gdp_build(ctx_, nullptr) : gdp_generate_dog(ctx_, nullptr);
    check_(ctx_, gdp_set_window_centre(ctx_, GDP_CENTRE_SERIAL), "GenerateDoG_mpi");
    check_(ctx_, rc, "GenerateDoG_mpi");
    fresh_ = false;
    check_(ctx_, gdp_sync(ctx_), "GenerateDoG_mpi");
    if (mirror_host) publish_();
}

inline void GaussPyramid_hip::output() {  // :89-104
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

inline GaussPyramid_hip::~GaussPyramid_hip() {
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
    gdp_destroy(ctx_);
}

#endif  // SIFT_GAUSSDEPYRAMID_HIP_H
