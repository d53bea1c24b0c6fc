// libgdp_comm.so — RCCL collector for row-band pyramids (include/gdp_comm.h).
// Host-only code (no kernels): RCCL grouped point-to-point transfers of finished band levels
// into the collector's whole-image context, plus the band arithmetic shared with bench.py /
// distributed.py (plan_band, band_level_rows).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "gdp_comm.h"

struct gdp_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    // A grouped transfer failed: the group was closed (ncclGroupEnd) but the peers may still wait
    // for this rank's half of it, so the communicator is unusable — every later collective on it
    // returns GDP_ERR_STATE at once, and gdp_comm_destroy aborts it instead of a (possibly
    // blocking) ncclCommDestroy.
    bool failed = false;
    int inject = 0;  // gdp_comm_test_inject_fault: the next group adds a send to an invalid peer
    std::string err;
};

namespace {
thread_local std::string g_comm_error;

int fail(gdp_comm* c, int code, const std::string& m) {
    if (c)
        c->err = m;
    else
        g_comm_error = m;
    return code;
}

// Inside ncclGroupStart() .. ncclGroupEnd(): a failing ncclSend / ncclRecv must still close the
// group, or every later RCCL call of this thread is swallowed by the open group.
#define GDP_NCCL_IN_GROUP(c, call)                                                                        \
    do {                                                                                                  \
        ncclResult_t r_ = (call);                                                                         \
        if (r_ != ncclSuccess) return group_fail((c), std::string(#call ": ") + ncclGetErrorString(r_));   \
    } while (0)
#define GDP_HIPC(c, call)                                                                                 \
    do {                                                                                                  \
        hipError_t e_ = (call);                                                                           \
        if (e_ != hipSuccess) return fail((c), GDP_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)

// Close the open group after a failed transfer and mark the communicator failed.
int group_fail(gdp_comm* c, const std::string& m) {
    const ncclResult_t e = ncclGroupEnd();
    c->failed = true;
    return fail(c, GDP_ERR_HIP, m + (e == ncclSuccess ? "" : std::string("; ncclGroupEnd: ") + ncclGetErrorString(e)) +
                                    " (group closed; communicator marked failed)");
}
// Entry check of every collective: a communicator that failed earlier is refused, never reused.
int refuse_failed(gdp_comm* c, const char* who) {
    return fail(c, GDP_ERR_STATE, std::string(who) + ": an earlier collective on this communicator failed ("
                                      + c->err + "); destroy it and create a new one");
}
// Open a group; with a test fault armed, its first transfer targets peer `nranks` (invalid).
int group_start(gdp_comm* c, hipStream_t st) {
    const ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) {
        c->failed = true;
        return fail(c, GDP_ERR_HIP, std::string("ncclGroupStart: ") + ncclGetErrorString(r));
    }
    if (c->inject) {
        c->inject = 0;
        static float dummy_dev_ptr_unused;  // never dereferenced: RCCL rejects the peer first
        GDP_NCCL_IN_GROUP(c, ncclSend(&dummy_dev_ptr_unused, 1, ncclFloat, c->nranks, c->comm, st));
    }
    return GDP_OK;
}
int group_end(gdp_comm* c) {
    const ncclResult_t r = ncclGroupEnd();
    if (r != ncclSuccess) {
        c->failed = true;
        return fail(c, GDP_ERR_HIP, std::string("ncclGroupEnd: ") + ncclGetErrorString(r) + " (communicator marked failed)");
    }
    return GDP_OK;
}

int band_align(int octaves) { return 1 << (std::max(octaves, 5) - 1); }

// (first global row, rows) of octave o for the band [r0, r1) of an H-row image — gdp_level_dims
// of a band context, computed for any rank without its context.
void band_level(int H, int o, int r0, int r1, int* first, int* rows) {
    const int Hg = H >> o;
    *first = (r0 + (1 << o) - 1) >> o;
    const int hi = (r1 == H) ? Hg : std::min(Hg, (r1 + (1 << o) - 1) >> o);
    *rows = std::max(0, hi - *first);
}
// The collector's schedule (gdp_comm_plan): a non-root rank sends each non-empty level of its
// band, octave-major then scale; the root posts, for every other rank in rank order, the matching
// receives in the same order, then copies its own band's levels.
std::vector<gdp_transfer> make_plan(int H, int W, int S, int O, int nranks, int rank, int root) {
    std::vector<gdp_transfer> plan;
    const int L = S + 3;
    auto band_levels = [&](int r, int kind, int peer) {
        int r0 = 0, r1 = 0;
        gdp_band_rows(H, nranks, r, O, &r0, &r1);
        if (r1 <= r0) return;
        for (int o = 0; o < O; ++o) {
            int first, rows;
            band_level(H, o, r0, r1, &first, &rows);
            for (int s = 0; s < L && rows > 0; ++s) plan.push_back({kind, peer, o, s, first, rows, W >> o});
        }
    };
    if (rank != root) {
        band_levels(rank, GDP_XFER_SEND, root);
        return plan;
    }
    for (int r = 0; r < nranks; ++r)
        if (r != root) band_levels(r, GDP_XFER_RECV, r);
    band_levels(root, GDP_XFER_COPY, root);
    return plan;
}

// The reference's role map (gdp_comm_scale_plan): worker i < L sends level (o, i) of every octave
// to collector L; the collector receives worker-major, then octave.
int make_scale_plan(int S, int O, int nranks, int rank, std::vector<gdp_scale_transfer>& plan) {
    const int L = S + 3;
    if (nranks < L + 1) return GDP_ERR_ARG;
    if (rank < L) {
        for (int o = 0; o < O; ++o) plan.push_back({GDP_SCALE_SEND, L, o, rank});
    } else if (rank == L) {
        for (int j = 0; j < L; ++j)
            for (int o = 0; o < O; ++o) plan.push_back({GDP_SCALE_RECV, j, o, j});
    }
    return GDP_OK;
}

// The halo exchange schedule (gdp_comm_halo_plan): rows a band's convolution reads beyond it are
// 6 * 2^(O-1) clipped to the image (gdp_conv_halo_rows), exchanged with the adjacent bands.
int halo_counts_side(int H, int O, int r0, int r1, int side) {
    const int hh = 6 << (O - 1);
    return side == 0 ? std::min(hh, r0) : std::min(hh, H - r1);
}
int make_halo_plan(int H, int nranks, int rank, int O, std::vector<gdp_halo_transfer>& plan) {
    int r0 = 0, r1 = 0;
    gdp_band_rows(H, nranks, rank, O, &r0, &r1);
    if (r1 <= r0) return GDP_OK;
    if (rank > 0 && r0 > 0) {
        int p0 = 0, p1 = 0;
        gdp_band_rows(H, nranks, rank - 1, O, &p0, &p1);
        const int need = halo_counts_side(H, O, p0, p1, 1), mine = halo_counts_side(H, O, r0, r1, 0);
        if (need > r1 - r0 || mine > p1 - p0) return GDP_ERR_ARG;
        plan.push_back({GDP_HALO_SEND, rank - 1, 0, need});
        plan.push_back({GDP_HALO_RECV_ABOVE, rank - 1, 0, mine});
    }
    if (r1 < H) {
        int n0 = 0, n1 = 0;
        gdp_band_rows(H, nranks, rank + 1, O, &n0, &n1);
        const int need = halo_counts_side(H, O, n0, n1, 0), mine = halo_counts_side(H, O, r0, r1, 1);
        if (need > r1 - r0 || mine > n1 - n0) return GDP_ERR_ARG;
        plan.push_back({GDP_HALO_SEND, rank + 1, r1 - r0 - need, need});
        plan.push_back({GDP_HALO_RECV_BELOW, rank + 1, 0, mine});
    }
    return GDP_OK;
}

int fail_nothrow(gdp_comm* c, int code, const char* m) noexcept {
    try {
        return fail(c, code, m);
    } catch (...) {
        return code;
    }
}
// no C++ exception crosses the C ABI (std::bad_alloc -> GDP_ERR_NOMEM, others -> GDP_ERR_INTERNAL)
#define GDP_COMM_CATCH(c)                                                                                  \
    catch (const std::bad_alloc&) { return fail_nothrow((c), GDP_ERR_NOMEM, "host allocation failed"); }    \
    catch (const std::exception& e_) { return fail_nothrow((c), GDP_ERR_INTERNAL, e_.what()); }            \
    catch (...) { return fail_nothrow((c), GDP_ERR_INTERNAL, "unknown C++ exception"); }
}  // namespace

extern "C" {

int gdp_band_rows(int H, int nranks, int rank, int octaves, int* row_begin, int* row_end) try {
    if (H <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || octaves <= 0 || !row_begin || !row_end)
        return GDP_ERR_ARG;
    // per = ceil(ceil(H / nranks) / align) * align — distributed.plan_band, same numbers
    const long long align = band_align(octaves);
    const long long hn = ((long long)H + nranks - 1) / nranks;
    const long long per = (hn + align - 1) / align * align;
    *row_begin = (int)std::min<long long>(H, (long long)rank * per);
    *row_end = (int)std::min<long long>(H, (long long)(rank + 1) * per);
    return GDP_OK;
} GDP_COMM_CATCH(nullptr)

int gdp_comm_unique_id(unsigned char id[GDP_COMM_ID_BYTES]) try {
    static_assert(sizeof(ncclUniqueId) == GDP_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(nullptr, GDP_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id, &u, sizeof u);
    return GDP_OK;
} GDP_COMM_CATCH(nullptr)

int gdp_comm_init(gdp_comm** out, const unsigned char id[GDP_COMM_ID_BYTES], int nranks, int rank, int device) try {
    if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks) return fail(nullptr, GDP_ERR_ARG, "gdp_comm_init: bad argument");
    *out = nullptr;
    gdp_comm* c = new (std::nothrow) gdp_comm();
    if (!c) return fail(nullptr, GDP_ERR_NOMEM, "host allocation failed");
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete c;
        return fail(nullptr, GDP_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(nullptr, GDP_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    *out = c;
    return GDP_OK;
} GDP_COMM_CATCH(nullptr)

void gdp_comm_destroy(gdp_comm* c) {
    if (!c) return;
    // a failed communicator may have operations its peers never matched: abort, do not wait
    if (c->comm) (void)(c->failed ? ncclCommAbort(c->comm) : ncclCommDestroy(c->comm));
    delete c;
}

int gdp_comm_failed(const gdp_comm* c) { return c ? (c->failed ? 1 : 0) : -1; }

int gdp_comm_test_inject_fault(gdp_comm* c) try {
    if (!c) return GDP_ERR_ARG;
    c->inject = 1;
    return GDP_OK;
} GDP_COMM_CATCH(c)

int gdp_comm_check(gdp_comm* c, void* stream) try {
    // ring: rank r sends kWords words of r to (r + 1) % n and receives (r - 1 + n) % n's; with one
    // rank that is a send to itself.  Verified on the host.
    if (!c) return GDP_ERR_ARG;
    if (c->failed) return refuse_failed(c, "gdp_comm_check");
    constexpr size_t kWords = 4096;
    GDP_HIPC(c, hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;
    int* d = nullptr;
    GDP_HIPC(c, hipMalloc(&d, 2 * kWords * sizeof(int)));
    std::vector<int> h(kWords, c->rank);
    int rc = GDP_OK;
    auto step = [&]() -> int {
        GDP_HIPC(c, hipMemcpyAsync(d, h.data(), kWords * sizeof(int), hipMemcpyHostToDevice, st));
        GDP_HIPC(c, hipMemsetAsync(d + kWords, 0xff, kWords * sizeof(int), st));
        const int next = (c->rank + 1) % c->nranks, prev = (c->rank + c->nranks - 1) % c->nranks;
        int r = group_start(c, st);
        if (r != GDP_OK) return r;
        GDP_NCCL_IN_GROUP(c, ncclSend(d, kWords, ncclInt32, next, c->comm, st));
        GDP_NCCL_IN_GROUP(c, ncclRecv(d + kWords, kWords, ncclInt32, prev, c->comm, st));
        if ((r = group_end(c)) != GDP_OK) return r;
        GDP_HIPC(c, hipMemcpyAsync(h.data(), d + kWords, kWords * sizeof(int), hipMemcpyDeviceToHost, st));
        GDP_HIPC(c, hipStreamSynchronize(st));
        for (size_t k = 0; k < kWords; ++k)
            if (h[k] != prev)
                return fail(c, GDP_ERR_STATE, "gdp_comm_check: word " + std::to_string(k) + " from rank " +
                                                  std::to_string(prev) + " reads " + std::to_string(h[k]));
        return GDP_OK;
    };
    rc = step();
    (void)hipFree(d);
    return rc;
} GDP_COMM_CATCH(c)

int gdp_comm_rank(const gdp_comm* c) { return c ? c->rank : -1; }
int gdp_comm_size(const gdp_comm* c) { return c ? c->nranks : -1; }
const char* gdp_comm_last_error(const gdp_comm* c) { return c ? c->err.c_str() : g_comm_error.c_str(); }

int gdp_comm_plan(int H, int W, int S, int O, int nranks, int rank, int root, gdp_transfer* out, int capacity,
                  int* count) try {
    if (H <= 0 || W <= 0 || S < 0 || O <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || root < 0 ||
        root >= nranks || !count || capacity < 0 || (capacity > 0 && !out))
        return fail(nullptr, GDP_ERR_ARG, "gdp_comm_plan: bad argument");
    std::vector<gdp_transfer> plan = make_plan(H, W, S, O, nranks, rank, root);
    *count = (int)plan.size();
    if ((int)plan.size() > capacity) return fail(nullptr, GDP_ERR_ARG, "gdp_comm_plan: capacity too small");
    std::copy(plan.begin(), plan.end(), out);
    return GDP_OK;
} GDP_COMM_CATCH(nullptr)

int gdp_comm_gather_bands(gdp_comm* c, gdp_ctx* band, int band_image, gdp_ctx* full, int full_image, int root,
                          void* stream) try {
    // band == NULL: this rank's band is empty (more ranks than aligned row bands); it sends nothing
    if (!c || root < 0 || root >= c->nranks || (c->rank == root && !full))
        return fail(c, GDP_ERR_ARG, "gdp_comm_gather_bands: bad argument");
    if (c->failed) return refuse_failed(c, "gdp_comm_gather_bands");
    int H, W, S, O, B;
    if (gdp_get_geometry(band ? band : full, &H, &W, &S, &O, &B) != GDP_OK) {
        if (band || c->rank == root) return fail(c, GDP_ERR_ARG, "band geometry");
    }
    if (band && (band_image < 0 || band_image >= B)) return fail(c, GDP_ERR_ARG, "gdp_comm_gather_bands: band_image out of range");
    if (c->rank == root) {
        int H2, W2, S2, O2, B2;
        gdp_get_geometry(full, &H2, &W2, &S2, &O2, &B2);
        int rows0, cols0, first0;
        gdp_level_dims(full, 0, &rows0, &cols0, &first0);
        if (H2 != H || W2 != W || S2 != S || O2 != O || first0 != 0 || rows0 != H)
            return fail(c, GDP_ERR_ARG, "collector context must be the whole image of the same geometry");
        if (full_image < 0 || full_image >= B2) return fail(c, GDP_ERR_ARG, "gdp_comm_gather_bands: full_image out of range");
    }
    GDP_HIPC(c, hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)gdp_stream(band ? band : full);
    if (!band && c->rank != root) return GDP_OK;  // empty band: nothing to send, nothing to receive
    const std::vector<gdp_transfer> plan = make_plan(H, W, S, O, c->nranks, c->rank, root);
    if (band) {  // the band context must hold exactly the rows the plan sends / copies
        for (const gdp_transfer& t : plan) {
            if (t.kind == GDP_XFER_RECV) continue;
            int rows, cols, first;
            gdp_level_dims(band, t.octave, &rows, &cols, &first);
            if (rows != t.rows || cols != t.cols || first != t.first_row)
                return fail(c, GDP_ERR_ARG, "band context rows differ from gdp_band_rows' band of this rank");
        }
    }
    int rc = group_start(c, st);
    if (rc != GDP_OK) return rc;
    for (const gdp_transfer& t : plan) {
        const size_t n = (size_t)t.rows * t.cols;
        if (t.kind == GDP_XFER_SEND)
            GDP_NCCL_IN_GROUP(c, ncclSend(gdp_device_level(band, band_image, t.octave, t.scale), n, ncclFloat, t.peer,
                                          c->comm, st));
        else if (t.kind == GDP_XFER_RECV)
            GDP_NCCL_IN_GROUP(c, ncclRecv(const_cast<float*>(gdp_device_level(full, full_image, t.octave, t.scale)) +
                                              (size_t)t.first_row * t.cols,
                                          n, ncclFloat, t.peer, c->comm, st));
    }
    if ((rc = group_end(c)) != GDP_OK) return rc;
    for (const gdp_transfer& t : plan) {  // the collector's own band: device-to-device copies
        if (t.kind != GDP_XFER_COPY || !band) continue;
        float* dst = const_cast<float*>(gdp_device_level(full, full_image, t.octave, t.scale)) + (size_t)t.first_row * t.cols;
        GDP_HIPC(c, hipMemcpyAsync(dst, gdp_device_level(band, band_image, t.octave, t.scale),
                                   (size_t)t.rows * t.cols * 4, hipMemcpyDeviceToDevice, st));
    }
    GDP_HIPC(c, hipStreamSynchronize(st));
    return GDP_OK;
} GDP_COMM_CATCH(c)

int gdp_comm_scale_plan(int S, int O, int nranks, int rank, gdp_scale_transfer* out, int capacity, int* count) try {
    if (S < 0 || O <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || !count || capacity < 0 || (capacity > 0 && !out))
        return fail(nullptr, GDP_ERR_ARG, "gdp_comm_scale_plan: bad argument");
    std::vector<gdp_scale_transfer> plan;
    if (make_scale_plan(S, O, nranks, rank, plan) != GDP_OK)
        return fail(nullptr, GDP_ERR_ARG, "gdp_comm_scale_plan: the reference's role map needs >= S+4 ranks");
    *count = (int)plan.size();
    if ((int)plan.size() > capacity) return fail(nullptr, GDP_ERR_ARG, "gdp_comm_scale_plan: capacity too small");
    std::copy(plan.begin(), plan.end(), out);
    return GDP_OK;
} GDP_COMM_CATCH(nullptr)

int gdp_comm_collect_scales(gdp_comm* c, gdp_ctx* ctx, int image, void* stream) try {
    if (!c || !ctx) return fail(c, GDP_ERR_ARG, "gdp_comm_collect_scales: bad argument");
    if (c->failed) return refuse_failed(c, "gdp_comm_collect_scales");
    int H, W, S, O, B;
    if (gdp_get_geometry(ctx, &H, &W, &S, &O, &B) != GDP_OK || image < 0 || image >= B)
        return fail(c, GDP_ERR_ARG, "gdp_comm_collect_scales: bad context / image");
    int rows0, cols0, first0;
    gdp_level_dims(ctx, 0, &rows0, &cols0, &first0);
    if (first0 != 0 || rows0 != H) return fail(c, GDP_ERR_ARG, "gdp_comm_collect_scales needs a whole-image context");
    std::vector<gdp_scale_transfer> plan;
    if (make_scale_plan(S, O, c->nranks, c->rank, plan) != GDP_OK)
        return fail(c, GDP_ERR_ARG, "gdp_comm_collect_scales: the reference's role map needs >= S+4 ranks");
    if (plan.empty()) return GDP_OK;  // ranks > S+3 take no part (GaussDePyramid-MPI.h:269-335)
    GDP_HIPC(c, hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)gdp_stream(ctx);
    int rc = group_start(c, st);
    if (rc != GDP_OK) return rc;
    for (const gdp_scale_transfer& t : plan) {
        int rows, cols, first;
        gdp_level_dims(ctx, t.octave, &rows, &cols, &first);
        const size_t n = (size_t)rows * cols;
        if (n == 0) continue;
        float* lev = const_cast<float*>(gdp_device_level(ctx, image, t.octave, t.scale));
        if (t.kind == GDP_SCALE_SEND)
            GDP_NCCL_IN_GROUP(c, ncclSend(lev, n, ncclFloat, t.peer, c->comm, st));
        else
            GDP_NCCL_IN_GROUP(c, ncclRecv(lev, n, ncclFloat, t.peer, c->comm, st));
    }
    if ((rc = group_end(c)) != GDP_OK) return rc;
    GDP_HIPC(c, hipStreamSynchronize(st));
    return GDP_OK;
} GDP_COMM_CATCH(c)

int gdp_comm_halo_plan(int H, int nranks, int rank, int O, gdp_halo_transfer* out, int capacity, int* count) try {
    if (H <= 0 || nranks <= 0 || rank < 0 || rank >= nranks || O <= 0 || !count || capacity < 0 || (capacity > 0 && !out))
        return fail(nullptr, GDP_ERR_ARG, "gdp_comm_halo_plan: bad argument");
    std::vector<gdp_halo_transfer> plan;
    if (make_halo_plan(H, nranks, rank, O, plan) != GDP_OK)
        return fail(nullptr, GDP_ERR_ARG, "gdp_comm_halo_plan: a row band is thinner than the halo");
    *count = (int)plan.size();
    if ((int)plan.size() > capacity) return fail(nullptr, GDP_ERR_ARG, "gdp_comm_halo_plan: capacity too small");
    std::copy(plan.begin(), plan.end(), out);
    return GDP_OK;
} GDP_COMM_CATCH(nullptr)

int gdp_comm_exchange_halo(gdp_comm* c, gdp_ctx* band, void* stream) try {
    if (!c) return GDP_ERR_ARG;
    if (c->failed) return refuse_failed(c, "gdp_comm_exchange_halo");
    if (!band) return GDP_OK;  // empty band: its neighbours do not count it as one
    int H, W, S, O, B;
    if (gdp_get_geometry(band, &H, &W, &S, &O, &B) != GDP_OK) return fail(c, GDP_ERR_ARG, "band geometry");
    int r0 = 0, r1 = 0, rows0, cols0, first0;
    gdp_band_rows(H, c->nranks, c->rank, O, &r0, &r1);
    gdp_level_dims(band, 0, &rows0, &cols0, &first0);
    if (first0 != r0 || rows0 != r1 - r0) return fail(c, GDP_ERR_ARG, "band context rows differ from gdp_band_rows' band of this rank");
    std::vector<gdp_halo_transfer> plan;
    if (make_halo_plan(H, c->nranks, c->rank, O, plan) != GDP_OK)
        return fail(c, GDP_ERR_ARG, "a row band is thinner than the convolution halo");
    const bool u8 = gdp_get_input_format(band) == GDP_INPUT_U8;
    const size_t esz = u8 ? 1 : 4;
    void* halo[2] = {nullptr, nullptr};
    size_t hpitch[2] = {0, 0};
    for (int side = 0; side < 2; ++side) {  // binds the band's owned halo rows (a no-op once bound)
        const int rc = gdp_input_halo(band, side, &halo[side], &hpitch[side]);
        if (rc != GDP_OK) return fail(c, rc, gdp_last_error(band));
    }
    int na = 0, nb = 0;
    gdp_conv_halo_rows(band, &na, &nb);
    GDP_HIPC(c, hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)gdp_stream(band);
    std::vector<std::pair<const void*, size_t>> inputs((size_t)B);
    for (int b = 0; b < B; ++b) {
        gdp_device_input(band, b, &inputs[(size_t)b].first, &inputs[(size_t)b].second);
        if (inputs[(size_t)b].second != hpitch[0])
            return fail(c, GDP_ERR_ARG, "band input pitch differs from its halo rows' (bind an input of pitch round_up(W, 4))");
    }
    const ncclDataType_t ty = u8 ? ncclUint8 : ncclInt32;
    int rc = group_start(c, st);
    if (rc != GDP_OK) return rc;
    for (int b = 0; b < B; ++b) {
        const char* in = static_cast<const char*>(inputs[(size_t)b].first);
        const size_t pitch = inputs[(size_t)b].second;
        for (const gdp_halo_transfer& t : plan) {
            const size_t n = (size_t)t.rows * pitch;  // whole padded rows (the same pitch on both sides)
            if (t.kind == GDP_HALO_SEND) {
                GDP_NCCL_IN_GROUP(c, ncclSend(in + (size_t)t.first_row * pitch * esz, n, ty, t.peer, c->comm, st));
            } else {
                const int side = t.kind == GDP_HALO_RECV_ABOVE ? 0 : 1;
                const size_t rows_side = side ? (size_t)nb : (size_t)na;
                GDP_NCCL_IN_GROUP(c, ncclRecv(static_cast<char*>(halo[side]) + (size_t)b * rows_side * hpitch[side] * esz, n,
                                              ty, t.peer, c->comm, st));
            }
        }
    }
    return group_end(c);
} GDP_COMM_CATCH(c)

}  // extern "C"
