// GaussDePyramid-HIP-AVX512.h — drop-in MI355X replacements for the reference's AVX-512 classes,
// the two CPU paths its main.cpp selects by #include (main.cpp:8, :11):
//
//   GaussPyramid_a512omp  (GaussDePyramid-AVX512xOpenMP.h:20-48)  -> GaussPyramid_a512omp_hip
//   GaussPyramid_a512xp   (GaussDePyramid-AVX512xPTHREAD.h:21-40) -> GaussPyramid_a512xp_hip
//
// Swap the include line and the class name; link with -lgdp.  Both derive from GaussPyramid_hip
// (GaussDePyramid-HIP.h: constructor, GaussPy host mirror, GaussPyInit, output, destructor) and
// differ only where the reference classes differ from GuassDePyramid.h:
//
// GaussPy is two-way state exactly as in GaussPyramid_hip (mirror_host / host_dirty / SyncDevice).
//
// GaussPyramid_a512omp_hip
//  - GenerateDoG_nomp_dynamic() (:240-364), the path the reference times: scales 0..S-1 windowed
//    with the integer-length centre float(len_o - 1) / 2 (:251, :279), then level i -= level i+1
//    for i < S-1 (:324-357) — {DoG_0 .. DoG_{S-2}, G_{S-1}, x, x, x}.  On fresh GaussPyInit
//    contents one fused launch (gdp_build_subset), else in place (gdp_generate_dog_subset).  The
//    reference's DoG loop is an `omp for` over i with level i+1 modified in place by the next
//    iteration, so with counnt > 1 and S >= 3 its output depends on thread timing; this computes
//    the sequential (counnt = 1) result, which is the only one for S <= 2.
//  - GaussFilter(int) does nothing: the reference's body is commented out (:128-181).
//  - GenerateDoG() is therefore the DoG pass alone, level j -= level j+1 for j = 0..S+1 per
//    octave (:183-193), applied a second time on octaves of side <= 2 (:194-201).
//  - GenerateDoG_nomp_static() is empty (:366-368).
//  - `counnt` (:18, the OpenMP thread count callers set) exists and is ignored.
// GaussPyramid_a512xp_hip
//  - GenerateDoG() (:143-155 / thread_Filter_Sub :178-261): GuassDePyramid.h's full semantics, but
//    with the integer-length window centre (:193, :218); identical to the serial header for every
//    side its 16-float vector loops support (powers of two) and different for sides 3, 5, 6, 7.
//  - GaussFilter(int) (:113-141) keeps the serial header's float-halved centre.
#ifndef SIFT_GAUSSDEPYRAMID_HIP_AVX512_H
#define SIFT_GAUSSDEPYRAMID_HIP_AVX512_H

#include "GaussDePyramid-HIP.h"

// GaussDePyramid-AVX512xOpenMP.h:18 — the caller-visible OpenMP thread count (no threads here)
__attribute__((unused)) static int counnt = 2;
#ifndef THREAD_COUNT_a512t
#define THREAD_COUNT_a512t 7  // GaussDePyramid-AVX512xPTHREAD.h's worker count (unused here)
#endif

class GaussPyramid_a512omp_hip : public GaussPyramid_hip {
public:
    GaussPyramid_a512omp_hip() {}
    GaussPyramid_a512omp_hip(int** img, int len, int S, int device = 0) : GaussPyramid_hip(img, len, S, device) {
        check_(ctx_, gdp_set_window_centre(ctx_, GDP_CENTRE_INTLEN), "GaussPyramid_a512omp_hip");
    }
    void GaussFilter(int) {}
    void GenerateDoG();
    void GenerateDoG_nomp_dynamic();
    void GenerateDoG_nomp_static() {}
    // not members of the reference class (GaussPyramid_hip's MPI-variant entry points)
    void GenerateDoG_mpi(int, char**) = delete;
    void GenerateDoG_mgpu(int, char**) = delete;
};

inline void GaussPyramid_a512omp_hip::GenerateDoG_nomp_dynamic() {
    CallScope scope(this);
    pull_host_();  // GaussPy is two-way state (GaussDePyramid-HIP.h)
    check_(ctx_, fresh_ ? gdp_build_subset(ctx_, nullptr) : gdp_generate_dog_subset(ctx_, nullptr),
           "GenerateDoG_nomp_dynamic");
    fresh_ = false;
    check_(ctx_, gdp_sync(ctx_), "GenerateDoG_nomp_dynamic");
    if (mirror_host) publish_();
}

inline void GaussPyramid_a512omp_hip::GenerateDoG() {
    CallScope scope(this);
    // per octave (:183-201): the DoG pass, then once more where the side is <= 2 — as two
    // launches, all octaves and then the tiny ones
    pull_host_();
    int tiny = 0;
    while (tiny < layer && (length >> tiny) > 2) ++tiny;
    check_(ctx_, gdp_dog_range(ctx_, 0, layer, nullptr), "GenerateDoG");
    if (tiny < layer) check_(ctx_, gdp_dog_range(ctx_, tiny, layer, nullptr), "GenerateDoG");
    fresh_ = false;
    check_(ctx_, gdp_sync(ctx_), "GenerateDoG");
    if (mirror_host) publish_();
}

class GaussPyramid_a512xp_hip : public GaussPyramid_hip {
public:
    GaussPyramid_a512xp_hip() {}
    GaussPyramid_a512xp_hip(int** img, int len, int S, int device = 0) : GaussPyramid_hip(img, len, S, device) {
        check_(ctx_, gdp_set_window_centre(ctx_, GDP_CENTRE_INTLEN), "GaussPyramid_a512xp_hip");
    }
    void GaussFilter(int theLayer) {
        // the serial header's float-halved centre for this method only (:113-141); each centre
        // has its own device tap table, so the two switches are pointer swaps (no drain/upload)
        check_(ctx_, gdp_set_window_centre(ctx_, GDP_CENTRE_SERIAL), "GaussFilter");
        GaussPyramid_hip::GaussFilter(theLayer);
        check_(ctx_, gdp_set_window_centre(ctx_, GDP_CENTRE_INTLEN), "GaussFilter");
    }
    // GenerateDoG: GaussPyramid_hip's (fused on fresh contents, else in place) with this
    // context's integer-length centre
    void GenerateDoG_mpi(int, char**) = delete;  // not members of the reference class
    void GenerateDoG_mgpu(int, char**) = delete;
};

#endif  // SIFT_GAUSSDEPYRAMID_HIP_AVX512_H
