// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// Runs the reference's own MULTI-PROCESS variants, compiled in place from /root/reference (see
// oracle/Makefile targets `ref-mpi`), so the collector's output can be pinned as golden vectors:
//
//   -DREF_MPI_CLASS : GaussPyramid_mpi::GenerateDoG_mpi (GaussDePyramid-MPI.h:265-335)
//   -DREF_MPITEST   : mpitest.cpp's GenerateDoG_mpi (:114-189) / GenerateDoG_mpi_omp (:35-113) on
//                     its globals (GaussPyInit(int* data[MAX]) :438-473); mpitest.cpp is #included
//                     with its `main` renamed, nothing of it is copied here
//
//   mpiexec -n <S+4> ref_mpi  hash <n> <S> <input>               collector prints per-level hashes
//   mpiexec -n <S+4> ref_mpi  dump <n> <S> <input> <out.f32>     collector writes the packed pyramid
//   mpiexec -n <S+4> ref_mpitest hash|dump <n> <S> <input> [out] <mpi|mpi_omp>
//
// Both variants hard-wire rank S+3 as the collector and need >= S+4 ranks; the
// other ranks end with partially filtered data and print nothing.  They call MPI_Init/MPI_Finalize
// themselves, so the harness learns its rank from the launcher's environment (PMI_RANK, MPICH
// hydra) and only reads the pyramid after the call returns.  <input> as in ref_harness.cpp.
#ifdef REF_MPI_CLASS
#include "GaussDePyramid-MPI.h"
#endif
#ifdef REF_MPITEST
#define main gdp_unused_mpitest_main
#include "mpitest.cpp"
#undef main
#endif

#include <cstdio>
#include <cstdlib>
#include <string>

#include "ref_common.h"

static int launcher_rank() {
    for (const char* v : {"PMI_RANK", "OMPI_COMM_WORLD_RANK", "PMIX_RANK"})
        if (const char* e = std::getenv(v)) return std::atoi(e);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: see the header of oracle/ref_mpi_harness.cpp\n");
        return 2;
    }
    const std::string mode = argv[1];
    const int nn = std::atoi(argv[2]);
    const int SS = std::atoi(argv[3]);
    int** img = refh::make_input(nn, argv[4]);
    const char* out = mode == "dump" ? (argc > 5 ? argv[5] : nullptr) : nullptr;
    if (mode == "dump" && !out) return 2;
    // the reference's GenerateDoG_mpi takes (argc, argv) for MPI_Init: hand it a copy
    int margc = 1;
    char* margv_store[2] = {argv[0], nullptr};
    char** margv = margv_store;
    const int rank = launcher_rank();
#ifdef REF_MPI_CLASS
    GaussPyramid_mpi g(img, nn, SS);
    g.GenerateDoG_mpi(margc, margv);
    float**** G = g.GaussPy;
#endif
#ifdef REF_MPITEST
    const std::string fn = argv[argc - 1];
    n = nn;   // mpitest.cpp:29 global (GaussPyInit sets length = n, :440)
    S = SS;   // :30
    GaussPyInit(img);
    if (fn == "mpi_omp")
        GenerateDoG_mpi_omp(margc, margv);
    else
        GenerateDoG_mpi(margc, margv);
    float**** G = GaussPy;
#endif
    if (rank == SS + 3) {  // the collector (GaussDePyramid-MPI.h:292, mpitest.cpp:65,142)
        std::fflush(stdout);
        if (mode == "hash")
            refh::hash(G, nn, SS);
        else
            refh::dump(G, nn, SS, out);
        std::fflush(stdout);
    }
    return 0;
}
