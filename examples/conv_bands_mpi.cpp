// Convolution extension on row bands across MPI ranks, one GPU per rank, halo rows over RCCL:
// the C-ABI path of distributed.exchange_halo.
//
//   mpiexec -n N examples/conv_bands_mpi [n] [S]
//
// Rank r builds row band gdp_band_rows(n, N, r) of the synthetic n x n image (generated on its GPU),
// receives its halo rows from ranks r - 1 / r + 1 (gdp_comm_exchange_halo), runs
// gdp_build_gaussian on the band, and the band checksums are summed on rank 0, which compares them
// with the whole image built on its own GPU.  Prints "bands == whole image" and the slowest rank's
// exchange + build time.  MPI is only the launcher and the id broadcast; the data moves over RCCL.
#include <mpi.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "gdp.h"
#include "gdp_comm.h"

static void check(int rc, const char* what, gdp_ctx* c = nullptr) {
    if (rc != GDP_OK) {
        std::fprintf(stderr, "%s failed: %s (%s)\n", what, gdp_status_string(rc), gdp_last_error(c));
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank = 0, size = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    const int n = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int S = argc > 2 ? std::atoi(argv[2]) : 2;
    const int O = 5;
    const int ndev = gdp_device_count();
    if (ndev <= 0) check(GDP_ERR_NODEV, "gdp_device_count");
    const int device = rank % ndev;

    unsigned char id[GDP_COMM_ID_BYTES] = {};
    if (rank == 0 && gdp_comm_unique_id(id) != GDP_OK) check(GDP_ERR_HIP, gdp_comm_last_error(nullptr));
    MPI_Bcast(id, GDP_COMM_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
    gdp_comm* comm = nullptr;
    if (gdp_comm_init(&comm, id, size, rank, device) != GDP_OK) check(GDP_ERR_HIP, gdp_comm_last_error(nullptr));

    int r0 = 0, r1 = 0;
    check(gdp_band_rows(n, size, rank, O, &r0, &r1), "gdp_band_rows");
    gdp_ctx* band = nullptr;
    uint64_t mine = 0;
    double secs = 0;
    if (r1 > r0) {
        check(gdp_create_band(&band, n, n, S, O, 1, r0, r1, device), "gdp_create_band");
        check(gdp_fill_synthetic(band, 0x5EED, 0, nullptr), "gdp_fill_synthetic", band);
        check(gdp_sync(band), "gdp_sync", band);
    }
    MPI_Barrier(MPI_COMM_WORLD);
    const auto t0 = std::chrono::steady_clock::now();
    if (gdp_comm_exchange_halo(comm, band, nullptr) != GDP_OK) check(GDP_ERR_HIP, gdp_comm_last_error(comm));
    if (band) {
        check(gdp_build_gaussian(band, nullptr), "gdp_build_gaussian", band);
        check(gdp_sync(band), "gdp_sync", band);
    }
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (band) check(gdp_checksum(band, 0, &mine), "gdp_checksum", band);
    unsigned long long sum = 0, local = mine;
    double slowest = 0;
    MPI_Reduce(&local, &sum, 1, MPI_UNSIGNED_LONG_LONG, MPI_SUM, 0, MPI_COMM_WORLD);
    MPI_Reduce(&secs, &slowest, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    int status = 0;
    if (rank == 0) {
        gdp_ctx* whole = nullptr;
        check(gdp_create(&whole, n, n, S, O, 1, device), "gdp_create");
        check(gdp_fill_synthetic(whole, 0x5EED, 0, nullptr), "gdp_fill_synthetic", whole);
        check(gdp_build_gaussian(whole, nullptr), "gdp_build_gaussian", whole);
        uint64_t want = 0;
        check(gdp_checksum(whole, 0, &want), "gdp_checksum", whole);
        gdp_destroy(whole);
        status = sum == want ? 0 : 1;
        std::printf("%s: %d band(s) of %dx%d, checksum %016llx vs whole image %016llx; exchange + build %.3f ms\n",
                    status ? "MISMATCH" : "bands == whole image", size, n, n, sum, (unsigned long long)want,
                    slowest * 1e3);
    }
    MPI_Bcast(&status, 1, MPI_INT, 0, MPI_COMM_WORLD);
    gdp_destroy(band);
    gdp_comm_destroy(comm);
    MPI_Finalize();
    return status;
}
