/*
 * gdp_comm.h — C ABI of libgdp_comm.so: the multi-GPU collector over RCCL (xGMI).
 *
 * The RCCL counterpart of the reference's MPI collector (GaussPyramid_mpi::GenerateDoG_mpi,
 * GaussDePyramid-MPI.h:265-335: ranks < S+3 filter one scale each and MPI_Send every row to rank
 * S+3, which receives them, :295-303, and forms all DoG levels, :304-318).  Here every rank builds
 * one ROW BAND of the whole pyramid on its own GPU (gdp_create_band; DoG fused, any world size)
 * and the collector receives each band's finished levels straight into a whole-image context with
 * RCCL point-to-point transfers — one grouped send per level instead of one MPI_Send per row.
 *
 * Bootstrap is the caller's: rank 0 calls gdp_comm_unique_id and broadcasts the 128 bytes with
 * whatever launcher it has (MPI_Bcast in include/GaussDePyramid-HIP-mpi.h), then every rank calls
 * gdp_comm_init.  Uses only the public gdp.h ABI of the contexts it is given.
 */
#ifndef GDP_COMM_H_
#define GDP_COMM_H_

#include "gdp.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gdp_comm gdp_comm;
#define GDP_COMM_ID_BYTES 128

/* Rows [row_begin, row_end) of rank `rank`'s band of an H-row image split over `nranks` ranks:
 * multiples of 2^(max(octaves,5)-1), the last band ends at H (what gdp_create_band accepts). */
int gdp_band_rows(int height, int nranks, int rank, int octaves, int* row_begin, int* row_end);

/* One point-to-point transfer of the collector's schedule: `rows` x `cols` floats of level
 * (octave, scale).  SEND: this rank's whole band level to `peer` (the root); RECV: the root takes
 * sender `peer`'s band level into the whole image's level at row `first_row`; COPY: the root's own
 * band, device to device, to row `first_row`.  For SEND `first_row` is the band's first row of the
 * level in the whole image (where the root will put it). */
enum { GDP_XFER_SEND = 0, GDP_XFER_RECV = 1, GDP_XFER_COPY = 2 };
typedef struct gdp_transfer {
    int kind, peer, octave, scale, first_row, rows, cols;
} gdp_transfer;

/* The transfer schedule gdp_comm_gather_bands executes on rank `rank` of `nranks` (pure host
 * arithmetic, no device): the sends of a non-root rank in issue order, or the root's receives
 * (rank-major, then octave, then scale: RCCL matches the sends and receives of one peer pair in
 * order) followed by its local copies.  Levels with no rows of a band are skipped.  Writes up to
 * `capacity` records to `out` (may be NULL with capacity 0) and the total count to `*count`;
 * GDP_ERR_ARG if the schedule does not fit (call again with a larger buffer).  The RCCL
 * counterpart of the reference's per-row MPI_Send/MPI_Recv loops (GaussDePyramid-MPI.h:285,298). */
int gdp_comm_plan(int height, int width, int S, int octaves, int nranks, int rank, int root, gdp_transfer* out,
                  int capacity, int* count);

int gdp_comm_unique_id(unsigned char id[GDP_COMM_ID_BYTES]);
int gdp_comm_init(gdp_comm** out, const unsigned char id[GDP_COMM_ID_BYTES], int nranks, int rank, int device);
void gdp_comm_destroy(gdp_comm* comm);
int gdp_comm_rank(const gdp_comm* comm);
int gdp_comm_size(const gdp_comm* comm);
const char* gdp_comm_last_error(const gdp_comm* comm); /* comm may be NULL: last init failure */

/* Failure contract of every collective below (the counterpart of an MPI error on the reference's
 * per-row MPI_Send / MPI_Recv, GaussDePyramid-MPI.h:285,298).  The transfers of one call are one
 * ncclGroupStart() .. ncclGroupEnd(); when any ncclSend / ncclRecv inside it fails, the group is
 * closed before returning (so no later RCCL call of the thread is captured by an open group), the
 * call returns GDP_ERR_HIP, and the communicator is marked failed: the peers may still wait for
 * this rank's half of the exchange, so every later collective on it returns GDP_ERR_STATE at
 * once instead of hanging, and gdp_comm_destroy aborts it (ncclCommAbort) instead of waiting.
 * gdp_comm_failed: 1 once that happened, 0 before, -1 for NULL. */
int gdp_comm_failed(const gdp_comm* comm);
/* Health check, collective over all ranks: a ring exchange (rank r sends 4096 words holding r to
 * r + 1 and receives r - 1's; a one-rank communicator sends to itself), verified on the host.
 * GDP_OK when every word arrived; same failure contract as the collectives. stream may be NULL. */
int gdp_comm_check(gdp_comm* comm, void* stream);
/* Test hook: the NEXT collective on `comm` adds, first in its group, a send to peer `nranks`
 * (out of range), which RCCL rejects inside the group — exercises the failure contract above. */
int gdp_comm_test_inject_fault(gdp_comm* comm);

/* Collective over all ranks of `comm`: every rank passes its band context (built with
 * gdp_band_rows' rows of the same H, W, S, octaves) and image index `band_image`; rank `root`
 * also passes `full`, a whole-image context of the same geometry, whose image `full_image`
 * receives every band's levels (other ranks pass NULL).  A non-root rank whose band is empty
 * (more ranks than aligned bands) passes band = NULL and returns at once.  Stream-ordered on `stream` (NULL = the
 * band context's stream); blocking until the transfers are complete on return. */
int gdp_comm_gather_bands(gdp_comm* comm, gdp_ctx* band, int band_image, gdp_ctx* full, int full_image, int root,
                          void* stream);

/* ---- the reference's own role map (GaussPyramid_mpi::GenerateDoG_mpi, GaussDePyramid-MPI.h:265-335)
 * Ranks i < S+3 ("workers") window scale i of every octave of their OWN pyramid and send it, level
 * by level, to rank S+3 (the collector), which receives scale j from worker j and forms every DoG
 * level; ranks > S+3 take no part.  Needs nranks >= S+4, as the reference does.  The drop-in class
 * uses it when the world is that large (GaussDePyramid-HIP-mpi.h), leaving every rank's GaussPy
 * where the reference leaves it: worker i with scale i windowed, the collector with the pyramid.
 * gdp_comm_scale_plan: rank `rank`'s transfers (pure host arithmetic): a worker's sends (octave
 * order), the collector's receives (worker-major, then octave: RCCL matches one peer pair's
 * transfers in order), nothing for the others; GDP_ERR_ARG when nranks < S+4. */
enum { GDP_SCALE_SEND = 0, GDP_SCALE_RECV = 1 };
typedef struct gdp_scale_transfer {
    int kind, peer, octave, scale;
} gdp_scale_transfer;
int gdp_comm_scale_plan(int S, int octaves, int nranks, int rank, gdp_scale_transfer* out, int capacity, int* count);
/* Collective over the ranks of `comm` (>= S+4): executes gdp_comm_scale_plan on `ctx`, a
 * whole-image context of the same geometry on every rank, image `image`: a worker's level
 * (o, rank) goes to the collector's level (o, rank), whole levels, RCCL point-to-point in one
 * group.  The window multiply (gdp_gauss_scales) before and the collector's DoG pass
 * (gdp_dog_range) after are the caller's.  Stream-ordered on `stream` (NULL = the context's
 * stream); blocking until the transfers are complete on return. */
int gdp_comm_collect_scales(gdp_comm* comm, gdp_ctx* ctx, int image, void* stream);

/* ---- halo exchange of the convolution extension on row bands (gdp_build_gaussian) ----------
 * The one step of the path with a real exchange: a band's convolution reads up to 6 * 2^(O-1)
 * input rows of each neighbouring band (gdp_conv_halo_rows).  Rank r sends its first rows to
 * r - 1 (that band's "below" halo) and its last rows to r + 1 (its "above" halo), and receives
 * its own two halos.  The reference's pointwise window needs no exchange.
 * gdp_comm_halo_plan: the schedule on rank `rank` (pure host arithmetic; neighbours are the
 * adjacent non-empty bands of gdp_band_rows; GDP_ERR_ARG when a band is thinner than the halo).
 * SEND: rows [first_row, first_row + rows) of this band (band-local); RECV_ABOVE / RECV_BELOW:
 * the whole halo buffer of that side.  Issue order: per neighbour (above, then below) the send
 * then the receive. */
enum { GDP_HALO_SEND = 0, GDP_HALO_RECV_ABOVE = 1, GDP_HALO_RECV_BELOW = 2 };
typedef struct gdp_halo_transfer {
    int kind, peer, first_row, rows;
} gdp_halo_transfer;
int gdp_comm_halo_plan(int height, int nranks, int rank, int octaves, gdp_halo_transfer* out, int capacity,
                       int* count);
/* Collective over the ranks holding bands: fills `band`'s own halo buffers (gdp_input_halo) with
 * the neighbours' input rows for every image of the batch, RCCL point-to-point grouped in one
 * ncclGroupStart/End.  `band` must be gdp_band_rows' band of this rank (NULL on a rank whose band
 * is empty), its input pitch the width rounded up to 4 (the owned input, or a bound input of that
 * pitch).  Stream-ordered on `stream` (NULL = the band's stream); returns when enqueued (the
 * following gdp_build_gaussian on the same stream sees the rows).  The FIRST call on a band
 * allocates and binds its halo buffers (gdp_input_halo: a blocking geometry upload that drains the
 * device); every later call only enqueues the transfers.  A failure returns the status of the
 * step that failed (GDP_ERR_NOMEM only for an allocation). */
int gdp_comm_exchange_halo(gdp_comm* comm, gdp_ctx* band, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* GDP_COMM_H_ */
