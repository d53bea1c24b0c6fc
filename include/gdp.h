/*
 * gdp.h — C ABI of libgdp.so, the MI355X (gfx950) Gaussian / Difference-of-Gaussians pyramid.
 *
 * This is the drop-in boundary for the reference's pyramid hot path
 * (ZhangShuui/SIFT-parallel-optimization, GuassDePyramid.h and the GaussDePyramid-*.h variants).
 * The reference exposes a duck-typed C++ class surface selected by #include (main.cpp:2-13);
 * every entry point below names the reference member it replaces (file:line).  The C++ class
 * `GaussPyramid_hip` (include/GaussDePyramid-HIP.h) and the Python mirror
 * (sift-parallel-optimization_amd/gausspyramid.py) are thin callers of exactly these functions.
 *
 * Conventions
 *  - Every function returns an int status (GDP_OK == 0) unless documented otherwise; no C++
 *    exception crosses the ABI.  gdp_last_error(ctx) / gdp_status_string() describe failures.
 *  - Only plain pointers and sizes cross the boundary.  `stream` is a hipStream_t passed as
 *    void*: NULL = the context's own stream, GDP_STREAM_NULL = HIP's default (null) stream; all
 *    compute and copy calls are stream-ordered and asynchronous unless documented otherwise.
 *  - The context owns its device buffers (input, pyramid, tap tables); the caller keeps
 *    ownership of every host array it passes in.  One context per host thread and device.
 *  - Semantics are the reference's, bit for bit: float32 taps from glibc expf/sqrtf computed on
 *    the host (GuassDePyramid.h:119-121), products ((float)x * f[c]) * f[r] with no FMA
 *    contraction and denormals kept, DoG_s = G_s - G_{s+1} in ascending s (:140-146),
 *    level S+2 keeps the last Gaussian.
 *
 * Pyramid geometry (per image b of a batch):
 *   octave o has rows_o x cols_o pixels, cols_o = W >> o and (whole image) rows_o = H >> o;
 *   scale s in [0, S+3).  Octave o decimates the ORIGINAL image: input pixel (r<<o, c<<o)
 *   (GuassDePyramid.h:80).  `octaves` = 0 selects floor(log2(min(H, W))) + 1, the reference's
 *   `layer` (GuassDePyramid.h:48-53).  The reference is square-only; H != W is an extension
 *   (W-derived window along columns, H-derived window along rows).
 *   A "band" context computes the output rows whose input rows lie in [row_begin, row_end) of
 *   an H-row image (multi-GPU row-band partition; the operation is pointwise, halo = 0).
 */
#ifndef GDP_H_
#define GDP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gdp_ctx gdp_ctx;

/* Stream argument selecting HIP's default (null) stream; NULL selects the context's stream. */
#define GDP_STREAM_NULL ((void*)1)

enum {
    GDP_OK = 0,
    GDP_ERR_ARG = 1,      /* invalid argument (sizes, indices, null pointers)        */
    GDP_ERR_HIP = 2,      /* a HIP runtime call failed (message in gdp_last_error)   */
    GDP_ERR_STATE = 3,    /* call not valid in the context's current state           */
    GDP_ERR_NOMEM = 4,    /* host or device allocation failed                        */
    GDP_ERR_NODEV = 5,    /* no usable gfx950 device                                 */
    GDP_ERR_INTERNAL = 6  /* unexpected internal failure (a C++ exception stopped at the ABI) */
};

/* ABI version of this header; gdp_abi_version() returns the library's. */
#define GDP_ABI_VERSION 1
int gdp_abi_version(void);

/* Number of visible HIP devices (0 when none / no driver). */
int gdp_device_count(void);

/* Number of octaves the reference builds for an n-pixel axis: floor(log2 n) + 1
 * (GaussPyramid ctor, GuassDePyramid.h:48-53). */
int gdp_octaves_for(int n);

/* Allocate a context for `batch` images of H x W int32 pixels, S (+3 Gaussian scales per octave)
 * and `octaves` octaves (0 = all) on HIP device `device`, and upload the tap tables.
 * Replaces the allocation half of GaussPyramid(int** img, int len, int S)
 * (GuassDePyramid.h:36-58) and GaussPyInit's first-call allocation (:60-73). */
int gdp_create(gdp_ctx** out, int height, int width, int S, int octaves, int batch, int device);

/* Same as gdp_create for the row band [row_begin, row_end) of an H-row image.  row_begin must
 * be a multiple of 2^(max(octaves,5)-1); row_end must be too, or equal `height`.  Extension for
 * the multi-GPU row-band split (no reference counterpart). */
int gdp_create_band(gdp_ctx** out, int height, int width, int S, int octaves, int batch, int row_begin,
                    int row_end, int device);

/* Free every device buffer.  Replaces ~GaussPyramid() (GuassDePyramid.h:151-170). */
void gdp_destroy(gdp_ctx* ctx);

/* Geometry queries.  gdp_level_dims gives the rows held by this context for octave o (the whole
 * image, or the band), their first global row, and the columns. */
int gdp_get_geometry(const gdp_ctx* ctx, int* height, int* width, int* S, int* octaves, int* batch);
int gdp_level_dims(const gdp_ctx* ctx, int octave, int* rows, int* cols, int* first_row);
size_t gdp_pyramid_bytes(const gdp_ctx* ctx); /* device bytes of all pyramids of the batch */
/* The pyramid's backing: by default one reserved address range backed by separately
 * created 2 MiB physical pieces (GDP_TUNE_PYRAMID_CHUNK_KB reports it); GDP_SPREAD_VMM=0 in the
 * environment when the context is created gives one hipMalloc instead (e.g. to share the pyramid
 * with another process through IPC).  Identical bits and offsets either way.  Each image starts
 * on an allocation granule only where that wastes at most 1/16 of an image: gdp_pyramid_bytes and
 * gdp_level_offset follow that stride, gdp_image_floats stays one image's dense extent.  (The
 * layout experiments of DESIGN.md §4 read further variables only in the research build,
 * `make -C sift-parallel-optimization_amd/csrc exp`.) */

/* ---- input ---------------------------------------------------------------------------------
 * The reference deep-copies `int** img` in its constructor (GuassDePyramid.h:38-46).  These
 * upload image b of the batch (band contexts: the band's rows only, given as rows of the band). */
/* int** row-pointer form, exactly the reference ctor's argument. */
int gdp_set_input_rows(gdp_ctx* ctx, int b, const int32_t* const* rows, void* stream);
/* contiguous host image with a row pitch of `pitch` int32 elements. */
int gdp_set_input_host(gdp_ctx* ctx, int b, const int32_t* base, size_t pitch, void* stream);
/* Zero-copy: read every image straight from caller-owned DEVICE memory.  Image b, row r starts
 * at base + b*image_stride + r*pitch (int32 elements).  Pass base = NULL to go back to the
 * context's own input buffer.  The memory must stay valid while builds run. */
int gdp_set_input_device(gdp_ctx* ctx, const int32_t* base, size_t pitch, size_t image_stride);
/* Input pixel format of the context: GDP_INPUT_I32 (default; the reference's int) or
 * GDP_INPUT_U8 (8-bit images: a quarter of the input bytes, identical pyramid bits since every
 * uint8 value is an int).  Switching reallocates the context's input buffer (contents zeroed). */
enum { GDP_INPUT_I32 = 0, GDP_INPUT_U8 = 1 };
int gdp_set_input_format(gdp_ctx* ctx, int format);
int gdp_get_input_format(const gdp_ctx* ctx);
int gdp_set_input_host_u8(gdp_ctx* ctx, int b, const uint8_t* base, size_t pitch, void* stream);
int gdp_set_input_device_u8(gdp_ctx* ctx, const uint8_t* base, size_t pitch, size_t image_stride);
/* Benchmark/test input generated on the device (SURVEY.md §8d counter hash): image b of the
 * batch gets global index first_image + b; pixel = lowbias32(seed ^ fold(idx)) >> 24 with
 * idx = (index*H + r)*W + c over the WHOLE image (band contexts generate their rows only).
 * Writes the input the builds read: the context's own buffer, or the caller's device buffer
 * bound by gdp_set_input_device* (its pitch and image stride; the pitch padding is untouched). */
int gdp_fill_synthetic(gdp_ctx* ctx, uint32_t seed, long first_image, void* stream);

/* ---- compute ------------------------------------------------------------------------------- */
/* Fused GaussPyInit() + GenerateDoG() for every image of the batch in one launch: reads each
 * input pixel once and writes the final pyramid once.  Equivalent, bit for bit, to
 * GuassDePyramid.h:74-86 followed by :136-149. */
int gdp_build(gdp_ctx* ctx, void* stream);
/* GaussPyInit() refill: every scale of octave o := (float) decimated input
 * (GuassDePyramid.h:74-86). */
int gdp_init(gdp_ctx* ctx, void* stream);
/* GaussFilter(o) in place: every scale of octave o *= column window then row window
 * (GuassDePyramid.h:106-134). */
int gdp_gauss_octave(gdp_ctx* ctx, int octave, void* stream);
/* GaussFilter(o) for every o in [o_begin, o_end) in ONE launch (the reference calls it per octave
 * from GenerateDoG, :139); the "row + column window pass" the north star's roofline target names. */
int gdp_gauss_range(gdp_ctx* ctx, int o_begin, int o_end, void* stream);
/* The window multiply of scales [s_begin, s_end) only, for every octave in [o_begin, o_end), in
 * ONE launch: what worker rank i of the reference's MPI variant does to its own scale i before
 * sending it to the collector (GaussPyramid_mpi::GenerateDoG_mpi, GaussDePyramid-MPI.h:271-290;
 * its integer-length centre is GDP_CENTRE_INTLEN).  gdp_gauss_range is s = [0, S+3). */
int gdp_gauss_scales(gdp_ctx* ctx, int s_begin, int s_end, int o_begin, int o_end, void* stream);
/* DoG of octave o in place: level s -= level s+1 for s = 0..S+1 ascending
 * (GuassDePyramid.h:140-146). */
int gdp_dog_octave(gdp_ctx* ctx, int octave, void* stream);
/* The DoG pass of every octave in [o_begin, o_end) in ONE launch (no window multiply). */
int gdp_dog_range(gdp_ctx* ctx, int o_begin, int o_end, void* stream);
/* GenerateDoG() in place on the CURRENT contents, all octaves in one launch
 * (GuassDePyramid.h:136-149).  After gdp_init this equals gdp_build; called again it re-filters,
 * like the reference's repeated-call timing loop (main.cpp:66-73). */
int gdp_generate_dog(gdp_ctx* ctx, void* stream);
/* GaussPyramid_a512omp::GenerateDoG_nomp_dynamic (GaussDePyramid-AVX512xOpenMP.h:240-364), the
 * reference's AVX-512 x OpenMP path, whose output is a SUBSET of GenerateDoG's: only scales
 * 0..S-1 are windowed (:242-318) and level i -= level i+1 only for i < S-1 (:337-357), so the
 * pyramid holds {DoG_0..DoG_{S-2}, G_{S-1}, x, x, x} with x the GaussPyInit value.  The header
 * computes its windows with the integer-length centre float(len_o - 1) / 2 (:251, :279): use
 * GDP_CENTRE_INTLEN (gdp_set_window_centre) to reproduce it (identical to the serial centre when
 * the side is a multiple of 2^(octaves-1), the only sizes its 16-float vector loops handle).
 *   gdp_build_subset:        fused GaussPyInit + GenerateDoG_nomp_dynamic from the input
 *   gdp_generate_dog_subset: GenerateDoG_nomp_dynamic in place on the CURRENT contents (repeated
 *                            calls re-filter, like the reference's timing loop) */
int gdp_build_subset(gdp_ctx* ctx, void* stream);
int gdp_generate_dog_subset(gdp_ctx* ctx, void* stream);

/* ---- extension: true Gaussian convolution pyramid --------------------------
 * NOT the reference's algorithm (which multiplies by a window, :119-131) and carries no parity
 * claim: G_s = base_o (*) k_s, the separable Gaussian with sigma_s = 2/(s+1) (the reference's
 * schedule), normalised taps over radius ceil(3 sigma_s) (<= 6), clamp-to-edge borders; same octave
 * bases, DoG and level layout as gdp_build.  Row bands need their halo rows (below).
 * gdp_conv_taps returns scale s's 13 taps (zero beyond 2R+1) and radius R. */
int gdp_build_gaussian(gdp_ctx* ctx, void* stream);
int gdp_conv_taps(int S, int scale, float* taps13, int* radius);
/* Row bands (multi-GPU split of one image): unlike the reference's
 * pointwise window, the convolution reads 6 rows of every octave beyond a band's own rows, i.e.
 * up to 6 * 2^(octaves-1) input rows above and below it (clipped to the image): *above / *below
 * (0 for whole-image contexts).  A band's gdp_build_gaussian reads them from halo buffers
 * [batch][rows][pitch] (the context's input format): the context's own (gdp_input_halo allocates
 * one on first call, binds it and returns its device address — later calls only return it, with
 * no geometry upload — for a neighbour's rows to be written into —
 * gdp_comm_exchange_halo over RCCL, or any copy) or caller device memory (gdp_bind_input_halo,
 * zero copy; pitch and image stride multiples of 4, rows 16-B aligned).  gdp_device_input returns
 * the device address and pitch of image b's input rows (the context's own or a bound buffer), the
 * rows a neighbour needs.  A band build fails with GDP_ERR_STATE until both halos it needs are
 * set, and only the block-tile kernel (GDP_TUNE_CONV_KERNEL 2, S <= 5, width a multiple of
 * 2^(octaves+1)) runs on bands; its output equals the whole image's rows bit for bit. */
int gdp_conv_halo_rows(const gdp_ctx* ctx, int* above, int* below);
int gdp_input_halo(gdp_ctx* ctx, int side /* 0 above, 1 below */, void** rows, size_t* pitch);
int gdp_bind_input_halo(gdp_ctx* ctx, const void* above, const void* below, size_t pitch, size_t image_stride);
int gdp_device_input(const gdp_ctx* ctx, int b, const void** rows, size_t* pitch);

/* ---- output --------------------------------------------------------------------------------
 * The blocking copies below are ordered after work on the context's OWN stream; if a build was
 * launched on another stream, synchronize that stream first. */
/* Device pointer to level (o, s) of image b: rows x cols float32, row-major, dense. */
const float* gdp_device_level(const gdp_ctx* ctx, int b, int octave, int scale);
/* Copy level (o, s) of image b to a dense host array (blocking). */
int gdp_download_level(gdp_ctx* ctx, int b, int octave, int scale, float* host);
/* Copy level (o, s) of image b into host row pointers — materialises the reference's
 * float**** GaussPy[o][s] rows (GuassDePyramid.h:16) (blocking). */
int gdp_download_level_rows(gdp_ctx* ctx, int b, int octave, int scale, float* const* rows);
/* Mirror image b's whole pyramid into the reference's host layout GaussPy[o][s][row] (the
 * float**** of GuassDePyramid.h:16; rows as held by this context), staging the levels through a
 * double-buffered pinned buffer (the D2H copy of one 32 MiB batch overlaps the host scatter of the
 * previous one; GDP_TUNE_STAGE_KB / _THREADS) (blocking).  What the drop-in classes call after
 * each mutating method. */
int gdp_download_pyramid_rows(gdp_ctx* ctx, int b, float* const* const* const* gauss_py);
/* Copy rows [first_row, first_row + nrows) of level (o, s) of image b (rows as held by this
 * context; a band context's row 0 is its first row) to a dense host array (blocking).  Reads one
 * GaussPy[o][s][r] row range without materialising the level (e.g. 65536^2 images). */
int gdp_download_level_range(gdp_ctx* ctx, int b, int octave, int scale, int first_row, int nrows, float* host);
/* Copy the whole pyramid of image b in the packed layout [o][s][rows][cols] (blocking). */
int gdp_download_pyramid(gdp_ctx* ctx, int b, float* host);
/* Upload a packed pyramid of image b (state restore; used by re-entry tests). */
int gdp_upload_pyramid(gdp_ctx* ctx, int b, const float* host);
/* Host -> device state: the reference's float**** GaussPy IS its pyramid, and GaussFilter /
 * GenerateDoG work on whatever the caller left in it (GuassDePyramid.h:16, :122-131, :140-146).
 * These copy a caller-edited host pyramid back into the device levels (blocking), so an in-place
 * call that follows processes the caller's edits.  The drop-in classes call them before every
 * mutating method when `mirror_host` is set or the caller flagged `host_dirty`
 * (include/GaussDePyramid-HIP.h).
 *   gdp_upload_level:        level (o, s) of image b from a dense rows x cols host array
 *   gdp_upload_level_rows:   the same from host row pointers (GaussPy[o][s])
 *   gdp_upload_pyramid_rows: every level of image b from GaussPy[o][s][row] (the inverse of
 *                            gdp_download_pyramid_rows; rows gathered through the double-buffered
 *                            pinned staging, the H2D copy of one batch overlapping the gather of
 *                            the next)
 *   gdp_upload_image_raw:    image b's pyramid in the device layout (gdp_image_floats floats,
 *                            level (o, s) at gdp_level_offset(ctx, 0, o, s)) in ONE H2D copy — the
 *                            inverse of gdp_download_image_raw */
int gdp_upload_level(gdp_ctx* ctx, int b, int octave, int scale, const float* host);
int gdp_upload_level_rows(gdp_ctx* ctx, int b, int octave, int scale, const float* const* rows);
int gdp_upload_pyramid_rows(gdp_ctx* ctx, int b, const float* const* const* const* gauss_py);
int gdp_upload_image_raw(gdp_ctx* ctx, int b, const float* host);
/* Float elements of one image's packed pyramid (what gdp_download_pyramid writes). */
size_t gdp_packed_floats(const gdp_ctx* ctx);
/* Zero-copy output: write the pyramids into caller-owned DEVICE memory of at least
 * gdp_pyramid_bytes() bytes, 256-B aligned (e.g. a torch tensor that a collective then moves).
 * Level (o, s) of image b starts gdp_level_offset() floats into it.  base = NULL restores the
 * context's own buffer. */
int gdp_set_output_device(gdp_ctx* ctx, float* base, size_t bytes);
size_t gdp_level_offset(const gdp_ctx* ctx, int b, int octave, int scale);

/* ---- host mirror in the device layout (the drop-in classes' fast path) ---------------------
 * gdp_host_alloc: pinned (page-locked) host memory, which one DMA copy fills at the full PCIe
 * rate (gdp_host_free releases it).  gdp_image_floats: floats of one image's pyramid in the device
 * layout — level (o, s) at gdp_level_offset(ctx, 0, o, s), dense rows of cols_o floats, levels
 * 256-B aligned (the dense extent, also under a spread layout).  gdp_download_image_raw: copy
 * image b's pyramid in that layout to `host` in ONE
 * D2H copy (blocking).  A caller that points the reference's float**** rows into such a buffer
 * (GaussPy[o][s][r] = host + gdp_level_offset(ctx, 0, o, s) + r * cols_o) mirrors the device with
 * no per-row scatter (include/GaussDePyramid-HIP.h does). */
int gdp_host_alloc(size_t bytes, void** host);
void gdp_host_free(void* host);
size_t gdp_image_floats(const gdp_ctx* ctx);
int gdp_download_image_raw(gdp_ctx* ctx, int b, float* host);
/* GenerateDoG (in place, all octaves, the context's window centre) of image `b` held in HOST
 * memory in the raw device layout (gdp_download_image_raw's format, `gdp_image_floats` floats):
 * bit-identical to gdp_upload_image_raw(b, host) + gdp_generate_dog + gdp_download_image_raw(b,
 * host) for that image, but pipelined over row chunks so the host-to-device copies, the kernel and
 * the device-to-host copies overlap (two copy streams beside the context's).  `host` should be
 * pinned (gdp_host_alloc) for the copies to be asynchronous.  Blocking.  The overlap is
 * best-effort: the two copy streams share the process's hardware queues (4 on the MI355X boxes)
 * with every other stream and context, so under concurrent work the copies may serialise with
 * the kernel — the result is the same either way.  This is what the C++ drop-ins run for
 * GenerateDoG() when GaussPy is mirrored (mirror_host, the default) and not write-tracked. */
int gdp_generate_dog_mirrored(gdp_ctx* ctx, int b, float* host);

/* ---- write-tracked host mirrors (GuassDePyramid.h:16's two-way GaussPy, main.cpp:66-73) ------
 * A mirror that the caller usually does not write (main.cpp's loop never writes GaussPy) need not
 * be uploaded before every call.  gdp_host_alloc_tracked: `bytes` of host memory for such a mirror
 * — one shared-memory object mapped twice, a view registered with HIP that libgdp's copies use
 * (gdp_upload_image_raw / gdp_download_image_raw / gdp_generate_dog_mirrored* and the single-buffer
 * level / pyramid copies given an address inside it DMA through it at the pinned rate) and the returned CPU view, which is the one ever
 * write-protected (protecting memory the GPU driver registered — hipHostMalloc / hipHostRegister —
 * invalidates the registration and stalls the process's GPU queues, so gdp_host_track refuses such
 * memory).  Freed by gdp_host_free.  GDP_ERR_STATE / _HIP / _NOMEM: not available (use
 * gdp_host_alloc and whole uploads).  It is tracked from the start, not armed.
 * gdp_host_track registers other, plain (unregistered, page-granular) host memory and re-enables
 * tracking of an untracked gdp_host_alloc_tracked buffer; the first call installs a SIGSEGV
 * handler (once per process; faults elsewhere go to the handler installed before it, or take the
 * default action).  gdp_host_arm write-protects the buffer's pages — the caller asserts that the
 * buffer now equals the device copy it mirrors; the first CPU write to each page then faults once,
 * is recorded, and the page is writable again.  gdp_upload_image_written /
 * gdp_generate_dog_mirrored_written are gdp_upload_image_raw / gdp_generate_dog_mirrored that
 * upload only the pages written since the buffer was armed (the caller asserts image b's device
 * pyramid equals the buffer as of arming), and re-arm it; on a buffer that is not tracked or not
 * armed they upload everything (and arm it if tracked).  gdp_host_written_bytes: bytes of the
 * buffer in pages written since arming (GDP_ERR_STATE when not armed).  gdp_host_untrack makes
 * every page writable and stops recording (a gdp_host_alloc_tracked buffer keeps its DMA view).
 * Not seen (untrack such buffers): writes that do not fault on the CPU view — DMA into it, or a
 * system call such as read(2), which fails with EFAULT on a protected page.  GDP_ERR_STATE from
 * gdp_host_track: page protection is unavailable for this memory, it is registered with the GPU,
 * or no slot is free (64). */
int gdp_host_alloc_tracked(size_t bytes, void** host);
int gdp_host_track(void* host, size_t bytes);
int gdp_host_untrack(void* host);
int gdp_host_arm(void* host);
int gdp_host_written_bytes(const void* host, size_t* bytes);
int gdp_upload_image_written(gdp_ctx* ctx, int b, const float* host);
int gdp_generate_dog_mirrored_written(gdp_ctx* ctx, int b, float* host);
/* Deferred download (opt-in; the drop-in's GaussPyramid_hip::DeferDownload).  gdp_host_defer: the
 * caller asserts that image b's device pyramid of `ctx` is now NEWER than the tracked
 * gdp_host_alloc_tracked buffer `host` (at most gdp_image_floats floats), instead of downloading
 * it: every page of the CPU view becomes inaccessible, and the first CPU access to one (read or
 * write) faults, has a block of pages around it copied from the device — 64 pages, doubling to 8192
 * while the faults walk forward, then the next block ahead of the reader too (its first page stays
 * inaccessible until touched, which queues the one after) — on the context's stream by a libgdp
 * helper thread, and arms them
 * (a write then faults once more and is recorded, as above).  Not blocking: the fetches are ordered
 * after the work queued on the context's stream.  Host writes not uploaded yet are discarded (the
 * device copy is declared the newer one).  gdp_host_fetch completes a deferred buffer now (every
 * inaccessible page fetched; gdp_download_image_raw(b, host) of the whole image ends the deferral
 * by overwriting it).  Every libgdp entry taking caller host memory completes deferred buffers
 * first, and gdp_destroy completes those deferred to its context; gdp_host_untrack / gdp_host_arm
 * of a deferred buffer complete it first.  gdp_host_deferred_stats: bytes not fetched yet (whole
 * pages) and the bytes / copies fetched since the last gdp_host_defer (any argument may be NULL).
 * Limits on top of write tracking's: a system call READING a deferred page (write(2), send(2) from
 * it) fails with EFAULT, and a fault while the faulting thread holds a HIP runtime lock (the
 * buffer's CPU view handed straight to a HIP copy) cannot be served — call gdp_host_fetch before
 * either.  GDP_ERR_STATE: `host` is not a tracked gdp_host_alloc_tracked buffer. */
int gdp_host_defer(gdp_ctx* ctx, int b, void* host);
int gdp_host_fetch(void* host);
int gdp_host_deferred_stats(const void* host, size_t* stale_bytes, size_t* fetched_bytes, uint64_t* fetches);
/* Order-independent 64-bit checksum of image b's pyramid (blocking): the sum, mod 2^64, over
 * every word of every level of splitmix64_fin(idx * 0x9E3779B97F4A7C15 + (o*64+s) *
 * 0xD1B54A32D192ED03 + float_bits), idx = global_row * cols + col.  Row-band checksums add up
 * to the whole image's, so multi-GPU runs are verified by gathering 8 bytes per rank. */
int gdp_checksum(gdp_ctx* ctx, int b, uint64_t* out);

/* ---- taps ---------------------------------------------------------------------------------- */
/* The column (axis = 0, from W) or row (axis = 1, from H) window of (o, s) the context uploaded,
 * copied to host (cols_o or rows-of-whole-image_o floats).  Lets tests pin the host taps against
 * the reference's own (tests/golden/taps.npz). */
int gdp_get_taps(gdp_ctx* ctx, int axis, int octave, int scale, float* host);

/* ---- window centre ------------------------------------------------------------------------
 * Where the 1-D window of octave o is centred.  GDP_CENTRE_SERIAL (default): c = (len_f - 1) / 2
 * with len_f the FLOAT axis length halved o times (GuassDePyramid.h:107-115, also
 * GaussPyramid_mpi::GaussFilter, GaussDePyramid-MPI.h:134-143).  GDP_CENTRE_INTLEN:
 * c = float(len_o - 1) / 2 with the INTEGER length len_o = n >> o, what the multi-process variants
 * compute (GaussPyramid_mpi::GenerateDoG_mpi, GaussDePyramid-MPI.h:273; mpitest.cpp:44,123).  The
 * two agree bit for bit whenever every octave's float length is whole (n a multiple of
 * 2^(octaves-1)); they differ for e.g. n = 100 from octave 3 on.  Each mode has its own device
 * tap table, built and uploaded on its first use (a blocking copy); after that a switch only
 * selects the table the NEXT launch reads — no device drain, launches already queued keep the
 * table they were launched with.  Pure layout of the taps: kernels and bytes are unchanged. */
enum { GDP_CENTRE_SERIAL = 0, GDP_CENTRE_INTLEN = 1 };
int gdp_set_window_centre(gdp_ctx* ctx, int mode);
int gdp_get_window_centre(const gdp_ctx* ctx);

/* ---- band state ----------------------------------------------------------------------------
 * Copy the band's rows of every level of `full` (a whole-image context of the same H, W, S and
 * octaves) image `full_image` into band context `band` image `band_image`: the band then holds
 * exactly its rows of the whole pyramid's CURRENT contents, so an in-place call on the band
 * (gdp_generate_dog, gdp_gauss_octave, ...) continues where the whole image left off (the
 * operation is pointwise).  Device-to-device, ordered on `stream` (NULL = the band's stream),
 * blocking.  Before copying it waits for `full`'s OWN stream only: work the caller queued for
 * `full` on any other stream must be complete (or ordered before `stream`) when this is called.
 * (The C++ MPI drop-in does not use it: after single-process calls each rank re-enters on its
 * whole-image context instead, GaussDePyramid-HIP-mpi.h.) */
int gdp_copy_band(gdp_ctx* band, int band_image, const gdp_ctx* full, int full_image, void* stream);

/* ---- tuning (performance only; results are bit-identical for every setting) --------------- */
enum {
    GDP_TUNE_NONTEMPORAL = 1,   /* 1 (default): pyramid stores bypass cache allocation (nt)   */
    GDP_TUNE_BLOCKS_PER_CU = 2, /* value > 0: persistent build grid = CUs x value;
                                   0 (default): one 16x256 tile per block                      */
    GDP_TUNE_GRID = 3,          /* explicit build grid size; 0 (default) = automatic         */
    GDP_TUNE_VARIANT = 4,       /* build kernel code variant (block size / tile shape): one of
                                   the ids gdp_build_variants lists (others GDP_ERR_ARG); default
                                   chosen from the image width and the pyramid backing          */
    GDP_TUNE_TILE_ORDER = 5,    /* build tile order: 0 linear (default), 1 XCD-chunked,
                                   2 XCD row-interleaved                                       */
    GDP_TUNE_INPLACE_SUB = 6,   /* in-place DoG / re-entry passes: blocks per 1024-group chunk,
                                   1 / 2 / 4 / 8 / 16 (default 16 for one image, else 4 up to
                                   32 Mpix per launch, else 1); 0 = one level per wave (k_levels_x);
                                   -16 = 16 x 256 block tiles of k_build's shape (k_levels_tile) */
    GDP_TUNE_WINDOW_SUB = 7,    /* in-place window pass: blocks per chunk (4 default; 1, 2, 8, 16) */
    GDP_TUNE_CONV_KERNEL = 8,   /* gdp_build_gaussian: 0 register sweep (S <= 3), 1 LDS tiles,
                                   2 block tiles (default; one output row per wave, S <= 5) */
    GDP_TUNE_CONV_ROWS = 9,     /* gdp_build_gaussian: block tiles' rows per block (48 default;
                                   16 / 32 with 16 waves, 8 / 16 / 24 / 32 with 8); the sweep's
                                   rows per wave strip (16 / 32) */
    GDP_TUNE_CONV_ORDER = 11,   /* gdp_build_gaussian block order: bit 0 XCD-chunked, bit 1 odd
                                   sweep waves go bottom-up (sweep only), bit 2 octave o's block
                                   rows issued right after the octave-0 rows covering their input
                                   rows.  Default 5 (4 for one image of >= 2^27 pixels) */
    GDP_TUNE_BUILD_LDS = 12,    /* gdp_build: dynamic LDS bytes requested per block (0 default);
                                   used only to cap resident blocks per CU (occupancy) */
    GDP_TUNE_STAGE_KB = 13,     /* row-pointer downloads: KiB per half of the double-buffered
                                   pinned staging buffer (32768 default) */
    GDP_TUNE_STAGE_THREADS = 14, /* row-pointer downloads: host threads scattering a staged batch
                                   into the caller's rows (8 default, at most the host's threads) */
    GDP_TUNE_CONV_WAVES = 15,   /* gdp_build_gaussian block tiles: waves per block (16 default, 8) */
    GDP_TUNE_ZERO_WINDOW = 16,  /* 1 = 4-pixel groups outside the support of every window (all
                                   taps of their row or columns +0, any scale, either centre) skip
                                   their window loads: gdp_build stores their DoG levels as +0
                                   before the input lands and level S+2 as copysign(0, x); the
                                   in-place window passes (gdp_generate_dog, gdp_gauss_*) form
                                   v * 0.0f.  The same bits either way; 0 (default) off */
    GDP_TUNE_STORE_PACE = 17,   /* -1 (default) off; n = 0..3: after each pyramid store of the
                                   build (full, subset and outside-support paths), wait until at
                                   most n memory operations of the wave are outstanding
                                   (s_waitcnt vmcnt(n)); the same bits either way */
    GDP_TUNE_CONV_PACE = 18,    /* the same for gdp_build_gaussian's block tiles (default 2) */
    GDP_TUNE_INPLACE_PACE = 19, /* the same for the in-place re-entry (gdp_generate_dog, k_levels;
                                   default -1): its own field, so tuning the build's pacing never
                                   changes the in-place passes' speed */
    GDP_TUNE_PYRAMID_CHUNK_KB = 20 /* read-only: how the context-owned pyramid is backed — KiB per
                                      separately created physical piece (default 2 MiB, at most
                                      4096 pieces), -1 one piece per image, 0 one hipMalloc */
};
int gdp_set_tuning(gdp_ctx* ctx, int key, int value);
/* The build-kernel variant ids this library holds (GDP_TUNE_VARIANT values): writes up to
 * `capacity` of them to `ids` (may be NULL) and returns how many there are.  Pure table read: no
 * device, no context. */
int gdp_build_variants(int* ids, int capacity);
/* Benchmark every build-kernel variant x tile order x store mode (GDP_TUNE_ZERO_WINDOW,
 * GDP_TUNE_STORE_PACE) in (0, off) (0, 1) (1, off) (1, 0) on the context's current input (`iters`
 * launches each, HIP events on `stream`) and keep the fastest; reports the variant, tile order
 * (the store mode: gdp_get_tuning) and its per-launch ms.  Results are bit-identical for every
 * candidate.  Overwrites the pyramid.  NB: GDP_TUNE_ZERO_WINDOW is context-wide — the pick also
 * applies to the in-place window passes that run later on this context (bit-identical either
 * way); GDP_TUNE_STORE_PACE applies to the builds only (the re-entry has GDP_TUNE_INPLACE_PACE). */
int gdp_autotune(gdp_ctx* ctx, int iters, void* stream, int* variant, int* tile_order, float* ms_per_build);
int gdp_get_tuning(const gdp_ctx* ctx, int key, int* value);

/* ---- misc ---------------------------------------------------------------------------------- */
int gdp_sync(gdp_ctx* ctx);                    /* wait for the context's stream */
void* gdp_stream(const gdp_ctx* ctx);          /* the context's own hipStream_t */
const char* gdp_last_error(const gdp_ctx* ctx); /* ctx may be NULL: last create() failure */
const char* gdp_status_string(int status);
/* Time `iters` back-to-back gdp_build launches on `stream` with HIP events recorded on that same
 * stream; writes the total milliseconds.  Used by bench.py for the per-launch kernel time. */
int gdp_time_builds(gdp_ctx* ctx, int iters, void* stream, float* total_ms);

#ifdef __cplusplus
}
#endif

#endif /* GDP_H_ */
