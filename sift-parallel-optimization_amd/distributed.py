"""Multi-GPU drivers: one process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm).

The pyramid is pointwise in the input (halo 0) and images are independent, so the work
partitions with NO data-path collective:

* image sharding (configs 3/4): rank r owns a contiguous block of global image indices;
* row bands (config 5): rank r owns input rows [r0, r1) of one image, aligned to 2^(max(O,5)-1)
  rows so every octave's band rows are whole.

Collectives appear only where the caller asks for a result on one rank:

* `generate_dog_mgpu` — the RCCL counterpart of `GaussPyramid_mpi::GenerateDoG_mpi`
  (GaussDePyramid-MPI.h:265-335).  The reference splits by SCALE (rank i < S+3 filters scale i of
  every octave and streams rows to collector rank S+3, which does all DoG; needs >= S+4 ranks).
  Here ranks split by ROW BAND (any world size, DoG fused on every rank) and the collector,
  rank 0, receives each band's finished pyramid with one gather — the same result on the
  collector: the full pyramid, bit-identical to the serial reference.
* `gather_checksums` — 8 bytes per image/band instead of the pyramids (verification at scale).
* `exchange_halo` — the one real exchange step, and only for the true-Gaussian convolution
  extension on row bands (gdp_build_gaussian): a convolution reads 6 rows of every octave beyond
  a band, so each rank receives up to 6 * 2^(O-1) input rows from each neighbour (point-to-point,
  RCCL over xGMI under "nccl") before its band build.  The reference's pointwise window needs none.

The band/shard arithmetic and the assembly are pure torch / Python so the N > 1 logic runs under
`gloo` on CPU in tests (tests/test_distributed.py) with the same code the GPU path uses.
"""
import numpy as np


def octaves_for(n):
    x = 0
    while n > 0:
        x += 1
        n //= 2
    return x


# ---------------------------------------------------------------------------------- planning
def plan_images(total_images, world, rank):
    """Contiguous block of global image indices for `rank`: (first, count)."""
    base, extra = divmod(int(total_images), int(world))
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def band_alignment(octaves):
    return 1 << (max(int(octaves), 5) - 1)


def plan_band(H, world, rank, octaves):
    """Input rows [r0, r1) of `rank`'s band; every band but the last is a multiple of the
    alignment, so octave o of band r is rows [r0 >> o, r1 >> o) of the whole image."""
    align = band_alignment(octaves)
    per = -(-int(H) // int(world) // align) * align
    r0 = min(H, rank * per)
    r1 = min(H, (rank + 1) * per)
    return r0, r1


def conv_halo_rows(H, octaves, r0, r1):
    """(above, below) input rows a band [r0, r1)'s convolution reads beyond it: 6 * 2^(O-1)
    clipped to the image (libgdp's gdp_conv_halo_rows)."""
    hh = 6 << (int(octaves) - 1)
    return min(hh, r0), min(hh, int(H) - r1)


def halo_plan(H, world, rank, octaves):
    """Point-to-point schedule of `exchange_halo` for `rank`: [(kind, peer, first_row, rows)], kind
    "send" (rows of this band, band-local first row) or "recv_above" / "recv_below" (the whole
    halo buffer).  Neighbours are the adjacent non-empty bands; a band thinner than the rows a
    neighbour needs is an error (the halo would span several bands)."""
    r0, r1 = plan_band(H, world, rank, octaves)
    if r1 <= r0:
        return []
    ops = []
    above, below = conv_halo_rows(H, octaves, r0, r1)
    if rank > 0 and r0 > 0:  # rank - 1 owns the rows just above: it needs our first rows as its "below"
        p0, p1 = plan_band(H, world, rank - 1, octaves)
        need = conv_halo_rows(H, octaves, p0, p1)[1]
        if need > r1 - r0 or above > p1 - p0:
            raise ValueError(f"row bands of {r1 - r0} / {p1 - p0} rows are thinner than the {max(need, above)}-row halo")
        ops.append(("send", rank - 1, 0, need))
        ops.append(("recv_above", rank - 1, 0, above))
    if r1 < H:
        n0, n1 = plan_band(H, world, rank + 1, octaves)
        need = conv_halo_rows(H, octaves, n0, n1)[0]
        if need > r1 - r0 or below > n1 - n0:
            raise ValueError(f"row bands of {r1 - r0} / {n1 - n0} rows are thinner than the {max(need, below)}-row halo")
        ops.append(("send", rank + 1, r1 - r0 - need, need))
        ops.append(("recv_below", rank + 1, 0, below))
    return ops


def exchange_halo(band, above, below, H, world, rank, octaves, dist=None):
    """Fill this rank's halo buffers from its neighbours: `band` [B, rows, W] is this rank's input
    band, `above` / `below` [B, n, W] receive the neighbours' rows (None when not needed).  Under
    "nccl" the tensors are device tensors and the transfers are RCCL point-to-point over xGMI
    (ordered after the current stream's work; the current stream waits for them); under "gloo"
    they are CPU tensors.  One send/recv pair per neighbour and image."""
    if dist is None or world == 1:
        return
    ops = []
    for kind, peer, first, rows in halo_plan(H, world, rank, octaves):
        for b in range(band.shape[0]):
            if kind == "send":
                ops.append(dist.P2POp(dist.isend, band[b, first:first + rows].contiguous(), peer))
            else:
                ops.append(dist.P2POp(dist.irecv, (above if kind == "recv_above" else below)[b], peer))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def band_level_rows(H, octaves, r0, r1):
    """[(first_row, rows)] per octave for the band [r0, r1) of an H-row image (matches
    gdp_level_dims of a band context)."""
    out = []
    for o in range(octaves):
        Hg = H >> o
        first = (r0 + (1 << o) - 1) >> o
        hi = Hg if r1 == H else min(Hg, (r1 + (1 << o) - 1) >> o)
        out.append((first, max(0, hi - first)))
    return out


def packed_band_floats(H, W, S, octaves, r0, r1):
    return sum((S + 3) * rows * (W >> o) for o, (_, rows) in enumerate(band_level_rows(H, octaves, r0, r1)))


# ---------------------------------------------------------------------------------- collectives
def max_over_ranks(values, dist=None, device="cpu"):
    """Element-wise max of a list of floats over all ranks (the bench's slowest-rank time)."""
    import torch

    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.cpu()]


def sum_over_ranks(value, dist=None, device="cpu"):
    """Sum of one integer over all ranks (exact in int64: the job's algorithmic bytes per step)."""
    import torch

    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.cpu()[0])


def gather_checksums(local, dist=None, dst=0):
    """Gather each rank's list of 64-bit checksums to rank `dst` (None elsewhere)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [list(local)]
    out = [None] * dist.get_world_size() if dist.get_rank() == dst else None
    dist.gather_object(list(local), out, dst=dst)
    return out


def scatter_images(per_rank, fill, dist=None, device="cpu", dtype=None):
    """The image-batch split of SURVEY.md §8e's optional path: rank 0 holds every rank's images
    (`fill(chunk, r)` writes rank r's `per_rank` elements into `chunk`) and one collective scatter
    (RCCL over xGMI on GPUs, gloo on CPU) hands each rank its share.  Returns (this rank's
    elements, seconds of the scatter between two barriers)."""
    import time

    import torch

    dtype = dtype or torch.int32
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    recv = torch.empty(per_rank, dtype=dtype, device=device)
    chunks = None
    if rank == 0:
        big = torch.empty(world * per_rank, dtype=dtype, device=device)
        chunks = [big[r * per_rank:(r + 1) * per_rank] for r in range(world)]
        for r, ch in enumerate(chunks):
            fill(ch, r)
    sync = torch.cuda.synchronize if torch.device(device).type == "cuda" else (lambda: None)
    sync()
    if world == 1:
        t0 = time.perf_counter()
        recv.copy_(chunks[0])
        sync()
        return recv, time.perf_counter() - t0
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    dist.scatter(recv, chunks, src=0)
    sync()
    dist.barrier()
    return recv, time.perf_counter() - t0


def gather_packed_bands(band, sizes, dist=None, dst=0):
    """The collector's exchange as ONE collective (the reference sends every level row by row,
    MPI_Send / MPI_Recv at GaussDePyramid-MPI.h:285,298): each rank's packed band pyramid `band`
    (sizes[r] float32 elements on rank r) is padded to the largest band and gathered to rank `dst`
    (RCCL over xGMI for GPU tensors, gloo for CPU tensors).  Returns (the per-rank bands trimmed to
    their sizes on `dst`, None elsewhere; seconds of the gather between two barriers)."""
    import time

    import torch

    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    if world == 1:
        return [band[:sizes[0]]], 0.0
    if band.numel() != sizes[rank]:
        raise ValueError(f"rank {rank}: band of {band.numel()} floats, plan says {sizes[rank]}")
    buf = torch.zeros(max(sizes), dtype=torch.float32, device=band.device)
    buf[:band.numel()] = band
    gathered = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    sync = torch.cuda.synchronize if buf.is_cuda else (lambda: None)
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    dist.gather(buf, gathered, dst=dst)
    sync()
    secs = time.perf_counter() - t0
    dist.barrier()
    if rank != dst:
        return None, secs
    return [g[:sizes[r]] for r, g in enumerate(gathered)], secs


def assemble_bands(H, W, S, octaves, world, packed_bands, like=None):
    """Collector-side assembly: the packed band pyramids of ranks 0..world-1 (torch tensors,
    any device) -> the packed pyramid of the whole image, in the oracle's [o][s][rows][cols]
    layout.  Pure device copies; no arithmetic touches the values."""
    import torch

    total = sum((S + 3) * (H >> o) * (W >> o) for o in range(octaves))
    ref = like if like is not None else packed_bands[0]
    full = torch.empty(total, dtype=torch.float32, device=ref.device)
    layouts = [band_level_rows(H, octaves, *plan_band(H, world, r, octaves)) for r in range(world)]
    off_full = 0
    band_off = [0] * world
    for o in range(octaves):
        cols = W >> o
        rows_full = H >> o
        for s in range(S + 3):
            for r in range(world):
                first, rows = layouts[r][o]
                if rows:
                    n = rows * cols
                    dst = off_full + first * cols
                    full[dst:dst + n] = packed_bands[r][band_off[r]:band_off[r] + n]
                    band_off[r] += n
            off_full += rows_full * cols
    return full


def scale_plan(S, octaves, world, rank):
    """The reference's role map (GaussPyramid_mpi::GenerateDoG_mpi, GaussDePyramid-MPI.h:265-335) on
    `rank`: [(kind, peer, octave, scale)] — worker i < S+3 sends level (o, i) of every octave to the
    collector S+3 (octave order, :285); the collector receives worker-major, then octave (:295-303);
    ranks > S+3 take no part.  Needs world >= S+4 (the reference's own requirement).  Equals
    libgdp_comm's gdp_comm_scale_plan."""
    L = int(S) + 3
    if world < L + 1:
        raise ValueError(f"the reference's role map needs >= S+4 = {L + 1} ranks, world is {world}")
    if rank < L:
        return [("send", L, o, rank) for o in range(octaves)]
    if rank == L:
        return [("recv", j, o, j) for j in range(L) for o in range(octaves)]
    return []


def generate_dog_mgpu(img, n, S, octaves=0, dist=None, compute=None, device=None, centre="serial", roles="bands",
                      scale_compute=None, collect=None):
    """Collector semantics of GenerateDoG_mpi (GaussDePyramid-MPI.h:265-335) over RCCL.

    Every rank passes the same `img` (the reference also replicates the input on every rank,
    GaussDePyramid-MPI.h:60-84); rank r builds the row band plan_band(n, world, r, octaves) on its
    GPU; rank 0 gathers the bands and returns the full packed pyramid (torch tensor, on its GPU);
    other ranks return None.  `compute(img_band, r0, r1) -> packed float32 torch tensor` may be
    injected (tests use it to run this logic under gloo on CPU); by default it is the HIP build.
    `centre="intlen"` reproduces the MPI variant's own window centre (GaussDePyramid-MPI.h:273;
    differs from the serial header only when n is not a multiple of 2^(octaves-1)).

    roles="reference" runs the reference's own role map instead (scale_plan; world >= S+4): worker
    i windows scale i of every octave of its pyramid with the variant's integer-length centre
    (`scale_compute(img, i) -> [O flat float32 tensors]`, default: a libgdp context's
    gdp_gauss_scales), sends it to the collector S+3, which forms every DoG level
    (`collect(levels[j][o]) -> packed pyramid`, default: the collector's context, gdp_dog_range)
    and returns the pyramid; every other rank returns None.
    """
    import torch

    if roles == "reference":
        return _generate_dog_roles(img, n, S, octaves, dist, device, scale_compute, collect)
    if roles != "bands":
        raise ValueError(f"roles must be 'bands' or 'reference', not {roles!r}")

    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    O = octaves or octaves_for(n)
    r0, r1 = plan_band(n, world, rank, O)
    img = np.asarray(img, dtype=np.int32)[:n, :n]
    if compute is None:
        compute = _gpu_band_compute(n, n, S, O, device, centre)
    band = compute(np.ascontiguousarray(img[r0:r1]), r0, r1)
    if world == 1:
        return assemble_bands(n, n, S, O, 1, [band])
    sizes = [packed_band_floats(n, n, S, O, *plan_band(n, world, r, O)) for r in range(world)]
    bands, _ = gather_packed_bands(band, sizes, dist=dist, dst=0)
    if rank != 0:
        return None
    return assemble_bands(n, n, S, O, world, bands)


def _generate_dog_roles(img, n, S, octaves, dist, device, scale_compute, collect):
    """generate_dog_mgpu(roles="reference"): the reference's scale split over point-to-point
    transfers (RCCL over xGMI under "nccl", gloo in CPU tests)."""
    import torch

    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if world > 1 else 0
    O = octaves or octaves_for(n)
    L = S + 3
    plan = scale_plan(S, O, world, rank)  # raises below S+4 ranks, as the reference cannot run either
    img = np.ascontiguousarray(np.asarray(img, dtype=np.int32)[:n, :n])
    sizes = [(n >> o) * (n >> o) for o in range(O)]
    if scale_compute is None or collect is None:
        dflt_scale, dflt_collect = _gpu_role_compute(n, S, O, device)
        scale_compute, collect = scale_compute or dflt_scale, collect or dflt_collect
    if rank < L:
        levels = scale_compute(img, rank)  # GaussDePyramid-MPI.h:271-284: window this rank's scale
        ops = [dist.P2POp(dist.isend, levels[o].contiguous(), peer) for kind, peer, o, _ in plan]
    elif rank == L:
        dev = torch.device("cpu") if dist.get_backend() == "gloo" else torch.device("cuda", torch.cuda.current_device())
        recv = [[torch.empty(sizes[o], dtype=torch.float32, device=dev) for o in range(O)] for _ in range(L)]
        ops = [dist.P2POp(dist.irecv, recv[j][o], peer) for kind, peer, o, j in plan]
    else:
        return None  # ranks > S+3 take no part (:269-335)
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    if rank != L:
        return None
    return collect(recv)  # :304-318: every DoG level on the collector


def _gpu_role_compute(n, S, O, device):
    """Default worker / collector steps of the reference role map on a libgdp whole-image context
    (integer-length window centre, GaussDePyramid-MPI.h:273)."""
    import torch

    from .gausspyramid import PyramidContext

    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)

    def bound_ctx():
        ctx = PyramidContext(n, n, S=S, octaves=O, batch=1, device=dev.index, centre="intlen")
        out = torch.empty(ctx.pyramid_bytes() // 4 + 64, dtype=torch.float32, device=dev)
        shift = (-out.data_ptr() % 256) // 4
        view = out[shift:shift + ctx.pyramid_bytes() // 4]
        ctx.bind_device_output(view.data_ptr(), ctx.pyramid_bytes(), keepalive=out)
        return ctx, view

    def levels_of(ctx, view, s):
        return [view[ctx.level_offset(0, o, s):ctx.level_offset(0, o, s) + (n >> o) * (n >> o)] for o in range(O)]

    def scale_compute(img, i):
        ctx, view = bound_ctx()
        ctx.set_input(img)
        ctx.init()                              # GaussPyInit (the constructor's state)
        ctx.gauss_scales(i, i + 1)              # this worker's scale, every octave
        ctx.sync()
        return levels_of(ctx, view, i)

    def collect(recv):
        ctx, view = bound_ctx()
        for j in range(S + 3):
            for o, dst in enumerate(levels_of(ctx, view, j)):
                dst.copy_(recv[j][o])
        torch.cuda.current_stream(dev).synchronize()
        ctx.dog_range(0, O)
        ctx.sync()
        return torch.cat([lv for o in range(O) for s in range(S + 3) for lv in [levels_of(ctx, view, s)[o]]])

    return scale_compute, collect


def _gpu_band_compute(H, W, S, O, device, centre="serial"):
    """Default band compute: a libgdp band context writing straight into a torch tensor."""
    import torch

    from .gausspyramid import PyramidContext

    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)

    def compute(img_band, r0, r1):
        if r1 <= r0:  # more ranks than aligned bands: this rank holds no rows
            return torch.empty(0, dtype=torch.float32, device=dev)
        with PyramidContext(H, W, S=S, octaves=O, batch=1, device=dev.index, row_begin=r0, row_end=r1,
                            centre=centre) as ctx:
            out = torch.empty(ctx.pyramid_bytes() // 4 + 64, dtype=torch.float32, device=dev)
            base = out.data_ptr()
            shift = (-base % 256) // 4  # 256-B aligned view
            view = out[shift:shift + ctx.pyramid_bytes() // 4]
            ctx.bind_device_output(view.data_ptr(), ctx.pyramid_bytes(), keepalive=out)
            ctx.set_input(img_band)
            ctx.build(torch.cuda.current_stream(dev))
            parts = []
            for o in range(O):
                rows, cols, _ = ctx.level_dims(o)
                for s in range(S + 3):
                    off = ctx.level_offset(0, o, s)
                    parts.append(view[off:off + rows * cols])
            packed = torch.cat(parts) if parts else view[:0].clone()
            torch.cuda.current_stream(dev).synchronize()
            return packed

    return compute
