"""The N > 1 path on CPU: sharding / band arithmetic, and the collector (`generate_dog_mgpu`,
the RCCL counterpart of GenerateDoG_mpi, GaussDePyramid-MPI.h:265-335) run for real across
`gloo` ranks (world 2 and 3) with the same assembly code the GPU path uses.  The band compute is
injected: here it slices the oracle's whole-image pyramid (the GPU path builds band contexts)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dist_mod(pkg):
    import importlib

    return importlib.import_module(pkg.__name__ + ".distributed")


def test_image_plan_covers_every_image_once(pkg):
    d = _dist_mod(pkg)
    for total, world in [(512, 8), (64, 3), (5, 8), (1, 2), (1000, 7)]:
        seen = []
        for r in range(world):
            first, count = d.plan_images(total, world, r)
            seen.extend(range(first, first + count))
        assert seen == list(range(total))


@pytest.mark.parametrize("H,O,world", [(16384, 5, 8), (1080, 5, 4), (100, 7, 2), (4096, 13, 8), (96, 5, 3)])
def test_band_plan_tiles_every_octave(pkg, H, O, world):
    d = _dist_mod(pkg)
    align = d.band_alignment(O)
    bands = [d.plan_band(H, world, r, O) for r in range(world)]
    assert bands[0][0] == 0 and bands[-1][1] == H
    for (a0, a1), (b0, b1) in zip(bands, bands[1:]):
        assert a1 == b0
    for r0, r1 in bands:
        assert r0 % align == 0 and (r1 == H or r1 % align == 0)
    for o in range(O):
        rows = []
        for r0, r1 in bands:
            first, n = d.band_level_rows(H, O, r0, r1)[o]
            rows.extend(range(first, first + n))
        assert rows == list(range(H >> o)), (o, rows[:5])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, S, O, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    pkg = entry.load_package()
    oracle = entry.load_oracle()
    d = __import__(pkg.__name__ + ".distributed", fromlist=["x"])
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # loopback pairs: no host-name lookup
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        img = oracle.lcg_image(n, n, 12345)
        full = oracle.levels(oracle.build_pyramid(img, S, O), n, n, S, O)

        def compute(img_band, r0, r1):  # injected CPU band "build": rows of the oracle's levels
            parts = []
            for o, (first, rows) in enumerate(d.band_level_rows(n, O, r0, r1)):
                for s in range(S + 3):
                    parts.append(torch.from_numpy(full[(o, s)][first:first + rows].ravel().copy()))
            return torch.cat(parts)

        res = d.generate_dog_mgpu(img, n, S, octaves=O, dist=dist, compute=compute)
        t = d.max_over_ranks([1.0 + rank, 5.0 - rank], dist=dist)
        sums = d.gather_checksums([rank * 10 + 1, rank * 10 + 2], dist=dist)
        if rank == 0:
            want = oracle.build_pyramid(img, S, O)
            q.put(("ok", bool(np.array_equal(res.numpy().view(np.uint32), want.view(np.uint32))), t, sums))
        else:
            q.put(("rank", res is None, t, sums))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,S,O,world", [(64, 2, 5, 2), (100, 2, 7, 2), (96, 3, 5, 3)])
def test_collector_generate_dog_mgpu_over_gloo(pkg, n, S, O, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, S, O, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    root = [r for r in results if r[0] == "ok"]
    assert len(root) == 1 and root[0][1], "rank 0 pyramid differs from the oracle"
    assert all(r[1] for r in results if r[0] == "rank"), "non-root ranks must return None"
    assert root[0][2] == [float(world), 5.0]
    assert root[0][3] == [[r * 10 + 1, r * 10 + 2] for r in range(world)]


def _scatter_worker(rank, world, port, per, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    pkg = entry.load_package()
    d = __import__(pkg.__name__ + ".distributed", fromlist=["x"])
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # loopback pairs: no host-name lookup
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        # rank 0 fills rank r's share with the synthetic images' generator stand-in r*1000 + i
        fill = lambda ch, r: ch.copy_(torch.arange(per, dtype=torch.int32) + r * 1000)
        got, secs = d.scatter_images(per, fill, dist=dist)
        ok = bool(torch.equal(got, torch.arange(per, dtype=torch.int32) + rank * 1000))
        t = d.max_over_ranks([secs], dist=dist)
        q.put((rank, ok, t[0] >= 0.0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,per", [(2, 4096), (3, 1000)])
def test_scatter_images_over_gloo(pkg, world, per):
    """The image-batch split (bench.py's scatter of rank 0's batch, RCCL on GPUs) on gloo ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scatter_worker, args=(r, world, port, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in results] == list(range(world))
    assert all(r[1] and r[2] for r in results), results


def test_checksum_restatement_is_order_independent(oracle):
    """Band checksums add up to the whole image's (the property gdp_checksum relies on)."""
    n, S, O = 64, 2, 5
    pyr = oracle.build_pyramid(oracle.lcg_image(n, n, 1), S, O)
    whole = oracle.pyramid_checksum(pyr, n, n, S, O)
    lv = oracle.levels(pyr, n, n, S, O)
    parts = 0
    for r0, r1 in [(0, 16), (16, 48), (48, 64)]:
        for o in range(O):
            a, b = (r0 + (1 << o) - 1) >> o, (r1 + (1 << o) - 1) >> o
            for s in range(S + 3):
                parts = (parts + oracle.level_checksum(lv[(o, s)][a:b], o, s, a)) & 0xFFFFFFFFFFFFFFFF
    assert parts == whole


# ---- halo exchange of the convolution extension on row bands ---------------------------------
@pytest.mark.parametrize("H,O,world", [(16384, 5, 8), (4096, 5, 3), (1080, 5, 4), (512, 4, 2), (300, 3, 5)])
def test_halo_plan_pairs_sends_with_receives(pkg, H, O, world):
    """distributed.halo_plan (what exchange_halo executes): each band's received halo rows are
    exactly its neighbours' rows above / below it (conv_halo_rows of the band), every send has the
    neighbour's matching receive of the same size, and empty bands take no part."""
    d = _dist_mod(pkg)
    plans = {r: d.halo_plan(H, world, r, O) for r in range(world)}
    bands = [d.plan_band(H, world, r, O) for r in range(world)]
    for r, ops in plans.items():
        r0, r1 = bands[r]
        if r1 <= r0:
            assert ops == []
            continue
        above, below = d.conv_halo_rows(H, O, r0, r1)
        recv = {k: (p, n) for k, p, _, n in ops if k.startswith("recv")}
        assert ("recv_above" in recv) == (above > 0) and ("recv_below" in recv) == (below > 0)
        for kind, peer, first, rows in ops:
            p0, p1 = bands[peer]
            if kind == "send":  # the neighbour receives exactly these global rows
                g0 = r0 + first
                mine = [o for o in plans[peer] if o[0].startswith("recv") and o[1] == r]
                assert len(mine) == 1 and mine[0][3] == rows
                if peer == r - 1:  # its halo below = rows [p1, p1 + n)
                    assert mine[0][0] == "recv_below" and g0 == p1
                else:               # its halo above = rows [p0 - n, p0)
                    assert mine[0][0] == "recv_above" and g0 + rows == p0
            elif kind == "recv_above":
                assert peer == r - 1 and rows == above and p1 == r0
            else:
                assert peer == r + 1 and rows == below and p0 == r1


def test_halo_plan_matches_the_rccl_plan(pkg):
    """gdp_comm_halo_plan (the C++ RCCL exchange's schedule) == distributed.halo_plan."""
    import ctypes

    class _Halo(ctypes.Structure):
        _fields_ = [(f, ctypes.c_int) for f in ("kind", "peer", "first_row", "rows")]

    pkg.lib()
    L = ctypes.CDLL(os.path.join(REPO, "sift-parallel-optimization_amd", "lib", "libgdp_comm.so"))
    d = _dist_mod(pkg)
    kinds = {0: "send", 1: "recv_above", 2: "recv_below"}
    for H, O, world in [(16384, 5, 8), (4096, 5, 3), (1080, 5, 4), (300, 3, 5), (4096, 13, 2)]:
        for r in range(world):
            count = ctypes.c_int()
            buf = (_Halo * 8)()
            assert L.gdp_comm_halo_plan(H, world, r, O, buf, 8, ctypes.byref(count)) == 0
            got = [(kinds[buf[i].kind], buf[i].peer, buf[i].first_row, buf[i].rows) for i in range(count.value)]
            assert got == d.halo_plan(H, world, r, O), (H, O, world, r)
    # a band thinner than the halo: 4 x 16-row bands of a 64-row image need 96 halo rows at O = 5
    assert L.gdp_comm_halo_plan(64, 4, 1, 5, buf, 8, ctypes.byref(count)) != 0
    with pytest.raises(ValueError):
        d.halo_plan(64, 4, 1, 5)


def _halo_worker(rank, world, port, H, W, O, B, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    pkg = entry.load_package()
    d = __import__(pkg.__name__ + ".distributed", fromlist=["x"])
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")  # loopback pairs: no host-name lookup
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        full = torch.arange(B * H * W, dtype=torch.int32).reshape(B, H, W)
        r0, r1 = d.plan_band(H, world, rank, O)
        above, below = d.conv_halo_rows(H, O, r0, r1)
        band = full[:, r0:r1].contiguous()
        top = torch.full((B, above, W), -1, dtype=torch.int32)
        bot = torch.full((B, below, W), -1, dtype=torch.int32)
        d.exchange_halo(band, top, bot, H, world, rank, O, dist=dist)
        ok = torch.equal(top, full[:, r0 - above:r0]) and torch.equal(bot, full[:, r1:r1 + below])
        q.put((rank, bool(ok), above, below))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("H,W,O,B,world", [(512, 24, 4, 2, 2), (1080, 16, 5, 1, 3)])
def test_exchange_halo_over_gloo(pkg, H, W, O, B, world):
    """exchange_halo (RCCL point-to-point on GPUs) on gloo ranks: every band receives exactly the
    rows above and below it that its convolution reads, for every image of the batch."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, H, W, O, B, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in results), results
    assert results[0][2] == 0 and results[-1][3] == 0 and any(a > 0 for _, _, a, _ in results)


@pytest.mark.parametrize("H,O,world", [(16384, 5, 8), (4096, 5, 3), (1080, 5, 4), (512, 4, 2), (300, 3, 5), (4096, 9, 2),
                                       (1000, 6, 3)])
def test_halo_rows_cover_every_row_the_band_convolution_reads(pkg, H, O, world):
    """The band convolution stages, for octave o, global octave-o rows [row0_o - 6, row0_o + rows_o
    + 5] clamped to the image (row0_o = ceil(r0 / 2^o), rows_o the band's octave-o rows), i.e.
    input rows (r << o): conv_halo_rows' 6 * 2^(O-1) rows above / below cover all of them (what
    gdp_build_gaussian's host check enforces before launching)."""
    d = _dist_mod(pkg)
    for r in range(world):
        r0, r1 = d.plan_band(H, world, r, O)
        if r1 <= r0:
            continue
        above, below = d.conv_halo_rows(H, O, r0, r1)
        for o, (first, rows) in enumerate(d.band_level_rows(H, O, r0, r1)):
            if rows == 0:
                continue
            Hg = H >> o
            lo = max(0, first - 6) << o
            hi = min(Hg - 1, first + rows - 1 + 6) << o
            assert r0 - above <= lo and hi < r1 + below, (H, O, world, r, o, lo, hi, r0 - above, r1 + below)


# ------------------------------------------------------------ the reference's own role map
def test_scale_plan_matches_the_rccl_plan(pkg):
    """the reference's role map (GaussDePyramid-MPI.h:265-335 — worker i < S+3
    sends scale i of every octave to the collector S+3; ranks > S+3 idle) — distributed.scale_plan
    == gdp_comm_scale_plan for worlds S+4 .. S+6, every rank; the collector receives exactly one
    copy of every (octave, scale) from the worker that owns that scale, each send has the matching
    receive in the same per-pair order; fewer than S+4 ranks is refused by both."""
    import ctypes

    class _Sc(ctypes.Structure):
        _fields_ = [(f, ctypes.c_int) for f in ("kind", "peer", "octave", "scale")]

    pkg.lib()
    L = ctypes.CDLL(os.path.join(REPO, "sift-parallel-optimization_amd", "lib", "libgdp_comm.so"))
    d = _dist_mod(pkg)
    kinds = {0: "send", 1: "recv"}
    for S, O in [(2, 5), (1, 7), (3, 4), (0, 10)]:
        Lv = S + 3
        for world in (Lv + 1, Lv + 2, Lv + 3):
            plans = {}
            for r in range(world):
                count = ctypes.c_int()
                buf = (_Sc * 256)()
                assert L.gdp_comm_scale_plan(S, O, world, r, buf, 256, ctypes.byref(count)) == 0
                got = [(kinds[buf[i].kind], buf[i].peer, buf[i].octave, buf[i].scale) for i in range(count.value)]
                assert got == d.scale_plan(S, O, world, r), (S, O, world, r)
                plans[r] = got
            recv = plans[Lv]
            assert sorted((o, s) for _, _, o, s in recv) == sorted((o, s) for o in range(O) for s in range(Lv))
            for kind, peer, o, s in recv:
                assert kind == "recv" and peer == s
            for r in range(Lv):  # worker r's sends, in order, are the collector's receives from r
                assert plans[r] == [("send", Lv, o, r) for o in range(O)]
                assert [(o, s) for _, p, o, s in recv if p == r] == [(o, s) for _, _, o, s in plans[r]]
            assert all(plans[r] == [] for r in range(Lv + 1, world))
        count = ctypes.c_int()
        assert L.gdp_comm_scale_plan(S, O, Lv, 0, None, 0, ctypes.byref(count)) != 0
        with pytest.raises(ValueError):
            d.scale_plan(S, O, Lv, 0)


def _roles_worker(rank, world, port, n, S, spec, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    pkg = entry.load_package()
    oracle = entry.load_oracle()
    d = __import__(pkg.__name__ + ".distributed", fromlist=["x"])
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        img = oracle.image_from_spec(n, spec)
        O = oracle.octaves(n)
        Lv = S + 3

        def scale_compute(im, i):  # the worker's own step, restated: (x * fc) * fr, integer-length centre
            init = oracle.levels(oracle.init_pyramid(im, S), n, n, S, O)
            out = []
            for o in range(O):
                fc = oracle.taps(n, o, i, centre="intlen")
                lev = (init[(o, i)] * fc[None, :]) * fc[:, None]
                out.append(torch.from_numpy(np.ascontiguousarray(lev, dtype=np.float32).ravel()))
            return out

        def collect(recv):  # the collector's DoG pass (GaussDePyramid-MPI.h:304-318), restated
            pyr = np.concatenate([recv[s][o].numpy() for o in range(O) for s in range(Lv)]).astype(np.float32)
            for o in range(O):
                oracle.dog_octave(pyr, n, n, S, o)
            return torch.from_numpy(pyr)

        res = d.generate_dog_mgpu(img, n, S, dist=dist, roles="reference", scale_compute=scale_compute, collect=collect)
        q.put((rank, None if res is None else res.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,S,spec,world", [(100, 2, "lcg:12345", 6), (512, 2, "lcg:12345", 7), (96, 1, "lcg:7", 5)])
def test_reference_role_map_over_gloo_matches_the_mpi_variant(pkg, oracle, n, S, spec, world):
    """generate_dog_mgpu(roles="reference") on S+4 .. S+5 gloo ranks: the collector (rank S+3) ends
    with the pyramid the reference's own GaussPyramid_mpi::GenerateDoG_mpi collector produced under
    mpiexec (tests/golden/mpi_hashes.json), every other rank with None."""
    import json

    with open(os.path.join(REPO, "tests", "golden", "mpi_hashes.json")) as f:
        recs = [r for r in json.load(f) if r["variant"] == "GaussDePyramid-MPI.h:GenerateDoG_mpi" and r["n"] == n
                and r["S"] == S and r["input"] == spec]
    assert recs, (n, S, spec)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_roles_worker, args=(r, world, port, n, S, spec, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(results[r] is None for r in range(world) if r != S + 3)
    got = results[S + 3]
    O = oracle.octaves(n)
    lv = oracle.levels(got, n, n, S, O)
    for o, row in enumerate(recs[0]["octaves"]):
        for s, h in enumerate(row):
            assert oracle.fnv(lv[(o, s)]) == int(h, 16), (o, s)
