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
