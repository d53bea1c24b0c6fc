#!/usr/bin/env python3
"""Benchmark of the Gaussian / DoG pyramid build on MI355X — BASELINE.json's metric:
"Mpix/s full Gaussian+DoG pyramid build; % HBM roofline at 1/2/4/8 GPU".

A step is one fused pyramid build (GaussPyInit + GenerateDoG of GuassDePyramid.h, S = 2,
5 octaves) over each rank's resident batch of synthetic int32 images, through the C ABI
(libgdp.so, one kernel launch per step).  Input pixels are generated on each GPU before the timed
region; nothing leaves HBM inside it.  Consecutive steps cycle through independent buffer sets
(input + pyramid) totalling > 2 GiB per GPU (--rotate), so a small workload cannot be served from
the 256 MB Infinity Cache between steps: the rate is the HBM rate.  One process per GPU (torchrun), ranks shard the images
(no data-path collective: images are independent), max-over-ranks timing.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

--gpus N > 1 without a launcher (WORLD_SIZE unset) starts N rank processes itself — one per GPU,
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 and a file rendezvous (GDP_BENCH_RDV) in
their environment — before anything touches the GPU, and exits with the first failing rank's
status; under torchrun
(WORLD_SIZE set) it is one of the ranks.  A world size that differs from --gpus, or more ranks
than visible GPUs under "nccl", is an error.

Workloads (BASELINE.json configs; c2 is the default, the single-GPU config the metric names):
  c2: 4096x4096, 5 octaves, 1 image per GPU per step
  c3: 64 x 1080x1920 (HxW), 5 octaves, per GPU per step (persistent kernel)
  c4: 64 x 4096x4096, 5 octaves, per GPU per step (MPI-variant image sharding)
  c5: 16384x16384, 5 octaves, ONE image split into row bands across the ranks
Prints ONE JSON line on rank 0 (contract in the task description).
"""
import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mpix/s full Gaussian+DoG pyramid build; % HBM roofline at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
SEED = 0x5EED
# A step's working set (input + pyramid) is rotated over enough independent buffer sets to exceed
# this many bytes, 8x MI355X's 256 MB Infinity Cache (MALL): otherwise a small workload (config 2:
# 514 MB per image) re-writes lines the MALL still holds from the previous step and the "HBM" rate
# exceeds what HBM can do (measured: 8.17 TB/s on config 2 without rotation).
ROTATE_BYTES = 2 << 30

CONFIGS = {
    "c2": dict(H=4096, W=4096, batch=1, O=5, band=False, name="1xMI355X 4096x4096 image, 5 octaves x 5 scales"),
    "c3": dict(H=1080, W=1920, batch=64, O=5, band=False, name="batch of 64 x 1920x1080 images, 5 octaves x 5 scales"),
    "c4": dict(H=4096, W=4096, batch=64, O=5, band=False, name="64 x 4096x4096 images per GPU, 5 octaves x 5 scales"),
    "c5": dict(H=16384, W=16384, batch=1, O=5, band=True, name="16384x16384 single image in row bands, 5 octaves"),
}


def pyramid_pixels(H, W, O, rows=None):
    """P = sum over octaves of rows_o * cols_o."""
    return sum(((rows if rows is not None else H) >> o) * (W >> o) for o in range(O))


def algorithmic_bytes(H, W, S, O, batch, in_bytes=4):
    """B = 4*H*W (read every int32 input pixel once; 1*H*W for uint8 input) + 4*(S+3)*P (write the
    final pyramid once)."""
    return batch * (in_bytes * H * W + 4 * (S + 3) * pyramid_pixels(H, W, O))


def cpu_info():
    model = platform.processor() or "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def host_threads():
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(budget_s):
    """The reference's AVX512xOpenMP path (GaussDePyramid-AVX512xOpenMP.h:240-364) on the host cores,
    timed on a bounded sample: 4096x4096 image (the c2 workload's input), all its octaves, reps
    sized to ~budget_s.  Falls back to the oracle's restatement ("port") when oracle/_ref is absent
    or the host lacks AVX-512.  Uses the oracle only as the CPU baseline, never on the GPU path."""
    import __graft_entry__ as entry

    oracle = entry.load_oracle()
    n, S = 4096, 2
    threads = host_threads()
    spec = f"synth:{SEED:#x}:0"
    have_bin, have_isa = oracle.ref_binary("avx512"), oracle.host_has_avx512()
    if have_bin and have_isa:
        probe = oracle.ref_time("time-a512omp", n, S, spec, 2, threads)
        reps = max(3, min(400, int(budget_s / max(probe["ms_median"] / 1e3, 1e-4))))
        rec = oracle.ref_time("time-a512omp", n, S, spec, reps, threads)
        serial = oracle.ref_time("time-serial", n, S, spec, 5) if oracle.ref_binary("serial") else None
        out = {
            "value": round(n * n / (rec["ms_median"] / 1e3) / 1e6, 3), "unit": "Mpix/s", "cores": threads,
            "kind": "reference",
            "sample": (f"GaussPyramid_a512omp::GenerateDoG_nomp_dynamic (reference header compiled in place, "
                       f"counnt={threads}) on one {n}x{n} synthetic image, all {rec['octaves']} octaves, "
                       f"median of {rec['reps']} calls after a warm-up; GaussPyInit untimed as in the reference. "
                       f"NB: that path filters only S of the S+3 scales and forms 1 of the S+2 DoG levels "
                       f"(~34% of the full build's bytes)"),
            "cpu": cpu_info(),
            # which reference text the timed binary was compiled from: oracle/Makefile's stamp
            # (sha256 of every source the compile read, compiler, flags; oracle/stamp.py)
            "provenance": _ref_stamp(have_bin),
        }
        if serial:
            out["serial_full_semantics"] = {"value": round(n * n / (serial["ms_median"] / 1e3) / 1e6, 3),
                                            "unit": "Mpix/s", "cores": 1,
                                            "sample": f"GuassDePyramid.h GenerateDoG, {n}x{n}, median of {serial['reps']}"}
        # the reference's fastest FULL-semantics CPU path: AVX-512 x pthreads, octaves round-robin
        # over its own 7 worker threads (GaussDePyramid-AVX512xPTHREAD.h:143-261)
        xp_probe = oracle.ref_time("time-a512xp", n, S, spec, 2)
        if xp_probe:
            xp_reps = max(3, min(200, int(0.3 * budget_s / max(xp_probe["ms_median"] / 1e3, 1e-4))))
            xp = oracle.ref_time("time-a512xp", n, S, spec, xp_reps)
            out["a512xp_full_semantics"] = {
                "value": round(n * n / (xp["ms_median"] / 1e3) / 1e6, 3), "unit": "Mpix/s", "cores": 7,
                "sample": f"GaussPyramid_a512xp::GenerateDoG (reference header compiled in place, 7 pthreads), "
                          f"{n}x{n}, all {xp.get('octaves', '?')} octaves, median of {xp['reps']} calls; GaussPyInit untimed"}
        return out
    import numpy as np

    reason = ("oracle/_ref/ref_avx512 (the reference header compiled in place) is not in this tree"
              if not have_bin else "this host's CPU lacks AVX-512F, which the reference header needs")
    print(f"bench.py: cpu_baseline falls back to the oracle restatement (kind 'port'): {reason}",
          file=sys.stderr, flush=True)
    img = oracle.synthetic_image(n, n, SEED, 0)
    base = oracle.init_pyramid(img, S)
    O = oracle.octaves(n)
    times = []
    t_end = time.perf_counter() + budget_s
    while time.perf_counter() < t_end or len(times) < 3:
        pyr = base.copy()
        t0 = time.perf_counter()
        oracle.subset_a512omp(pyr, n, n, S, O)
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    return {"value": round(n * n / med / 1e6, 3), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "reason": reason,
            "sample": f"oracle restatement of GenerateDoG_nomp_dynamic (OpenMP, {threads} threads), {n}x{n}, "
                      f"median of {len(times)} calls", "cpu": cpu_info()}


def _ref_stamp(binary):
    """oracle/_ref/<binary>.stamp.json (written by `make -C oracle ref`), or why it is missing."""
    try:
        with open(binary + ".stamp.json") as f:
            st = json.load(f)
    except (OSError, ValueError, TypeError):
        return {"status": "no stamp next to the binary (built before oracle/stamp.py existed): provenance unrecorded"}
    import hashlib

    with open(binary, "rb") as f:
        actual = hashlib.sha256(f.read()).hexdigest()
    return {"binary_sha256": st.get("binary_sha256"), "binary_matches_stamp": actual == st.get("binary_sha256"),
            "sources_sha256": {os.path.basename(k): v for k, v in st.get("sources", {}).items()},
            "compiler": st.get("compiler"), "flags": st.get("flags"), "built_utc": st.get("built_utc")}


def complete_line(result, args, rank, world, dist, mg, device, bytes_launch, wall):
    """The parts of the line every N needs: the whole-job roofline — every
    rank's algorithmic bytes per step over the job's step time, against N GPUs' peak
    (`frac_aggregate`; `frac` is the per-launch rate of rank 0's kernel, its bytes over its launch)
    — and the CPU baseline (attach_cpu_baseline).  Collective: every rank calls it."""
    total = mg.sum_over_ranks(bytes_launch, dist=dist, device=device)
    if rank == 0:
        result["roofline"]["aggregate_bytes_per_step"] = total
        result["roofline"]["frac_aggregate"] = round(total / (wall / args.steps) / (world * HBM_PEAK_GBS * 1e9), 4)
    attach_cpu_baseline(result, args, rank, world, dist)


def attach_cpu_baseline(result, args, rank, world, dist):
    """The reference's CPU path timed on this box's host cores in the same run (north star), on
    rank 0 only and after every rank's timed region: at N > 1 the other ranks wait at a barrier
    until rank 0 has sampled it, so no GPU step overlaps the CPU sample and the line is complete at
    every N (mpitest.cpp:95-96 times its collector in the same run)."""
    if args.no_cpu:
        if rank == 0:
            result["cpu_baseline"] = None
    elif rank == 0:
        base = cpu_baseline(args.cpu_budget)
        base["semantics_vs_this_line"] = {
            "build": "the GPU line computes the full GenerateDoG output; the timed CPU path its subset (see sample); "
                     "serial_full_semantics / a512xp_full_semantics are the full-output CPU rates",
            "subset": "identical: the GPU line computes GenerateDoG_nomp_dynamic's output",
            "conv": "none: the reference has no convolution (the extension has no CPU counterpart)",
        }.get(args.op, "in-place pass vs the CPU build path (different work)")
        if world > 1:
            base["when"] = (f"rank 0, after all {world} ranks finished their timed steps; ranks 1..{world - 1} "
                            f"waited at a barrier meanwhile (no GPU work during the sample)")
        result["cpu_baseline"] = base
        if args.op == "build" and world == 1:
            result["dropin_call"] = dropin_call_cost()
    if dist is not None and world > 1:
        dist.barrier()


PMC_ARCHIVE = "pmc_records.json"  # the kept records of earlier rounds, one list (tools/prune_profiles.py)


def pmc_records():
    """Every PMC record under profiles/ as (name, record), in name order (later = newer): the
    individual pmc_*.json files the collectors write, and the records gathered into
    profiles/pmc_records.json (each keeps its original file name under "file").  A record's
    citation is profiles/<file> when that file exists, else profiles/pmc_records.json#<file>."""
    pdir = os.path.join(REPO, "profiles")
    out = {}
    if not os.path.isdir(pdir):
        return []
    names = sorted(f for f in os.listdir(pdir) if f.startswith("pmc_") and f.endswith(".json"))
    stamp = tuple((f, os.path.getmtime(os.path.join(pdir, f))) for f in names)
    if _PMC_CACHE.get("stamp") == stamp:
        return _PMC_CACHE["records"]
    agg = os.path.join(pdir, PMC_ARCHIVE)
    if os.path.exists(agg):
        with open(agg) as fh:
            for rec in json.load(fh):
                out[rec["file"]] = (f"{PMC_ARCHIVE}#{rec['file']}", {k: v for k, v in rec.items() if k != "file"})
    for f in os.listdir(pdir):
        if f.startswith("pmc_") and f.endswith(".json") and f != PMC_ARCHIVE:
            try:
                with open(os.path.join(pdir, f)) as fh:
                    out[f] = (f, json.load(fh))
            except (OSError, ValueError):
                continue
    _PMC_CACHE.update(stamp=stamp, records=[out[k] for k in sorted(out)])
    return _PMC_CACHE["records"]


_PMC_CACHE = {}


def concurrent_streams(ctxs, bytes_launch, n_streams=4, launches=200):
    """Informational, after the timed region (never `value`): the serving mode of INTEGRATION §5 —
    independent single-image builds of the rotated contexts launched round-robin on `n_streams`
    torch streams, so one launch's drain overlaps the next one's ramp.  Ms per image over
    `launches` builds (host clock around synchronizes), its fraction of 8 TB/s for the same
    algorithmic bytes, and whether every context's checksum is unchanged."""
    import torch

    n_streams = max(1, min(n_streams, len(ctxs)))
    sums = [c.checksum(0) for c in ctxs]
    streams = [torch.cuda.Stream() for _ in range(n_streams)]
    for it in range(2):  # a warm pass over every context, then the timed pass
        k_max = len(ctxs) * 2 if it == 0 else launches
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(k_max):
            ctxs[k % len(ctxs)].build(streams[k % n_streams])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    ms = dt * 1e3 / launches
    return {"streams": n_streams, "contexts": len(ctxs), "launches": launches, "ms_per_image": round(ms, 6),
            "frac_of_8TBps": round(bytes_launch / (ms / 1e3) / (HBM_PEAK_GBS * 1e9), 4),
            "checksums_unchanged": all(c.checksum(0) == v for c, v in zip(ctxs, sums)),
            "note": "informational: one image per launch, launches of different contexts overlapping on "
                    "several streams (INTEGRATION §5); `value` and `roofline` time one launch at a time"}


def dropin_call_cost(n=4096, calls=5):
    """Per-call cost of the C++ drop-in class (include/GaussDePyramid-HIP.h, main.cpp's timing loop:
    GenerateDoG() on the same object) through examples/state_hip, outside the timed region: with
    the default two-way GaussPy (mirror_host, write-tracked: the caller writes nothing, so only the
    in-place pass and the pyramid's download over PCIe, pipelined over row chunks), with the write
    tracking off (TrackWrites(false): the whole pyramid uploaded too, round 5's default) and with
    mirror_host = false (the device pyramid is the state; no PCIe), and with the deferred download
    (DeferDownload(true): nothing copied back until GaussPy is read; the read_all_* pair prices the
    first full read after a call, eager against deferred).  ADVICE r4 / VERDICT r5 item 2."""
    import re
    import subprocess

    exe = os.path.join(REPO, "examples", "state_hip")
    if not os.path.exists(exe):
        return None
    out = {"n": n, "S": 2, "calls": calls,
           "source": "examples/state_hip hip <n> 2 ones - [track:0 | mirror:0 | defer:1] dog time:<calls>; "
                     "[defer:1] dog read"}
    for key, ops in (("mirror_host_ms", []), ("mirror_untracked_ms", ["track:0"]), ("device_state_ms", ["mirror:0"]),
                     ("mirror_deferred_ms", ["defer:1"])):
        # one untimed call first (the mirror's copy streams and events are created on first use)
        r = subprocess.run([exe, "hip", str(n), "2", "ones", "-", *ops, "dog", f"time:{calls}"], capture_output=True,
                           text=True, timeout=120)
        m = re.search(r"([0-9.]+) ms per GenerateDoG", r.stderr)
        out[key] = float(m.group(1)) if (r.returncode == 0 and m) else None
    # main.cpp's own size (n = 512, main.cpp:19): the default mirror and the deferred one
    for key, ops in (("n512_mirror_host_ms", []), ("n512_mirror_deferred_ms", ["defer:1"])):
        r = subprocess.run([exe, "hip", "512", "2", "ones", "-", *ops, "dog", f"time:{20 * calls}"], capture_output=True,
                           text=True, timeout=120)
        m = re.search(r"([0-9.]+) ms per GenerateDoG", r.stderr)
        out[key] = float(m.group(1)) if (r.returncode == 0 and m) else None
    # reading every GaussPy float once after a call: eager mirror (already on the host) against the
    # deferred one (each page fetched on first touch) — the difference is what deferral moves to the
    # first read
    for key, ops in (("read_all_eager_ms", ["dog", "read"]), ("read_all_deferred_ms", ["defer:1", "dog", "read"])):
        r = subprocess.run([exe, "hip", str(n), "2", "ones", "-", *ops], capture_output=True, text=True, timeout=120)
        m = re.search(r"read_ms=([0-9.]+)", r.stderr)
        out[key] = float(m.group(1)) if (r.returncode == 0 and m) else None
    pyr = 4 * 5 * pyramid_pixels(n, n, octaves_for(n))  # bytes each way per call
    if out.get("mirror_host_ms"):
        out["pcie_GBps_d2h"] = round(pyr / (out["mirror_host_ms"] / 1e3) / 1e9, 1)
    if out.get("mirror_untracked_ms"):
        out["pcie_GBps_each_way_untracked"] = round(pyr / (out["mirror_untracked_ms"] / 1e3) / 1e9, 1)
    return out


def octaves_for(n):
    x = 0
    while n > 0:
        x, n = x + 1, n // 2
    return x


def latest_conv_pmc(config_key, tun):
    """PMC record of the convolution extension's kernel on this workload with the run's conv
    kernel / rows / order (profiles/pmc_<cfg>_conv*_*.json), or None."""
    best = None
    for f, rec in pmc_records():
        if rec.get("config") == config_key and rec.get("op") == "conv" and rec.get("kernel_bytes_per_launch") and \
                (rec.get("conv_kernel"), rec.get("conv_rows"), rec.get("conv_order"), rec.get("conv_halo", 2)) == \
                (tun["conv_kernel"], tun["conv_rows"], tun["conv_order"], tun.get("conv_halo", 2)):
            best = dict(rec, file=f)
    return best


def latest_pmc(config_key, variant, tile_order, op="build", levels=5, zero_window=0, band_of=None,
               image_stride_mb=None, chunk_kb=None):
    """PMC-derived HBM bytes per launch of THIS kernel instance on this workload, from the newest
    PMC record (pmc_records()) written by tools/pmc_variants.py from separate rocprofv3 --pmc passes,
    whose recorded build variant, tile order and zero-window mode equal the run's; None when no profile of that
    instance exists (the traffic of another variant would describe a different kernel).  band_of = N:
    the row-band config's per-rank launch at N ranks (rank 0's band of N, profiled on one GPU by
    tools/pmc_variants.py --band-of N), not the whole image's.  image_stride_mb: the spread layout's
    records (a GDP_EXPERIMENTS build), kept apart from the dense layout's.  chunk_kb: the run's pyramid
    backing (GDP_TUNE_PYRAMID_CHUNK_KB); a record of the same backing is preferred, else one of
    another backing (the backing moves pages, not bytes: DESIGN.md §4) — the file is named either way."""
    best, same = None, None
    # the template instance too: k_build<5, ...> (S + 3 = 5 levels unrolled) or k_build<0, ...>
    lt = f"k_build<{5 if levels == 5 else 0},"
    for f, rec in pmc_records():
        if rec.get("config") == config_key and rec.get("op", "build") == op and \
                rec.get("kernel_bytes_per_launch") and rec.get("variant") == variant and \
                rec.get("tile_order") == tile_order and rec.get("input_format", "i32") == "i32" and \
                rec.get("zero_window", 0) == zero_window and rec.get("band_of") == band_of and \
                rec.get("image_stride_mb") == image_stride_mb and \
                lt in rec.get("kernel", lt):
            best = dict(rec, file=f)
            if rec.get("pyramid_chunk_kb", 0) == (chunk_kb or 0):
                same = best
    return same or best


def latest_inplace_pmc(config_key, op, tun):
    """PMC record of an in-place pass (--op regen: k_levels<MODE 3> / k_levels_x, keyed by
    GDP_TUNE_INPLACE_SUB; --op gauss: k_window, keyed by GDP_TUNE_WINDOW_SUB) with the run's block
    shape, or None."""
    key = "inplace_sub" if op == "regen" else "window_sub"
    best = None
    for f, rec in pmc_records():
        if rec.get("config") == config_key and rec.get("op") == op and rec.get("kernel_bytes_per_launch") and \
                rec.get(key) == tun[key] and rec.get("zero_window", 0) == tun.get("zero_window", 0):
            best = dict(rec, file=f)
    return best


def launch_ranks(n, argv, script=None):
    """`bench.py --gpus N` with no launcher: start N rank processes of this script (one per GPU)
    and wait for them.  Runs before anything imports torch or touches the GPU; the parent never
    does.  If a rank fails the others are stopped (they would wait in a collective forever).

    Rendezvous: a FILE in a fresh private directory (GDP_BENCH_RDV, torch.distributed's file://
    init method), not a TCP port.  Round 2 picked MASTER_PORT by binding port 0 and closing the
    socket before the children bound it: between the close and rank 0's TCPStore bind the port was
    free for anyone — another process's bind, or (the port is in the ephemeral range) a rank's own
    TCPStore client connect() retrying on 127.0.0.1:P while rank 0 was still importing torch, which
    the kernel can complete as a TCP self-connect (source port == P), so the client reads its own
    request back.  A file rendezvous has no port to lose.

    Each rank's stderr also goes to <GDP_BENCH_RANK_LOGS>/rank<r>.stderr when that directory is
    set (tests keep it); a failing rank's tail is printed with the path either way."""
    import shutil
    import signal
    import subprocess
    import tempfile

    rdv_dir = tempfile.mkdtemp(prefix="gdp_bench_rdv_")
    own_logs = not os.environ.get("GDP_BENCH_RANK_LOGS")  # a private log directory: removed unless a rank fails
    log_dir = tempfile.mkdtemp(prefix="gdp_bench_ranks_") if own_logs else os.environ["GDP_BENCH_RANK_LOGS"]
    os.makedirs(log_dir, exist_ok=True)
    procs, logs = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", GDP_BENCH_RDV=os.path.join(rdv_dir, "rendezvous"))
        env.pop("MASTER_PORT", None)
        path = os.path.join(log_dir, f"rank{r}.stderr")
        logs.append(path)
        with open(path, "wb") as err:
            procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env,
                                          stderr=err))
    rc = 0

    def forward(signum, frame):  # the launcher itself told to stop (timeout, Ctrl-C): stop the ranks too
        raise SystemExit(128 + signum)

    old_handlers = {sig: signal.signal(sig, forward) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    r = procs.index(p)
                    try:
                        with open(logs[r], "rb") as f:
                            tail = f.read()[-4000:].decode(errors="replace")
                    except OSError:
                        tail = "(stderr log unreadable)"
                    print(f"bench.py: rank {r} exited with {code}; stopping the other ranks. Its stderr "
                          f"({logs[r]}), last 4000 bytes:\n{tail}", file=sys.stderr, flush=True)
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    except BaseException:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        raise
    finally:
        for sig, h in old_handlers.items():
            signal.signal(sig, h)
        for p in procs:
            if p.poll() is None:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
        if rc == 0:  # a passing rank's stderr (warnings) still reaches the caller
            for path in logs:
                try:
                    with open(path, "rb") as f:
                        sys.stderr.write(f.read().decode(errors="replace"))
                except OSError:
                    pass
            if own_logs:
                shutil.rmtree(log_dir, ignore_errors=True)
        shutil.rmtree(rdv_dir, ignore_errors=True)  # the failing rank's log (named above) is kept
    return rc


def gpu_state(pci):
    """Clocks, power and temperatures of this rank's GPU right after its timed steps (`rocm-smi`,
    informational: boxes of this part differ by up to +-3 % on the same command, and this is what
    such a difference can be read against).  None when rocm-smi is missing or says nothing."""
    import shutil
    import subprocess

    smi = shutil.which("rocm-smi") or ("/opt/rocm/bin/rocm-smi" if os.path.exists("/opt/rocm/bin/rocm-smi") else None)
    if not smi or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        # under rocprofv3 the child inherits the profiler's preload, which initialises the GPU
        # before rocm-smi's `#!/usr/bin/env python3` re-execs: skip the informational query
        return None
    try:
        r = subprocess.run([smi, "--showclocks", "--showpower", "--showtemp", "--showbus", "--json"],
                           capture_output=True, text=True, timeout=20)
        cards = json.loads(r.stdout[r.stdout.index("{"):])
    except Exception:  # noqa: BLE001 - informational only
        return None
    card = next((v for v in cards.values() if isinstance(v, dict) and str(v.get("PCI Bus", "")).lower() == pci.lower()),
                next(iter(cards.values())) if len(cards) == 1 else None)
    if not isinstance(card, dict):
        return None
    keep = ("mclk clock speed:", "fclk clock speed:", "sclk clock speed:", "socclk clock speed:",
            "Current Socket Graphics Package Power (W)", "Temperature (Sensor junction) (C)",
            "Temperature (Sensor memory) (C)", "PCI Bus")
    return {k.rstrip(":"): card[k] for k in keep if k in card} or None


def rank_topology(world, rank, local, backend, dist, args):
    """Which device each rank drives, and how many ranks the collective backend sees — so an
    N-rank line proves "N ranks on N distinct GPUs" from its own record: every rank's device
    ordinal, PCI address and UUID (all_gather_object), and an all_reduce of ones over the process
    group (RCCL under "nccl": `rccl_world`).  Under nccl a shared device or a count other than
    --gpus is fatal (before any timing); a gloo rehearsal records its shared device explicitly."""
    import torch

    props = torch.cuda.get_device_properties(local)
    me = {"rank": rank, "device": local, "name": props.name,
          "pci": "%04x:%02x:%02x.0" % (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", 0),
                                        getattr(props, "pci_device_id", 0)),
          "uuid": str(getattr(props, "uuid", "")),
          "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES"))}
    if dist is None:
        return {"backend": None, "collective_world": 1, "devices": [me], "distinct_devices": 1}
    devs = [None] * world
    dist.all_gather_object(devs, me)
    ones = torch.ones(1, dtype=torch.int64, device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(ones)
    counted = int(ones.item())
    ids = {(d["pci"], d["uuid"]) for d in devs}
    topo = {"backend": "rccl" if backend == "nccl" else backend, "collective_world": counted, "devices": devs,
            "distinct_devices": len(ids)}
    if backend == "nccl":
        topo["rccl_world"] = counted
        if counted != args.gpus or len(ids) != world:
            sys.exit(f"bench.py: RCCL counted {counted} ranks on {len(ids)} distinct devices for --gpus {args.gpus}: "
                     f"{devs}")
    else:
        topo["note"] = (f"{backend} rehearsal: {world} ranks on {len(ids)} device(s) — not a multi-GPU measurement"
                        if len(ids) < world else f"{backend} ranks on distinct devices")
    return topo


def autotune_rotating(ctxs, stream, iters, rounds=5, op="build"):
    """gdp_autotune's search (every build variant x tile order 0/1, and for the full build x
    store mode: (GDP_TUNE_ZERO_WINDOW, GDP_TUNE_STORE_PACE) in (0, off) (0, 1) (1, off) (1, 0)) over the
    ROTATED step sequence
    the benchmark times (one set when it alone exceeds the MALL), so the pick is made on cold
    buffers; candidates are interleaved round-robin over `rounds` rounds and ranked by their
    median (drift hits all alike, unlike gdp_autotune's one-candidate-at-a-time timing).  All
    candidates give identical bits.  op "subset" times the subset build (gdp_build_subset)."""
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    cands = []
    for v in pkg.build_variants():
        # the subset build has no zero window (its levels S..S+2 keep x) but its five stores per group
        # go out with only two windows' loads between them: pacing alone
        modes = ((0, -1), (0, 1), (1, -1), (1, 0)) if op == "build" else ((0, -1), (0, 0), (0, 1))
        cands += [(v, o, z, p) for z, p in modes for o in (0, 1)]
    times = {c: [] for c in cands}
    for _ in range(rounds):
        for v, order, zw, sp in cands:
            for c in ctxs:
                c.set_tuning(variant=v, tile_order=order, zero_window=zw, store_pace=sp)
            run = [c.build_subset if op == "subset" else c.build for c in ctxs]
            for r in run:
                r(stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(iters * len(ctxs)):
                run[i % len(ctxs)](stream)
            e1.record(stream)
            e1.synchronize()
            times[(v, order, zw, sp)].append(e0.elapsed_time(e1) / (iters * len(ctxs)))
    med = {c: sorted(t)[len(t) // 2] for c, t in times.items()}
    best = min(cands, key=lambda c: med[c])
    for c in ctxs:
        c.set_tuning(variant=best[0], tile_order=best[1], zero_window=best[2], store_pace=best[3])
    return best[0], best[1], med[best]


def autotune_inplace(ctxs, steps_fn, stream, iters, key, values, rounds=5):
    """The in-place passes' block shape (GDP_TUNE_INPLACE_SUB / _WINDOW_SUB: 1024 / 512 / 256-thread
    blocks, or k_levels_x) chosen like the build variant: every candidate timed over the ROTATED
    cold step sequence, interleaved round-robin over `rounds`, median wins.  Bit-identical
    outputs; the best shape depends on the workload (profiles/ab_regen_c*_r02ae.log).  Every shape
    runs with GDP_TUNE_ZERO_WINDOW off and on (profiles/zwi_*_r03an.log) and, for the re-entry's five
    stores per thread, paced at vmcnt(1) (GDP_TUNE_STORE_PACE; profiles/spi_regen_c*_r03as.log)."""
    import torch

    modes = ((0, -1), (1, -1), (0, 1)) if key == "inplace_sub" else ((0, -1), (1, -1))
    cands = [(v, z, p) for v in values for z, p in modes]
    times = {cand: [] for cand in cands}
    for _ in range(rounds):
        for cand in cands:
            v, z, p = cand
            for c in ctxs:
                c.set_tuning(**{key: v}, zero_window=z, inplace_pace=p)
            for f in steps_fn:
                f(stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(iters * len(ctxs)):
                steps_fn[i % len(ctxs)](stream)
            e1.record(stream)
            e1.synchronize()
            times[cand].append(e0.elapsed_time(e1) / (iters * len(ctxs)))
    best = min(cands, key=lambda cand: sorted(times[cand])[len(times[cand]) // 2])
    for c in ctxs:
        c.set_tuning(**{key: best[0]}, zero_window=best[1], inplace_pace=best[2])
    return best[0]


def scatter_split(ctx, cfg, world, rank, dist, mg, backend, in_fmt):
    """SURVEY.md §8e's optional image-batch split, measured OUTSIDE the timed region: rank 0
    generates every rank's images (the same global indices the ranks otherwise generate locally),
    one collective scatter (RCCL over xGMI; gloo + host staging in rehearsals) hands each rank
    its share, and every rank builds from the scattered images and checks that each image's
    pyramid checksum equals the one built from its locally generated copy."""
    import torch

    H, W, B = cfg["H"], cfg["W"], cfg["batch"]
    dt = torch.uint8 if in_fmt == "u8" else torch.int32
    dev = torch.device("cuda", torch.cuda.current_device())
    if cfg["band"]:
        return scatter_band_split(ctx, cfg, world, rank, dist, mg, backend, in_fmt, dt, dev)
    per = B * H * W

    def fill(chunk, r):  # the device generator writes straight into rank r's share
        stage = chunk if chunk.is_cuda else torch.empty(per, dtype=dt, device=dev)
        ctx.bind_device_input(stage.data_ptr(), W, H * W, keepalive=stage)
        ctx.fill_synthetic(SEED, r * B)
        ctx.sync()
        ctx.unbind_device_input()
        if stage is not chunk:
            chunk.copy_(stage.cpu())

    recv, secs = mg.scatter_images(per, fill, dist=dist, device=dev if backend == "nccl" else "cpu", dtype=dt)
    recv = recv.to(dev)
    ctx.build()
    ctx.sync()
    local = [ctx.checksum(b) for b in range(B)]
    ctx.bind_device_input(recv.data_ptr(), W, H * W, keepalive=recv)
    ctx.build()
    ctx.sync()
    got = [ctx.checksum(b) for b in range(B)]
    ctx.unbind_device_input()
    secs, bad = mg.max_over_ranks([secs, float(local != got)], dist=dist,
                                  device="cuda" if backend == "nccl" else "cpu")
    nbytes = world * per * (1 if in_fmt == "u8" else 4)
    return {"mode": f"collective scatter of rank 0's batch ({'RCCL over xGMI' if backend == 'nccl' else backend + ' via host'}), "
                    "outside the timed region", "bytes": nbytes, "ms": round(secs * 1e3, 3),
            "GBps": round(nbytes / secs / 1e9, 1) if secs > 0 else None, "bit_exact": bad == 0.0}


def scatter_band_split(ctx, cfg, world, rank, dist, mg, backend, in_fmt, dt, dev):
    """The row-band config's input split (optional): rank 0 generates the whole
    image and one collective scatter hands every rank its rows (padded to the largest band);
    each rank builds its band from them and checks the pyramid checksum against its locally
    generated band.  Outside the timed region."""
    import torch

    import __graft_entry__ as entry

    H, W, O = cfg["H"], cfg["W"], cfg["O"]
    bands = [mg.plan_band(H, world, r, O) for r in range(world)]
    per = max(r1 - r0 for r0, r1 in bands) * W
    whole_img = None
    if rank == 0:
        pkg = entry.load_package()
        whole_img = torch.empty((H, W), dtype=dt, device=dev)
        with pkg.PyramidContext(H, W, S=2, octaves=O, batch=1, device=ctx.device, input_format=in_fmt) as whole:
            whole.bind_device_input(whole_img.data_ptr(), W, H * W, keepalive=whole_img)
            whole.fill_synthetic(SEED, 0)
            whole.sync()
            whole.unbind_device_input()

    def fill(chunk, r):
        r0, r1 = bands[r]
        chunk[:(r1 - r0) * W].copy_(whole_img[r0:r1].reshape(-1))

    recv, secs = mg.scatter_images(per, fill, dist=dist, device=dev if backend == "nccl" else "cpu", dtype=dt)
    recv = recv.to(dev)
    r0, r1 = bands[rank]
    ctx.build()
    ctx.sync()
    local = ctx.checksum(0)
    ctx.bind_device_input(recv.data_ptr(), W, max(1, r1 - r0) * W, keepalive=recv)
    ctx.build()
    ctx.sync()
    got = ctx.checksum(0)
    ctx.unbind_device_input()
    secs, bad = mg.max_over_ranks([secs, float(local != got)], dist=dist,
                                  device="cuda" if backend == "nccl" else "cpu")
    nbytes = sum(r1 - r0 for r0, r1 in bands[1:]) * W * (1 if in_fmt == "u8" else 4)
    return {"mode": f"collective scatter of rank 0's image in row bands ({'RCCL over xGMI' if backend == 'nccl' else backend + ' via host'}), "
                    "outside the timed region", "bytes_to_other_ranks": nbytes, "ms": round(secs * 1e3, 3),
            "GBps": round(nbytes / secs / 1e9, 1) if secs > 0 else None, "bit_exact": bad == 0.0}


def gather_bands(ctx, cfg, world, rank, dist, mg, backend, in_fmt):
    """The row-band config's output gather (optional; the MPI variant's collector,
    GaussDePyramid-MPI.h:285-298): every rank packs its band pyramid, one collective gather brings
    the bands to rank 0 (timed between barriers), and rank 0 lays them into a whole-image context
    and checks gdp_checksum of the assembled pyramid against the reference's output for the
    image.  Outside the timed region."""
    import torch

    import __graft_entry__ as entry

    H, W, S, O = cfg["H"], cfg["W"], 2, cfg["O"]
    dev = torch.device("cuda", torch.cuda.current_device())

    def aligned(nbytes):  # 256-B aligned float32 view for gdp_set_output_device
        raw = torch.empty(nbytes // 4 + 64, dtype=torch.float32, device=dev)
        shift = (-raw.data_ptr() % 256) // 4
        return raw, raw[shift:shift + nbytes // 4]

    raw, view = aligned(ctx.pyramid_bytes())
    ctx.bind_device_output(view.data_ptr(), ctx.pyramid_bytes(), keepalive=raw)
    ctx.build()
    ctx.sync()
    parts = []
    for o in range(O):
        rows, cols, _ = ctx.level_dims(o)
        for s in range(S + 3):
            off = ctx.level_offset(0, o, s)
            parts.append(view[off:off + rows * cols])
    packed = torch.cat(parts) if parts else view[:0].clone()
    ctx.unbind_device_output()
    del raw, view, parts
    sizes = [mg.packed_band_floats(H, W, S, O, *mg.plan_band(H, world, r, O)) for r in range(world)]
    bands, secs = mg.gather_packed_bands(packed if backend == "nccl" else packed.cpu(), sizes, dist=dist)
    del packed
    secs = mg.max_over_ranks([secs], dist=dist, device="cuda" if backend == "nccl" else "cpu")[0]
    if rank != 0:
        return None
    full = mg.assemble_bands(H, W, S, O, world, [b.to(dev) for b in bands])
    del bands
    pkg = entry.load_package()
    with pkg.PyramidContext(H, W, S=S, octaves=O, batch=1, device=ctx.device, input_format=in_fmt) as whole:
        wraw, wview = aligned(whole.pyramid_bytes())
        whole.bind_device_output(wview.data_ptr(), whole.pyramid_bytes(), keepalive=wraw)
        wview.zero_()
        at = 0
        for o in range(O):
            rows, cols, _ = whole.level_dims(o)
            for s in range(S + 3):
                off = whole.level_offset(0, o, s)
                wview[off:off + rows * cols] = full[at:at + rows * cols]
                at += rows * cols
        torch.cuda.synchronize()
        got = whole.checksum(0)
        whole.unbind_device_output()
    want = _fixture_checksums(cfg).get(0)
    nbytes = 4 * sum(sizes[1:])
    return {"mode": f"collective gather of every row band's pyramid to rank 0 ({'RCCL over xGMI' if backend == 'nccl' else backend + ' via host'}), "
                    "outside the timed region", "bytes_to_rank0": nbytes, "ms": round(secs * 1e3, 3),
            "GBps": round(nbytes / secs / 1e9, 1) if secs > 0 else None,
            "assembled_checksum": f"{got:016x}",
            "status": ("unchecked (no reference fixture)" if want is None else
                       "bit-exact vs the reference's output for the whole image" if got == want[0] else "MISMATCH")}


def _fixture_checksums(cfg, subset=False):
    """global image index -> the gdp_checksum of the reference's output for that synthetic image
    (tests/golden/checksums.json; square images, generated by the reference binary), or of the
    oracle's closed form for non-square images (checksums_oracle.json: the reference only builds
    square pyramids; the oracle is pinned to it on every square fixture, tests/test_oracle.py)."""
    H, W, O = cfg["H"], cfg["W"], cfg["O"]
    prefix = f"synth:{SEED:#x}:".lower()
    out = {}
    if subset:  # GenerateDoG_nomp_dynamic's output (tests/golden/checksums_a512omp.json, the reference header)
        with open(os.path.join(REPO, "tests", "golden", "checksums_a512omp.json")) as f:
            for r in json.load(f):
                if r["n"] == H == W and r["S"] == 2 and r["input"].lower().startswith(prefix) and f"octaves_{O}" in r:
                    out[int(r["input"].split(":")[2])] = (int(r[f"octaves_{O}"], 16), "reference")
        return out
    if H == W:
        with open(os.path.join(REPO, "tests", "golden", "checksums.json")) as f:
            for r in json.load(f):
                if r["n"] == H and r["S"] == 2 and r["input"].lower().startswith(prefix) and f"octaves_{O}" in r:
                    out[int(r["input"].split(":")[2])] = (int(r[f"octaves_{O}"], 16), "reference")
    else:
        with open(os.path.join(REPO, "tests", "golden", "checksums_oracle.json")) as f:
            for r in json.load(f):
                if (r["H"], r["W"], r["S"], r["octaves"]) == (H, W, 2, O) and r["input"].lower().startswith(prefix):
                    out[int(r["input"].split(":")[2])] = (int(r["checksum"], 16), "oracle")
    return out


def verify(ctx, cfg, key, world, rank, dist, mg, first_image, subset=False):
    """After the timed region: gdp_checksum of what the benchmark built vs the checksum of the
    reference's own output for the same input.  Image configs: EVERY rank checksums the first and
    last image of its shard and rank 0 checks each against the fixtures (tests/golden/), so an
    N-rank line certifies every rank's images; the row-band config sums every rank's band
    checksum into the image's."""
    fixtures = _fixture_checksums(cfg, subset)
    if cfg["band"]:
        sums = mg.gather_checksums([ctx.checksum(0)], dist=dist)
        if rank != 0:
            return None
        got = sum(v[0] for v in sums) & 0xFFFFFFFFFFFFFFFF
        want = fixtures.get(0)
        if want is None:
            return {"status": "unchecked (no reference fixture for this input)", "checksum": f"{got:016x}"}
        return {"status": "bit-exact" if got == want[0] else "MISMATCH",
                "checked": f"sum of {world} row-band checksums = image 0", "checksum": f"{got:016x}",
                "reference_checksum": f"{want[0]:016x}"}
    B = cfg["batch"]
    local = sorted({0, B - 1})
    mine = [[first_image + b, ctx.checksum(b)] for b in local]
    per_rank = mg.gather_checksums([v for pair in mine for v in pair], dist=dist)
    if rank != 0:
        return None
    checked, unchecked, bad = [], [], []
    for r, flat in enumerate(per_rank):
        for idx, got in zip(flat[0::2], flat[1::2]):
            want = fixtures.get(int(idx))
            if want is None:
                unchecked.append(int(idx))
                continue
            (checked if got == want[0] else bad).append(int(idx))
    status = "MISMATCH" if bad else ("bit-exact" if checked else "unchecked (no fixture for these images)")
    against = {v[1] for v in fixtures.values()}
    return {"status": status,
            "checked": f"first and last image of each of {world} rank(s): global images {sorted(checked + bad)}",
            "bit_exact_images": len(checked), "mismatched_images": bad, "images_without_fixture": unchecked,
            "ranks_certified": sorted({i // B for i in checked} - {i // B for i in bad}),
            "against": (("reference output (tests/golden/checksums_a512omp.json: GenerateDoG_nomp_dynamic)" if subset
                         else "reference output (tests/golden/checksums.json)") if against == {"reference"} else
                        "oracle closed form (non-square input: no reference output exists)")}


INPLACE_CALLS = {"regen": 3, "gauss": 2}  # checksums_inplace.json's K per op


def verify_inplace(ctx, cfg, op, stream, world, rank, dist, mg, first_image):
    """The in-place passes (--op regen: GenerateDoG re-entry, main.cpp:66-73's loop; --op gauss:
    GaussFilter of every octave) after the timed region, with the timed kernel instance: rotated
    set 0 is refilled (gdp_init = GaussPyInit) and K calls of the op run on it; the first and last
    image of every rank are then checksummed against the serial reference's output after the same
    K calls on the same input (tests/golden/checksums_inplace.json, oracle/_ref/ref_serial
    regen/gauss).  Image configs only (no fixture of the 16384^2 or non-square re-entry)."""
    K = INPLACE_CALLS[op]
    H, W, O, B = cfg["H"], cfg["W"], cfg["O"], cfg["batch"]
    ctx.init(stream)
    for _ in range(K):
        if op == "regen":
            ctx.generate_dog(stream)
        else:
            ctx.gauss_range(0, O, stream)
    stream.synchronize()
    fixtures = {}
    with open(os.path.join(REPO, "tests", "golden", "checksums_inplace.json")) as f:
        for r in json.load(f):
            if r["op"] == op and r["calls"] == K and r["n"] == H == W and r["S"] == 2 and f"octaves_{O}" in r and \
                    r["input"].lower().startswith(f"synth:{SEED:#x}:".lower()):
                fixtures[int(r["input"].split(":")[2])] = int(r[f"octaves_{O}"], 16)
    local = sorted({0, B - 1})
    mine = [v for b in local for v in (first_image + b, ctx.checksum(b))]
    per_rank = mg.gather_checksums(mine, dist=dist)
    if rank != 0:
        return None
    checked, bad, unchecked = [], [], []
    for flat in per_rank:
        for idx, got in zip(flat[0::2], flat[1::2]):
            want = fixtures.get(int(idx))
            (unchecked if want is None else checked if got == want else bad).append(int(idx))
    return {"status": "MISMATCH" if bad else ("bit-exact" if checked else "unchecked (no fixture for these images)"),
            "checked": f"GaussPyInit + {K} x {'GenerateDoG' if op == 'regen' else 'GaussFilter(every octave)'} "
                       f"after the timed region, same kernel instance; first and last image of each of {world} "
                       f"rank(s): global images {sorted(checked + bad)}",
            "against": "reference output (tests/golden/checksums_inplace.json: oracle/_ref/ref_serial "
                       f"{op} {K})", "bit_exact_images": len(checked), "mismatched_images": bad,
            "images_without_fixture": unchecked, "post_timing_launches": K}


def verify_conv_bands(ctx, cfg, world, rank, dist, mg, in_fmt):
    """Convolution extension on row bands (no reference output exists for this mode): the sum of
    every rank's band checksum must equal the checksum of the whole image built on ONE GPU (rank
    0, after the timed region) — the halo exchange delivered exactly the rows the bands read."""
    import __graft_entry__ as entry

    pkg = entry.load_package()
    sums = mg.gather_checksums([ctx.checksum(0)], dist=dist)
    if rank != 0:
        return None
    got = sum(v[0] for v in sums) & 0xFFFFFFFFFFFFFFFF
    with pkg.PyramidContext(cfg["H"], cfg["W"], S=2, octaves=cfg["O"], batch=1, device=ctx.device,
                            input_format=in_fmt) as whole:
        whole.fill_synthetic(SEED, 0)
        whole.build_gaussian()
        whole.sync()
        want = whole.checksum(0)
    return {"status": "bands == whole image (bit-exact)" if got == want else "MISMATCH",
            "checked": f"sum of {world} row-band checksums (halo rows exchanged every step) vs the whole image "
                       f"built on one GPU", "checksum": f"{got:016x}", "whole_image_checksum": f"{want:016x}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="override images per GPU")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds of CPU-baseline sampling")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--variant", type=int, default=None,
                    help="force a build-kernel variant (and skip autotuning), e.g. for profiling runs")
    ap.add_argument("--tile-order", type=int, default=None,
                    help="with --variant: force the build tile order too (0 linear, 1 XCD-chunked)")
    ap.add_argument("--zero-window", type=int, default=None, choices=[0, 1],
                    help="with --variant / --inplace-sub: force GDP_TUNE_ZERO_WINDOW too (groups outside every "
                         "window's support skip their window loads; the autotunes otherwise pick it)")
    ap.add_argument("--store-pace", type=int, default=None, choices=[-1, 0, 1, 2, 3],
                    help="with --variant / --inplace-sub: force GDP_TUNE_STORE_PACE too (-1 off; n: s_waitcnt vmcnt(n) "
                         "after each store)")
    ap.add_argument("--no-autotune", action="store_true",
                    help="skip gdp_autotune (by default the build kernel variant is chosen by timing every "
                         "variant on this device before the warm-up; all variants give identical bits)")
    ap.add_argument("--inplace-sub", type=int, default=None, choices=[0, 1, 2, 4, 8, 16, -16],
                    help="--op regen/gauss: force the in-place block shape (GDP_TUNE_INPLACE_SUB / _WINDOW_SUB: "
                         "1024 / N threads, 0 = k_levels_x, -16 = 16 x 256 block tiles) and skip its autotune, e.g. "
                         "for profiling runs")
    ap.add_argument("--input", default="i32", choices=["i32", "u8"],
                    help="input pixel format (i32 = the reference's int image; u8 = 8-bit images)")
    ap.add_argument("--op", default="build", choices=["build", "regen", "gauss", "conv", "subset"],
                    help="build: fused GaussPyInit+GenerateDoG (headline); regen: in-place GenerateDoG "
                         "re-entry; gauss: in-place row+column window pass of every octave; conv: the "
                         "true-Gaussian-convolution extension (not the reference's algorithm)")
    ap.add_argument("--conv-kernel", type=int, default=None,
                    help="--op conv: 0 register sweep, 1 LDS tiles, 2 block tiles (default)")
    ap.add_argument("--conv-rows", type=int, default=None,
                    help="--op conv: block tiles' rows per block (48 default) / the sweep's rows per strip (16/32)")
    ap.add_argument("--concurrent-streams", type=int, default=0, metavar="N",
                    help="--op build, one GPU, one image per set: also report `concurrent_streams`, the rotated "
                         "sets' single-image builds overlapped on N streams (INTEGRATION §5's serving mode; "
                         "informational, before the warm-up; never `value`)")
    ap.add_argument("--conv-waves", type=int, default=None, choices=[8, 16],
                    help="--op conv: waves per block tile (GDP_TUNE_CONV_WAVES; 16 waves: 16 / 32 / 48 rows, "
                         "8 waves: 8 / 16 / 24 / 32 rows)")
    ap.add_argument("--conv-order", type=int, default=None,
                    help="--op conv: block order bits (1 XCD-chunked, 2 alternate sweep directions, 4 octave rows "
                         "after their input rows; default 5, and 4 for one image of >= 2^27 pixels — gdp.h "
                         "GDP_TUNE_CONV_ORDER)")
    ap.add_argument("--scatter", action="store_true",
                    help="N > 1: also measure the input split (rank 0's image batch, or for the row-band config its "
                         "image's rows, scattered over RCCL, SURVEY.md §8e), outside the timed region, and check the "
                         "ranks build the same bits from it")
    ap.add_argument("--gather", action="store_true",
                    help="N > 1, row-band config: also measure the collector's gather of every band's pyramid to "
                         "rank 0 (outside the timed region) and check the assembled pyramid against the reference")
    ap.add_argument("--rotate", type=int, default=None,
                    help="independent input+pyramid buffer sets the steps cycle through (default: enough to "
                         "exceed %d MiB, so no step finds its lines in the 256 MB Infinity Cache)" % (ROTATE_BYTES >> 20))
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks here, before torch is imported or a GPU is touched
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    import torch

    import __graft_entry__ as entry

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    # one process per GPU; GDP_BENCH_BACKEND=gloo lets a 1-GPU box rehearse N ranks on device 0
    backend = os.environ.get("GDP_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        sys.exit(f"bench.py: {world} ranks need {world} GPUs under nccl (RCCL), {ndev} visible "
                 f"(GDP_BENCH_BACKEND=gloo rehearses several ranks on one GPU)")
    pkg = entry.load_package()
    local = local if backend == "nccl" else local % max(1, ndev)
    torch.cuda.set_device(local)
    dist = None
    # GDP_BENCH_FORCE_PG=1 (under torchrun --nproc-per-node 1): open the process group at N = 1 too,
    # so a 1-GPU box exercises the RCCL init, barriers and object gathers the N > 1 line takes
    if world > 1 or os.environ.get("GDP_BENCH_FORCE_PG") == "1":
        import torch.distributed as dist

        # self-launched ranks meet through a file (launch_ranks); under torchrun, env:// as usual
        rdv = os.environ.get("GDP_BENCH_RDV")
        init = dict(init_method="file://" + rdv, rank=rank, world_size=world) if rdv else {}
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local), **init)
        else:
            # one-node rehearsal: gloo's pairs on loopback (otherwise gloo picks its interface by
            # resolving this host's name, which this pool's boxes cannot always do)
            if os.environ.get("MASTER_ADDR", "127.0.0.1") in ("127.0.0.1", "localhost"):
                os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
            dist.init_process_group(backend=backend, **init)
    topology = rank_topology(world, rank, local, backend, dist, args)
    red_dev = "cuda" if backend == "nccl" else "cpu"

    cfg = dict(CONFIGS[args.config])
    if args.batch:
        cfg["batch"] = args.batch
    H, W, S, O, B = cfg["H"], cfg["W"], 2, cfg["O"], cfg["batch"]
    mg = __import__(pkg.__name__ + ".distributed", fromlist=["plan_band"])
    in_bytes = 1 if args.input == "u8" else 4
    if cfg["band"]:
        # one image, row bands aligned to 2^(max(O,5)-1) rows: each rank owns rows [r0, r1)
        r0, r1 = mg.plan_band(H, world, rank, O)
        make = lambda: pkg.PyramidContext(H, W, S=S, octaves=O, batch=1, device=local, row_begin=r0, row_end=r1,
                                          input_format=args.input)
        first_image = 0
        scaling = "strong"
        units_all = H * W  # input pixels of the whole job per step
        set_bytes = in_bytes * (r1 - r0) * W + 4 * (S + 3) * pyramid_pixels(H, W, O) * (r1 - r0) // H
    else:
        make = lambda: pkg.PyramidContext(H, W, S=S, octaves=O, batch=B, device=local, input_format=args.input)
        first_image = rank * B  # rank r owns global images [r*B, (r+1)*B)
        scaling = "weak"
        units_all = world * B * H * W
        set_bytes = algorithmic_bytes(H, W, S, O, B, in_bytes)
    rotate = args.rotate or max(1, -(-ROTATE_BYTES // max(1, set_bytes)))
    # the convolution extension on row bands reads its neighbours' rows: each band's input lives in
    # a torch tensor (the rows its neighbours need are sent from it) and its halo rows are received
    # into bound tensors by distributed.exchange_halo — RCCL point-to-point over xGMI, part of every
    # timed step (the reference's pointwise window needs no exchange)
    halo_exchange = args.op == "conv" and cfg["band"] and world > 1
    ctxs, halos = [], []
    for _ in range(rotate):  # identical sets (same images) at different addresses
        c = make()
        if halo_exchange:
            dev = torch.device("cuda", local)
            edt = torch.uint8 if args.input == "u8" else torch.int32
            inp = torch.empty((1, r1 - r0, W), dtype=edt, device=dev)
            c.bind_device_input(inp.data_ptr(), W, (r1 - r0) * W, keepalive=inp)
            above, below = c.conv_halo_rows()
            top = torch.empty((1, max(above, 1), W), dtype=edt, device=dev)
            bot = torch.empty((1, max(below, 1), W), dtype=edt, device=dev)
            c.bind_input_halo(top.data_ptr() if above else None, bot.data_ptr() if below else None, pitch=W,
                              keepalive=(top, bot))
            # gloo rehearsals exchange through host memory: a host image of the band, refreshed
            # only in the rows the neighbours need, and host halo buffers
            host = ((torch.empty(inp.shape, dtype=edt), torch.empty(top[:, :above].shape, dtype=edt),
                     torch.empty(bot[:, :below].shape, dtype=edt)) if backend != "nccl" else None)
            halos.append((inp, top[:, :above], bot[:, :below], host))
        c.fill_synthetic(SEED, first_image)
        ctxs.append(c)
    ctx = ctxs[0]
    for c in ctxs:
        c.sync()
    # a dedicated (non-null) torch stream: the builds and the HIP events share it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)

    distribution = None
    if args.scatter and world > 1 and not halo_exchange:
        distribution = scatter_split(ctx, cfg, world, rank, dist, mg, backend, args.input)
    for c in ctxs:
        c.set_tuning(conv_kernel=args.conv_kernel, conv_rows=args.conv_rows, conv_order=args.conv_order,
                     conv_waves=args.conv_waves)
        if args.op == "subset":  # that header's integer-length window centre (the same taps at these sizes)
            c.set_window_centre("intlen")
    autotuned = None
    t_tune = time.perf_counter()
    if args.variant is not None:
        for c in ctxs:
            c.set_tuning(variant=args.variant, tile_order=args.tile_order, zero_window=args.zero_window,
                         store_pace=args.store_pace)
    elif args.op in ("build", "subset") and not args.no_autotune:
        # candidates interleaved round-robin (drift hits all alike), over the rotated sets
        autotuned = autotune_rotating(ctxs, stream, 3 if B * H * W > (1 << 28) else 10, op=args.op)
    if args.op == "build":
        steps_fn = [c.build for c in ctxs]
    elif args.op == "subset":  # GaussPyramid_a512omp::GenerateDoG_nomp_dynamic, the CPU baseline's semantics
        steps_fn = [c.build_subset for c in ctxs]
    elif args.op == "conv" and halo_exchange:
        def conv_step(i, st):
            inp, top, bot, host = halos[i]
            if backend == "nccl":
                mg.exchange_halo(inp, top, bot, H, world, rank, O, dist=dist)
            else:  # gloo rehearsal: the same exchange through host copies of the rows it moves
                h_in, h_top, h_bot = host
                for kind, _, first, n in mg.halo_plan(H, world, rank, O):
                    if kind == "send":
                        h_in[:, first:first + n].copy_(inp[:, first:first + n])
                mg.exchange_halo(h_in, h_top, h_bot, H, world, rank, O, dist=dist)
                top.copy_(h_top)
                bot.copy_(h_bot)
            ctxs[i].build_gaussian(st)

        steps_fn = [lambda st, i=i: conv_step(i, st) for i in range(rotate)]
    elif args.op == "conv":
        steps_fn = [c.build_gaussian for c in ctxs]
    else:
        for c in ctxs:
            c.build(stream)  # materialise the pyramid the in-place passes work on
        steps_fn = [c.generate_dog if args.op == "regen" else (lambda st, c=c: c.gauss_range(0, O, st))
                    for c in ctxs]
        key, values = (("inplace_sub", [1, 4, 2, 0, 8, 16, -16]) if args.op == "regen" else
                       ("window_sub", [1, 4, 2, 8, 16]))
        if args.inplace_sub is not None:
            if args.inplace_sub not in values:
                sys.exit(f"bench.py: --inplace-sub {args.inplace_sub} is not a {key} value ({values})")
            for c in ctxs:
                c.set_tuning(**{key: args.inplace_sub}, zero_window=args.zero_window, inplace_pace=args.store_pace)
        elif not args.no_autotune:
            autotuned = (key, autotune_inplace(ctxs, steps_fn, stream, 3 if B * H * W > (1 << 28) else 10, key, values))
    tune_s = time.perf_counter() - t_tune if autotuned else 0.0
    n_step = [0]

    def step(st):  # step i works on buffer set i mod rotate
        steps_fn[n_step[0] % rotate](st)
        n_step[0] += 1

    # the serving-mode figure runs BEFORE the warm-up, so the timed launches stay the last ones of
    # their kernel in a trace (tools/timed_dispatches.py takes the last `steps` dispatches)
    # (opt-in: its overlapped launches of the same kernel instance would otherwise enter a
    # `rocprofv3 --stats` average of the default command)
    streams_fig = None
    if args.concurrent_streams and args.op == "build" and world == 1 and not cfg["band"] and B == 1 and rotate > 1:
        streams_fig = concurrent_streams(ctxs, algorithmic_bytes(H, W, S, O, B, in_bytes), args.concurrent_streams)
        torch.cuda.set_stream(stream)
    for _ in range(args.warmup):
        step(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step(stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    # this rank's wall time for exactly K steps ends when its GPU drains; the closing barrier
    # fences the ranks but its own latency is not a step's (the max over ranks below takes the
    # slowest rank's K steps)
    wall = time.perf_counter() - t0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # per-launch, HIP events on the launch stream
    topology["gpu_state_after_timed_steps"] = gpu_state(topology["devices"][0]["pci"]) if rank == 0 else None
    if dist:  # every rank's own timing, recorded beside the max that the line reports
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "ms_per_step": round(wall * 1e3 / args.steps, 6),
                                          "kernel_ms": round(kernel_ms, 6)})
        topology["per_rank"] = per_rank
    wall, kernel_ms = mg.max_over_ranks([wall, kernel_ms], dist=dist, device=red_dev)
    parity = (verify(ctx, cfg, args.config, world, rank, dist, mg, first_image, subset=args.op == "subset")
              if args.op in ("build", "subset") else None)
    if halo_exchange:
        parity = verify_conv_bands(ctx, cfg, world, rank, dist, mg, args.input)
    if args.op in ("regen", "gauss") and not cfg["band"]:
        parity = verify_inplace(ctx, cfg, args.op, stream, world, rank, dist, mg, first_image)
    if parity is not None and rotate > 1 and args.op not in ("regen", "gauss"):
        # every rotated set built the same images: their checksums must all equal set 0's
        sums = {c.checksum(0) for c in ctxs}
        parity["rotated_sets_agree"] = len(sums) == 1
        if len(sums) != 1:
            parity["status"] = "MISMATCH (rotated sets differ)"
    collect = None
    if args.gather and world > 1 and cfg["band"] and args.op == "build":
        collect = gather_bands(ctx, cfg, world, rank, dist, mg, backend, args.input)

    # roofline of the (only) kernel of a step, per launch on THIS rank's share
    rows_local = ctx.row_end - ctx.row_begin
    pyr_px = sum(ctx.level_dims(o)[0] * ctx.level_dims(o)[1] for o in range(O)) * (1 if cfg["band"] else B)
    if args.op not in ("build", "conv", "subset"):  # in-place passes read and write every level once: 8*(S+3)*P bytes
        bytes_launch = 8 * (S + 3) * pyr_px
    elif cfg["band"]:
        bytes_launch = in_bytes * rows_local * W + 4 * (S + 3) * pyr_px
    else:
        bytes_launch = algorithmic_bytes(H, W, S, O, B, in_bytes)
    achieved = bytes_launch / (kernel_ms / 1e3) / 1e9
    tun = ctx.tuning()
    # PMC records are of the whole workload on one GPU; a row band (config 5 at N > 1) is another
    # launch, profiled separately as rank 0's band of N on one GPU (tools/pmc_variants.py --band-of N)
    band_of = world if (cfg["band"] and world > 1) else None
    pmc = (latest_pmc(args.config, tun["variant"], tun["tile_order"], args.op, S + 3,
                      tun["zero_window"] if args.op == "build" else 0, band_of=band_of,
                      chunk_kb=tun.get("pyramid_chunk_kb", 0))
           if args.op in ("build", "subset") and args.input == "i32" and (band_of is None or rank == 0) else None)
    if args.op == "conv" and args.input == "i32" and not (cfg["band"] and world > 1):
        pmc = latest_conv_pmc(args.config, tun)
    if args.op in ("regen", "gauss") and not (cfg["band"] and world > 1):
        pmc = latest_inplace_pmc(args.config, args.op, tun)

    result = {
        "metric": METRIC,
        "value": round(units_all * args.steps / wall / 1e6, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1e3 / args.steps, 6),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (on-device counter-hash int32 images, SURVEY.md §8d)",
        "config": {
            "workload": cfg["name"], "H": H, "W": W, "S": S, "octaves": O, "scales": S + 3,
            "images_per_gpu": 1 if cfg["band"] else B,
            "parallelism": (f"row-band x{world}" if cfg["band"] else f"image-sharded x{world}"),
            "input_mpix_per_step": units_all / 1e6,
            "input_format": "int32" if args.input == "i32" else "uint8",
            "rotated_buffer_sets": rotate,
            "working_set_bytes_per_gpu": rotate * set_bytes,
            "pyramid_backing": ("one hipMalloc" if ctx.tuning()["pyramid_chunk_kb"] == 0 else
                                "one physical piece per image (VMM)" if ctx.tuning()["pyramid_chunk_kb"] < 0 else
                                "%d KiB physical pieces mapped into one range (VMM)" % ctx.tuning()["pyramid_chunk_kb"]),
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": round(pmc["kernel_bytes_per_launch"]) if pmc else None,
            "traffic_source": (f"profiles/{pmc['file']}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the same "
                               + (f"kernel instance (conv kernel {pmc['conv_kernel']}, rows {pmc['conv_rows']}, order "
                                  f"{pmc['conv_order']}) on this workload" if args.op == "conv" else
                                  f"kernel instance (inplace_sub {pmc['inplace_sub']}, zero window {pmc.get('zero_window', 0)}) "
                                  f"on this workload" if args.op == "regen" else
                                  f"kernel instance (window_sub {pmc['window_sub']}, zero window {pmc.get('zero_window', 0)}) "
                                  f"on this workload" if args.op == "gauss" else
                                  f"kernel instance (variant {pmc['variant']}, tile order {pmc['tile_order']}, zero window "
                                  f"{pmc.get('zero_window', 0)}) on this workload (store pacing waits change no bytes)")
                               if pmc else "no PMC profile of this kernel instance (variant/tile order) on this workload"),
            "kernel": ("k_build (fused decimate+window+DoG), variant %d, tile order %d, zero window %d, store pace %s%s"
                       % (tun["variant"], tun["tile_order"], tun["zero_window"],
                          "off" if tun["store_pace"] < 0 else "vmcnt(%d)" % tun["store_pace"],
                          " (autotuned)" if autotuned else "")
                       if args.op == "build" else
                       "k_build<SUB> (fused decimate+window+DoG, GenerateDoG_nomp_dynamic's subset of levels), "
                       "variant %d, tile order %d, store pace %s" % (tun["variant"], tun["tile_order"],
                                                                     "off" if tun["store_pace"] < 0 else
                                                                     "vmcnt(%d)" % tun["store_pace"])
                       if args.op == "subset" else
                       {"regen": ("k_levels_x (in-place window+DoG, one level per wave)" if tun["inplace_sub"] == 0 else
                                  "k_levels_tile<MODE=3> (in-place window+DoG, all octaves, 16-row x 256-column block "
                                  "tiles of k_build's shape)" if tun["inplace_sub"] < 0 else
                                  "k_levels<MODE=3> (in-place window+DoG, all octaves, %d-thread blocks)"
                                  % (1024 // tun["inplace_sub"])) + ", zero window %d, store pace %s" % (
                                     tun["zero_window"], "off" if tun["inplace_pace"] < 0 else "vmcnt(%d)" % tun["inplace_pace"])
                                 + (" (autotuned)" if autotuned else ""),
                        "gauss": "k_window (in-place row+column window, all octaves, %d-thread blocks), zero window %d%s"
                                 % (1024 // tun["window_sub"], tun["zero_window"], " (autotuned)" if autotuned else ""),
                        "conv": ("k_conv_blk (extension: separable Gaussian convolution, LDS-staged %d-row x "
                                 "%d-column block tiles on %d waves, DPP lane shifts, store pace %s)"
                                 % (ctx.tuning()["conv_rows"], 240,
                                    ctx.tuning().get("conv_waves") or 16,
                                    "off" if tun["conv_pace"] < 0 else "vmcnt(%d)" % tun["conv_pace"])
                                 if ctx.tuning()["conv_kernel"] == 2 and S <= 5 else
                                 "k_conv_sweep (extension: separable Gaussian convolution, register sweep + "
                                 "DPP lane shifts, %d-row strips)" % ctx.tuning()["conv_rows"]
                                 if ctx.tuning()["conv_kernel"] == 0 and S <= 3 else
                                 "k_conv (extension: separable Gaussian convolution, LDS halo tiles)")}[args.op]),
            "kernel_ms": round(kernel_ms, 6),
            **({"step_includes": "halo exchange (distributed.exchange_halo, RCCL point-to-point) before each band build"}
               if halo_exchange else {}),
            "algorithmic_bytes_per_launch": bytes_launch,
        },
    }
    result["parity"] = parity if (args.op in ("build", "subset", "regen", "gauss") or halo_exchange) else (
        {"status": "extension: no reference output (tests/ check it against a float64 convolution)"})
    if result["parity"] is None:  # an in-place op on the row-band config
        result["parity"] = {"status": "unchecked (no reference re-entry fixture of this workload)"}
    if autotuned:  # outside the timed region: the search that picked the kernel instance
        result["autotune"] = {"seconds": round(tune_s, 2), "candidates": (
            len(pkg.build_variants()) * (8 if args.op == "build" else 6) if args.op in ("build", "subset")
            else None), "rounds": 5}
    result["tuning"] = {k: tun[k] for k in ("variant", "tile_order", "zero_window", "store_pace", "inplace_sub",
                                            "window_sub", "inplace_pace", "conv_kernel", "conv_rows", "conv_order",
                                            "conv_waves", "conv_pace", "pyramid_chunk_kb") if k in tun}
    result["topology"] = topology
    if distribution is not None:
        result["distribution"] = distribution
    if collect is not None:
        result["collect"] = collect
    if args.op != "build":
        result["metric"] = METRIC + (" [op=conv: true-Gaussian extension, not the reference's algorithm]"
                                     if args.op == "conv" else
                                     " [op=subset: GaussPyramid_a512omp::GenerateDoG_nomp_dynamic's output, the "
                                     "CPU baseline's own semantics]" if args.op == "subset" else
                                     f" [op={args.op}: in-place pass]")
    if streams_fig is not None:
        result["concurrent_streams"] = streams_fig
    complete_line(result, args, rank, world, dist, mg, red_dev, bytes_launch, wall)
    for c in ctxs:
        c.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
