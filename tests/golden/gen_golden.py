#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REFERENCE ITSELF.

The reference (ZhangShuui/SIFT-parallel-optimization) ships no tests, fixtures or golden
vectors.  Every expected value here is therefore produced by the reference's own
`GuassDePyramid.h` (and, for the CPU-baseline semantics, `GaussDePyramid-AVX512xOpenMP.h` /
`-AVX512xPTHREAD.h`), compiled in place by `make -C oracle ref` into oracle/_ref/.  This script
only runs that binary and stores its outputs as data; it needs /root/reference to exist
(this container), never the GPU box, which only reads the committed fixtures.

Outputs (all plain data, loadable without pickle):
  hashes.json   per-level FNV hashes (oracle/gdp_oracle.c:gdo_fnv) of GenerateDoG() output
  dumps.npz     complete packed pyramids for small n, GenerateDoG re-entry results,
                the AVX512xOpenMP subset output, and centre windows for n = 512 / 4096
  taps.npz      the reference's `filter` taps for every (octave, scale) — read from the
                reference object itself (TapProbe in oracle/ref_harness.cpp)
  checksums.json gdp_checksum values of the reference's output for the bench inputs
  mpi_hashes.json per-level hashes of the COLLECTOR's pyramid of the reference's multi-process
                variants — GaussPyramid_mpi::GenerateDoG_mpi (GaussDePyramid-MPI.h:265-335) and
                mpitest.cpp's GenerateDoG_mpi / GenerateDoG_mpi_omp (:35-189) — run under
                conda MPICH's mpiexec with S+4 ranks (oracle/_ref/ref_mpi, ref_mpitest)
  checksums_a512omp.json gdp_checksum values of GenerateDoG_nomp_dynamic's output for the bench inputs
  checksums_inplace.json gdp_checksum values after K in-place calls on the constructor's
                GaussPyInit — GenerateDoG() K times ("regen", main.cpp:66-73's loop) or GaussFilter
                of every octave K rounds ("gauss") — for the bench inputs (bench.py --op regen|gauss)
  a512_hashes.json per-level hashes after repeated calls of GaussPyramid_a512omp's
                GenerateDoG_nomp_dynamic (the AVX-512 x OpenMP subset, :240-364) and GenerateDoG
                (its DoG-only form, :183-213) — oracle/_ref/ref_avx512 hash-a512omp
  meta.json     generator provenance (glibc, g++, input definitions)

Usage:  make -C oracle ref ref-mpi && python tests/golden/gen_golden.py [--only PART,...]
        PART: hashes, dumps, taps, checksums, mpi, a512, inplace (default: all)
"""
import json
import os
import platform
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SERIAL = os.path.join(REPO, "oracle", "_ref", "ref_serial")
REF_AVX512 = os.path.join(REPO, "oracle", "_ref", "ref_avx512")
REF_MPI = os.path.join(REPO, "oracle", "_ref", "ref_mpi")
REF_MPITEST = os.path.join(REPO, "oracle", "_ref", "ref_mpitest")
MPIEXEC = os.environ.get("MPIEXEC", "/opt/conda/bin/mpiexec")

# (n, S, input) cases hashed over EVERY octave the reference builds (floor(log2 n)+1).
HASH_CASES = [
    (1, 2, "lcg:12345"), (2, 2, "lcg:12345"), (3, 2, "lcg:12345"), (7, 2, "lcg:12345"),
    (16, 2, "lcg:12345"), (64, 2, "lcg:12345"), (64, 0, "lcg:12345"), (64, 1, "lcg:12345"),
    (64, 5, "lcg:12345"), (100, 2, "lcg:12345"), (256, 3, "lcg:12345"), (512, 2, "lcg:12345"),
    (512, 2, "ones"), (513, 3, "lcg:12345"), (1000, 2, "lcg:12345"), (1024, 2, "lcg:777"),
    (4096, 2, "lcg:12345"),
    # the benchmark's own input (bench.py / SURVEY.md §8d counter hash), image 0 and 1
    (4096, 2, "synth:0x5EED:0"), (4096, 2, "synth:0x5EED:1"),
    (8192, 2, "synth:0x5EED:0"),
]
# complete pyramids (every octave, every level) — small enough to commit
DUMP_CASES = [(1, 2, "lcg:12345"), (2, 2, "lcg:12345"), (3, 2, "lcg:12345"), (7, 2, "lcg:12345"),
              (16, 2, "lcg:12345"), (64, 2, "lcg:12345"), (64, 3, "lcg:99"), (100, 2, "lcg:12345")]
# GenerateDoG() called repeatedly without GaussPyInit (main.cpp:66-73 timing loop semantics)
REGEN_CASES = [(64, 2, "lcg:12345", 2), (64, 2, "lcg:12345", 3), (37, 1, "lcg:5", 2)]
# AVX512xOpenMP::GenerateDoG_nomp_dynamic output (subset semantics) and AVX512xPTHREAD output
SUBSET_CASES = [(64, 2, "lcg:12345"), (256, 2, "lcg:12345")]
WINDOW_CASES = [(512, 2, "lcg:12345"), (4096, 2, "lcg:12345")]
WINDOW = 96
# bench inputs (config 2/4 image 0 and 1; config 5 image 0) for gdp_checksum fixtures
CHECKSUM_CASES = [(4096, 2, "synth:0x5EED:0"), (4096, 2, "synth:0x5EED:1"), (512, 2, "lcg:12345"),
                  (16384, 2, "synth:0x5EED:0"),
                  # config 4 (512 x 4096^2, 64 per GPU): rank 0's last image and rank 7's first and
                  # last (global indices past 2^32 pixels: the counter hash folds the index)
                  (4096, 2, "synth:0x5EED:63"), (4096, 2, "synth:0x5EED:448"), (4096, 2, "synth:0x5EED:511")]
# bench.py verifies the first and last image of EVERY rank: config 2 at N <= 8 (image r on rank r)
# and config 4 at N = 8 (images 64r and 64r + 63)
CHECKSUM_CASES += [(4096, 2, f"synth:0x5EED:{i}") for i in
                   list(range(2, 8)) + [x for r in range(1, 7) for x in (64 * r, 64 * r + 63)]]
# the multi-process variants' collector output: (variant, n, S, input); power-of-two n agree with
# the serial header, non-power-of-two n use the integer-length window centre (GaussDePyramid-MPI.h:273)
MPI_CASES = [(v, n, S, inp) for v in ("GaussDePyramid-MPI.h:GenerateDoG_mpi", "mpitest.cpp:GenerateDoG_mpi",
                                       "mpitest.cpp:GenerateDoG_mpi_omp")
             for n, S, inp in [(512, 2, "lcg:12345"), (256, 2, "ones"), (256, 2, "lcg:12345"),
                               (100, 2, "lcg:12345"), (1000, 2, "lcg:12345"), (96, 1, "lcg:7")]]
# GaussPyramid_a512omp / _a512xp methods, (method, n, S, input, calls): power-of-two n only (its 16-float
# vector loops run past the row end otherwise); n <= 8 octaves take its scalar branch
A512_CASES = [("nomp_dynamic", n, S, inp, calls) for n, S, inp, calls in [
    (64, 2, "lcg:12345", 1), (256, 2, "lcg:12345", 2), (512, 2, "lcg:12345", 1), (512, 2, "ones", 3),
    (1024, 3, "lcg:7", 1), (2048, 1, "lcg:5", 2), (16, 2, "lcg:3", 1), (8, 2, "lcg:3", 2), (256, 5, "lcg:9", 1),
    (128, 0, "lcg:1", 1), (4096, 2, "synth:0x5EED:0", 1)]] + \
    [("GenerateDoG", n, S, inp, calls) for n, S, inp, calls in [
        (64, 2, "lcg:12345", 1), (64, 2, "lcg:12345", 2), (256, 3, "ones", 1), (512, 2, "lcg:12345", 1),
        (16, 2, "lcg:3", 3)]] + \
    [("xp.GenerateDoG", n, S, inp, calls) for n, S, inp, calls in [
        (3, 2, "lcg:12345", 1), (5, 2, "lcg:12345", 1), (6, 1, "lcg:4", 2), (7, 3, "lcg:12345", 1),
        (64, 2, "lcg:12345", 2), (512, 2, "lcg:12345", 1)]]
A512_CHECKSUM_CASES = [(4096, 2, "synth:0x5EED:0"), (4096, 2, "synth:0x5EED:1")]
# in-place re-entry ops after the bench's timed region: (op, calls, n, S, input) — config 2's image
# and config 4's rank-0 first / last image
INPLACE_CHECKSUM_CASES = [(op, calls, 4096, 2, f"synth:0x5EED:{i}") for op, calls in (("regen", 3), ("gauss", 2))
                          for i in (0, 63)]
TAP_CASES = [(512, 2), (100, 2), (1000, 2), (513, 3), (4096, 2), (1080, 2), (1920, 2), (37, 1)]


def octaves_of(n):
    x = 0
    while n:
        x += 1
        n //= 2
    return x


def level_slices(n, S):
    """(o, s) -> slice of the packed float32 layout of oracle/ref_harness.cpp:dump()."""
    out, off = {}, 0
    for o in range(octaves_of(n)):
        m = n >> o
        for s in range(S + 3):
            out[(o, s)] = (off, m)
            off += m * m
    return out, off


def run(*args):
    return subprocess.run(list(args), check=True, capture_output=True, text=True).stdout


def dump(binary, mode, n, S, inp, *extra):
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "out.f32")
        run(binary, mode, str(n), str(S), inp, *extra, path)
        return np.fromfile(path, dtype=np.float32)


def key(*parts):
    return "_".join(str(p).replace(":", "-") for p in parts)


def gen_checksums():
    # gdp_checksum values (definition in include/gdp.h) of the reference's output for the bench's
    # own input images, over the first 5 octaves (bench configs) and over all octaves
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # the checksum formula's numpy restatement (test infrastructure)

    # incremental: cases already in checksums.json are kept (the 16384^2 dump alone is 7 GB); pass
    # --force to regenerate every case
    path = os.path.join(HERE, "checksums.json")
    have = {}
    if os.path.exists(path) and "--force" not in sys.argv:
        with open(path) as f:
            have = {(r["n"], r["S"], r["input"]): r for r in json.load(f)}
    checks = []
    for n, S, inp in CHECKSUM_CASES:
        if (n, S, inp) in have:
            checks.append(have[(n, S, inp)])
            continue
        pyr = dump(REF_SERIAL, "dump", n, S, inp)
        sl, _ = level_slices(n, S)
        acc, rec = 0, {"n": n, "S": S, "input": inp}
        for o in range(octaves_of(n)):
            m = n >> o
            for s in range(S + 3):
                off, _ = sl[(o, s)]
                acc = (acc + oracle.level_checksum(pyr[off:off + m * m].reshape(m, m), o, s)) & 0xFFFFFFFFFFFFFFFF
            rec[f"octaves_{o + 1}"] = f"{acc:016x}"
        checks.append(rec)
        print("checksum", n, inp, flush=True)
    with open(os.path.join(HERE, "checksums.json"), "w") as f:
        json.dump(checks, f, indent=1)


def run_mpi(variant, n, S, inp):
    """Collector-rank hashes of one multi-process reference run (S+4 ranks, rank S+3 prints)."""
    binary = REF_MPI if variant.startswith("GaussDePyramid-MPI.h") else REF_MPITEST
    args = [MPIEXEC, "-n", str(S + 4), binary, "hash", str(n), str(S), inp]
    if binary == REF_MPITEST:
        args.append("mpi_omp" if variant.endswith("_omp") else "mpi")
    out = run(*args)
    recs = [json.loads(line) for line in out.splitlines() if line.startswith("{")]
    assert len(recs) == 1, out
    return recs[0]


def gen_mpi():
    for b in (REF_MPI, REF_MPITEST, REF_SERIAL):
        if not os.path.exists(b):
            sys.exit(f"missing {b}: run `make -C oracle ref ref-mpi` first")
    out = []
    for variant, n, S, inp in MPI_CASES:
        rec = run_mpi(variant, n, S, inp)
        ser = json.loads(run(REF_SERIAL, "hash", str(n), str(S), inp))
        rec.update({"variant": variant, "input": inp, "ranks": S + 4, "collector_rank": S + 3,
                    "equals_serial": rec["octaves"] == ser["octaves"]})
        out.append(rec)
        print("mpi", variant, n, S, inp, "equals serial:", rec["equals_serial"], flush=True)
    with open(os.path.join(HERE, "mpi_hashes.json"), "w") as f:
        json.dump(out, f, indent=1)


def gen_a512():
    if not os.path.exists(REF_AVX512):
        sys.exit(f"missing {REF_AVX512}: run `make -C oracle ref` first")
    out = []
    for method, n, S, inp, calls in A512_CASES:
        # counnt = 1: with more threads its DoG loop (an `omp for` over i < S-1, level i -= level
        # i+1 in place, :324-357) is a data race once S >= 3 — the output is then timing-dependent
        rec = json.loads(run(REF_AVX512, "hash-a512omp", str(n), str(S), inp, str(calls), method, "1"))
        name = {"nomp_dynamic": "GaussPyramid_a512omp::GenerateDoG_nomp_dynamic",
                "GenerateDoG": "GaussPyramid_a512omp::GenerateDoG",
                "xp.GenerateDoG": "GaussPyramid_a512xp::GenerateDoG"}[method]
        rec.update({"method": name, "input": inp, "calls": calls, "counnt": 1})
        if method == "xp.GenerateDoG":  # recorded as a fact about the reference
            ser = json.loads(run(REF_SERIAL, "regen-hash", str(n), str(S), inp, str(calls)))
            rec["equals_serial"] = rec["octaves"] == ser["octaves"]
        out.append(rec)
        print("a512", method, n, S, inp, calls, flush=True)
    with open(os.path.join(HERE, "a512_hashes.json"), "w") as f:
        json.dump(out, f, indent=1)
    # gdp_checksum of GenerateDoG_nomp_dynamic's output for the bench inputs (bench.py --op subset)
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # the checksum formula's numpy restatement (test infrastructure)

    checks = []
    for n, S, inp in A512_CHECKSUM_CASES:
        pyr = dump(REF_AVX512, "dump-a512omp", n, S, inp)  # S = 2: one DoG iteration, no race
        sl, _ = level_slices(n, S)
        acc, rec = 0, {"n": n, "S": S, "input": inp, "method": "GaussPyramid_a512omp::GenerateDoG_nomp_dynamic"}
        for o in range(octaves_of(n)):
            m = n >> o
            for s in range(S + 3):
                off, _ = sl[(o, s)]
                acc = (acc + oracle.level_checksum(pyr[off:off + m * m].reshape(m, m), o, s)) & 0xFFFFFFFFFFFFFFFF
            rec[f"octaves_{o + 1}"] = f"{acc:016x}"
        checks.append(rec)
        print("a512 checksum", n, inp, flush=True)
    with open(os.path.join(HERE, "checksums_a512omp.json"), "w") as f:
        json.dump(checks, f, indent=1)


def gen_inplace():
    # gdp_checksum after K in-place calls of the serial reference (oracle/_ref/ref_serial regen /
    # gauss), for bench.py's post-timing parity check of --op regen / --op gauss
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # the checksum formula's numpy restatement (test infrastructure)

    checks = []
    for op, calls, n, S, inp in INPLACE_CHECKSUM_CASES:
        pyr = dump(REF_SERIAL, op, n, S, inp, str(calls))
        sl, _ = level_slices(n, S)
        acc = 0
        rec = {"op": op, "calls": calls, "n": n, "S": S, "input": inp,
               "method": ("GuassDePyramid.h GenerateDoG() x%d" % calls) if op == "regen" else
                         ("GuassDePyramid.h GaussFilter(o) for every octave, x%d" % calls)}
        for o in range(octaves_of(n)):
            m = n >> o
            for s in range(S + 3):
                off, _ = sl[(o, s)]
                acc = (acc + oracle.level_checksum(pyr[off:off + m * m].reshape(m, m), o, s)) & 0xFFFFFFFFFFFFFFFF
            rec[f"octaves_{o + 1}"] = f"{acc:016x}"
        checks.append(rec)
        print("inplace checksum", op, calls, n, inp, flush=True)
    with open(os.path.join(HERE, "checksums_inplace.json"), "w") as f:
        json.dump(checks, f, indent=1)


def main():
    parts = {"hashes", "dumps", "taps", "checksums", "mpi", "a512", "inplace"}
    if "--only" in sys.argv:
        parts = set(sys.argv[sys.argv.index("--only") + 1].split(","))
    if "mpi" in parts:
        gen_mpi()
    if "a512" in parts:
        gen_a512()
    if "inplace" in parts:
        gen_inplace()
    if not parts - {"mpi", "a512", "inplace"}:
        return
    for b in (REF_SERIAL, REF_AVX512):
        if not os.path.exists(b):
            sys.exit(f"missing {b}: run `make -C oracle ref` first")
    if parts & {"hashes", "dumps", "taps"} != {"hashes", "dumps", "taps"} and parts & {"hashes", "dumps", "taps"}:
        sys.exit("hashes, dumps and taps are generated together")
    if "hashes" not in parts:
        return gen_checksums() if "checksums" in parts else None
    hashes = []
    for n, S, inp in HASH_CASES:
        rec = json.loads(run(REF_SERIAL, "hash", str(n), str(S), inp))
        rec["input"] = inp
        hashes.append(rec)
        print("hash", n, S, inp, flush=True)

    arrays = {}
    for n, S, inp in DUMP_CASES:
        arrays[key("full", n, S, inp)] = dump(REF_SERIAL, "dump", n, S, inp)
    for n, S, inp, calls in REGEN_CASES:
        arrays[key("regen", n, S, inp, calls)] = dump(REF_SERIAL, "regen", n, S, inp, str(calls))
    for n, S, inp in SUBSET_CASES:
        arrays[key("a512omp", n, S, inp)] = dump(REF_AVX512, "dump-a512omp", n, S, inp)
        full = dump(REF_AVX512, "dump-a512xp", n, S, inp)
        ser = dump(REF_SERIAL, "dump", n, S, inp)
        # recorded as a fact about the reference, checked again by tests/test_oracle.py
        arrays[key("a512xp_equals_serial", n, S, inp)] = np.array([np.array_equal(full.view(np.uint32), ser.view(np.uint32))])
    for n, S, inp in WINDOW_CASES:
        pyr = dump(REF_SERIAL, "dump", n, S, inp)
        sl, _ = level_slices(n, S)
        for o in range(4):
            m = n >> o
            h = min(WINDOW, m)
            r0 = m // 2 - h // 2
            for s in range(S + 3):
                off, _ = sl[(o, s)]
                lev = pyr[off:off + m * m].reshape(m, m)
                arrays[key("win", n, S, inp, o, s)] = lev[r0:r0 + h, r0:r0 + h].copy()
        arrays[key("winorigin", n, S, inp)] = np.array([m // 2 - min(WINDOW, m) // 2 for m in (n >> o for o in range(4))])
        print("window", n, flush=True)
    np.savez_compressed(os.path.join(HERE, "dumps.npz"), **arrays)

    taps = {}
    with tempfile.TemporaryDirectory() as td:
        for n, S in TAP_CASES:
            path = os.path.join(td, "t.f32")
            run(REF_SERIAL, "taps", str(n), str(S), path)
            t = np.fromfile(path, dtype=np.float32)
            off = 0
            for s in range(S + 3):
                for o in range(octaves_of(n)):
                    m = n >> o
                    taps[key("taps", n, S, o, s)] = t[off:off + m]
                    off += m
            assert off == t.size
    np.savez_compressed(os.path.join(HERE, "taps.npz"), **taps)

    with open(os.path.join(HERE, "hashes.json"), "w") as f:
        json.dump(hashes, f, indent=1)

    gen_checksums()
    gxx = run("g++", "--version").splitlines()[0]
    meta = {
        "generator": "tests/golden/gen_golden.py via oracle/_ref/ref_serial + ref_avx512 "
                     "(reference headers compiled in place by oracle/Makefile)",
        "reference_files": ["GuassDePyramid.h", "GaussDePyramid-AVX512xOpenMP.h", "GaussDePyramid-AVX512xPTHREAD.h"],
        "glibc": platform.libc_ver()[1], "gxx": gxx,
        "hash": "h0=0xcbf29ce484222325; h=(h^bits32)*0x100000001b3 mod 2^64 over float32 bits, row-major per level",
        "inputs": {
            "lcg:SEED": "s=SEED; per pixel row-major: s=s*1664525+1013904223 mod 2^32; px=s>>24",
            "ones": "every pixel 1 (main.cpp:31-35)",
            "synth:SEED:B": "idx=(B*n+r)*n+c (u64); x=SEED^(u32)(idx^(idx>>32)); lowbias32(x)>>24",
        },
        "layout": "packed: levels in (octave, scale) order, each (n>>o)x(n>>o) row-major float32",
        "window": f"centre window of {WINDOW}x{WINDOW} (or the whole level), origin listed in winorigin_*",
    }
    with open(os.path.join(HERE, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("done")


if __name__ == "__main__":
    main()
