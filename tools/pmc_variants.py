#!/usr/bin/env python3
"""HBM bytes per launch of EVERY build-kernel instance bench.py's autotune can pick, in one process:
each (variant, tile order) builds `--reps` times over the rotated cold buffer sets bench.py uses,
in a fixed order written to a manifest, so the per-dispatch counters of one rocprofv3 --pmc pass
map back to (variant, tile order).  Run once per counter (passes never share counters):

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcv_fetch -o run --output-format csv -- \
        python3 tools/pmc_variants.py --config c2 --manifest gpurun_out/pmcv_manifest.json
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcv_write ...  (same command)

then, in the container: python3 tools/pmc_variants.py --summarise --config c2 --round r02 \
    --manifest gpurun_out/pmcv_manifest.json --fetch gpurun_out/pmcv_fetch --write gpurun_out/pmcv_write
which writes profiles/pmc_<config>_v<V>o<T>_<round>.json for every instance (bench.py attaches
`roofline.traffic` from the record whose variant and tile order equal the run's)."""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def run(args):
    import __graft_entry__ as entry

    pkg = entry.load_package()
    cfg = bench.CONFIGS[args.config]
    H, W, O, B = cfg["H"], cfg["W"], cfg["O"], cfg["batch"]
    r0, r1 = band_rows(pkg, cfg, args.band_of)
    set_bytes = band_bytes(cfg, r0, r1)
    rotate = max(1, -(-bench.ROTATE_BYTES // set_bytes))
    # --band-of N: rank 0's row band of the N-rank row-band job (bench.py's context on that rank)
    ctxs = [pkg.PyramidContext(H, W, S=2, octaves=O, batch=B, row_begin=r0, row_end=r1) for _ in range(rotate)]
    for c in ctxs:
        c.fill_synthetic(bench.SEED, 0)
        c.set_tuning(zero_window=args.zero_window)
        if args.op == "subset":  # bench.py --op subset's contexts
            c.set_window_centre("intlen")
        c.sync()
    order = []
    only = {int(x) for x in args.variants.split(",")} if args.variants else None
    for v in pkg.build_variants():
        if only is None or v in only:
            order += [(v, 0), (v, 1)]
    manifest = []
    for v, t in order:
        for c in ctxs:
            c.set_tuning(variant=v, tile_order=t)
        n = 0
        for i in range(args.warm + args.reps):  # consecutive launches cycle through the cold sets
            (ctxs[i % rotate].build_subset if args.op == "subset" else ctxs[i % rotate].build)()
            n += 1
        for c in ctxs:
            c.sync()
        manifest.append({"variant": v, "tile_order": t, "dispatches": n, "warm": args.warm})
    chunk_kb = ctxs[0].tuning().get("pyramid_chunk_kb", 0)
    for c in ctxs:
        c.close()
    with open(args.manifest, "w") as f:
        json.dump({"config": args.config, "op": args.op, "rotate": rotate, "zero_window": args.zero_window,
                   "band_of": args.band_of, "band": [r0, r1], "instances": manifest,
                   "image_stride_mb": int(os.environ["GDP_IMAGE_STRIDE_MB"]) if os.environ.get("GDP_IMAGE_STRIDE_MB")
                   else None, "pyramid_chunk_kb": chunk_kb}, f)


def band_rows(pkg, cfg, band_of):
    """Rows of the profiled context: the whole image, or rank 0's band of `band_of` ranks."""
    if not band_of:
        return 0, cfg["H"]
    if not cfg["band"]:
        sys.exit("--band-of needs the row-band config (c5)")
    mg = __import__(pkg.__name__ + ".distributed", fromlist=["plan_band"])
    return mg.plan_band(cfg["H"], band_of, 0, cfg["O"])


def band_bytes(cfg, r0, r1):
    """Algorithmic bytes of one launch over input rows [r0, r1): 4 B per input pixel + 4 (S+3) B
    per pyramid pixel of the band (bench.py's per-rank accounting)."""
    H, W, O, B = cfg["H"], cfg["W"], cfg["O"], cfg["batch"]
    if (r0, r1) == (0, H):
        return bench.algorithmic_bytes(H, W, 2, O, B)
    px = sum((((r1 + (1 << o) - 1) >> o) - ((r0 + (1 << o) - 1) >> o)) * (W >> o) for o in range(O))
    return B * (4 * (r1 - r0) * W + 4 * 5 * px)


def per_dispatch(d, counter):
    rows = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if "k_build" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def summarise(args):
    with open(args.manifest) as f:
        man = json.load(f)
    fetch, write = per_dispatch(args.fetch, "FETCH_SIZE"), per_dispatch(args.write, "WRITE_SIZE")
    total = sum(m["dispatches"] for m in man["instances"])
    if len(fetch) != total or len(write) != total:
        sys.exit(f"dispatch count mismatch: manifest {total}, FETCH_SIZE {len(fetch)}, WRITE_SIZE {len(write)}")
    cfg = bench.CONFIGS[man["config"]]
    band_of = man.get("band_of")
    r0, r1 = man.get("band", [0, cfg["H"]])
    alg = band_bytes(cfg, r0, r1)
    k = 0
    for m in man["instances"]:
        fs, ws = fetch[k:k + m["dispatches"]], write[k:k + m["dispatches"]]
        k += m["dispatches"]
        fs, ws = fs[m["warm"]:], ws[m["warm"]:]
        read_b = 2 * statistics.median(v for _, v, _ in fs) * 1024
        write_b = statistics.median(v for _, v, _ in ws) * 1024
        rec = {"config": man["config"], "round": args.round, "kernel": fs[0][2], "variant": m["variant"],
               "tile_order": m["tile_order"], "input_format": "i32", "op": man.get("op", "build"),
               "zero_window": man.get("zero_window", 0),
               **({"band_of": band_of, "band_rows": [r0, r1]} if band_of else {}),
               **({"image_stride_mb": man["image_stride_mb"]} if man.get("image_stride_mb") else {}),
               **({"pyramid_chunk_kb": man["pyramid_chunk_kb"]} if man.get("pyramid_chunk_kb") else {}),
               "source": "tools/pmc_variants.py: every instance in one process, its own FETCH_SIZE and WRITE_SIZE "
                         "rocprofv3 --pmc passes, launches cycling over %d cold buffer sets as in bench.py" % man["rotate"],
               "dispatches_counted": [len(fs), len(ws)],
               "fetch_size_kib_median": read_b / 2048, "write_size_kib_median": write_b / 1024,
               "read_bytes_corrected": read_b, "write_bytes": write_b,
               "kernel_bytes_per_launch": read_b + write_b, "algorithmic_bytes_per_launch": alg,
               "traffic_over_algorithmic": (read_b + write_b) / alg,
               "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count of wide streaming reads); write = WRITE_SIZE KiB"}
        tag = man["config"] + (f"b{band_of}" if band_of else "") + ("_subset" if man.get("op") == "subset" else "")
        zw = ("z1" if man.get("zero_window", 0) else "") + (f"s{man['image_stride_mb']}" if man.get("image_stride_mb") else "") \
            + (f"k{man['pyramid_chunk_kb']}" if man.get("pyramid_chunk_kb") else "")
        out = os.path.join(REPO, "profiles", f"pmc_{tag}_v{m['variant']}o{m['tile_order']}{zw}_{args.round}.json")
        if os.path.exists(out) and not args.overwrite:
            print("keep", out)
            continue
        with open(out, "w") as f:
            json.dump(rec, f, indent=1)
        print(os.path.basename(out), round(rec["traffic_over_algorithmic"], 4))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--manifest", default="gpurun_out/pmcv_manifest.json")
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--summarise", action="store_true")
    ap.add_argument("--op", default="build", choices=["build", "subset"],
                    help="subset: the GenerateDoG_nomp_dynamic build (bench.py --op subset)")
    ap.add_argument("--zero-window", type=int, default=0, choices=[0, 1],
                    help="GDP_TUNE_ZERO_WINDOW of every instance (records pmc_<cfg>_v<V>o<T>z1_*.json)")
    ap.add_argument("--variants", default=None, help="comma-separated variant numbers to profile (default: all)")
    ap.add_argument("--band-of", type=int, default=None,
                    help="row-band config: profile rank 0's band of N ranks (bench.py --gpus N --config c5's "
                         "per-rank launch; records pmc_c5b<N>_*.json)")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--round", default="r02")
    ap.add_argument("--overwrite", action="store_true", help="replace records written by tools/pmc_session.sh")
    args = ap.parse_args()
    summarise(args) if args.summarise else run(args)


if __name__ == "__main__":
    main()
