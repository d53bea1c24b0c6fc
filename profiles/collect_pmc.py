#!/usr/bin/env python3
"""Summarise rocprofv3 runs of bench.py into profiles/ (committed evidence for bench.py's roofline).

Inputs (written on the GPU box under gpurun_out/ by tools/gpu_session.sh steps):
  <trace>/run_kernel_stats.csv          rocprofv3 --kernel-trace --stats
  <fetch>/run_counter_collection.csv    rocprofv3 --pmc FETCH_SIZE   (its own pass)
  <write>/run_counter_collection.csv    rocprofv3 --pmc WRITE_SIZE   (its own pass)
Corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE
are KiB; on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read,
so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for 16-B-per-lane streaming stores.

Writes profiles/pmc_<tag>_<round>.json (read by bench.py for roofline.traffic when the run's build
variant and tile order equal the recorded ones) and copies the kernel-stats CSV to
profiles/rocprof_<tag>_<round>_kernel_stats.csv.  The profiled bench runs are forced to one
variant / tile order (bench.py --variant V --tile-order T), recorded here.
"""
import argparse
import csv
import json
import os
import shutil
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))



def counter_values(path, counter, name):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Kernel_Name"] == name and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--bench-json", help="bench.py output line of the traced run (optional)")
    ap.add_argument("--kernel", default="k_build", help="substring of the kernel to summarise")
    ap.add_argument("--op", default="build", help="bench.py --op of the profiled run")
    ap.add_argument("--variant", type=int, default=None, help="build variant the profiled runs were forced to")
    ap.add_argument("--tile-order", type=int, default=None, help="build tile order of the profiled runs")
    ap.add_argument("--inplace-sub", type=int, default=None,
                    help="--op regen: GDP_TUNE_INPLACE_SUB the profiled runs were forced to (0 = k_levels_x)")
    ap.add_argument("--window-sub", type=int, default=None, help="--op gauss: GDP_TUNE_WINDOW_SUB of the profiled runs")
    ap.add_argument("--zero-window", type=int, default=0, help="GDP_TUNE_ZERO_WINDOW of the profiled runs")
    ap.add_argument("--tag", default=None, help="file tag (default: config, or config_op)")
    args = ap.parse_args()
    if args.op in ("build", "subset") and (args.variant is None or args.tile_order is None):
        ap.error("--op build/subset records need --variant and --tile-order")
    if args.op == "regen" and args.inplace_sub is None or args.op == "gauss" and args.window_sub is None:
        ap.error("--op regen needs --inplace-sub, --op gauss --window-sub")

    import bench

    stats = None  # the timed kernel: the matching row with the most calls
    with open(os.path.join(args.trace, "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            if args.kernel in r["Name"] and (stats is None or int(r["Calls"]) > int(stats["Calls"])):
                stats = r
    name = stats["Name"]
    fetch = counter_values(os.path.join(args.fetch, "run_counter_collection.csv"), "FETCH_SIZE", name)
    write = counter_values(os.path.join(args.write, "run_counter_collection.csv"), "WRITE_SIZE", name)
    cfg = bench.CONFIGS[args.config]
    if args.op in ("build", "conv", "subset"):
        alg = bench.algorithmic_bytes(cfg["H"], cfg["W"], 2, cfg["O"], cfg["batch"])
    else:  # in-place passes read and write every level: 8*(S+3)*P
        alg = 8 * 5 * cfg["batch"] * bench.pyramid_pixels(cfg["H"], cfg["W"], cfg["O"])
    read_b = 2 * statistics.median(fetch) * 1024
    write_b = statistics.median(write) * 1024
    rec = {
        "config": args.config, "round": args.round, "kernel": name,
        "variant": args.variant, "tile_order": args.tile_order, "input_format": "i32",
        **({"inplace_sub": args.inplace_sub} if args.inplace_sub is not None else {}),
        **({"window_sub": args.window_sub} if args.window_sub is not None else {}),
        "zero_window": args.zero_window,
        "trace_calls": int(stats["Calls"]) if stats else None,
        "trace_avg_ns": float(stats["AverageNs"]) if stats else None,
        "trace_min_ns": float(stats["MinNs"]) if stats else None,
        "fetch_size_kib_median": statistics.median(fetch), "write_size_kib_median": statistics.median(write),
        "dispatches_counted": [len(fetch), len(write)],
        "read_bytes_corrected": read_b, "write_bytes": write_b,
        "kernel_bytes_per_launch": read_b + write_b,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read_b + write_b) / alg,
        "trace_GBps_algorithmic": alg / (float(stats["AverageNs"]) * 1e-9) / 1e9 if stats else None,
        "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count of wide streaming reads); write = WRITE_SIZE KiB",
    }
    if args.bench_json and os.path.exists(args.bench_json):
        with open(args.bench_json) as f:
            for line in f:
                if line.startswith("{"):
                    rec["bench_line_of_traced_run"] = json.loads(line)
    # the timed region alone: the last `steps` dispatches of the kernel in the trace (the stats
    # row also averages the autotuning and warm-up launches)
    trace_csv = os.path.join(args.trace, "run_kernel_trace.csv")
    line = rec.get("bench_line_of_traced_run")
    if line and os.path.exists(trace_csv):
        with open(trace_csv) as f:
            durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                    for r in sorted((r for r in csv.DictReader(f) if r["Kernel_Name"] == name),
                                    key=lambda r: int(r["Start_Timestamp"]))]
        # launches of the same kernel after the timed region (the in-place ops' parity calls)
        post = int((line.get("parity") or {}).get("post_timing_launches", 0))
        timed = durs[-int(line["steps"]) - post:len(durs) - post]
        if timed:
            rec["trace_timed_steps"] = len(timed)
            rec["trace_timed_avg_ns"] = statistics.mean(timed)
            rec["bench_kernel_ms"] = line["roofline"]["kernel_ms"]
    tag = args.tag or (args.config if args.op == "build" else f"{args.config}_{args.op}")
    rec["op"] = args.op
    out = os.path.join(HERE, f"pmc_{tag}_{args.round}.json")
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    shutil.copy(os.path.join(args.trace, "run_kernel_stats.csv"),
                os.path.join(HERE, f"rocprof_{tag}_{args.round}_kernel_stats.csv"))
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
