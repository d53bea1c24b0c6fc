#!/usr/bin/env python3
"""PMC record of the kernel a bench.py line timed (any --op), from two separate rocprofv3 --pmc
passes of the SAME bench.py command (FETCH_SIZE, then WRITE_SIZE):

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/p_fetch -o run --output-format csv -- python3 bench.py <args> --no-cpu
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/p_write -o run --output-format csv -- python3 bench.py <args> --no-cpu
    python3 tools/pmc_bench.py --fetch gpurun_out/p_fetch --write gpurun_out/p_write \\
        --bench-log gpurun_out/<the FETCH pass's stdout> --kernel k_conv_blk --round r05 --tag c2_conv_h8

Reads = 2 x FETCH_SIZE KiB (the guide's gfx950 correction, calibrated for this kernel's access
widths in round 4: profiles/calib_fetch_r04a.json), writes = WRITE_SIZE KiB; the median over the
dispatches of the named kernel (the bench's warm-up, autotune and timed launches alike: every
candidate moves the same bytes).  Writes profiles/pmc_<tag>_<round>.json with the bench line's
config / tuning keys, which bench.py's selectors (latest_conv_pmc / latest_inplace_pmc /
latest_pmc) match against later runs."""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(d, counter, kernel):
    vals = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    vals.append((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r["Kernel_Name"]))
    vals.sort()
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--bench-log", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--round", required=True)
    ap.add_argument("--tag", required=True)
    args = ap.parse_args()
    kernel = args.kernel
    if kernel == "from-bench":  # exactly the instance the bench line timed (the autotune ran others)
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from timed_dispatches import instance_name

        kernel = instance_name(json.loads([x for x in open(args.bench_log) if x.startswith("{")][-1])["roofline"]["kernel"])
    fs = per_dispatch(args.fetch, "FETCH_SIZE", kernel)
    ws = per_dispatch(args.write, "WRITE_SIZE", kernel)
    if not fs or not ws:
        sys.exit(f"no {kernel} dispatches in the PMC output")
    line = [x for x in open(args.bench_log) if x.startswith("{")][-1]
    bench = json.loads(line)
    roof = bench["roofline"]
    read_b = 2 * statistics.median(v for _, v, _ in fs) * 1024
    write_b = statistics.median(v for _, v, _ in ws) * 1024
    alg = roof["algorithmic_bytes_per_launch"]
    op = "conv" if "[op=conv" in bench["metric"] else "regen" if "[op=regen" in bench["metric"] else \
        "gauss" if "[op=gauss" in bench["metric"] else "subset" if "[op=subset" in bench["metric"] else "build"
    rec = {"config": None,
           "round": args.round, "op": op, "kernel": fs[0][2], "input_format": "i32",
           **{k: v for k, v in bench.get("tuning", {}).items()
              if (op == "conv" and k.startswith("conv_")) or (op in ("build", "subset") and k in (
                  "variant", "tile_order", "zero_window", "pyramid_chunk_kb")) or
              (op in ("regen", "gauss") and k in ("inplace_sub", "window_sub", "zero_window"))},
           "dispatches_counted": [len(fs), len(ws)],
           "read_bytes_corrected": read_b, "write_bytes": write_b, "kernel_bytes_per_launch": read_b + write_b,
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (read_b + write_b) / alg,
           "bench_kernel_ms": roof["kernel_ms"], "bench_line_of_traced_run": bench,
           "source": "tools/pmc_bench.py: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes of the same bench.py command",
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count of wide streaming reads); write = WRITE_SIZE KiB"}
    sys.path.insert(0, REPO)
    import bench as bench_py  # the workload names of bench.py's CONFIGS

    wl = bench["config"]["workload"]
    rec["config"] = next((k for k, c in bench_py.CONFIGS.items() if c["name"] == wl), None)
    out = os.path.join(REPO, "profiles", f"pmc_{args.tag}_{args.round}.json")
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(os.path.basename(out), round(rec["traffic_over_algorithmic"], 4), "read", round(read_b / 1e6, 1), "MB",
          "write", round(write_b / 1e6, 1), "MB")


if __name__ == "__main__":
    main()
