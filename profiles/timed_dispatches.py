#!/usr/bin/env python3
"""Extract the TIMED dispatches of a bench run from its rocprofv3 kernel trace into a small tracked
CSV (the headline's per-launch average must be recomputable from tracked files,
not only from the gpurun_out/ scratch trace).

    python3 profiles/timed_dispatches.py <run_kernel_trace.csv> <bench.log or bench json line> <out.csv>

The timed region is the last `steps` dispatches of the kernel the line names (bench.py launches
nothing after its timed steps for --op build); the CSV keeps, per dispatch, its index, start / end
timestamps (ns) and duration, plus a trailing summary row; the mean duration and the line's
algorithmic bytes give the roofline fraction."""
import csv
import json
import statistics
import sys


def main(trace, bench, out):
    line = None
    with open(bench) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
    if line is None:
        sys.exit("no bench line in " + bench)
    steps = int(line["steps"])
    with open(trace) as f:
        rows = [r for r in csv.DictReader(f) if r["Kernel_Name"].startswith("void (anonymous namespace)::k_build")]
    # the timed kernel instance: the name of the last dispatch (autotune candidates come earlier)
    name = max(rows, key=lambda r: int(r["Start_Timestamp"]))["Kernel_Name"]
    mine = sorted((r for r in rows if r["Kernel_Name"] == name), key=lambda r: int(r["Start_Timestamp"]))
    timed = mine[-steps:]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    nbytes = line["roofline"]["algorithmic_bytes_per_launch"]
    mean = statistics.mean(durs)
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["dispatch", "start_ns", "end_ns", "duration_ns"])
        for i, (r, d) in enumerate(zip(timed, durs)):
            w.writerow([i, r["Start_Timestamp"], r["End_Timestamp"], d])
        w.writerow(["# kernel", name])
        w.writerow(["# timed_dispatches", len(durs), "mean_ns", round(mean, 1), "median_ns", statistics.median(durs)])
        w.writerow(["# algorithmic_bytes_per_launch", nbytes, "TBps", round(nbytes / mean / 1e3, 4),
                    "frac_of_8TBps", round(nbytes / mean / 8e3, 4)])
        w.writerow(["# bench_kernel_ms", line["roofline"]["kernel_ms"], "bench_frac", line["roofline"]["frac"]])
    print(json.dumps({"kernel": name, "timed": len(durs), "mean_ns": mean, "frac": nbytes / mean / 8e3}))


if __name__ == "__main__":
    main(*sys.argv[1:4])
