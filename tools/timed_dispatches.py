#!/usr/bin/env python3
"""The TIMED launches of a bench.py run, out of its rocprofv3 kernel trace.

bench.py's autotune and warm-up launch many kernel instances before the timed region, so the
`--stats` average of an instance mixes them in.  The timed region is the LAST `steps` dispatches of
the instance the bench line names (its kernel string: variant / tile order for k_build) on the
bench's own stream — the stream that carries most of that instance's dispatches (the serving-mode
`concurrent_streams` figure launches on four others); this writes them as
profiles/timed_dispatches_<tag>.csv (dispatch, start_ns, end_ns, duration_ns) and prints their mean
next to the bench line's kernel_ms:

    python3 tools/timed_dispatches.py --trace gpurun_out/prof_c2_trace --bench-log gpurun_out/prof_c2_trace.log \\
        --tag c2_r05e
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bench.py's kernel string -> the template arguments of that k_build instance
VARIANTS = {0: (1024, 256, 0, 16), 8: (512, 256, 0, 8), 11: (768, 384, 0, 8), 15: (1024, 256, 3, 16),
            16: (512, 256, 3, 8), 17: (768, 384, 3, 8), 18: (512, 128, 3, 16), 20: (512, 512, 4, 0),
            23: (768, 768, 4, 0), 27: (512, 512, 5, 0)}


def instance_name(kernel_string):
    """The kernel-trace name fragment of the instance a bench line's roofline.kernel names."""
    m = re.search(r"variant (\d+)", kernel_string)
    if kernel_string.startswith("k_build") and m:
        blk, tc, path, tr = VARIANTS[int(m.group(1))]
        sub = "true" if "SUB" in kernel_string.split(" ")[0] else "false"
        return f"k_build<5, true, {blk}, {tc}, {path}, {tr}, {sub}>"
    return kernel_string.split(" ")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True, help="rocprofv3 -d directory of the --kernel-trace run")
    ap.add_argument("--bench-log", required=True)
    ap.add_argument("--tag", required=True)
    args = ap.parse_args()
    line = json.loads([x for x in open(args.bench_log) if x.startswith("{")][-1])
    steps = line["steps"]
    want = instance_name(line["roofline"]["kernel"])
    rows = []
    for p in glob.glob(os.path.join(args.trace, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if want in r["Kernel_Name"]:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                                 r.get("Stream_Id", "0")))
    rows.sort()
    streams = [x[3] for x in rows]
    main = max(set(streams), key=streams.count) if streams else None
    timed = [x for x in rows if x[3] == main][-steps:]
    out = os.path.join(REPO, "profiles", f"timed_dispatches_{args.tag}.csv")
    with open(out, "w") as f:
        f.write("dispatch,start_ns,end_ns,duration_ns\n")
        for i, (s, e, _, _) in enumerate(timed):
            f.write(f"{i},{s},{e},{e - s}\n")
    d = [e - s for s, e, _, _ in timed]
    print(json.dumps({"file": os.path.relpath(out, REPO), "kernel": timed[0][2] if timed else want,
                      "dispatches": len(timed), "mean_us": round(statistics.mean(d) / 1e3, 3) if d else None,
                      "median_us": round(statistics.median(d) / 1e3, 3) if d else None,
                      "bench_kernel_ms": line["roofline"]["kernel_ms"],
                      "frac_from_trace": round(line["roofline"]["algorithmic_bytes_per_launch"] /
                                               (statistics.mean(d) * 1e-9) / 8e12, 4) if d else None}))


if __name__ == "__main__":
    main()
