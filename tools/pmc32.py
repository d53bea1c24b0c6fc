#!/usr/bin/env python3
"""Exact-byte traffic of a kernel from the TCC's 32-byte request counters (round 5).

FETCH_SIZE on gfx950 tallies a 128-B read request as 64 B (the guide's x2 correction, calibrated
per access width); TCC_EA0_RDREQ_32B counts every read request in 32-B units (a 128-B request as
4), TCC_EA0_RDREQ_DRAM_32B the ones destined for DRAM, TCC_EA0_WRREQ_WRITE_DRAM_32B the DRAM
writes likewise — bytes = count x 32 with no correction.  Reads the counter_collection CSVs of
rocprofv3 --pmc passes and prints, per kernel instance matching --kernel, the median over its
dispatches of every counter found, in bytes:

    rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_32B_sum -d gpurun_out/p32r -o run \\
        --output-format csv -- python3 bench.py ... --no-cpu
    rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_DRAM_32B_sum TCC_EA0_WRREQ_64B_sum -d gpurun_out/p32w ...
    python3 tools/pmc32.py --kernel k_build --dirs gpurun_out/p32r gpurun_out/p32w [--algorithmic B]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--dirs", nargs="+", required=True)
    ap.add_argument("--algorithmic", type=float, default=None, help="algorithmic bytes per launch")
    a = ap.parse_args()
    vals = {}
    for d in a.dirs:
        for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(p) as f:
                for r in csv.DictReader(f):
                    if a.kernel in r["Kernel_Name"]:
                        key = (r["Kernel_Name"], r["Counter_Name"])
                        vals.setdefault(key, []).append(float(r["Counter_Value"]))
    out = {}
    for (kname, cname), v in sorted(vals.items()):
        scale = 32.0 if cname.endswith("_32B_sum") or cname.endswith("_32B") else 64.0 if "64B" in cname else 1.0
        rec = out.setdefault(kname, {})
        rec[cname] = {"dispatches": len(v), "median": statistics.median(v), "bytes": statistics.median(v) * scale}
        if a.algorithmic:
            rec[cname]["over_algorithmic"] = round(statistics.median(v) * scale / a.algorithmic, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
