#!/usr/bin/env python3
"""Summarise tools/fetch_calib under rocprofv3: per access width, the bytes
FETCH_SIZE reports and the raw read requests, against the bytes of the lines the case reads.

    python3 tools/calib_summary.py --fetch gpurun_out/calib_fetch --req gpurun_out/calib_req \
        --log gpurun_out/calib_fetch_r04a.log --out profiles/calib_fetch_r04.json

The dispatches of fetch_calib run in the order its stdout lists; per case the record holds
fetch_bytes = FETCH_SIZE x 1024, the factor bytes_of_lines / fetch_bytes (2.0 = the guide's
half-count of wide streaming reads), and RDREQ / RDREQ_32B when that pass was collected."""
import argparse
import csv
import glob
import json
import os


def per_dispatch(d, counters):
    rows = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] in counters and ("k_b128" in r["Kernel_Name"] or "k_b32" in r["Kernel_Name"]):
                    rows.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--req", default=None)
    ap.add_argument("--log", required=True, help="fetch_calib's stdout (one JSON line per case, in order)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    cases = []
    with open(a.log) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{") and '"case"' in line:
                cases.append(json.loads(line))
    fetch = per_dispatch(a.fetch, {"FETCH_SIZE"})
    req = per_dispatch(a.req, {"TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ", "TCC_EA0_RDREQ_32B"}) \
        if a.req else []
    if len(fetch) != len(cases):
        raise SystemExit(f"{len(fetch)} FETCH_SIZE dispatches for {len(cases)} cases")
    out = []
    for i, c in enumerate(cases):
        fb = fetch[i]["FETCH_SIZE"] * 1024
        rec = dict(c, fetch_bytes=fb, lines_over_fetch=c["bytes_of_lines"] / fb if fb else None)
        if req and len(req) == len(cases):
            r = req[i]
            rd = r.get("TCC_EA0_RDREQ_sum", r.get("TCC_EA0_RDREQ"))
            r32 = r.get("TCC_EA0_RDREQ_32B_sum", r.get("TCC_EA0_RDREQ_32B"))
            rec.update(rdreq=rd, rdreq_32b=r32, lines_per_rdreq=(c["lines"] / rd) if rd else None)
        out.append(rec)
    with open(a.out, "w") as f:
        json.dump({"source": "tools/fetch_calib.hip under rocprofv3 --pmc (one pass per counter set)", "cases": out}, f,
                  indent=1)
    for r in out:
        print(json.dumps({k: r.get(k) for k in ("case", "fetch_bytes", "lines_over_fetch", "rdreq", "rdreq_32b",
                                                 "lines_per_rdreq")}))


if __name__ == "__main__":
    main()
