#!/usr/bin/env python3
"""Per-launch medians of the counter passes of tools/c3_counters.sh (k_build dispatches only,
summed over counter instances), normalised per TCC_EA0_WRREQ (one memory-side write request).
    python profiles/c3_counters_r02/summarise.py"""
import collections
import csv
import glob
import json
import os
import statistics

HERE = os.path.dirname(os.path.abspath(__file__))
rows = {}
for f in sorted(glob.glob(os.path.join(HERE, "cnt_*.csv"))):
    tag = os.path.basename(f)[4:].rsplit("_", 1)[0]
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_build" in r["Kernel_Name"]:
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for (_, c), v in agg.items():
        per[c].append(v)
    rows.setdefault(tag, {}).update({c: statistics.median(v) for c, v in per.items()})
out = {}
for tag, c in rows.items():
    wr = c["TCC_EA0_WRREQ_sum"]
    out[tag] = {"SQ_BUSY_CYCLES_per_WRREQ": round(c["SQ_BUSY_CYCLES"] / wr, 4),
                "WRREQ_STALL_per_WRREQ": round(c["TCC_EA0_WRREQ_STALL_sum"] / wr, 4),
                "TAG_STALL_per_WRREQ": round(c["TCC_TAG_STALL_sum"] / wr, 4),
                "SQ_WAIT_ANY_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
                "SQ_WAIT_INST_ANY_frac": round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4),
                "RDREQ_per_WRREQ": round(c["TCC_EA0_RDREQ_sum"] / wr, 4),
                "WAVE_CYCLES_per_wave": round(c["SQ_WAVE_CYCLES"] / c["SQ_WAVES"], 1),
                "raw": c}
print(json.dumps(out, indent=1))
