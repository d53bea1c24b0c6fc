#!/usr/bin/env python3
"""Ramp and tail of one cold k_build launch, from per-block timestamps (diagnostic build).

    make -C tools/trace && python tools/trace/trace_blocks.py [--shape 4096x4096x1] [--variant 0]
    python tools/trace/trace_blocks.py --op conv [--conv-rows 48 --conv-waves 16]   (k_conv_blk)

Builds tools/trace/libgdp_trace.so's k_build over `--rotate` buffer sets (so the traced launch is
cold, as in bench.py), then traces one launch: per WAVE the 100 MHz real-time clock at entry and
after its last store was issued, and its XCC.  Prints one JSON line per repeat: launch span, when
the last wave STARTED, the spread of wave end times, mean wave lifetime per dispatch round,
per-XCC first-start / last-end.
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
os.environ.setdefault("GDP_LIBRARY", os.path.join(HERE, "libgdp_trace.so"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4096x4096x1")
    ap.add_argument("--variant", type=int, default=15)
    ap.add_argument("--zero-window", type=int, default=1)
    ap.add_argument("--store-pace", type=int, default=-1)
    ap.add_argument("--order", type=int, default=0)
    ap.add_argument("--rotate", type=int, default=5)
    ap.add_argument("--op", choices=("build", "conv"), default="build")
    ap.add_argument("--conv-rows", type=int, default=None)
    ap.add_argument("--conv-waves", type=int, default=None)
    ap.add_argument("--conv-order", type=int, default=None)
    args = ap.parse_args()
    import numpy as np
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    from importlib import import_module

    lib = import_module(pkg.__name__ + "._lib").lib()
    lib.gdp_debug_set_block_trace.argtypes = [ctypes.c_void_p]
    H, W, B = (int(x) for x in args.shape.split("x"))
    ctxs = [pkg.PyramidContext(H, W, S=2, octaves=5, batch=B) for _ in range(args.rotate)]
    for c in ctxs:
        c.fill_synthetic(0x5EED, 0)
        if args.op == "conv":
            c.set_tuning(conv_kernel=2, conv_rows=args.conv_rows, conv_waves=args.conv_waves,
                         conv_order=args.conv_order)
        else:
            c.set_tuning(variant=args.variant, tile_order=args.order, zero_window=args.zero_window,
                         store_pace=args.store_pace)
    run = (lambda c, st=None: c.build_gaussian(st)) if args.op == "conv" else (lambda c, st=None: c.build(st))
    for _ in range(3):
        for c in ctxs:
            run(c)
    for c in ctxs:
        c.sync()
    blocks = 1 << 24  # wave records
    buf = torch.zeros(3 * blocks, dtype=torch.int64, device="cuda")
    out = []
    for rep in range(3):
        for c in ctxs[1:]:
            run(c)
        for c in ctxs:
            c.sync()
        buf.zero_()
        torch.cuda.synchronize()
        assert lib.gdp_debug_set_block_trace(ctypes.c_void_p(buf.data_ptr())) == 0
        ev_ms = ctypes.c_float()
        if args.op == "conv":  # one traced launch between torch events on torch's current stream
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run(ctxs[0], st)
            e1.record(st)
            e1.synchronize()
            ev_ms.value = e0.elapsed_time(e1)
        else:  # one traced launch between HIP events on the context's stream (gdp_time_builds, iters 1)
            assert lib.gdp_time_builds(ctxs[0]._ctx, 1, None, ctypes.byref(ev_ms)) == 0
        ctxs[0].sync()
        assert lib.gdp_debug_set_block_trace(None) == 0
        t = buf.cpu().numpy().reshape(-1, 3)
        t = t[t[:, 0] != 0]
        t0 = t[:, 0].min()
        start = (t[:, 0] - t0) / 100.0  # us
        end = (t[:, 1] - t0) / 100.0
        xcc = (t[:, 2] >> 32) & 0xF
        life = end - start
        order = np.argsort(start)
        n = len(t)
        span = float(end.max())
        # dispatch rounds: blocks sorted by start, cut into groups of the resident count
        resident = int((start < float(end.min())).sum())  # waves started before the first one ended
        rounds = [float(life[order[i:i + resident]].mean()) for i in range(0, n, max(resident, 1))]
        rec = {"rep": rep, "waves": n, "span_us": round(span, 2), "last_block_start_us": round(float(start.max()), 2),
               "first_block_end_us": round(float(end.min()), 2),
               "end_p10_p50_p90_us": [round(float(np.percentile(end, p)), 2) for p in (10, 50, 90)],
               "lifetime_mean_us": round(float(life.mean()), 2), "resident_at_start": resident,
               "lifetime_by_round_us": [round(x, 2) for x in rounds[:12]],
               "idle_tail_us": round(span - float(np.percentile(end, 50)), 2),
               "xcc_first_start_last_end_us": {int(x): [round(float(start[xcc == x].min()), 2),
                                                        round(float(end[xcc == x].max()), 2)] for x in np.unique(xcc)}}
        # fraction of the span with fewer than half the resident blocks running
        grid = np.linspace(0, span, 400)
        running = np.array([((start <= g) & (end > g)).sum() for g in grid])
        rec["us_below_half_resident"] = round(float((running < resident / 2).mean() * span), 2)
        # ramp / drain split: the launch's HIP-event time vs the waves' span;
        # ramp = first wave start -> running waves first reach 90 % of their peak; drain = running
        # waves last at 90 % of the peak -> last wave's last store issued; after = event time not
        # covered by any wave (dispatch before the first wave + completion after the last store)
        peak = running.max()
        hi = np.flatnonzero(running >= 0.9 * peak)
        rec["event_us"] = round(ev_ms.value * 1e3, 2)
        rec["ramp_us"] = round(float(grid[hi[0]]), 2)
        rec["drain_us"] = round(span - float(grid[hi[-1]]), 2)
        rec["steady_us"] = round(float(grid[hi[-1]] - grid[hi[0]]), 2)
        rec["outside_waves_us"] = round(ev_ms.value * 1e3 - span, 2)
        # running waves over the launch in 20 equal bins (mean per bin), and per XCC the time its
        # last wave issued its last store relative to the launch's last one
        edges = np.linspace(0, span, 21)
        rec["running_waves_20_bins"] = [int(running[(grid >= a) & (grid < b)].mean()) if ((grid >= a) & (grid < b)).any()
                                        else 0 for a, b in zip(edges[:-1], edges[1:])]
        ends = sorted(float(end[xcc == x].max()) for x in np.unique(xcc))
        rec["xcc_end_spread_us"] = round(ends[-1] - ends[0], 2)
        rec["xcc_end_mean_gap_us"] = round(ends[-1] - float(np.mean(ends)), 2)
        rec["max_running_waves"] = int(running.max())
        rec["running_p50_over_span"] = int(np.median(running))
        # per CU (XCC, SE, SA?, CU from HW_ID) peak concurrency at the busiest sampled instant
        hw = t[:, 2] & 0xFFFFFFFF
        cu = (xcc << 16) | ((hw >> 13) & 0x7) << 8 | ((hw >> 12) & 0x1) << 4 | ((hw >> 8) & 0xF)
        g = grid[int(np.argmax(running))]
        live = (start <= g) & (end > g)
        _, per_cu = np.unique(cu[live], return_counts=True)
        rec["waves_per_cu_at_peak"] = [int(per_cu.min()), int(np.median(per_cu)), int(per_cu.max()), int(len(per_cu))]
        out.append(rec)
        print(json.dumps(rec), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
