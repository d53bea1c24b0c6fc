#!/usr/bin/env python3
"""Research A/B of the convolution block tiles' register budget (round 5): k_conv_blk (product:
one output row of a wave at a time, 64 VGPRs, two 16-wave blocks per CU) against k_conv_blk_x of
the research build (tools/ab/libgdp_exp.so: UR rows of a wave unrolled branch-free so their
chains interleave, at exactly W waves per SIMD), over rows-per-block / waves-per-block shapes.

Each case runs in its own process (the research build reads GDP_CONV_UNROLL /
GDP_CONV_WAVES_PER_SIMD once), builds the 4096^2 convolution pyramid over 5 rotated contexts,
times `--launches` launches with HIP events on one stream and checks image 0's checksum against
the product kernel's.  Cases are alternated `--reps` times.  One JSON line per run.
    python3 tools/conv_unroll_ab.py [--reps 2] [--n 4096] [--batch 1]
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
EXP = os.path.join(HERE, "ab", "libgdp_exp.so")

# (rows per block, waves per block, UR, waves per SIMD); UR 0 = the product kernel
CASES = [(48, 16, 0, 8), (48, 16, 3, 8), (48, 16, 3, 4), (32, 8, 2, 6), (32, 8, 0, 8), (24, 8, 3, 6),
         (32, 16, 2, 8), (32, 16, 2, 4)]


def child(rows, waves, launches, n, batch):
    import torch

    sys.path.insert(0, REPO)
    import __graft_entry__ as entry

    pkg = entry.load_package()
    ctxs = [pkg.PyramidContext(n, n, S=2, octaves=5, batch=batch) for _ in range(5)]
    for c in ctxs:
        c.fill_synthetic(0x5EED, 0)
        c.set_tuning(conv_kernel=2, conv_rows=rows, conv_waves=waves, conv_order=4)
    st = torch.cuda.Stream()
    for k in range(10):
        ctxs[k % 5].build_gaussian(st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for k in range(launches):
        ctxs[k % 5].build_gaussian(st)
    e1.record(st)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / launches
    ctxs[0].build_gaussian()
    ctxs[0].sync()
    total = 4 * n * n * batch + ctxs[0].pyramid_bytes()
    print(json.dumps({"ms": round(ms, 5), "frac": round(total / (ms / 1e3) / 8e12, 4), "checksum": f"{ctxs[0].checksum(0):016x}"}))
    for c in ctxs:
        c.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--launches", type=int, default=60)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--child", nargs=2, type=int, default=None)
    a = ap.parse_args()
    if a.child:
        child(a.child[0], a.child[1], a.launches, a.n, a.batch)
        return
    want = None
    for rep in range(a.reps):
        for rows, waves, ur, w in CASES:
            env = dict(os.environ, GDP_LIBRARY=EXP, GDP_CONV_UNROLL=str(ur), GDP_CONV_WAVES_PER_SIMD=str(w))
            r = subprocess.run([sys.executable, __file__, "--child", str(rows), str(waves), "--launches", str(a.launches),
                                "--n", str(a.n), "--batch", str(a.batch)], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            rec = {"rep": rep, "rows": rows, "waves": waves, "unroll": ur, "waves_per_simd": w, "n": a.n,
                   "batch": a.batch}
            if r.returncode != 0 or not line:
                rec["error"] = (r.stderr or r.stdout)[-400:]
                print(json.dumps(rec), flush=True)
                sys.exit(1)
            rec.update(json.loads(line[-1]))
            if (rows, waves, ur) == (48, 16, 0):
                want = want or rec["checksum"]
            rec["same_bits_as_product"] = rec["checksum"] == want
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
