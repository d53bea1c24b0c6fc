"""Single-image builds from independent callers: does running them on separate HIP streams hide
the per-launch ramp + drain (~10 us of a 0.084 ms cold 4096^2 launch)?

    python tools/overlap_bench.py [--n 4096] [--sets 6] [--iters 300] [--streams 1,2,3,6]

`--sets` contexts of one image each (cold: their pyramids together exceed the 256 MB MALL),
built round-robin; with s streams, context i launches on stream i % s.  Prints ms per image and
the algorithmic HBM rate (4 B/input px + 4 (S+3) B/pyramid px) for each stream count, and checks
that every context's checksum is unchanged.  A diagnostic: bench.py's `value` stays one stream."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--sets", type=int, default=6)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--streams", default="1,2,3,6")
    a = ap.parse_args()
    ctxs = [pkg.PyramidContext(a.n, a.n, S=2, octaves=5) for _ in range(a.sets)]
    for i, c in enumerate(ctxs):
        c.fill_synthetic(0x5EED, i)
        c.build()
        c.sync()
    sums = [c.checksum(0) for c in ctxs]
    nbytes = 4 * a.n * a.n + ctxs[0].pyramid_bytes()
    for ns in (int(x) for x in a.streams.split(",")):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        for it in range(2):  # warm-up pass, then the timed pass
            iters = a.iters if it else a.sets * 2
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(iters):
                ctxs[k % a.sets].build(streams[(k % a.sets) % ns])
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        ok = all(c.checksum(0) == s for c, s in zip(ctxs, sums))
        ms = 1e3 * dt / a.iters
        print(json.dumps({"n": a.n, "streams": ns, "sets": a.sets, "ms_per_image": round(ms, 5),
                          "GB/s": round(nbytes / ms / 1e6, 1), "frac_8TBps": round(nbytes / ms / 8e9, 4),
                          "checksums_unchanged": ok}), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
