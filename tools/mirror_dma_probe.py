#!/usr/bin/env python3
"""DMA rate of the drop-in mirror's host memory (round 6): one 4096^2 pyramid image (447 MB) copied
device -> host and host -> device through libgdp's raw copies (gdp_download_image_raw /
gdp_upload_image_raw), into (a) hipHostMalloc memory (gdp_host_alloc, round 5's mirror) and (b) the
registered view of gdp_host_alloc_tracked memory (round 6's mirror; addressed through its CPU
view, as the drop-in classes do), alternated, `--reps` times each.  One JSON line per measurement.
    python3 tools/mirror_dma_probe.py [--reps 5] [--n 4096]
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--n", type=int, default=4096)
    a = ap.parse_args()
    import __graft_entry__ as entry

    pkg = entry.load_package()
    L = pkg.lib()
    with pkg.PyramidContext(a.n, a.n, S=2) as ctx:
        ctx.fill_synthetic(0x5EED, 0)
        ctx.build()
        ctx.sync()
        nbytes = L.gdp_image_floats(ctx._ctx) * 4
        bufs = {}
        p = ctypes.c_void_p()
        assert L.gdp_host_alloc(nbytes, ctypes.byref(p)) == 0
        bufs["hipHostMalloc"] = ctypes.c_void_p(p.value)
        q = ctypes.c_void_p()
        rc = L.gdp_host_alloc_tracked(nbytes, ctypes.byref(q))
        if rc == 0:
            bufs["tracked_alias"] = ctypes.c_void_p(q.value)
            assert L.gdp_host_untrack(bufs["tracked_alias"]) == 0  # DMA rate only: no protection
        thp = {}
        for k in ("enabled", "shmem_enabled", "defrag"):
            try:
                thp[k] = open(f"/sys/kernel/mm/transparent_hugepage/{k}").read().strip()
            except OSError:
                thp[k] = None
        # how the mappings of the two host buffers are backed (huge pages or not)
        maps = {}
        cur = None
        for line in open("/proc/self/smaps"):
            if "-" in line.split(" ")[0] and len(line.split(" ")[0].split("-")) == 2 and \
                    all(c in "0123456789abcdef-" for c in line.split(" ")[0]):
                lo, hi = (int(x, 16) for x in line.split(" ")[0].split("-"))
                cur = None
                for name, ptr in bufs.items():
                    if lo <= ptr.value < hi:
                        cur = name
                        maps[cur] = {"vma": line.strip()[:120]}
            elif cur and line.split(":")[0] in ("Size", "Rss", "AnonHugePages", "ShmemPmdMapped", "FilePmdMapped",
                                                 "KernelPageSize", "MMUPageSize"):
                maps[cur][line.split(":")[0]] = line.split(":")[1].strip()
        huge = {}
        for line in open("/proc/meminfo"):
            if line.startswith(("HugePages_", "Hugepagesize", "ShmemHugePages")):
                huge[line.split(":")[0]] = line.split(":")[1].strip()
        print(json.dumps({"thp": thp, "hugetlb": huge, "mappings": maps}), flush=True)
        try:
            for rep in range(a.reps):
                for name, ptr in bufs.items():
                    for direction, fn in (("d2h", L.gdp_download_image_raw), ("h2d", L.gdp_upload_image_raw)):
                        t = time.perf_counter()
                        assert fn(ctx._ctx, 0, ptr) == 0
                        dt = time.perf_counter() - t
                        print(json.dumps({"rep": rep, "memory": name, "dir": direction, "ms": round(dt * 1e3, 3),
                                          "GBps": round(nbytes / dt / 1e9, 1), "bytes": nbytes}), flush=True)
        finally:
            for ptr in bufs.values():
                L.gdp_host_free(ptr)


if __name__ == "__main__":
    main()
