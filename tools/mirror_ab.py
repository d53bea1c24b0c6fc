#!/usr/bin/env python3
"""A/B of the drop-in class's mirrored GenerateDoG on one box (round 5):
serial upload + in-place pass + download (gdp_upload_image_raw, gdp_generate_dog,
gdp_download_image_raw) against the pipelined gdp_generate_dog_mirrored, alternated, on a pinned
device-layout host image; plus whether PCIe copies in the two directions overlap at all (torch:
447 MB host->device on one stream while 447 MB device->host runs on another).
    python3 tools/mirror_ab.py [n]
"""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch

    import __graft_entry__ as entry

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    pkg = entry.load_package()
    L = pkg.lib()
    ctx = pkg.PyramidContext(n, n, S=2, octaves=pkg.octaves_for(n))
    ctx.fill_synthetic(0x5EED, 0)
    ctx.build()
    ctx.sync()
    floats = L.gdp_image_floats(ctx._ctx)
    hp = ctypes.c_void_p()
    assert L.gdp_host_alloc(floats * 4, ctypes.byref(hp)) == 0
    assert L.gdp_download_image_raw(ctx._ctx, 0, hp) == 0
    res = {"n": n, "bytes_each_way": floats * 4, "serial_ms": [], "pipelined_ms": []}
    for rep in range(6):
        for mode in ("serial", "pipelined"):
            t = time.perf_counter()
            if mode == "serial":
                assert L.gdp_upload_image_raw(ctx._ctx, 0, hp) == 0
                assert L.gdp_generate_dog(ctx._ctx, None) == 0
                assert L.gdp_download_image_raw(ctx._ctx, 0, hp) == 0
            else:
                assert L.gdp_generate_dog_mirrored(ctx._ctx, 0, hp) == 0
            res[mode + "_ms"].append(round((time.perf_counter() - t) * 1e3, 3))
    L.gdp_host_free(hp)
    ctx.close()
    # duplex probe
    m = floats
    d1 = torch.empty(m, dtype=torch.float32, device="cuda")
    d2 = torch.ones(m, dtype=torch.float32, device="cuda")
    h1 = torch.ones(m, dtype=torch.float32).pin_memory()
    h2 = torch.empty(m, dtype=torch.float32).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        d1.copy_(h1, non_blocking=True)
        torch.cuda.synchronize()
        up = time.perf_counter() - t
        t = time.perf_counter()
        h2.copy_(d2, non_blocking=True)
        torch.cuda.synchronize()
        down = time.perf_counter() - t
        t = time.perf_counter()
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
        torch.cuda.synchronize()
        both = time.perf_counter() - t
        res.setdefault("duplex", []).append({"up_ms": round(up * 1e3, 2), "down_ms": round(down * 1e3, 2),
                                             "both_concurrent_ms": round(both * 1e3, 2)})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
