#!/usr/bin/env python3
"""Interleaved A/B of build-kernel tunings in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python tools/tune.py [--config c2] [--iters 50] [--rounds 7]

Every variant builds the same resident synthetic batch; each round times every variant once
(HIP events around `iters` back-to-back launches on the context stream); prints per-variant
median / min per-launch ms and the algorithmic-byte rate, one JSON line per variant.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
import __graft_entry__ as entry  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--op", default="build", choices=["build", "regen", "gauss", "conv", "subset"],
                    help="default op; a variant may override it with op=... (e.g. 'v=15;v=15,op=subset')")
    ap.add_argument("--variants", default="v=0;v=8;v=11;v=15;v=16;v=17;v=18;v=20;v=23;v=27;v=15,nt=0")
    ap.add_argument("--no-check", action="store_true", help="skip the same-output check (timing experiments)")
    ap.add_argument("--S", type=int, default=2, help="scales parameter S (S + 3 levels per octave)")
    ap.add_argument("--shape", default=None, help="HxWxBATCH overriding the config's shape (O stays 5)")
    ap.add_argument("--octaves", type=int, default=None, help="octave count overriding the config's")
    ap.add_argument("--checksums", action="store_true",
                    help="print gdp_checksum of image 0 after each variant's warm-up build (A/B of library builds: "
                         "compare across GDP_LIBRARY runs)")
    ap.add_argument("--rotate", type=int, default=1,
                    help="buffer sets the timed launches cycle through (bench.py's cold-cache steps)")
    args = ap.parse_args()
    pkg = entry.load_package()
    cfg = bench.CONFIGS[args.config]
    H, W, O, B = cfg["H"], cfg["W"], cfg["O"], cfg["batch"]
    if args.shape:
        H, W, B = (int(x) for x in args.shape.split("x"))
    if args.octaves:
        O = args.octaves
    ctxs = [pkg.PyramidContext(H, W, S=args.S, octaves=O, batch=B) for _ in range(args.rotate)]
    for c in ctxs:
        c.fill_synthetic(bench.SEED, 0)
        c.sync()
    ctx = ctxs[0]
    refs = {}
    base_conv_order = ctx.tuning()["conv_order"]  # the library's geometry-dependent default
    variants = []
    for v in args.variants.split(";"):
        kv = dict(p.split("=") for p in v.split(","))
        variants.append((v, {"nontemporal": int(kv.get("nt", 1)), "grid": int(kv.get("grid", "0"), 0),
                             "variant": int(kv.get("v", -1)) if "v" in kv else None,
                             "tile_order": int(kv.get("ord", 0)), "inplace_sub": int(kv.get("sub", 1)), "window_sub": int(kv.get("wsub", 4)),
                             "conv_kernel": int(kv.get("ck", 0)), "conv_rows": int(kv.get("cr", 16)),
                             "conv_order": int(kv.get("co", base_conv_order)), "conv_waves": int(kv.get("cw", 16)), "build_lds": int(kv.get("lds", 0))}))
        variants[-1][1]["op"] = kv.get("op", args.op)
        if variants[-1][1]["variant"] is None:
            del variants[-1][1]["variant"]
        variants[-1][1]["zero_window"] = int(kv.get("zw", 0))  # every variant sets it (apply() keeps state)
        variants[-1][1]["store_pace"] = int(kv.get("sp", -1))
        variants[-1][1]["conv_pace"] = int(kv.get("cp", 2))
        if "bpc" in kv:
            variants[-1][1]["blocks_per_cu"] = int(kv["bpc"])
        if "ip" in kv or "is" in kv:  # timing-only: read a caller buffer with this input pitch / image stride
            ip = int(kv.get("ip", W))
            variants[-1][1]["in_layout"] = (ip, int(kv.get("is", H * ip)))
    times = {name: [] for name, _ in variants}

    padded = {}

    def apply(kw):  # fresh context state per variant: persistent only when bpc is given
        for i, c in enumerate(ctxs):
            c.set_tuning(**{k: v for k, v in kw.items() if k not in ("blocks_per_cu", "op", "in_layout")})
            c.set_tuning(blocks_per_cu=kw.get("blocks_per_cu", 0))
            if "in_layout" in kw:  # random pixels in a padded layout (timing only: needs --no-check)
                import torch
                ip, istride = kw["in_layout"]
                key = (i, ip, istride)
                if key not in padded:
                    padded[key] = torch.randint(0, 256, (B * istride + 64,), dtype=torch.int32, device="cuda")
                c.bind_device_input(padded[key].data_ptr(), ip, istride, keepalive=padded[key])
            elif c._bound is not None:
                c.unbind_device_input()

    for name, kw in variants:  # warm-up + identical-output check for every variant (per op)
        apply(kw)
        {"conv": ctx.build_gaussian, "subset": ctx.build_subset}.get(kw["op"], ctx.build)()
        if kw["op"] == "regen":  # the checksum below is then the re-entry's (GenerateDoG on the build)
            ctx.generate_dog()
        ctx.sync()
        if args.checksums:
            print(json.dumps({"variant": name, "shape": [H, W, B], "checksum0": f"{ctx.checksum(0):016x}"}), flush=True)
        lev = ctx.level(0, 0, 0)
        ref = refs.setdefault(kw["op"], lev)
        if args.no_check:
            pass
        elif kw["op"] == "conv":  # the two convolution kernels round differently (no parity contract)
            assert np.allclose(lev, ref, rtol=1e-5, atol=1e-3), name
        else:
            assert np.array_equal(lev.view(np.uint32), ref.view(np.uint32)), name
    import torch

    stream = torch.cuda.Stream()
    def steps_of(op):
        return [{"build": c.build, "regen": c.generate_dog, "gauss": lambda st, c=c: c.gauss_range(0, O, st),
                 "conv": c.build_gaussian, "subset": c.build_subset}[op] for c in ctxs]

    if any(kw["op"] in ("regen", "gauss") for _, kw in variants):
        for c in ctxs:
            c.build(stream)
    for _ in range(args.rounds):
        for name, kw in variants:
            apply(kw)
            steps = steps_of(kw["op"])
            if kw["op"] == "build" and args.rotate == 1:
                times[name].append(ctx.time_builds(args.iters) / args.iters)
            else:
                for st in steps:
                    st(stream)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for i in range(args.iters):
                    steps[i % len(steps)](stream)
                e1.record(stream)
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / args.iters)
    if args.op in ("build", "conv", "subset"):
        nbytes = bench.algorithmic_bytes(H, W, args.S, O, B)
    else:
        nbytes = 8 * (args.S + 3) * B * sum((H >> o) * (W >> o) for o in range(O))
    for name, _ in variants:
        t = np.array(times[name])
        print(json.dumps({"variant": name, "config": args.config, "shape": [H, W, B], "ms_median": round(float(np.median(t)), 5),
                          "ms_min": round(float(t.min()), 5),
                          "GBps_median": round(nbytes / (np.median(t) / 1e3) / 1e9, 1)}), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
