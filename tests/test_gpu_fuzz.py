"""Seeded randomized parity sweep of the HIP build against the oracle — bit-exact, 0 ULP.

Every case draws a shape (1..300 x 1..300), S (0..4), an octave count (default or fewer), a
batch, the input format (int32 / uint8), how the input arrives (host upload, or zero-copy from
a pitched device buffer), a build-kernel variant and tile order, and optionally a row-band
split; the pyramid of every image (or every band, reassembled) must equal the oracle's closed
form (oracle/gdp_oracle.c, pinned to the reference's own outputs by tests/test_oracle.py) word
for word, including signs of zero and subnormals.  The seed is fixed, so a failure names a
reproducible case.
"""
import os

import numpy as np
import pytest
from conftest import BUILD_VARIANTS

pytestmark = pytest.mark.gpu

# GDP_FUZZ_SCALE multiplies every sweep's case count, GDP_FUZZ_SEED offsets its seed and
# GDP_FUZZ_MAXDIM raises the build / subset sweeps' largest side (300), for
# one-off long sweeps on hardware (profiles/fuzz_*.log); the suite runs the defaults
SCALE = max(1, int(os.environ.get("GDP_FUZZ_SCALE", "1")))
SEED = int(os.environ.get("GDP_FUZZ_SEED", "0"))
MAXDIM = max(300, int(os.environ.get("GDP_FUZZ_MAXDIM", "300")))  # shapes 1..MAXDIM (build / subset)
N_CASES = 300 * SCALE
INPLACE_SUBS = (0, 1, 2, 4, 8, 16, -16)


def _progress(name, i):
    if SCALE > 1 and i % 100 == 0:  # long sweeps: a line every 100 cases (visible with -s)
        print(f"{name}: case {i}", flush=True)


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _case(rng):
    H = int(rng.integers(1, MAXDIM + 1))
    W = int(rng.integers(1, MAXDIM + 1))
    S = int(rng.integers(0, 5))
    omax = max(1, int(np.floor(np.log2(min(H, W)))) + 1)
    O = 0 if rng.random() < 0.5 else int(rng.integers(1, omax + 1))
    B = int(rng.integers(1, 4))
    fmt = "u8" if rng.random() < 0.3 else "i32"
    device_input = rng.random() < 0.3
    variant = int(rng.choice(BUILD_VARIANTS))
    order = int(rng.integers(0, 3))
    bands = rng.random() < 0.25 and B == 1 and not device_input
    return H, W, S, O, B, fmt, device_input, variant, order, bands


def _images(rng, H, W, B, fmt):
    if fmt == "u8":
        return [rng.integers(0, 256, size=(H, W), dtype=np.int64).astype(np.uint8) for _ in range(B)]
    # int32 over the whole range now and then (float rounding of the conversion, -0.0 products)
    hi = 2**31 - 1 if rng.random() < 0.2 else 256
    lo = -(2**31) if hi > 256 else 0
    return [rng.integers(lo, hi, size=(H, W), dtype=np.int64).astype(np.int32) for _ in range(B)]


def _follow_up(rng):
    """What runs after the build (whole-image cases): nothing, the GenerateDoG re-entry (in-place,
    random block split) or the GaussFilter pass of a random octave range."""
    r = rng.random()
    kind = "none" if r < 0.6 else "regen" if r < 0.85 else "gauss"
    return kind, int(rng.choice(INPLACE_SUBS)), int(rng.choice(INPLACE_SUBS[1:-1]))  # window: no tiles


def test_randomized_parity_sweep(pkg, oracle):
    """... plus, per case, the window centre (the serial float-halved one or the MPI variants'
    integer-length one) and, on whole images, a follow-up in-place pass checked after it."""
    import torch

    rng = np.random.default_rng(20261016 + SEED)
    for i in range(N_CASES):
        _progress("build", i)
        H, W, S, O, B, fmt, device_input, variant, order, bands = _case(rng)
        centre = "intlen" if rng.random() < 0.3 else "serial"
        follow, isub, wsub = _follow_up(rng)
        if centre == "intlen" and follow == "gauss":
            follow = "regen"  # the oracle's per-octave GaussFilter restates the serial centre only
        imgs = _images(rng, H, W, B, fmt)
        Oeff = O or oracle.default_octaves(H, W)
        wants = [oracle.build_pyramid(img.astype(np.int32), S, Oeff, centre=centre) for img in imgs]
        what = dict(case=i, H=H, W=W, S=S, O=O, B=B, fmt=fmt, device_input=device_input, variant=variant,
                    order=order, bands=bands, centre=centre, follow=follow, isub=isub, wsub=wsub)
        if bands:
            align = 1 << (max(Oeff, 5) - 1)
            cuts = sorted({0, H} | {c for c in range(align, H, align) if rng.random() < 0.5})
            want = oracle.levels(wants[0], H, W, S, Oeff)
            got = {k: np.zeros_like(v) for k, v in want.items()}
            for r0, r1 in zip(cuts[:-1], cuts[1:]):
                with pkg.PyramidContext(H, W, S=S, octaves=O, row_begin=r0, row_end=r1, input_format=fmt) as ctx:
                    ctx.set_tuning(variant=variant, tile_order=order)
                    ctx.set_window_centre(centre)
                    ctx.set_input(imgs[0][r0:r1])
                    ctx.build()
                    for o in range(Oeff):
                        rows, cols, first = ctx.level_dims(o)
                        for s in range(S + 3):
                            if rows:
                                got[(o, s)][first:first + rows] = ctx.level(0, o, s)
            for k in want:
                assert np.array_equal(_bits(got[k]), _bits(want[k])), (what, k)
            continue
        with pkg.PyramidContext(H, W, S=S, octaves=O, batch=B, input_format=fmt) as ctx:
            ctx.set_tuning(variant=variant, tile_order=order, inplace_sub=isub, window_sub=wsub)
            ctx.set_window_centre(centre)
            if device_input:
                pitch = W + int(rng.integers(0, 9))
                host = np.zeros((B, H, pitch), imgs[0].dtype)
                for b in range(B):
                    host[b, :, :W] = imgs[b]
                dev = torch.from_numpy(host).cuda()
                ctx.bind_device_input(dev.data_ptr(), pitch, H * pitch, keepalive=dev)
                ctx.build(torch.cuda.current_stream())
                torch.cuda.synchronize()
            else:
                for b in range(B):
                    ctx.set_input(imgs[b], b)
                ctx.build()
            if follow == "regen":
                ctx.generate_dog()
                for w in wants:
                    oracle.generate_dog(w, H, W, S, Oeff, centre=centre)
            elif follow == "gauss":
                ob = int(rng.integers(0, Oeff))
                oe = int(rng.integers(ob + 1, Oeff + 1))
                ctx.gauss_range(ob, oe)
                for w in wants:
                    for o in range(ob, oe):
                        oracle.gauss_octave(w, H, W, S, o)
                what["octaves"] = (ob, oe)
            for b in range(B):
                got = ctx.pyramid(b)
                assert got.shape == wants[b].shape, what
                bad = np.flatnonzero(_bits(got) != _bits(wants[b]))
                assert bad.size == 0, (what, b, bad[:5])


# ---- GenerateDoG_nomp_dynamic's subset (the AVX-512 x OpenMP header's semantics) ----------------
N_SUBSET_CASES = 120 * SCALE


def test_randomized_subset_sweep(pkg, oracle):
    """gdp_build_subset (+ a re-entry gdp_generate_dog_subset in half the cases) over the same random
    shapes / S / octave counts / batches / formats / variants / tile orders / row bands, against
    the oracle's restatement (pinned to the header run here by tests/test_oracle.py), with the
    header's integer-length window centre."""
    rng = np.random.default_rng(20261017 + SEED)
    for i in range(N_SUBSET_CASES):
        _progress("subset", i)
        H, W, S, O, B, fmt, _, variant, order, bands = _case(rng)
        again = rng.random() < 0.5
        imgs = _images(rng, H, W, B, fmt)
        Oeff = O or oracle.default_octaves(H, W)
        wants = []
        for img in imgs:
            w = oracle.init_pyramid(img.astype(np.int32), S, Oeff)
            for _ in range(2 if again else 1):
                oracle.subset_a512omp(w, H, W, S, Oeff)
            wants.append(w)
        what = dict(case=i, H=H, W=W, S=S, O=O, B=B, fmt=fmt, variant=variant, order=order, bands=bands, again=again)
        if bands:
            align = 1 << (max(Oeff, 5) - 1)
            cuts = sorted({0, H} | {c for c in range(align, H, align) if rng.random() < 0.5})
            want = oracle.levels(wants[0], H, W, S, Oeff)
            got = {k: np.zeros_like(v) for k, v in want.items()}
            for r0, r1 in zip(cuts[:-1], cuts[1:]):
                with pkg.PyramidContext(H, W, S=S, octaves=O, row_begin=r0, row_end=r1, input_format=fmt) as ctx:
                    ctx.set_tuning(variant=variant, tile_order=order)
                    ctx.set_window_centre("intlen")
                    ctx.set_input(imgs[0][r0:r1])
                    ctx.build_subset()
                    if again:
                        ctx.generate_dog_subset()
                    for o in range(Oeff):
                        rows, cols, first = ctx.level_dims(o)
                        for s in range(S + 3):
                            if rows:
                                got[(o, s)][first:first + rows] = ctx.level(0, o, s)
            for k in want:
                assert np.array_equal(_bits(got[k]), _bits(want[k])), (what, k)
            continue
        with pkg.PyramidContext(H, W, S=S, octaves=O, batch=B, input_format=fmt) as ctx:
            ctx.set_tuning(variant=variant, tile_order=order)
            ctx.set_window_centre("intlen")
            for b in range(B):
                ctx.set_input(imgs[b], b)
            ctx.build_subset()
            if again:
                ctx.generate_dog_subset()
            for b in range(B):
                bad = np.flatnonzero(_bits(ctx.pyramid(b)) != _bits(wants[b]))
                assert bad.size == 0, (what, b, bad[:5])


# ---- the convolution extension (no reference counterpart) -------------------------------------
N_CONV_CASES = 120 * SCALE
_CONV_TUNES = [dict(conv_kernel=2, conv_rows=32, conv_order=4), dict(conv_kernel=2, conv_rows=16, conv_order=0),
               dict(conv_kernel=2, conv_rows=48, conv_order=5), dict(conv_kernel=2, conv_rows=24, conv_waves=8, conv_order=1),
               dict(conv_kernel=2, conv_rows=8, conv_waves=8, conv_order=4), dict(conv_kernel=0, conv_rows=16, conv_order=5),
               dict(conv_kernel=0, conv_rows=32, conv_order=2), dict(conv_kernel=1)]


def _conv_ref(pkg, img, S, O):
    """float64 separable convolution with the library's taps, clamp-to-edge (tests/test_gpu_parity.py)."""
    H, W = img.shape
    out = {}
    for o in range(O):
        base = img[:: 1 << o, :: 1 << o][: H >> o, : W >> o].astype(np.float64)
        G = []
        for s in range(S + 3):
            k, R = pkg.conv_taps(S, s)
            k = k.astype(np.float64)
            p = np.pad(base, R, mode="edge")
            h = sum(k[d] * p[:, d:d + base.shape[1]] for d in range(2 * R + 1))
            G.append(sum(k[d] * h[d:d + base.shape[0]] for d in range(2 * R + 1)))
        for s in range(S + 3):
            out[(o, s)] = G[s] - G[s + 1] if s < S + 2 else G[s]
    return out


def test_randomized_convolution_sweep(pkg, oracle):
    """Seeded sweep of the convolution extension: shape 1..400 x 1..400, S 0..4, octave count,
    batch, int32 / uint8, every kernel / rows / waves / order the library has, against a float64
    convolution within the stated tolerance |err| <= 1e-3 + 1e-5 |ref|; and, when the width allows
    (a multiple of 2^(O+1), S <= 5), a random row-band split whose bands — given their halo rows —
    equal the whole image's build bit for bit."""
    import importlib

    import torch

    d = importlib.import_module(pkg.__name__ + ".distributed")
    rng = np.random.default_rng(20261017 + SEED)
    for i in range(N_CONV_CASES):
        _progress("conv", i)
        H = int(rng.integers(1, 401))
        W = int(rng.integers(1, 401)) if rng.random() < 0.6 else int(rng.integers(1, 13)) * 32
        S = int(rng.integers(0, 5))
        omax = max(1, int(np.floor(np.log2(min(H, W)))) + 1)
        O = int(rng.integers(1, min(omax, 6) + 1))
        B = int(rng.integers(1, 3))
        fmt = "u8" if rng.random() < 0.3 else "i32"
        tune = _CONV_TUNES[int(rng.integers(0, len(_CONV_TUNES)))]
        dt = np.uint8 if fmt == "u8" else np.int32
        imgs = [rng.integers(0, 256, size=(H, W), dtype=np.int64).astype(dt) for _ in range(B)]
        what = dict(case=i, H=H, W=W, S=S, O=O, B=B, fmt=fmt, tune=tune)
        with pkg.PyramidContext(H, W, S=S, octaves=O, batch=B, input_format=fmt) as ctx:
            ctx.set_tuning(**tune)
            for b, im in enumerate(imgs):
                ctx.set_input(im, b)
            ctx.build_gaussian()
            ctx.sync()
            whole = {(b, o, s): ctx.level(b, o, s) for b in range(B) for o in range(O) for s in range(S + 3)}
        for b, im in enumerate(imgs):
            for (o, s), ref in _conv_ref(pkg, im.astype(np.int32), S, O).items():
                got = whole[(b, o, s)].astype(np.float64)
                assert got.shape == ref.shape, what
                assert (np.abs(got - ref) - (1e-3 + 1e-5 * np.abs(ref))).max() <= 0, (what, b, o, s)
        align = 1 << (max(O, 5) - 1)
        if S <= 5 and W % (1 << (O + 1)) == 0 and H > 2 * align and rng.random() < 0.6:
            band_tune = dict(conv_kernel=2, conv_rows=tune.get("conv_rows", 32) if tune.get("conv_kernel") == 2 else 32,
                             conv_waves=tune.get("conv_waves", 16))
            if tune.get("conv_kernel") != 2:  # bands run the block tiles: compare with the same kernel's whole image
                with pkg.PyramidContext(H, W, S=S, octaves=O, batch=B, input_format=fmt) as ctx:
                    ctx.set_tuning(**band_tune)
                    for b, im in enumerate(imgs):
                        ctx.set_input(im, b)
                    ctx.build_gaussian()
                    ctx.sync()
                    whole = {(b, o, s): ctx.level(b, o, s) for b in range(B) for o in range(O) for s in range(S + 3)}
            nb = int(rng.integers(2, max(3, H // align) + 1))
            for r in range(nb):
                r0, r1 = d.plan_band(H, nb, r, O)
                if r1 <= r0:
                    continue
                try:
                    plan_ok = True
                    d.halo_plan(H, nb, r, O)
                except ValueError:
                    plan_ok = False  # bands thinner than the halo: a band context still works locally
                with pkg.PyramidContext(H, W, S=S, octaves=O, batch=B, row_begin=r0, row_end=r1, input_format=fmt) as bc:
                    bc.set_tuning(**band_tune)
                    for b, im in enumerate(imgs):
                        bc.set_input(np.ascontiguousarray(im[r0:r1]), b)
                    above, below = bc.conv_halo_rows()
                    rows = max(above, below, 1)
                    halo = [np.zeros((B, rows, W), dtype=dt) for _ in range(2)]
                    for b, im in enumerate(imgs):
                        halo[0][b, :above] = im[r0 - above:r0]
                        halo[1][b, :below] = im[r1:r1 + below]
                    dev = [torch.from_numpy(h).cuda() for h in halo]
                    bc.bind_input_halo(dev[0].data_ptr() if above else None, dev[1].data_ptr() if below else None,
                                       pitch=W, image_stride=rows * W, keepalive=dev)
                    bc.build_gaussian()
                    bc.sync()
                    for b in range(B):
                        for o in range(O):
                            n, _, first = bc.level_dims(o)
                            for s in range(S + 3):
                                assert np.array_equal(_bits(bc.level(b, o, s)), _bits(whole[(b, o, s)][first:first + n])), \
                                    (what, "band", r, nb, plan_ok, b, o, s)
