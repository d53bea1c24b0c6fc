"""Seeded randomized parity sweep of the HIP build against the oracle — bit-exact, 0 ULP.

Every case draws a shape (1..300 x 1..300), S (0..4), an octave count (default or fewer), a
batch, the input format (int32 / uint8), how the input arrives (host upload, or zero-copy from
a pitched device buffer), a build-kernel variant and tile order, and optionally a row-band
split; the pyramid of every image (or every band, reassembled) must equal the oracle's closed
form (oracle/gdp_oracle.c, pinned to the reference's own outputs by tests/test_oracle.py) word
for word, including signs of zero and subnormals.  The seed is fixed, so a failure names a
reproducible case.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N_CASES = 300


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def _case(rng):
    H = int(rng.integers(1, 301))
    W = int(rng.integers(1, 301))
    S = int(rng.integers(0, 5))
    omax = max(1, int(np.floor(np.log2(min(H, W)))) + 1)
    O = 0 if rng.random() < 0.5 else int(rng.integers(1, omax + 1))
    B = int(rng.integers(1, 4))
    fmt = "u8" if rng.random() < 0.3 else "i32"
    device_input = rng.random() < 0.3
    variant = int(rng.integers(0, 19))
    order = int(rng.integers(0, 2))
    bands = rng.random() < 0.25 and B == 1 and not device_input
    return H, W, S, O, B, fmt, device_input, variant, order, bands


def _images(rng, H, W, B, fmt):
    if fmt == "u8":
        return [rng.integers(0, 256, size=(H, W), dtype=np.int64).astype(np.uint8) for _ in range(B)]
    # int32 over the whole range now and then (float rounding of the conversion, -0.0 products)
    hi = 2**31 - 1 if rng.random() < 0.2 else 256
    lo = -(2**31) if hi > 256 else 0
    return [rng.integers(lo, hi, size=(H, W), dtype=np.int64).astype(np.int32) for _ in range(B)]


def test_randomized_parity_sweep(pkg, oracle):
    import torch

    rng = np.random.default_rng(20261016)
    for i in range(N_CASES):
        H, W, S, O, B, fmt, device_input, variant, order, bands = _case(rng)
        imgs = _images(rng, H, W, B, fmt)
        Oeff = O or oracle.default_octaves(H, W)
        wants = [oracle.build_pyramid(img.astype(np.int32), S, Oeff) for img in imgs]
        what = dict(case=i, H=H, W=W, S=S, O=O, B=B, fmt=fmt, device_input=device_input, variant=variant,
                    order=order, bands=bands)
        if bands:
            align = 1 << (max(Oeff, 5) - 1)
            cuts = sorted({0, H} | {c for c in range(align, H, align) if rng.random() < 0.5})
            want = oracle.levels(wants[0], H, W, S, Oeff)
            got = {k: np.zeros_like(v) for k, v in want.items()}
            for r0, r1 in zip(cuts[:-1], cuts[1:]):
                with pkg.PyramidContext(H, W, S=S, octaves=O, row_begin=r0, row_end=r1, input_format=fmt) as ctx:
                    ctx.set_tuning(variant=variant, tile_order=order)
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
            ctx.set_tuning(variant=variant, tile_order=order)
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
            for b in range(B):
                got = ctx.pyramid(b)
                assert got.shape == wants[b].shape, what
                bad = np.flatnonzero(_bits(got) != _bits(wants[b]))
                assert bad.size == 0, (what, b, bad[:5])
