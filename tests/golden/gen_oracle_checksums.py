#!/usr/bin/env python3
"""gdp_checksum fixtures for bench inputs the reference cannot run (non-square images).

The reference (GuassDePyramid.h) only builds square len x len pyramids, so config 3's 1080 x 1920
input has no reference output.  Its fixture comes from the oracle's closed form (oracle/, test
infrastructure), which tests/test_oracle.py pins bit-exact to the reference on every square
fixture; the non-square extension (column windows from W, row windows from H) is
the same code path with H != W.  Writes tests/golden/checksums_oracle.json.

    python tests/golden/gen_oracle_checksums.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import oracle  # noqa: E402

SEED = 0x5EED
# (H, W, S, O, image index) — bench config 3: images 0 and 1, and the first and last image of every
# rank at 64 images per GPU on up to 8 GPUs (bench.py verifies every rank's shard)
CASES = [(1080, 1920, 2, 5, i) for i in sorted({0, 1} | {x for r in range(8) for x in (64 * r, 64 * r + 63)})]


def main():
    out = []
    for H, W, S, O, idx in CASES:
        img = oracle.synthetic_image(H, W, SEED, idx)
        pyr = oracle.build_pyramid(img, S, O)
        out.append({"H": H, "W": W, "S": S, "octaves": O, "input": f"synth:{SEED:#x}:{idx}",
                    "checksum": f"{oracle.pyramid_checksum(pyr, H, W, S, O):016x}",
                    "source": "oracle closed form (non-square: no reference output exists)"})
        print(out[-1], flush=True)
    with open(os.path.join(HERE, "checksums_oracle.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
