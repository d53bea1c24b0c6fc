"""bench.py's roofline accounting, pinned to SURVEY.md §8(d)'s table of algorithmic bytes
(B = 4·H·W + 4·(S+3)·P per image, P = Σ_o H_o·W_o) and its per-config pyramid sizes."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


@pytest.mark.parametrize("H,W,O,P,B", [
    (512, 512, 4, 348_160, 8_011_776),             # config 1
    (4096, 4096, 5, 22_347_776, 514_064_384),      # config 2 (and 4, per image)
    (1080, 1920, 5, 2_762_040, 63_535_200),        # config 3, per image
    (16384, 16384, 5, 357_564_416, 8_225_030_144),  # config 5
])
def test_algorithmic_bytes_match_survey_table(H, W, O, P, B):
    assert bench.pyramid_pixels(H, W, O) == P
    assert bench.algorithmic_bytes(H, W, 2, O, 1) == B


def test_batch_and_uint8_accounting():
    one = bench.algorithmic_bytes(1080, 1920, 2, 5, 1)
    assert bench.algorithmic_bytes(1080, 1920, 2, 5, 64) == 64 * one == 4_066_252_800
    # uint8 input: a quarter of the input bytes, the same pyramid bytes
    assert bench.algorithmic_bytes(4096, 4096, 2, 5, 1, in_bytes=1) == 514_064_384 - 3 * 4096 * 4096


def test_configs_are_the_baseline_workloads():
    c = bench.CONFIGS
    assert (c["c2"]["H"], c["c2"]["W"], c["c2"]["batch"], c["c2"]["O"]) == (4096, 4096, 1, 5)
    assert (c["c3"]["H"], c["c3"]["W"], c["c3"]["batch"]) == (1080, 1920, 64)
    assert (c["c4"]["H"], c["c4"]["batch"]) == (4096, 64)
    assert c["c5"]["H"] == 16384 and c["c5"]["band"]


def test_rotation_exceeds_the_infinity_cache():
    # config 2's per-step working set (514 MB) is rotated over enough sets to exceed 2 GiB (8x MALL)
    set_bytes = bench.algorithmic_bytes(4096, 4096, 2, 5, 1)
    rotate = max(1, -(-bench.ROTATE_BYTES // set_bytes))
    assert rotate == 5 and rotate * set_bytes >= 8 * (256 << 20)
