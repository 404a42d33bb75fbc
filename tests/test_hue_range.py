"""The hue kernel's index arithmetic rests on a range fact about OpenCV's RGB2HSV_b over all 2^24
BGR triples (tools/hue_range.py): h before the +180 wrap lies in [-30, 150]."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools"))
import hue_range  # noqa: E402


def test_hue_h12_range():
    lo, hi = hue_range.check()
    assert -180 < lo and hi < 180 and (lo, hi) == (-30, 150)
