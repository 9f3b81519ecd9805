"""CPU check of the threshold algebra behind the chip-wide draws
(csrc/draws.h, tools/proto_thresholds.py): inside one mask region a 64-word
chunk of numpy's masked-rejection draws is exactly 64 thresholds plus a crossing
table, for every entering step.  Compared with the plain serial walk."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import proto_thresholds as pt  # noqa: E402


def test_chunk_thresholds_match_serial_walk():
    for b in (2, 3, 6, 8, 10):
        for seed in range(2):
            bad, n = pt.check(seed * 31 + b, b)
            assert bad == 0, f"mask {(1 << b) - 1}: {bad} of {n} entering steps differ"
