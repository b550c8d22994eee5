"""CPU test of the unit-timeline analysis (bench/unit_timeline.py) on a synthetic trace: the
same numbers the GPU probe's rows feed it (start, end, HW_ID | XCC_ID << 32, row << 32 | seg)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "bench"))
from unit_timeline import analyse  # noqa: E402


def _row(t0, t1, xcc, cu, row, seg):
    return [t0, t1, (cu << 8) | (xcc << 32), (row << 32) | seg]


def test_timeline_balanced_and_skewed_xcds():
    S = 10
    # 2 XCDs x 2 CUs x 2 slots = 8 slots; every slot runs 3 shell units of 100 ticks
    rows = []
    for x in range(2):
        for cu in range(2):
            for slot in range(2):
                for k in range(3):
                    rows.append(_row(1 + 100 * k, 1 + 100 * (k + 1), x, cu, slot, k))
    r = analyse(np.array(rows, dtype=np.uint64), S)
    assert r["units"] == 24 and r["cus_seen"] == 4 and r["slots"] == 8
    assert r["busy_frac"] == 1.0 and r["n_diag"] == 0
    assert r["xcd_end_ms"] == {0: 0.003, 1: 0.003}
    # XCD 1 runs 20 % slower: it sets the end, the launch is no longer packed
    slow = [[a, 1 + (b - 1) * 1.2 if (c >> 32) == 1 else b, c, d] for a, b, c, d in rows]
    slow = [[a if (c >> 32) == 0 else 1 + (a - 1) * 1.2, b, c, d] for a, b, c, d in slow]
    r2 = analyse(np.array(slow, dtype=np.uint64), S)
    assert r2["xcd_end_ms"][1] > r2["xcd_end_ms"][0]
    assert r2["busy_frac"] < 0.95
    assert r2["tail_ms"] > 0


def test_timeline_diag_units_and_empty_slots():
    S = 4
    rows = [_row(1, 101, 0, 0, 0, 0), _row(1, 51, 0, 0, 0, S), [0, 0, 0, 0]]  # last: no unit
    r = analyse(np.array(rows, dtype=np.uint64), S)
    assert r["units"] == 2 and r["n_shell"] == 1 and r["n_diag"] == 1
    assert r["diag_ms"] == 0.0005 and r["shell_ms"] == 0.001
    assert analyse(np.zeros((3, 4), dtype=np.uint64), S) == {"units": 0}
