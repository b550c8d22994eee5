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


def test_kernel_gaps_period_and_graph_boundaries(tmp_path):
    """scripts/kernel_gaps.py on a synthetic kernel trace: force 100 us, tail 10 us, no gap
    inside a graph, 14 us at every graph launch of two-step periods (r6_kernel_gaps_65k.txt)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "scripts"))
    import kernel_gaps

    rows, t = [], 0
    for step in range(8):
        rows.append((t, t + 100_000, "force_sym_kernel_f32"))
        rows.append((t + 100_000, t + 110_000, "sym_tail_kernel"))
        t += 110_000 + (14_000 if step % 2 == 1 else 0)  # (ns) graph launch after odd steps
    p = tmp_path / "kt_kernel_trace.csv"
    p.write_text("Kernel_Name,Start_Timestamp,End_Timestamp\n"
                 + "".join(f"{n},{s},{e}\n" for s, e, n in rows))
    r = kernel_gaps.summarise(kernel_gaps.load(str(p), ["force_sym", "sym_tail"]))
    assert r["kernels"] == 16 and r["force_us"] == 100.0 and r["tail_us"] == 10.0
    assert r["gap_force_tail_us"] == 0.0
    assert sorted([r["gap_tail_force_even_us"], r["gap_tail_force_odd_us"]]) == [0.0, 14.0]
    assert r["gaps_over_5us"] == 3  # (7 tail -> force gaps, 3 of them at a graph launch)
    assert r["idle_between_kernels_us_per_step"] == round(3 * 14.0 / 8, 2)
