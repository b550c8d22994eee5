"""Host-side geometry of the Newton-3 sym schedule (csrc/common/layout.cpp), CPU only.

The reference's CUDA kernel visits each pair once (j > i, cuda.cu:53-60) and scatters both
sides; the sym schedule does the same at chunk granularity: row A pairs with the next h(A)
chunks cyclically. These tests pin that every unordered chunk pair is covered exactly once
(with the parity split of the antipodal pairs), that ranks get equal work, and that the gated
launch's unit map (local units first) is a permutation with correct locality flags.
"""
import ctypes

import numpy as np
import pytest

from gravsim.ops import _native


def _geo(n_pad):
    lib = _native.cpu_lib()
    v = [ctypes.c_int32() for _ in range(5)]
    assert lib.gs_sym_geometry(n_pad, *[ctypes.byref(x) for x in v]) == 0
    return lib, dict(zip(("NC", "H", "L", "S", "D"), (x.value for x in v)))


@pytest.mark.parametrize("NC", [8, 32, 64, 512, 2048])
@pytest.mark.parametrize("parity", [0, 1])
def test_every_chunk_pair_exactly_once(NC, parity):
    lib = _native.cpu_lib()
    h = np.array([lib.gs_sym_shell_len(A, NC, parity) for A in range(NC)])
    assert set(h.tolist()) <= {NC // 2, NC // 2 - 1}
    A = np.repeat(np.arange(NC), NC // 2)
    d = np.tile(np.arange(1, NC // 2 + 1), NC)
    keep = d <= h[A]
    A, B = A[keep], (A[keep] + d[keep]) % NC
    cover = np.zeros((NC, NC), dtype=np.int32)
    np.add.at(cover, (np.minimum(A, B), np.maximum(A, B)), 1)
    assert (cover[np.triu_indices(NC, k=1)] == 1).all()
    assert cover.sum() == NC * (NC - 1) // 2


@pytest.mark.parametrize("P", [2, 4, 8])
def test_parity_balances_ranks(P):
    lib = _native.cpu_lib()
    NC = 512
    rows = NC // P
    work = [sum(lib.gs_sym_shell_len(A, NC, 1) for A in range(r * rows, (r + 1) * rows))
            for r in range(P)]
    assert max(work) - min(work) == 0
    old = [sum(lib.gs_sym_shell_len(A, NC, 0) for A in range(r * rows, (r + 1) * rows))
           for r in range(P)]
    assert max(old) - min(old) == rows  # round 1: the first half of the ranks held long rows


@pytest.mark.parametrize("n_pad,P", [(65536, 8), (262144, 4), (1 << 20, 8), (1 << 20, 2)])
@pytest.mark.parametrize("fill", [-1, 1024, 0])
def test_unit_map_permutation_and_locality(n_pad, P, fill):
    lib, g = _geo(n_pad)
    NC, L, S, D = g["NC"], g["L"], g["S"], g["D"]
    rows = NC // P
    for rank in (0, P - 1):
        out = (ctypes.c_int32 * (rows * (S + D)))()
        n = lib.gs_sym_unit_map(n_pad, rank, P, 1, fill, out, len(out))
        assert n == rows * (S + D)
        m = np.frombuffer(out, dtype=np.uint32)
        remote = (m >> 31).astype(bool)
        row = (m >> 16) & 0x7FFF
        unit = m & 0xFFFF
        key = row.astype(np.int64) * (S + D) + unit
        assert np.array_equal(np.sort(key), np.arange(rows * (S + D)))  # a permutation
        a0 = rank * rows
        A = a0 + row.astype(np.int64)
        u = unit.astype(np.int64)
        h = np.array([lib.gs_sym_shell_len(int(x), NC, 1) for x in range(NC)])[A]
        diag = u >= S
        assert not remote[diag].any()  # diagonal parts read only the own rows
        past = ~diag & (u * L >= 16 * h)  # past the row's shell: reads nothing
        seg = ~diag & ~past
        last_q = np.minimum((u + 1) * L, 16 * h)  # the segment's last quantum
        local = A + 1 + (last_q - 1) // 16 < a0 + rows
        assert np.array_equal(remote[seg], ~local[seg])
        if fill != 0:
            first = min(fill if fill > 0 else n, int((~remote).sum()))
            assert not remote[:first].any()  # local units lead the dispatch order


@pytest.mark.parametrize("n_pad,P", [(65536, 8), (262144, 4), (1 << 20, 8), (1 << 20, 2),
                                     (1 << 24, 8)])
@pytest.mark.parametrize("fill", [-1, 1024, 0])
def test_ring_unit_map_stages(n_pad, P, fill):
    """Ring strategy of the sym schedule: the slice of rank (r - k) mod P lands at stage k.
    Every unit carries the stage of the last slice it reads (0: own rows only), units are a
    permutation, the local prefix comes first and the rest is ordered by stage."""
    lib, g = _geo(n_pad)
    NC, L, S, D = g["NC"], g["L"], g["S"], g["D"]
    rows = NC // P
    for rank in (0, P - 1):
        out = (ctypes.c_int32 * (rows * (S + D)))()
        n = lib.gs_sym_unit_map_ring(n_pad, rank, P, 1, fill, out, len(out))
        assert n == rows * (S + D)
        m = np.frombuffer(out, dtype=np.uint32)
        remote = (m >> 31).astype(bool)
        stage = ((m >> 28) & 7).astype(np.int64)
        row = ((m >> 16) & 0xFFF).astype(np.int64)
        unit = (m & 0xFFFF).astype(np.int64)
        key = row * (S + D) + unit
        assert np.array_equal(np.sort(key), np.arange(rows * (S + D)))
        assert np.array_equal(remote, stage > 0)
        A = rank * rows + row
        h = np.array([lib.gs_sym_shell_len(int(x), NC, 1) for x in range(NC)])[A]
        want = np.zeros(len(m), dtype=np.int64)
        for i in np.nonzero((unit < S) & (unit * L < 16 * h))[0]:
            q0, q1 = unit[i] * L, (unit[i] + 1) * L - 1
            for d in range(1 + q0 // 16, 2 + q1 // 16):
                owner = ((A[i] + d) % NC) // rows
                want[i] = max(want[i], (rank - owner) % P)
        assert np.array_equal(stage, want)
        local_prefix = int(np.argmax(stage > 0)) if (stage > 0).any() else len(stage)
        assert (np.diff(stage[local_prefix:]) >= 0).all()  # stage order after the prefix
        if fill != 0:
            assert not remote[:min(fill if fill > 0 else n, int((~remote).sum()))].any()
    # too many rows for the 12-bit row field: no gated ring map (the launch stays ungated)
    big = 1 << 25
    assert lib.gs_sym_unit_map_ring(big, 0, 1, 1, -1, None, 0) == 0
