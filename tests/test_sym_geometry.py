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
from gravsim.parallel import partition


def _geo(n_pad):
    lib = _native.cpu_lib()
    v = [ctypes.c_int32() for _ in range(5)]
    assert lib.gs_sym_geometry(n_pad, *[ctypes.byref(x) for x in v]) == 0
    return lib, dict(zip(("NC", "H", "L", "S", "D"), (x.value for x in v)))


def _round1_shell_len(A, NC):
    """Round 1's rule (rows A < NC/2 take every antipodal pair), for the balance check."""
    return NC // 2 if A < NC // 2 else NC // 2 - 1


@pytest.mark.parametrize("NC", [8, 32, 64, 512, 2048])
@pytest.mark.parametrize("rule", ["parity", "round1"])
def test_every_chunk_pair_exactly_once(NC, rule):
    lib = _native.cpu_lib()
    f = lib.gs_sym_shell_len if rule == "parity" else _round1_shell_len
    h = np.array([f(A, NC) for A in range(NC)])
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
    work = [sum(lib.gs_sym_shell_len(A, NC) for A in range(r * rows, (r + 1) * rows))
            for r in range(P)]
    assert max(work) - min(work) == 0
    old = [sum(_round1_shell_len(A, NC) for A in range(r * rows, (r + 1) * rows))
           for r in range(P)]
    assert max(old) - min(old) == rows  # round 1: the first half of the ranks held long rows


@pytest.mark.parametrize("n_pad,P", [(65536, 8), (262144, 4), (1 << 20, 8), (1 << 20, 2),
                                     (1 << 20, 3), (1 << 20, 7), (262144, 6), (65536, 5)])
@pytest.mark.parametrize("fill", [-1, 1024, 0])
def test_unit_map_permutation_and_locality(n_pad, P, fill):
    lib, g = _geo(n_pad)
    NC, L, S, D = g["NC"], g["L"], g["S"], g["D"]
    for rank in (0, P - 1):
        a0, rows = partition.sym_rank_rows(n_pad, P, rank)
        out = (ctypes.c_int32 * (rows * (S + D)))()
        n = lib.gs_sym_unit_map(n_pad, rank, P, fill, out, len(out))
        assert n == rows * (S + D)
        m = np.frombuffer(out, dtype=np.uint32)
        remote = (m >> 31).astype(bool)
        row = (m >> 12) & 0xFFFF
        unit = m & 0xFFF
        key = row.astype(np.int64) * (S + D) + unit
        assert np.array_equal(np.sort(key), np.arange(rows * (S + D)))  # a permutation
        A = a0 + row.astype(np.int64)
        u = unit.astype(np.int64)
        h = np.array([lib.gs_sym_shell_len(int(x), NC) for x in range(NC)])[A]
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
                                     (1 << 24, 8), (1 << 20, 3), (262144, 6), (1 << 20, 7)])
@pytest.mark.parametrize("fill", [-1, 1024, 0])
def test_ring_unit_map_stages(n_pad, P, fill):
    """Ring strategy of the sym schedule: the slice of rank (r - k) mod P lands at stage k.
    Every unit carries the stage of the last slice it reads (0: own rows only), units are a
    permutation, the local prefix comes first and the rest is ordered by stage."""
    lib, g = _geo(n_pad)
    NC, L, S, D = g["NC"], g["L"], g["S"], g["D"]
    starts = [partition.sym_rank_rows(n_pad, P, q)[0] for q in range(P)]
    for rank in (0, P - 1):
        a0, rows = partition.sym_rank_rows(n_pad, P, rank)
        out = (ctypes.c_int32 * (rows * (S + D)))()
        n = lib.gs_sym_unit_map_ring(n_pad, rank, P, fill, out, len(out))
        assert n == rows * (S + D)
        m = np.frombuffer(out, dtype=np.uint32)
        remote = (m >> 31).astype(bool)
        stage = ((m >> 28) & 7).astype(np.int64)
        row = ((m >> 12) & 0xFFFF).astype(np.int64)
        unit = (m & 0xFFF).astype(np.int64)
        key = row * (S + D) + unit
        assert np.array_equal(np.sort(key), np.arange(rows * (S + D)))
        assert np.array_equal(remote, stage > 0)
        A = a0 + row
        h = np.array([lib.gs_sym_shell_len(int(x), NC) for x in range(NC)])[A]
        want = np.zeros(len(m), dtype=np.int64)
        owner_of_row = np.searchsorted(starts, np.arange(NC), side="right") - 1
        seg = np.nonzero((unit < S) & (unit * L < 16 * h))[0]
        d_lo = 1 + unit[seg] * L // 16
        d_hi = 1 + ((unit[seg] + 1) * L - 1) // 16
        for k in range(int((d_hi - d_lo).max()) + 1):  # the chunks each segment touches
            d = d_lo + k
            st = (rank - owner_of_row[(A[seg] + d) % NC]) % P
            want[seg] = np.where(d <= d_hi, np.maximum(want[seg], st), want[seg])
        assert np.array_equal(stage, want)
        local_prefix = int(np.argmax(stage > 0)) if (stage > 0).any() else len(stage)
        assert (np.diff(stage[local_prefix:]) >= 0).all()  # stage order after the prefix
        if fill != 0:
            assert not remote[:min(fill if fill > 0 else n, int((~remote).sum()))].any()
    # too many rows for the 16-bit row field: no gated ring map (the launch stays ungated)
    big = 1 << 28
    assert lib.gs_sym_unit_map_ring(big, 0, 1, -1, None, 0) == 0


@pytest.mark.parametrize("n_pad", [16384, 49152, 65536, 1 << 20, 1 << 24])
@pytest.mark.parametrize("P", range(1, 9))
def test_rank_blocks_and_nodes_match_native(n_pad, P):
    """Rows per rank (whole row blocks, mpi.c's remainder rule) and the dyadic reduction
    nodes each rank sends: native gs_sym_rank_rows / gs_sym_nodes equal the Python mirror;
    the ranks tile the rows in order and the nodes tile the blocks."""
    lib = _native.cpu_lib()
    NC = n_pad // 2048
    B = partition.sym_blocks(NC)
    if P > B:
        return
    nodes = partition.sym_nodes(n_pad, P)
    row = 0
    for r in range(P):
        a0, rows = ctypes.c_int32(), ctypes.c_int32()
        assert lib.gs_sym_rank_rows(n_pad, P, r, ctypes.byref(a0), ctypes.byref(rows)) == 0
        assert (a0.value, rows.value) == partition.sym_rank_rows(n_pad, P, r)
        assert a0.value == row and rows.value % (NC // B) == 0
        row += rows.value
        v = [ctypes.c_int32() for _ in range(5)]
        assert lib.gs_sym_nodes(n_pad, P, r, *[ctypes.byref(x) for x in v]) == 0
        Bn, RB, nn, nb, NN = (x.value for x in v)
        assert (Bn, RB) == (B, NC // B)
        assert nn == len(nodes[r]) and nb == sum(len(x) for x in nodes[:r])
        assert NN == sum(len(x) for x in nodes)
    assert row == NC
    cover = [b for rn in nodes for lo, l in rn for b in range(lo, lo + (1 << l))]
    assert cover == list(range(B))
    for rn in nodes:
        for lo, l in rn:
            assert lo % (1 << l) == 0  # aligned: a node of the canonical tree


def _tree(leaves):
    while len(leaves) > 1:
        leaves = [leaves[i] + leaves[i + 1] for i in range(0, len(leaves), 2)]
    return leaves[0]


def _counter_merge(nodes_vals):
    """The receiver's merge (nbody_sym.hip TreeAcc): nodes in global order, left + right."""
    acc, occ = {}, 0
    for level, v in nodes_vals:
        k = level
        while occ >> k & 1:
            v = acc[k] + v
            occ &= ~(1 << k)
            k += 1
        acc[k] = v
        occ |= 1 << k
    (k,) = [k for k in acc if occ >> k & 1]
    return acc[k]


@pytest.mark.parametrize("B", [8, 16, 32, 64, 128, 256])
def test_node_merge_equals_full_tree_bitwise_for_every_P(B):
    """fp32 leaves: every rank reduces its dyadic nodes (a sub-tree each) and the receiver
    merges them in global order. The result is the full tree's, bit for bit, for every P:
    the j-side sums do not depend on the rank count."""
    rng = np.random.default_rng(B)
    leaves = (rng.standard_normal((B, 1000)) * np.exp(rng.uniform(-20, 20, (B, 1)))).astype(
        np.float32)
    full = _tree(list(leaves))
    n_pad = B * (3 if B < 256 else 1) * 2048  # NC with sym_blocks(NC) == B
    assert partition.sym_blocks(n_pad // 2048) == B
    for P in range(1, min(8, B) + 1):
        vals = [(l, _tree(list(leaves[lo:lo + (1 << l)])))
                for rn in partition.sym_nodes(n_pad, P) for lo, l in rn]
        got = _counter_merge(vals)
        assert np.array_equal(got.view(np.uint32), full.view(np.uint32)), P


@pytest.mark.parametrize("n_pad,P", [(65536, 1), (65536, 8), (1 << 20, 1), (1 << 20, 8),
                                     (1 << 20, 3), (262144, 6)])
@pytest.mark.parametrize("np_", [None, 2])
def test_split_segment_map(n_pad, P, np_):
    """The last Kr shell segments of every row (Kr = S / 16 when a segment has >= 2 tiles) are
    split into Np parts (gs_sym_split_parts: 4 when a segment spans >= 4 quanta, else 2): the
    gated order lists every other unit once and each split segment as Np part units (bit 30,
    part in bits 28-29, rows in bits 12-27) at the very end, with the segment's locality."""
    lib, g = _geo(n_pad)
    S, D = g["S"], g["D"]
    kr = lib.gs_sym_split_segments(n_pad)
    assert kr == (S // 16 if g["L"] >= 2 else 0)
    npart = lib.gs_sym_split_parts(n_pad) if np_ is None else np_
    assert npart == (4 if g["L"] >= 4 else 2) or np_ is not None
    for rank in (0, P - 1):
        a0, rows = partition.sym_rank_rows(n_pad, P, rank)
        plain = (ctypes.c_int32 * (rows * (S + D)))()
        assert lib.gs_sym_unit_map(n_pad, rank, P, 1024, plain, len(plain)) == rows * (S + D)
        total = rows * (S + D + (npart - 1) * kr)
        out = (ctypes.c_int32 * total)()
        n = lib.gs_sym_unit_map_parts(n_pad, rank, P, 1024, kr, npart, out, len(out))
        assert n == total
        if npart == 2:  # the _kr entry point is the two-part map
            out2 = (ctypes.c_int32 * total)()
            assert lib.gs_sym_unit_map_kr(n_pad, rank, P, 1024, kr, out2, len(out2)) == total
            assert bytes(out2) == bytes(out)
        m = np.frombuffer(out, dtype=np.uint32)
        split = ((m >> 30) & 1).astype(bool)
        part = (m >> 28) & 3
        row = (m >> 12) & 0xFFFF
        unit = m & 0xFFF
        n_part = rows * kr * npart
        assert split[len(m) - n_part:].all() and not split[:len(m) - n_part].any()  # at the end
        whole = unit[~split].astype(np.int64) + ((m[~split] >> 12) & 0xFFFF).astype(np.int64) * (S + D)
        expect = [r * (S + D) + u for r in range(rows) for u in range(S + D)
                  if not (S - kr <= u < S)]
        assert np.array_equal(np.sort(whole), np.array(expect, dtype=np.int64))
        hk = (row[split].astype(np.int64) * S + unit[split]) * npart + part[split]
        want = sorted((r * S + u) * npart + h for r in range(rows) for u in range(S - kr, S)
                      for h in range(npart))
        assert np.array_equal(np.sort(hk), np.array(want, dtype=np.int64))
        # a split segment's parts carry its locality (remote = reads gathered rows)
        pm = np.frombuffer(plain, dtype=np.uint32)
        rem_plain = {(int((x >> 12) & 0xFFFF), int(x & 0xFFF)): bool(x >> 31) for x in pm}
        for x in m[split]:
            key = (int((x >> 12) & 0xFFFF), int(x & 0xFFF))
            assert bool(x >> 31) == rem_plain[key]


def test_unit_map_holds_16m_on_two_ranks():
    """16M bodies on 2 ranks: 4096 rows per rank. Round 4's 12-bit row field returned no map
    there, so the gated launch was silently replaced by the ungated one; the
    16-bit row field holds it, with split parts, for every P."""
    lib, g = _geo(1 << 24)
    S, D = g["S"], g["D"]
    kr, npart = lib.gs_sym_split_segments(1 << 24), lib.gs_sym_split_parts(1 << 24)
    for P in (1, 2, 3, 8):
        a0, rows = partition.sym_rank_rows(1 << 24, P, 0)
        total = rows * (S + D + (npart - 1) * kr)
        out = (ctypes.c_int32 * total)()
        assert lib.gs_sym_unit_map_parts(1 << 24, 0, P, 2048, kr, npart, out, total) == total
        m = np.frombuffer(out, dtype=np.uint32)
        assert int(((m >> 12) & 0xFFFF).max()) == rows - 1


@pytest.mark.parametrize("B", [4, 8, 64, 256])
def test_grouped_leaf_pushes_equal_single_pushes(B):
    """nbody_sym.hip push_leaves: four aligned leaves summed as ((l0 + l1) + (l2 + l3)) and
    pushed as one level-2 sub-tree give the bits of four level-0 pushes (and of the full
    tree), so grouping the node reduce's leaves by four changes only the work."""
    rng = np.random.default_rng(100 + B)
    leaves = (rng.standard_normal((B, 500)) * np.exp(rng.uniform(-15, 15, (B, 1)))).astype(
        np.float32)
    single = _counter_merge([(0, l) for l in leaves])
    grouped = _counter_merge([(2, (leaves[i] + leaves[i + 1]) + (leaves[i + 2] + leaves[i + 3]))
                              for i in range(0, B, 4)])
    assert np.array_equal(single.view(np.uint32), grouped.view(np.uint32))
    assert np.array_equal(single.view(np.uint32), _tree(list(leaves)).view(np.uint32))


@pytest.mark.parametrize("n_pad", [16384, 65536, 262144, 1 << 20, 1 << 24])
def test_split_geometry_matches_native(n_pad):
    """Split segments per row and their parts: native == the Python mirror."""
    lib = _native.cpu_lib()
    assert (lib.gs_sym_split_segments(n_pad), lib.gs_sym_split_parts(n_pad)) == \
        partition.sym_split(n_pad)


@pytest.mark.parametrize("n_pad", [65536, 1 << 20])
@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8])
def test_pair_live_matches_the_shell_definition(n_pad, P):
    """gs_sym_pair_live: rank src's node sums for rank dst are +0.0 for every body (the
    exchange skips the pair) exactly when no row of src's holds a chunk of dst's in its shell
    (distance 1 .. NC/2 - 1, or NC/2 for the rows that take the antipodal chunk). At P = 8 the
    three far-side destinations of every rank are dead: 24 of 56 sends skipped."""
    lib, g = _geo(n_pad)
    NC = g["NC"]
    takes = np.array([lib.gs_sym_shell_len(A, NC) == NC // 2 for A in range(NC)])
    rows = [partition.sym_rank_rows(n_pad, P, q) for q in range(P)]
    dead = 0
    for src in range(P):
        A = np.arange(rows[src][0], rows[src][0] + rows[src][1])[:, None]
        for dst in range(P):
            X = np.arange(rows[dst][0], rows[dst][0] + rows[dst][1])[None, :]
            d = (X - A) % NC
            want = src == dst or bool((((d >= 1) & (d < NC // 2)) |
                                       ((d == NC // 2) & takes[A])).any())
            got = lib.gs_sym_pair_live(n_pad, P, src, dst)
            assert got == int(want), (src, dst)
            dead += not want
    if P == 8:
        assert dead == 24
