"""Decomposition math and initial conditions (CPU).

Reference: mpi.c:184-187,218-225 (block partition with remainder spread), mpi.c:75-105 /
cuda.cu:81-96,127-138 / pyspark.py:124-149 (ICs, unseeded). Here the layout is padded and
world-size independent, and ICs are a pure function of (seed, index).
"""
import ctypes

import numpy as np
import pytest

from gravsim.models import initial_conditions as ic
from gravsim.ops import _native
from gravsim.parallel import partition


@pytest.mark.parametrize("n", [1, 2, 3, 8, 1000, 2048, 2049, 16383, 16384, 20000, 32768, 65536,
                               100_003, 1 << 20, 16_777_216])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("dtype", ["fp32", "fp64"])
def test_python_layout_matches_native(n, P, dtype):
    lib = _native.cpu_lib()
    for r in sorted({0, P - 1, P // 2}):
        c = _native.GsConfig(n=n, dtype=_native.GS_FP64 if dtype == "fp64" else _native.GS_FP32,
                             rank=r, nranks=P, device=0)
        L = _native.GsLayout()
        assert lib.gs_layout_compute(ctypes.byref(c), ctypes.byref(L)) == 0
        sym = partition.sym_auto(n, P, dtype=dtype)
        assert (L.mode == _native.MODE_IDS["sym"]) == sym
        p = partition.layout(n, r, P, sym=sym)
        assert (L.n_pad, L.n_local, L.local_begin, L.chunk, L.n_chunks) == \
            (p.n_pad, p.n_local, p.local_begin, p.chunk, p.n_chunks)
        assert p.n_pad >= n
        if not sym:
            assert p.n_pad % (P * p.chunk) == 0
        assert p.chunk == partition.auto_chunk(n)  # chunk depends on n only


def test_chunk_independent_of_world_size():
    for n in (5, 5000, 123457, 1 << 20):
        assert len({partition.layout(n, 0, P).chunk for P in (1, 2, 4, 8)}) == 1


def test_slices_tile_padded_range():
    n, P = 100_003, 8
    covered = []
    for r in range(P):
        L = partition.layout(n, r, P)
        covered.extend(range(L.local_begin, L.local_end))
        assert list(L.own_chunks) == [c for c in range(L.n_chunks)
                                      if L.local_begin <= c * L.chunk < L.local_end]
    assert covered == list(range(partition.layout(n, 0, P).n_pad))


def test_mpi_block_reference_partition():
    # mpi.c:184-187 with N=8, P=3: counts 3,3,2
    assert [partition.mpi_block(8, r, 3) for r in range(3)] == [(0, 3), (3, 3), (6, 2)]


@pytest.mark.parametrize("fam,ic_id", [("solar+random", 0), ("random", 1)])
def test_numpy_ics_match_native_bitwise(fam, ic_id):
    lib = _native.cpu_lib()
    n, seed = 5000, 987654321
    pos, vel, m = np.zeros((n, 3)), np.zeros((n, 3)), np.zeros(n)
    lib.gs_ic_fill_host(ic_id, seed, n, 0, n, _native.dptr(pos), _native.dptr(vel),
                        _native.dptr(m))
    b = ic.make(fam, n, seed)
    assert np.array_equal(pos, b.pos) and np.array_equal(vel, b.vel) and np.array_equal(m, b.mass)


def test_ic_slices_independent_of_partition():
    full = ic.solar_random(1000, 3)
    part = ic.solar_random(1000, 3, begin=400, end=700)
    assert np.array_equal(full.pos[400:700], part.pos)


def test_solar_bodies_and_ranges():
    b = ic.solar_random(2000, 1)
    assert b.mass[0] == 1.989e30 and tuple(b.pos[1]) == (1.496e11, 0.0, 0.0)
    assert tuple(b.vel[2]) == (0.0, 24.077e3, 0.0)
    r = b.pos[3:]
    assert r.min() >= -3e11 and r.max() < 3e11
    assert b.vel[3:].min() >= -3e4 and b.vel[3:].max() < 3e4
    assert b.mass[3:].min() >= 1e23 and b.mass[3:].max() < 1e25
    # uniform: mean near zero, std near 3e11/sqrt(3)
    assert abs(r.mean()) < 1e10 and abs(r.std() / (3e11 / np.sqrt(3)) - 1) < 0.03


def test_seed_changes_ics_and_is_reproducible():
    a, b, c = ic.random_cube(100, 1), ic.random_cube(100, 1), ic.random_cube(100, 2)
    assert np.array_equal(a.pos, b.pos) and not np.array_equal(a.pos, c.pos)


@pytest.mark.parametrize("fam", ic.FAMILIES)
def test_all_families_build(fam):
    n = 2 if fam == "kepler" else 300
    b = ic.make(fam, n, 5)
    assert b.pos.shape == (n, 3) and b.vel.shape == (n, 3) and b.mass.shape == (n,)
    assert np.isfinite(b.pos).all() and np.isfinite(b.vel).all() and (b.mass > 0).all()


def test_plummer_virial_ratio():
    from gravsim.models.diagnostics import kinetic_energy, potential_energy

    b = ic.plummer(2000, 4)
    ratio = 2 * kinetic_energy(b.vel, b.mass) / -potential_energy(b.pos, b.mass)
    assert 0.8 < ratio < 1.2


def test_mfma_kernel_config_validation():
    from gravsim.config import SimConfig

    SimConfig(n=1024, dtype="fp32", kernel="mfma").validate()
    for bad in (dict(dtype="fp64"), dict(dtype="fp32", ipl=4), dict(dtype="fp32", mode="fused")):
        with pytest.raises(ValueError):
            SimConfig(n=1024, kernel="mfma", **bad).validate()


@pytest.mark.parametrize("n", [1000, 20000, 100_003, 1 << 20])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8])
def test_sym_layout_independent_of_world_size(n, P):
    """mode=sym pads as an 8-rank run would: n_pad (hence the chunk/row/block structure and
    the summation order) is the same for every P up to 8, and matches the native layout."""
    lib = _native.cpu_lib()
    c = _native.GsConfig(n=n, dtype=0, rank=P - 1, nranks=P, device=0,
                         mode=_native.MODE_IDS["sym"])
    L = _native.GsLayout()
    assert lib.gs_layout_compute(ctypes.byref(c), ctypes.byref(L)) == 0
    assert L.mode == _native.MODE_IDS["sym"]
    p = partition.layout(n, P - 1, P, sym=True)
    assert (L.n_pad, L.n_local, L.local_begin) == (p.n_pad, p.n_local, p.local_begin)
    assert p.n_pad == partition.layout(n, 0, 1, sym=True).n_pad
    g = partition.sym_geometry(p.n_pad)
    assert g["NC"] % (partition.SYM_GROUPS) == 0
    # segments of L quanta (128 bodies, 16 per chunk) cover the H-chunk shell; the diagonal
    # chunk is cut into D parts of the same length when L < 16
    assert g["S"] * g["L"] >= 16 * g["H"] > (g["S"] - 1) * g["L"]
    assert g["D"] * min(g["L"], 16) == 16
    nc, h, seg, S, D = (ctypes.c_int32() for _ in range(5))
    assert lib.gs_sym_geometry(ctypes.c_int64(p.n_pad), ctypes.byref(nc), ctypes.byref(h),
                               ctypes.byref(seg), ctypes.byref(S), ctypes.byref(D)) == 0
    assert (nc.value, h.value, seg.value, S.value, D.value) == \
        (g["NC"], g["H"], g["L"], g["S"], g["D"])
    for esz in (4, 8):
        assert lib.gs_sym_bytes(p.n_pad, P, esz) == partition.sym_bytes(p.n_pad, P, esz)


def test_sym_layout_rejects_unsupported():
    lib = _native.cpu_lib()
    for kw in (dict(nranks=9, rank=0), dict(kernel=3)):
        base = dict(n=50000, dtype=0, rank=0, nranks=1, device=0, mode=_native.MODE_IDS["sym"])
        base.update(kw)
        L = _native.GsLayout()
        assert lib.gs_layout_compute(ctypes.byref(_native.GsConfig(**base)), ctypes.byref(L)) != 0


def test_sym_auto_at_headline_size():
    """N = 1M fp32 picks the Newton-3 schedule for every P from 1 to 8 with unchanged
    padding; ranks own whole row blocks of 2 rows (256 blocks), mpi.c's remainder rule."""
    for P in range(1, 9):
        assert partition.sym_auto(1 << 20, P)
        lays = [partition.layout(1 << 20, r, P, sym=True) for r in range(P)]
        assert all(L.n_pad == 1 << 20 for L in lays)
        counts = [L.n_local // (2 * 2048) for L in lays]  # blocks per rank
        assert sum(counts) == 256 and max(counts) - min(counts) <= 1
        assert counts == sorted(counts, reverse=True)  # the first 256 mod P ranks hold one more
        assert max(counts) * P / 256 <= 1.02  # at most 2 % over the mean for every P <= 8
        assert [L.local_begin for L in lays] == [sum(counts[:r]) * 2 * 2048 for r in range(P)]
