"""Canonical body decomposition (pure-Python mirror of csrc/common/layout.cpp).

Reference: mpi.c:184-187 gives rank r the block [r*floor(N/P) + min(r, N mod P), ...) and
rebuilds Allgatherv counts/displacements every step (mpi.c:218-225). Equal-count collectives
(RCCL all-gather) need equal slices, and bitwise world-size independence needs the j-sum
order fixed, so instead:

* chunk  = C(N): canonical j-chunk length, a function of N only;
* n_pad  = N rounded up to a multiple of P*C; rows [N, n_pad) are massless ghosts at the origin;
* rank r owns rows [r*n_pad/P, (r+1)*n_pad/P);
* every body's acceleration is sum over chunks c (in order) of a chunk sum that starts at 0,
  so partials computed on any rank, in any launch shape, add up to the same bits.

The Newton-3 (sym) schedule pads as an 8-rank run would and cuts its NC chunk rows into B
row blocks (B <= 256, a power of two dividing NC); rank r owns whole blocks by mpi.c's own
remainder rule (the first B mod P ranks hold one more), so every P from 1 to 8 is balanced to
within one block and the reduction tree over the blocks keeps the bits P-independent.
"""
from __future__ import annotations

from dataclasses import dataclass


def auto_chunk(n: int) -> int:
    p = 1
    while p < n:
        p <<= 1
    return int(min(65536, max(2048, p // 64)))


def round_up(a: int, b: int) -> int:
    return (a + b - 1) // b * b


@dataclass(frozen=True)
class Layout:
    n: int
    n_pad: int
    n_local: int
    local_begin: int
    chunk: int
    n_chunks: int
    rank: int
    nranks: int

    @property
    def local_end(self) -> int:
        return self.local_begin + self.n_local

    @property
    def real_local(self) -> range:
        """Global indices of the real (non-ghost) bodies this rank owns."""
        return range(self.local_begin, min(self.local_end, self.n))

    @property
    def own_chunks(self) -> range:
        c0 = min(self.local_begin // self.chunk, self.n_chunks)
        c1 = min(self.local_end // self.chunk, self.n_chunks)
        return range(c0, c1)


SYM_CHUNK = 2048  # Newton-3 schedule chunk (csrc/include/gs_kernels.h kSymC)
SYM_GROUPS = 8


def sym_pad(n: int, chunk: int) -> int:
    """Padding of the Newton-3 (sym) schedule: what an 8-rank run would use, so its chunk,
    row and group structure (hence its bits) is the same for every P dividing 8."""
    unit = 8 * (chunk if chunk % SYM_CHUNK == 0 else 2 * chunk)
    return round_up(n, unit)


def sym_geometry(n_pad: int) -> dict:
    """NC chunks, shell H = NC/2, segment length L (quanta of 128 bodies), S segments per row,
    D diagonal parts (layout.cpp gs_sym_geometry)."""
    if n_pad % (SYM_GROUPS * SYM_CHUNK):
        raise ValueError("sym n_pad must be a multiple of 16384")
    nc = n_pad // SYM_CHUNK
    h = nc // 2
    if nc >= 512:
        seg = 16 * (nc // 512)
    else:
        want = max(1, nc // 16)
        seg = 1
        while seg * 2 <= want:
            seg *= 2
    return {"NC": nc, "H": h, "L": seg, "S": -(-16 * h // seg), "D": 16 // seg if seg < 16 else 1}


SYM_MAX_BLOCKS = 256  # gs_common.h kSymMaxBlocks


def sym_blocks(nc: int) -> int:
    """Row blocks of the sym schedule: the largest power of two <= 256 dividing NC."""
    b = SYM_MAX_BLOCKS
    while b > 1 and nc % b:
        b >>= 1
    return b


def sym_blk_lo(B: int, P: int, r: int) -> int:
    """First block of rank r (mpi.c:184-187's remainder rule over the B blocks)."""
    base, rem = divmod(B, P)
    return r * base + min(r, rem)


def dyadic_nodes(lo: int, hi: int) -> list[tuple[int, int]]:
    """(first block, level) of the maximal aligned power-of-two pieces covering [lo, hi)."""
    out = []
    while lo < hi:
        l = 0
        while (lo >> l) & 1 == 0 and lo + (2 << l) <= hi:
            l += 1
        out.append((lo, l))
        lo += 1 << l
    return out


def sym_rank_rows(n_pad: int, nranks: int, rank: int) -> tuple[int, int]:
    """(first row, rows) of one rank in the sym schedule (layout.cpp gs_sym_rank_rows)."""
    nc = n_pad // SYM_CHUNK
    B = sym_blocks(nc)
    if not 1 <= nranks <= B or not 0 <= rank < nranks:
        raise ValueError("sym: nranks must be 1 .. the row-block count")
    rb = nc // B
    lo, hi = sym_blk_lo(B, nranks, rank), sym_blk_lo(B, nranks, rank + 1)
    return lo * rb, (hi - lo) * rb


def sym_nodes(n_pad: int, nranks: int) -> list[list[tuple[int, int]]]:
    """Per rank, the reduction-tree nodes it sends (layout.cpp gs_sym_nodes)."""
    B = sym_blocks(n_pad // SYM_CHUNK)
    return [dyadic_nodes(sym_blk_lo(B, nranks, q), sym_blk_lo(B, nranks, q + 1))
            for q in range(nranks)]


def sym_split(n_pad: int) -> tuple[int, int]:
    """(Kr, Np): the split shell segments per row and their parts (layout.cpp
    gs_sym_split_segments / gs_sym_split_parts): S / 16 segments when a segment spans >= 2
    quanta, in 4 parts when it spans >= 4, else 2."""
    g = sym_geometry(n_pad)
    return (g["S"] // 16 if g["L"] >= 2 else 0), (4 if g["L"] >= 4 else 2)


def sym_bytes(n_pad: int, nranks: int, esz: int = 4) -> int:
    """Partial-slot bytes of rank 0 (the largest share) if all its rows were held at once
    (one band), plus the node sums it sends and receives (layout.cpp gs_sym_bytes)."""
    g = sym_geometry(n_pad)
    kr, np_ = sym_split(n_pad)
    _, rows = sym_rank_rows(n_pad, nranks, 0)
    n_local = rows * SYM_CHUNK
    nodes = sym_nodes(n_pad, nranks)
    NN = sum(len(x) for x in nodes)
    return n_local * 3 * esz * (g["S"] + kr * (np_ - 1) + g["H"] + g["D"]) + \
        (len(nodes[0]) * n_pad + NN * n_local) * 3 * esz


SYM_MAX_IMBALANCE = 1.25  # layout.cpp kSymMaxImbalance


def sym_imbalance(n_pad: int, nranks: int) -> float:
    """Work of the busiest rank over the mean when P ranks own whole row blocks: the
    busiest holds ceil(B / P) of the B blocks (layout.cpp gs_sym_imbalance)."""
    B = sym_blocks(n_pad // SYM_CHUNK)
    return -(-B // nranks) * nranks / B


def sym_auto(n: int, nranks: int, chunk: int = 0, dtype: str = "fp32") -> bool:
    """Whether mode=auto picks the sym schedule (mirror of gs_layout_compute)."""
    # from 16K (fp32) / 32K (fp64) bodies sym wins, padding included
    # (profiles/r2_sizes_auto_vs_sym.txt); the partial slots are processed in bounded bands,
    # so memory does not limit the choice; a P up to 8 owns whole row blocks, unless that
    # leaves the busiest rank more than 25 % over the mean (few blocks, e.g. 8 blocks at P = 6
    # or 7: the split schedule's equal slices win there)
    if nranks > 8 or n < (16384 if dtype == "fp32" else 32768):
        return False
    c = chunk if chunk > 0 else auto_chunk(n)
    return sym_imbalance(sym_pad(n, c), nranks) <= SYM_MAX_IMBALANCE


def layout(n: int, rank: int = 0, nranks: int = 1, chunk: int = 0, sym: bool = False) -> Layout:
    if n < 1:
        raise ValueError("n must be >= 1")
    if not (0 <= rank < nranks):
        raise ValueError("bad rank/nranks")
    c = chunk or auto_chunk(n)
    if c % 1024:
        raise ValueError("chunk must be a multiple of 1024")
    if sym and nranks > 8:
        raise ValueError("the sym schedule needs nranks <= 8")
    if sym:
        n_pad = sym_pad(n, c)
        a0, rows = sym_rank_rows(n_pad, nranks, rank)
        begin, n_local = a0 * SYM_CHUNK, rows * SYM_CHUNK
    else:
        n_pad = round_up(n, nranks * c)
        n_local = n_pad // nranks
        begin = rank * n_local
    return Layout(n=n, n_pad=n_pad, n_local=n_local, local_begin=begin, chunk=c,
                  n_chunks=(n + c - 1) // c, rank=rank, nranks=nranks)


def mpi_block(n: int, rank: int, nranks: int) -> tuple[int, int]:
    """The reference's remainder-spread block (start, count) of mpi.c:184-187 (for parity docs)."""
    base, rem = divmod(n, nranks)
    return rank * base + min(rank, rem), base + (1 if rank < rem else 0)
