// Canonical decomposition shared by the CPU and GPU engines, plus host IC fill.
//
// Reference: mpi.c:184-187,218-225 spreads the N mod P remainder over the first ranks and
// rebuilds Allgatherv counts every step. Here the body array is padded once with massless
// ghost bodies (mu = 0, at the origin) to a multiple of P * chunk, so every rank owns an
// equal contiguous slice (RCCL all-gather needs equal counts) and the j-chunk boundaries,
// hence the floating-point summation order, do not depend on P.
#include <vector>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gravsim.h"
#include "gs_common.h"

namespace {
thread_local char g_err[512];
}

extern "C" const char* gs_last_error(void) { return g_err; }

void gs_set_error(const char* msg) {
  strncpy(g_err, msg, sizeof(g_err) - 1);
  g_err[sizeof(g_err) - 1] = 0;
}

extern "C" int32_t gs_auto_chunk(int64_t n) { return gs::auto_chunk(n); }

// Busiest rank's work over the mean when nranks ranks own whole row blocks of the sym
// schedule: ceil(B / P) * P / B (B row blocks of the n_pad geometry).
constexpr double kSymMaxImbalance = 1.25;
extern "C" double gs_sym_imbalance(int64_t n_pad, int32_t nranks) {
  if (nranks < 1) return 1e30;
  const int32_t B = gs::sym_blocks((int32_t)(n_pad / 2048));
  if (nranks > B) return 1e30;
  return (double)((B + nranks - 1) / nranks) * nranks / B;
}

extern "C" int gs_layout_compute(const gs_config* cfg, gs_layout* out) {
  if (!cfg || !out) { gs_set_error("layout: null argument"); return -1; }
  if (cfg->n < 1) { gs_set_error("layout: n must be >= 1"); return -1; }
  if (cfg->nranks < 1 || cfg->rank < 0 || cfg->rank >= cfg->nranks) {
    gs_set_error("layout: bad rank/nranks");
    return -1;
  }
  memset(out, 0, sizeof(*out));
  const int32_t chunk = cfg->chunk > 0 ? cfg->chunk : gs::auto_chunk(cfg->n);
  if (chunk % 1024 != 0) { gs_set_error("layout: chunk must be a multiple of 1024"); return -1; }
  out->n = cfg->n;
  out->chunk = chunk;
  out->n_pad = gs::round_up(cfg->n, (int64_t)cfg->nranks * chunk);
  // Newton-3 symmetric schedule, any P from 1 to 8. Its chunk/row/block structure must not
  // depend on P, so the padding is the one an 8-rank run would use; ranks own whole row
  // blocks (gs_common.h sym_blk_lo: mpi.c's remainder rule over the B blocks).
  const bool sym_ok = cfg->nranks <= 8 && cfg->kernel != GS_KERNEL_MFMA;
  if (cfg->mode == GS_MODE_SYM && !sym_ok) {
    gs_set_error("layout: the sym schedule needs nranks <= 8 (and not the mfma kernel)");
    return -1;
  }
  const int64_t sym_unit = 8 * (int64_t)(chunk % 2048 == 0 ? chunk : 2 * chunk);
  const int64_t sym_pad = gs::round_up(cfg->n, sym_unit);
  bool sym = cfg->mode == GS_MODE_SYM;
  // From 16K bodies (fp32) / 32K (fp64) the sym schedule beats the one-sided split/fused
  // kernels, padding included (all-ghost chunks are skipped). fp32: 16384 0.137 vs 0.196 ms,
  // 50000 (cuda.cu's N) 0.479 vs 0.630, 100000 1.64 vs 2.25, 300000 14.1 vs 21.5; fp64: 16384
  // 0.283 vs 0.250 (split wins), 50000 1.21 vs 1.75, 300000 37.5 vs 56.5
  // (profiles/r2_sizes_auto_vs_sym.txt). The partial slots are processed in bands of bounded
  // size (stepper.hip ensure_sym), so memory does not limit the choice either.
  // A rank owns whole row blocks: with few blocks (B = 8 when NC is an odd multiple of 8) some
  // P leave the busiest rank far above the mean (P = 7: 2 blocks against 1, twice the work),
  // which cancels the Newton-3 saving; auto then keeps the split schedule's equal slices.
  const int64_t sym_min = cfg->dtype == GS_FP32 ? 16384 : 32768;
  if (cfg->mode == GS_MODE_AUTO && sym_ok && cfg->n >= sym_min &&
      gs_sym_imbalance(sym_pad, cfg->nranks) <= kSymMaxImbalance)
    sym = true;
  if (sym) {
    out->n_pad = sym_pad;
    int32_t a0 = 0, rows = 0;
    if (gs_sym_rank_rows(sym_pad, cfg->nranks, cfg->rank, &a0, &rows)) return -1;
    out->local_begin = (int64_t)a0 * 2048;
    out->n_local = (int64_t)rows * 2048;
  } else {
    out->n_local = out->n_pad / cfg->nranks;
    out->local_begin = (int64_t)cfg->rank * out->n_local;
  }
  out->n_chunks = (int32_t)((cfg->n + chunk - 1) / chunk);
  // j source and i-bodies per lane, from in-process sweeps on MI355X with the explicit
  // 2-vector fp32 loop (profiles/r1_tune2_*.log):
  //  * fp32: SGPR streaming through the scalar cache at every size (no LDS barrier per tile;
  //    1M: 239.4 vs 252.1 ms, 64K: 1.09 vs 1.12 ms). IPL 8 at >= 256K bodies per rank,
  //    4 below (64K: IPL 8 leaves too few workgroups).
  //  * fp64: SGPR streaming at >= 128K per rank, LDS tiles below; IPL 2 (512K: 190.9 ms,
  //    IPL 4 192.3 ms).
  const bool f32 = cfg->dtype == GS_FP32;
  out->kernel = cfg->kernel != GS_KERNEL_AUTO ? cfg->kernel
                : (f32 || out->n_local >= 131072 ? GS_KERNEL_SMEM : GS_KERNEL_LDS);
  if (out->kernel == GS_KERNEL_MFMA) {
    // Experimental MFMA variant: fp32, 256 i-bodies per workgroup, split schedule only.
    if (cfg->dtype != GS_FP32 || (cfg->ipl > 1) || cfg->mode == GS_MODE_FUSED) {
      gs_set_error("layout: the mfma kernel is fp32, ipl 1, split schedule only");
      return -1;
    }
  }
  int32_t ipl = out->kernel == GS_KERNEL_MFMA ? 1 : cfg->ipl;
  if (ipl <= 0) {
    ipl = f32 ? (out->n_local >= 262144 ? 8 : 4) : 2;
    while (ipl > 1 && out->n_local % (gs::kForceBlock * ipl) != 0) ipl /= 2;
  }
  if (ipl != 1 && ipl != 2 && ipl != 4 && !(ipl == 8 && cfg->dtype == GS_FP32)) {
    gs_set_error("layout: ipl must be 1, 2, 4 (or 8 for fp32)");
    return -1;
  }
  if ((out->n_local % (gs::kForceBlock * ipl)) != 0) {
    gs_set_error("layout: block*ipl must divide the per-rank body count (raise chunk)");
    return -1;
  }
  out->ipl = ipl;
  const int64_t i_blocks = out->n_local / (gs::kForceBlock * ipl);
  int32_t mode = sym ? GS_MODE_SYM : cfg->mode;
  if (out->kernel == GS_KERNEL_MFMA) mode = GS_MODE_SPLIT;
  if (mode == GS_MODE_AUTO) {
    // Fused needs enough i-blocks to fill 256 CUs at >= 8 workgroups of 4 waves each;
    // otherwise split j over workgroups (deterministic per-chunk partials).
    mode = (i_blocks >= 2048) ? GS_MODE_FUSED : GS_MODE_SPLIT;
  }
  out->mode = mode;
  int32_t groups = cfg->split_groups;
  if (groups <= 0) {
    const int64_t target = 4096;  // workgroups per split launch (16 per CU)
    int64_t g = (target + i_blocks - 1) / i_blocks;
    if (g < 1) g = 1;
    if (g > out->n_chunks) g = out->n_chunks;
    groups = (int32_t)g;
  }
  out->split_groups = groups;
  return 0;
}

// Symmetric-schedule geometry (gs_kernels.h SymArgs), a function of n_pad only:
//   NC chunks of 2048 bodies; shell H = NC / 2 chunks;
//   L = segment length in quanta of 128 bodies (16 per chunk): 16 * (NC / 512) from
//       NC = 512 up (a row has about 256 segments: enough workgroups for one rank of
//       eight), else the largest power of two <= max(1, NC / 16) (about 128 segments: half
//       the i-side partial traffic; 1 GPU, profiles/r1_sym_seglen.jsonl: 65K 0.768 vs
//       0.788 ms at NC / 32, 131K 2.836 vs 2.850, 256K 11.04 vs 11.09, 512K 43.56 vs 43.65);
//   S = ceil(16 H / L) segments per row; D = max(1, 16 / L) parts of the diagonal chunk.
extern "C" int gs_sym_geometry(int64_t n_pad, int32_t* NC, int32_t* H, int32_t* L, int32_t* S,
                               int32_t* D) {
  if (n_pad % (8 * 2048) != 0) { gs_set_error("sym: n_pad must be a multiple of 16384"); return -1; }
  const int32_t nc = (int32_t)(n_pad / 2048);
  const int32_t h = nc / 2;
  int32_t l;
  if (nc >= 512) {
    l = 16 * (nc / 512);
  } else {
    const int32_t want = nc / 16 > 1 ? nc / 16 : 1;
    l = 1;
    while (l * 2 <= want) l *= 2;
  }
  const int32_t d = l < 16 ? 16 / l : 1;
  if (NC) *NC = nc;
  if (H) *H = h;
  if (L) *L = l;
  if (S) *S = (16 * h + l - 1) / l;
  if (D) *D = d;
  return 0;
}

// Split shell segments per row (the launch tail, gs_kernels.h SymArgs::Kr): S / 16 when a
// segment spans at least 2 quanta (1M / 8 per rank -0.7 %, 65K -0.7 %, 1M one GPU even;
// Kr 8 / 16 / 32 within noise: profiles/r3s2_split_segments_ab.jsonl, *_kr_sweep.jsonl).
extern "C" int32_t gs_sym_split_segments(int64_t n_pad) {
  int32_t NC, H, L, S, D;
  if (gs_sym_geometry(n_pad, &NC, &H, &L, &S, &D)) return 0;
  return L >= 2 ? S / 16 : 0;
}

// Parts per split segment (SymArgs::Np): the final units of a launch are 1 / Np of a segment.
// 4 when a segment spans at least 4 quanta (one fp32 tile each), else 2.
extern "C" int32_t gs_sym_split_parts(int64_t n_pad) {
  int32_t NC, H, L, S, D;
  if (gs_sym_geometry(n_pad, &NC, &H, &L, &S, &D)) return 2;
  return L >= 4 ? 4 : 2;
}

// Rows [a0, a0 + rows) of rank `rank` of `nranks` in the sym schedule: whole row blocks by
// mpi.c's remainder rule (gs_common.h sym_blk_lo). Equal for every P dividing 8.
extern "C" int gs_sym_rank_rows(int64_t n_pad, int32_t nranks, int32_t rank, int32_t* a0,
                                int32_t* rows) {
  if (n_pad % (8 * 2048) != 0) { gs_set_error("sym: n_pad must be a multiple of 16384"); return -1; }
  const int32_t NC = (int32_t)(n_pad / 2048), B = gs::sym_blocks(NC), RB = NC / B;
  if (nranks < 1 || nranks > B || rank < 0 || rank >= nranks) {
    gs_set_error("sym: nranks must be 1 .. the row-block count (>= 8)");
    return -1;
  }
  const int32_t lo = gs::sym_blk_lo(B, nranks, rank), hi = gs::sym_blk_lo(B, nranks, rank + 1);
  if (a0) *a0 = lo * RB;
  if (rows) *rows = (hi - lo) * RB;
  return 0;
}

// Row blocks and reduction-tree nodes: B blocks of RB rows; rank `rank` sends nn maximal
// dyadic nodes (sub-trees of its block range; one per rank for P dividing 64); nodes of lower
// ranks come first (nb of them); NN nodes in all. (Splitting one rank's range into 8 nodes,
// 8x the threads of the node reduce with the same bits, measured slower: reduce phase at 1M
// 1373-1381 us per step against 1342-1343, profiles/r3_reduce_fork_split_ab.txt.)
extern "C" int gs_sym_nodes(int64_t n_pad, int32_t nranks, int32_t rank, int32_t* B, int32_t* RB,
                            int32_t* nn, int32_t* nb, int32_t* NN) {
  if (gs_sym_rank_rows(n_pad, nranks, rank, nullptr, nullptr)) return -1;
  const int32_t NC = (int32_t)(n_pad / 2048), b = gs::sym_blocks(NC);
  int32_t before = 0, total = 0, mine = 0;
  for (int32_t q = 0; q < nranks; ++q) {
    const int32_t k = gs::sym_node_count(gs::sym_blk_lo(b, nranks, q),
                                         gs::sym_blk_lo(b, nranks, q + 1));
    if (q < rank) before += k;
    if (q == rank) mine = k;
    total += k;
  }
  if (B) *B = b;
  if (RB) *RB = NC / b;
  if (nn) *nn = mine;
  if (nb) *nb = before;
  if (NN) *NN = total;
  return 0;
}

// Owner rank of chunk row A.
static int32_t sym_row_owner(int32_t A, int32_t NC, int32_t nranks) {
  const int32_t B = gs::sym_blocks(NC), blk = A / (NC / B);
  int32_t q = 0;
  while (q + 1 < nranks && gs::sym_blk_lo(B, nranks, q + 1) <= blk) ++q;
  return q;
}

// Chunk rows of the sym schedule: row A pairs with the next h(A) chunks cyclically. Distances
// 1 .. NC/2 - 1 belong to the row below; each antipodal pair {A, A + NC/2} to one of its two
// rows, by parity (A < NC/2 takes it iff A is even; NC/2 is a multiple of 4, so A + NC/2 has
// A's parity and takes it iff A is odd), so any block of rows holds as many long rows as
// short ones. Mirrors shell_len() in nbody_sym.hip.
extern "C" int32_t gs_sym_shell_len(int32_t A, int32_t NC) {
  const bool takes = (A < NC / 2) == ((A & 1) == 0);
  return takes ? NC / 2 : NC / 2 - 1;
}

// Rank-local shell segments of row A: the prefix of the row's segments (L quanta of 128 bodies,
// 16 quanta per chunk) whose j-chunks A+1 .. all lie in the rank rows [a0, a0 + rows); wrapped
// chunks count as remote. The force kernel's units 4/5 test in quanta.
static int32_t sym_local_segs(int32_t A, int32_t NC, int32_t a0, int32_t rows, int32_t L,
                              int32_t S) {
  const int32_t h = gs_sym_shell_len(A, NC);
  const int32_t segs = (16 * h + L - 1) / L;
  const int32_t own_after = a0 + rows - 1 - A;
  int32_t n;
  if (own_after <= 0) n = 0;
  else if (h <= own_after) n = segs;
  else n = segs < own_after * 16 / L ? segs : own_after * 16 / L;
  return n < S ? n : S;
}

// Unit-map entry (gs_common.h sym_unit_entry): row in bits 12-27 (rows < 65536), unit in bits
// 0-11 (S + D < 4096; S is ~128-256 at every size), bit 31 remote, bit 30 a part unit with its
// part in bits 28-29 (all-gather order) or the ring stage in bits 28-30 (ring order). (Round 4
// kept the row in bits 16-27 next to a 16-bit unit field: rows < 4096, so a 16M run on 2 ranks,
// 4096 rows each, got no map and silently ran ungated.)
static inline int32_t unit_entry(uint32_t flags, int32_t row, int32_t unit) {
  return (int32_t)(flags | ((uint32_t)row << gs::kUnitRowShift) | (uint32_t)unit);
}

// The gated sym launch's unit order (units 6, gs_kernels.h) for rank `rank` of `nranks`, one
// band: entry = row, unit (unit < S: shell segment, >= S: diagonal part), bit 31 set
// for a remote unit (a j-chunk outside the rank's rows). The first `fill` entries (all local
// units when fill < 0) are rank-local ones, row by row (diagonal parts, then local
// segments); the rest follow the ungated order: shell segments row by row, then the diagonal
// parts. Returns the entry count (rows * (S + D)), 0 if the entry fields cannot hold the
// geometry, -1 on error (cap too small, bad arguments).
extern "C" int64_t gs_sym_unit_map(int64_t n_pad, int32_t rank, int32_t nranks, int64_t fill,
                                   int32_t* out, int64_t cap) {
  return gs_sym_unit_map_kr(n_pad, rank, nranks, fill, 0, out, cap);
}

// The same order with the last kr shell segments of every row split into np parts
// (gs_kernels.h SymArgs::Kr, Np): they leave the order above and are appended as np part units
// each (bit 30 set, bits 28-29 the part), row by row, so the launch ends with 1 / np-length
// units. rows * (S + D + (np - 1) kr) entries.
extern "C" int64_t gs_sym_unit_map_kr(int64_t n_pad, int32_t rank, int32_t nranks,
                                      int64_t fill, int32_t kr, int32_t* out, int64_t cap) {
  return gs_sym_unit_map_parts(n_pad, rank, nranks, fill, kr, 2, out, cap);
}

extern "C" int64_t gs_sym_unit_map_parts(int64_t n_pad, int32_t rank, int32_t nranks,
                                         int64_t fill, int32_t kr, int32_t np, int32_t* out,
                                         int64_t cap) {
  int32_t NC, H, L, S, D, a0, rows;
  if (nranks < 1 || rank < 0 || rank >= nranks || kr < 0 || np < 2 || np > 4 ||
      gs_sym_geometry(n_pad, &NC, &H, &L, &S, &D) ||
      gs_sym_rank_rows(n_pad, nranks, rank, &a0, &rows))
    return -1;
  if (kr > S) return -1;
  const int32_t per = S + D;
  const int64_t total = (int64_t)rows * (per + (int64_t)(np - 1) * kr);
  if (rows > gs::kUnitRowMax || per > gs::kUnitMax) return 0;
  if (!out || cap < total) return -1;
  std::vector<int32_t> nl(rows);
  std::vector<char> moved((size_t)rows * per, 0);
  for (int32_t r = 0; r < rows; ++r)  // split segments go to the end
    for (int32_t u = S - kr; u < S; ++u) moved[(size_t)r * per + u] = 1;
  int64_t k = 0;
  for (int32_t r = 0; r < rows; ++r) {
    nl[r] = sym_local_segs(a0 + r, NC, a0, rows, L, S);
    for (int32_t q = 0; q < D && (fill < 0 || k < fill); ++q) {
      out[k++] = unit_entry(0u, r, S + q);
      moved[(size_t)r * per + S + q] = 1;
    }
    for (int32_t g = 0; g < nl[r] && g < S - kr && (fill < 0 || k < fill); ++g) {
      out[k++] = unit_entry(0u, r, g);
      moved[(size_t)r * per + g] = 1;
    }
  }
  for (int pass = 0; pass < 2; ++pass)
    for (int32_t r = 0; r < rows; ++r)
      for (int32_t u = pass ? S : 0; u < (pass ? per : S); ++u) {
        if (moved[(size_t)r * per + u]) continue;
        const bool remote = u < S && u >= nl[r];
        out[k++] = unit_entry(remote ? 0x80000000u : 0u, r, u);
      }
  for (int32_t r = 0; r < rows; ++r)
    for (int32_t u = S - kr; u < S; ++u)
      for (uint32_t h = 0; h < (uint32_t)np; ++h) {
        const bool remote = u >= nl[r];
        out[k++] = unit_entry((remote ? 0x80000000u : 0u) | 0x40000000u | (h << 28), r, u);
      }
  return k;
}

// The gated sym launch's unit order for the ring strategy: the slice of rank (rank - k) mod P
// arrives at ring stage k (1 .. P-1), so a remote unit can start once the stage of the latest
// slice it reads has landed. Entry = bit 31 remote | stage << 28 | row | unit. Order: the first `fill` local units as in gs_sym_unit_map, then every other unit by
// stage (local ones first), row by row within a stage, shell segments before diagonal parts.
// Returns the entry count, 0 if the fields cannot hold the geometry, -1 on error.
extern "C" int64_t gs_sym_unit_map_ring(int64_t n_pad, int32_t rank, int32_t nranks,
                                        int64_t fill, int32_t* out, int64_t cap) {
  int32_t NC, H, L, S, D, a0, rows;
  if (nranks < 1 || rank < 0 || rank >= nranks || gs_sym_geometry(n_pad, &NC, &H, &L, &S, &D) ||
      gs_sym_rank_rows(n_pad, nranks, rank, &a0, &rows))
    return -1;
  const int32_t per = S + D;
  const int64_t total = (int64_t)rows * per;
  if (rows > gs::kUnitRowMax || per > gs::kUnitMax || nranks > 8) return 0;
  if (!out || cap < total) return -1;
  // ring stage of every unit (0: reads only the rank's own rows)
  std::vector<int8_t> stage((size_t)total, 0);
  for (int32_t r = 0; r < rows; ++r) {
    const int32_t A = a0 + r;
    const int32_t segs = (16 * gs_sym_shell_len(A, NC) + L - 1) / L;
    for (int32_t g = 0; g < S && g < segs; ++g) {
      const int32_t q0 = g * L, q1 = (g + 1) * L - 1;  // quanta of the shell, 16 per chunk
      int32_t st = 0;
      for (int32_t d = 1 + q0 / 16; d <= 1 + q1 / 16; ++d) {
        const int32_t owner = sym_row_owner((A + d) % NC, NC, nranks);
        const int32_t k = ((rank - owner) % nranks + nranks) % nranks;
        if (k > st) st = k;
      }
      stage[(size_t)r * per + g] = (int8_t)st;
    }
  }
  std::vector<int32_t> nl(rows);
  std::vector<char> moved((size_t)total, 0);
  int64_t k = 0;
  for (int32_t r = 0; r < rows; ++r) {  // the local prefix, exactly as gs_sym_unit_map
    nl[r] = sym_local_segs(a0 + r, NC, a0, rows, L, S);
    for (int32_t q = 0; q < D && (fill < 0 || k < fill); ++q) {
      out[k++] = unit_entry(0u, r, S + q);
      moved[(size_t)r * per + S + q] = 1;
    }
    for (int32_t g = 0; g < nl[r] && (fill < 0 || k < fill); ++g) {
      out[k++] = unit_entry(0u, r, g);
      moved[(size_t)r * per + g] = 1;
    }
  }
  for (int32_t st = 0; st < nranks; ++st)
    for (int pass = 0; pass < 2; ++pass)
      for (int32_t r = 0; r < rows; ++r)
        for (int32_t u = pass ? S : 0; u < (pass ? per : S); ++u) {
          const size_t i = (size_t)r * per + u;
          if (moved[i] || stage[i] != st) continue;
          const uint32_t remote = st > 0 ? 0x80000000u : 0u;
          out[k++] = unit_entry(remote | ((uint32_t)st << 28), r, u);
        }
  return k;
}

// Whether the node sums rank `src` sends rank `dst` can be nonzero (1) or are +0.0 for every
// body by the geometry alone (0): no row of src's holds a chunk of dst's in its shell (chunk X
// is in row A's shell iff d = (X - A) mod NC is in [1, NC/2 - 1], or d = NC/2 and row A takes
// its antipodal chunk). The j-side sums of such a pair skip every row and stay +0.0, the
// identity of the receiver's tree merge, so the send can be skipped: the receiver's slots for
// those nodes hold the +0.0 they were zeroed to. At P = 8 three of a rank's seven destinations
// are far side (d > NC/2): 43 % less exchange. -1 on bad arguments.
extern "C" int32_t gs_sym_pair_live(int64_t n_pad, int32_t nranks, int32_t src, int32_t dst) {
  int32_t sa0, srows, da0, drows;
  if (src == dst) return 1;
  if (gs_sym_rank_rows(n_pad, nranks, src, &sa0, &srows) ||
      gs_sym_rank_rows(n_pad, nranks, dst, &da0, &drows))
    return -1;
  const int32_t NC = (int32_t)(n_pad / 2048);
  for (int32_t A = sa0; A < sa0 + srows; ++A) {
    const bool anti = gs_sym_shell_len(A, NC) == NC / 2;
    for (int32_t X = da0; X < da0 + drows; ++X) {
      const int32_t d = ((X - A) % NC + NC) % NC;
      if ((d >= 1 && d < NC / 2) || (d == NC / 2 && anti)) return 1;
    }
  }
  return 0;
}

// Partial-slot bytes of rank 0 (the largest share) if all of its rows were held at once (one
// band): Pi + Px (the split segments' extra parts) + Pj + Pd (3 elements per body per slot),
// the node sums it sends (nn x 3 per body of the run) and the ones it receives (NN x 3 per own
// body).
extern "C" int64_t gs_sym_bytes(int64_t n_pad, int32_t nranks, int32_t esz) {
  int32_t nc, h, l, sg, dp, a0, rows, nn, NN;
  if (gs_sym_geometry(n_pad, &nc, &h, &l, &sg, &dp) ||
      gs_sym_rank_rows(n_pad, nranks, 0, &a0, &rows) ||
      gs_sym_nodes(n_pad, nranks, 0, nullptr, nullptr, &nn, nullptr, &NN))
    return -1;
  const int64_t n_local = (int64_t)rows * 2048;
  const int64_t kx = (int64_t)gs_sym_split_segments(n_pad) * (gs_sym_split_parts(n_pad) - 1);
  return n_local * 3 * esz * ((int64_t)sg + kx + h + dp) +
         ((int64_t)nn * n_pad + (int64_t)NN * n_local) * 3 * esz;
}

extern "C" void gs_ic_fill_host(int32_t ic, uint64_t seed, int64_t n, int64_t begin, int64_t end,
                                double* pos, double* vel, double* mass) {
  if (end > n) end = n;
  for (int64_t i = begin; i < end; ++i) {
    double p[3], v[3], m;
    gs::ic_body(ic, seed, i, p, v, &m);
    const int64_t k = i - begin;
    if (pos) { pos[3 * k] = p[0]; pos[3 * k + 1] = p[1]; pos[3 * k + 2] = p[2]; }
    if (vel) { vel[3 * k] = v[0]; vel[3 * k + 1] = v[1]; vel[3 * k + 2] = v[2]; }
    if (mass) mass[k] = m;
  }
}
