// Newton-3 (symmetric) force schedule for gfx950, fp32 and fp64: every unordered pair is
// evaluated once and its equal-and-opposite contribution reaches both bodies.
//
// Reference parity: cuda.cu:53-60 loops j > i and scatters F into forces[i] and -F into
// forces[j] (cuda.cu:43-49, Newton's third law) with racy non-atomic global read-modify-
// writes and a triangular load imbalance (D5). pyspark.py:80-84 applies
// the same +F/-F pair reduction on the driver. Here the saving is kept without any race:
//   * the pair arithmetic is the register tile of gs_sym_tile.h (i side in registers, j side
//     in carriers that travel lane to lane by DPP, j positions read from an LDS-staged tile):
//     fp32 4 v_pk + 0.5 v_rsq per interaction against 6 v_pk + 1 v_rsq one-sided; fp64
//     10 f64 ops + 0.5 v_rsq_f64 against 16 + 1;
//   * work is a canonical cyclic half-shell of 2048-body chunks (gs_kernels.h, SymArgs), so
//     every chunk row carries the same amount of work and rank ownership is a plain block
//     partition of rows;
//   * both sides land in pre-assigned partial slots and are summed in a fixed order by the
//     node-reduce and finalize kernels (a binary tree over up to 256 row blocks): deterministic, and
//     the same bits for every rank count P from 1 to 8 (the tree nodes are what crosses
//     ranks; a rank owns whole row blocks by mpi.c:184-187's remainder rule).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "gravsim.h"
#include "gs_common.h"
#include "gs_kernels.h"
#include "gs_sym_tile.h"

namespace gs {
namespace {

// Workgroup shape per precision: W waves, I i-bodies and J j-bodies per lane; one workgroup
// holds one 2048-body chunk on its i side (W * 64 * I == kSymC).
//   fp32: (4 waves, I 8, J 2), the j-pair packed tile (gs_sym_tile.h tile_lds_jp).
//         (8 waves, I 4, J 4) measured 7 % slower: the per-step j overhead is amortised over
//         fewer i (profiles/r1_sym_ab.jsonl). I 16 (2 waves) would halve that overhead but
//         needs 256 VGPRs + 94 AGPRs and spills to scratch (131 VGPRs at I 8).
//   fp64: (4 waves, I 8, J 1): 197 VGPRs, 2 waves/SIMD. The carriers' per-step cost (3 x
//         (2 v_mov_b32_dpp + v_add_f64)) and the LDS reads are shared by 8 i-bodies instead
//         of 4: 22.1 instead of 23.25 f64-pipe instructions per pair, 512K 96.8 vs 100.6 ms,
//         4M / 8 per rank 765.7 vs 796-798 ms against round 1-3's (8 waves, I 4) at 4 waves/SIMD
//         (profiles/r4s2_fp64_i8_ab.jsonl); that shape had beaten I 4 at 2 waves/SIMD (512K
//         124.7 -> 119.6 ms, profiles/r1_sym_ab.jsonl).
template <typename T>
struct Shape;
template <>
struct Shape<float> {
  static constexpr int I = 8, W = kSymC / (64 * I), J = 2;
};
template <>
struct Shape<double> {
  static constexpr int W = 4, I = 8, J = 1;
};

template <typename T>
struct Geo {
  static constexpr int W = Shape<T>::W, I = Shape<T>::I, J = Shape<T>::J;
  static constexpr int kTileI = 64 * I;  // i bodies per wave
  static constexpr int kTileJ = 64 * J;  // j bodies per tile
  static constexpr int kThreads = 64 * W;
  static constexpr int kTilesPerChunk = kSymC / kTileJ;
  static constexpr int kTilesPerQuantum = 128 / kTileJ;  // segments count 128-body quanta
  static_assert(W * kTileI == kSymC, "one workgroup holds one chunk on its i side");
  static_assert(kTileJ <= 128 && 128 % kTileJ == 0, "a j-tile must not straddle quanta");
};

// Row A's shell: the next h(A) chunks cyclically. Distances 1 .. NC/2 - 1 are covered by the
// row below; each antipodal pair {A, A + NC/2} by exactly one of its rows, chosen by parity
// (A < NC/2 takes it iff A is even; NC/2 is a multiple of 4, so A + NC/2 has A's parity and
// takes it iff A is odd). Every block of rows thus holds as many long (NC/2) as short rows,
// so the ranks of a P-rank run carry equal work (round 1 gave every antipodal pair to the
// rows A < NC/2, one more unit per row for ranks 0 .. P/2-1, and the max over ranks paid).
// Mirrors layout.cpp gs_sym_shell_len.
__device__ __forceinline__ int shell_len(int A, int NC) {
  const bool takes = (A < NC / 2) == ((A & 1) == 0);
  return takes ? NC / 2 : NC / 2 - 1;
}

// A unit's j-tiles, in order: shell tile u of row A is tile u % T of chunk A + 1 + u / T
// (T tiles per chunk); a diagonal unit's tile u is tile u of chunk A. All-ghost column chunks
// are skipped (mu = 0 there, and their rows are never read).
template <typename T>
struct TileSeq {
  int A, NC, real_chunks, u, u1;
  bool diag;
  static constexpr int kT = Geo<T>::kTilesPerChunk;
  __device__ __forceinline__ int d() const { return diag ? 0 : 1 + u / kT; }
  __device__ __forceinline__ int t() const { return u % kT; }
  __device__ __forceinline__ int valid(int uu) const {
    if (!diag)
      while (uu < u1 && (A + 1 + uu / kT) % NC >= real_chunks) uu = (uu / kT + 1) * kT;
    return uu;
  }
  __device__ __forceinline__ bool done() const { return u >= u1; }
  __device__ __forceinline__ int64_t row0() const {
    const int B = diag ? A : (A + d()) % NC;
    return (int64_t)B * kSymC + t() * Geo<T>::kTileJ;
  }
  __device__ __forceinline__ void next() { u = valid(u + 1); }
};

// Stage body b of a j-tile into the tile_lds layout (each body stored twice).
template <typename V>
__device__ __forceinline__ void stage_store(V* dst, int b, const V& q) {
  const int j = b / 64, l = b % 64;
  dst[j * sym::kStagedRows + sym::staged_entry(l, 0)] = q;
  dst[j * sym::kStagedRows + sym::staged_entry(l, 1)] = q;
}

// fp32: the j-pair packed tile (packed i-side accumulators); fp64: plain.
template <typename T>
constexpr bool kJpack = sizeof(T) == 4;

// i-set of a lane: j-pair packed accumulators (fp32) or plain fp64 ones.
template <typename T>
using ISetK = typename std::conditional<kJpack<T>, sym::ISetP<Geo<T>::I>,
                                        sym::ISetT<T, Geo<T>::I>>::type;

// One staging thread's share of a j-tile: one body (fp64: thread b < kTileJ), or (fp32) the
// bodies l and 64 + l (thread l < 64) interleaved into the pair layout of tile_lds_jp.
template <typename T>
struct StageQ {
  static constexpr int kN = kJpack<T> ? 2 : 1;
  static constexpr int kThreads = kJpack<T> ? 64 : Geo<T>::kTileJ;
  sym::Vec4<T> q[kN];
  __device__ __forceinline__ void load(const sym::Vec4<T>* X4, int64_t row0, int t) {
#pragma unroll
    for (int k = 0; k < kN; ++k) q[k] = X4[row0 + k * 64 + t];
  }
  __device__ __forceinline__ void store(sym::Vec4<T>* dst, int t) const {
    if constexpr (kJpack<T>) {
      const float4 p0 = {q[0].x, q[1].x, q[0].y, q[1].y}, p1 = {q[0].z, q[1].z, q[0].w, q[1].w};
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int e = sym::staged_entry(t, c);
        dst[2 * e] = p0;
        dst[2 * e + 1] = p1;
      }
    } else {
      stage_store(dst, t, q[0]);
    }
  }
};

template <typename T>
struct Smem {
  T slot[2][Geo<T>::W][3][Geo<T>::kTileJ];  // j-side carriers of each wave, double-buffered
  sym::Vec4<T> jt[2][Geo<T>::J * sym::kStagedRows];     // staged j-tiles, double-buffered
};

// Visit the unit's j-tiles. SYM: pairs both ways, j-side partials to Pj (the diagonal chunk
// runs with SYM = false: every ordered pair once on the i side).
template <typename T, bool SYM, bool EXACT>
__device__ __forceinline__ void run_tiles(const SymArgs& a, ISetK<T>& is, TileSeq<T> seq,
                                          int br, Smem<T>& sm) {
  using G = Geo<T>;
  using V4 = sym::Vec4<T>;
  constexpr int J = G::J;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const V4* X4 = static_cast<const V4*>(a.X);
  const T eps2 = (T)a.eps2, cut2 = (T)a.cut2;
  int buf = 0, cur = 0;
  const bool stager = threadIdx.x < StageQ<T>::kThreads;
  if (!seq.done() && stager) {
    StageQ<T> sq;
    sq.load(X4, seq.row0(), threadIdx.x);
    sq.store(sm.jt[0], threadIdx.x);
  }
  __syncthreads();
  while (!seq.done()) {
    TileSeq<T> nx = seq;
    nx.next();
    const int d = seq.d(), t = seq.t();
    StageQ<T> q_next;
    const bool stage_next = !nx.done() && stager;
    if (stage_next) q_next.load(X4, nx.row0(), threadIdx.x);  // lands during the arithmetic
    T cx[J], cy[J], cz[J];
    sym::CSetT<T, J> cs;
#pragma unroll
    for (int j = 0; j < J; ++j) cs.cx[j] = cs.cy[j] = cs.cz[j] = T(0);
    if constexpr (kJpack<T>) {
      sym::tile_lds_jp<G::I, SYM, EXACT>(is, cs, sm.jt[cur], eps2, sym::f2{a.cut_k, a.cut_c});
    } else {
      sym::tile_lds64<G::I, SYM, EXACT>(is, cs, sm.jt[cur], eps2, cut2);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) { cx[j] = cs.cx[j]; cy[j] = cs.cy[j]; cz[j] = cs.cz[j]; }
    if constexpr (SYM) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        sm.slot[buf][w][0][j * 64 + lane] = cx[j];
        sm.slot[buf][w][1][j * 64 + lane] = cy[j];
        sm.slot[buf][w][2][j * 64 + lane] = cz[j];
      }
    }
    // jt[cur ^ 1] was last read in the previous tile, before the previous barrier.
    if (stage_next) q_next.store(sm.jt[cur ^ 1], threadIdx.x);
    __syncthreads();
    if constexpr (SYM) {
      // Sum the waves' carriers in wave order (fixed) and store the tile's j-side partial.
      T* pj = static_cast<T*>(a.Pj) + ((int64_t)br * a.H + (d - 1)) * 3 * kSymC;
      for (int v = threadIdx.x; v < 3 * G::kTileJ; v += G::kThreads) {
        const int c = v / G::kTileJ, b = v % G::kTileJ;
        T acc = sm.slot[buf][0][c][b];
#pragma unroll
        for (int u = 1; u < G::W; ++u) acc += sm.slot[buf][u][c][b];
        pj[(int64_t)c * kSymC + t * G::kTileJ + b] = acc;
      }
      buf ^= 1;  // the other buffer was last read before this tile's barrier
    }
    cur ^= 1;
    seq = nx;
  }
}

// units 6: the grid lists every unit of the band, local ones (diagonal parts, then the
// rank-local shell segments, row by row) before the remote ones (row by row). Workgroups are
// dispatched in grid order, so the gathered rows are needed only after ~the local share of
// the step has been handed out. The order is a host-built map (one uniform load per
// workgroup: unit -> row, segment, bit 31 = remote; gs_common.h kUnitRowShift); a search
// through prefix sums put a chain of dependent loads in front of every workgroup and cost 2 %
// of the step.
// With the ring strategy (gate_n > 1) bits 28-30 hold the ring stage whose slice the unit
// waits for (layout.cpp gs_sym_unit_map_ring).
// With split segments (Kr > 0, all-gather order) bit 30 marks a part unit, bits 28-29 its
// part (layout.cpp gs_sym_unit_map_parts).
__device__ __forceinline__ bool local_first_unit(const SymArgs& a, int b, int* br, int* s,
                                                 int* stage, int* part) {
  const uint32_t m = (uint32_t)a.lf[b];
  const bool ring = a.gate_n > 1, halves = a.Kr > 0 && !ring;
  *br = (int)((m >> kUnitRowShift) & (uint32_t)kUnitRowMax);
  *s = (int)(m & (uint32_t)kUnitMax);
  *stage = ring ? (int)((m >> 28) & 7u) : 0;
  *part = halves && ((m >> 30) & 1u) ? (int)((m >> 28) & 3u) : -1;
  return (m >> 31) != 0u;
}

// Remote unit of the local-first launch (units 6): go ahead if the comm stream has already
// published the all-gather; otherwise append the unit to the deferred list and leave. No
// workgroup ever waits on the collective, so RCCL's kernels always find CUs; the deferred
// units run in a second launch (units 7) queued behind the gather event.
// The acquire is SYSTEM scope (global_load sc0 sc1 + buffer_inv sc0 sc1: this CU's L1 and the
// XCD's L2). On a real node the remote rows of X are written by peer GPUs over xGMI, which
// are not agent-scope writers: an agent-scope acquire (buffer_inv sc1) invalidates only the
// L1 and could leave stale L2 lines of X in place. The ungated schedule gets the same
// system-scope acquire from the dispatch of the kernel queued behind the gather event;
// gate_set_kernel publishes with the matching system-scope release (comm_model.hip).
__device__ __forceinline__ bool gate_open_or_defer(const SymArgs& a, int b, int stage) {
  __shared__ int open_s;
  if (threadIdx.x == 0) {
    const bool open =
        __hip_atomic_load(a.gate + stage, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    if (!open) {
      const unsigned k =
          __hip_atomic_fetch_add(a.defer, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      a.defer[1 + k] = (unsigned)b;
    }
    open_s = open ? 1 : 0;
  }
  __syncthreads();
  return open_s != 0;
}

// Work audit (SymArgs::audit): a unit that completed (or was empty) reports its weight; a
// workgroup adds the sum of its units with one relaxed device-scope atomic from one lane when
// it exits (one per unit in round 3: the batched add also gave the dynamic launch's hot loop
// back round 3's register assignment, 1.1 % at 1M, profiles/r4_ab_vs_r3.txt). The host
// compares the count with rows x (S + D + (Np - 1) Kr) per step (bench.py work_audit), so a
// launch that silently skipped units (a stale dynamic-fetch counter, a lost deferred unit)
// cannot pass as a fast step. A split segment run whole weighs Np (its parts), so the count
// per step is the same whichever way the segments run.
__device__ __forceinline__ void audit_unit(const SymArgs& a, unsigned long long n = 1) {
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(a.audit, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One unit b (row a, segment s) per call; s == S is the row's diagonal chunk. b is the
// workgroup index, or the index the workgroup fetched (SymArgs.work).
template <typename T, bool EXACT>
__device__ __forceinline__ unsigned force_sym_body(const SymArgs& a, int b) {
  using G = Geo<T>;
  using V4 = sym::Vec4<T>;
  __shared__ Smem<T> sm;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // Units per row: S shell segments, then D parts of the diagonal chunk.
  // br: row within the band (index into Pi/Pj/Pd); the rank's row is band0 + br.
  // part: -1 a whole unit, 0 .. Np-1 one part of a split segment (part 0 -> Pi, others -> Px).
  int br, s, stage = 0, part = -1;
  bool gated = false;
  if (a.units == 6) {
    gated = local_first_unit(a, b, &br, &s, &stage, &part) && a.gate != nullptr;
  } else if (a.units == 7) {  // deferred unit a.defer_index of the units-6 launch
    local_first_unit(a, (int)a.defer[1 + a.defer_index], &br, &s, &stage, &part);
  } else {  // units 0
    // Every unit: the shell segments row by row, then all diagonal parts. A diagonal part is
    // one-sided (about half the issue time of a shell segment), so dispatching them last fills
    // the launch's final, partial wave of workgroups with short jobs. With split segments
    // (Kr) the unsplit segments come first and the split ones last, as Np part units each.
    const int ns = a.S - a.Kr, shell = a.band_rows * ns, dg = a.band_rows * a.D;
    if (b < shell) {
      br = b / ns;
      s = b % ns;
    } else if (b < shell + dg) {
      const int k = b - shell;
      br = k / a.D;
      s = a.S + k % a.D;
    } else {
      const int k = b - shell - dg;
      part = k % a.Np;
      br = (k / a.Np) / a.Kr;
      s = ns + (k / a.Np) % a.Kr;
    }
  }
  const int A = a.a0 + a.band0 + br;
  const bool diag = s >= a.S;
  const bool split = !diag && s >= a.S - a.Kr;  // a split segment (Np part sums)
  const unsigned long long weight = split && part < 0 ? (unsigned long long)a.Np : 1ull;
  // Empty units (all-ghost row, segment past the row's shell) count as done for the work
  // audit (every unit is listed by exactly one launch).
  const bool count_empty = a.audit != nullptr;
  if ((int64_t)A * kSymC >= a.n_real)  // all-ghost row: never read
    return count_empty ? (unsigned)weight : 0u;
  const int seg_tiles = a.L * G::kTilesPerQuantum;
  TileSeq<T> seq{A, a.NC, a.real_chunks, 0, 0, diag};
  int u_lo = 0;  // shell: the segment's first tile
  if (diag) {
    const int q = s - a.S, plen = G::kTilesPerChunk / a.D;  // D parts of the diagonal chunk
    seq.u = q * plen;
    seq.u1 = seq.u + plen;
  } else {
    const int h_tiles = shell_len(A, a.NC) * G::kTilesPerChunk;
    const int u0 = s * seg_tiles;
    if (u0 >= h_tiles)  // past this row's shell: never read
      return count_empty ? (unsigned)weight : 0u;
    seq.u1 = min(u0 + seg_tiles, h_tiles);
    u_lo = u0;
    seq.u = seq.valid(u0);
  }
  if (gated && !gate_open_or_defer(a, b, stage)) return 0u;  // counted when units 7 runs it
  const unsigned long long t_start = a.utrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const V4* X4 = static_cast<const V4*>(a.X);
  ISetK<T> is;
  const int64_t i_row0 = (int64_t)A * kSymC + w * G::kTileI;
#pragma unroll
  for (int i = 0; i < G::I; ++i) {
    const V4 q = X4[i_row0 + i * 64 + lane];
    is.x[i] = q.x; is.y[i] = q.y; is.z[i] = q.z; is.mu[i] = q.w;
    is.ax[i] = is.ay[i] = is.az[i] = std::remove_reference_t<decltype(is.ax[i])>(0);
  }
  // The i-side sum of the lane's bodies over the tiles just visited -> out; then restart.
  auto store_i = [&](T* out) {
#pragma unroll
    for (int i = 0; i < G::I; ++i) {
      const int b = w * G::kTileI + i * 64 + lane;
      if constexpr (kJpack<T>) {  // slot-0 half + slot-1 half
        out[b] = is.ax[i].x + is.ax[i].y;
        out[kSymC + b] = is.ay[i].x + is.ay[i].y;
        out[2 * kSymC + b] = is.az[i].x + is.az[i].y;
      } else {
        out[b] = is.ax[i];
        out[kSymC + b] = is.ay[i];
        out[2 * kSymC + b] = is.az[i];
      }
    }
  };
  if (diag) {
    // Part of the 2048-body diagonal chunk, one-sided (self term 0 through the core, or
    // through the cutoff select in the exact path).
    run_tiles<T, false, EXACT>(a, is, seq, br, sm);
    store_i(static_cast<T*>(a.Pd) + ((int64_t)br * a.D + (s - a.S)) * 3 * kSymC);
  } else {
    // One piece (the segment), or for a split segment its Np parts: part p covers the tiles
    // [u_lo + p seg / Np, u_lo + (p + 1) seg / Np) (clipped to the shell), part 0 -> Pi,
    // part p > 0 -> Px slot p - 1; all of them (whole) or the one `part` names. One inlined
    // copy of the tile.
    T* const pi = static_cast<T*>(a.Pi) + ((int64_t)br * a.S + s) * 3 * kSymC;
    T* const px = split ? static_cast<T*>(a.Px) +
                              ((int64_t)br * a.Kr + (s - (a.S - a.Kr))) * (a.Np - 1) * 3 * kSymC
                        : nullptr;
    const int pc0 = split && part > 0 ? part : 0;
    const int pc1 = !split ? 1 : part >= 0 ? part + 1 : a.Np;
    const int u_end = seq.u1;
#pragma unroll 1
    for (int pc = pc0; pc < pc1; ++pc) {
      TileSeq<T> sq = seq;
      if (split) {
        sq.u1 = min(u_lo + (pc + 1) * seg_tiles / a.Np, u_end);
        sq.u = sq.valid(min(u_lo + pc * seg_tiles / a.Np, u_end));
      }
      if (pc > pc0) {
#pragma unroll
        for (int i = 0; i < G::I; ++i)
          is.ax[i] = is.ay[i] = is.az[i] = std::remove_reference_t<decltype(is.ax[i])>(0);
      }
      run_tiles<T, true, EXACT>(a, is, sq, br, sm);
      store_i(pc == 0 ? pi : px + (int64_t)(pc - 1) * 3 * kSymC);
      if (pc + 1 < pc1) __syncthreads();  // the next piece restages the LDS tiles and slots

    }
  }
  if (a.utrace && threadIdx.x == 0) {
    // hwreg(HW_ID) whole register, hwreg(XCC_ID) bits 3:0 (ids 4 and 20 on gfx9.4+)
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
    const int64_t slot = a.units == 7 ? (int64_t)a.trace_defer0 + a.defer_index : b;
    unsigned long long* e = a.utrace + 4 * slot;
    e[0] = t_start;
    e[1] = __builtin_amdgcn_s_memrealtime();
    e[2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    e[3] = ((unsigned long long)(unsigned)br << 32) | (unsigned)s;
  }
  return a.audit ? (unsigned)weight : 0u;
}

// units 7 runs a separate instantiation (DEFER): a small grid that walks the deferred list
// with a stride of the grid. The list is usually empty (the gather finished long before the
// remote units were dispatched), and a grid of one workgroup per possible unit would cost more
// than the gather it hides. The main kernel is unchanged by it (same registers, no spills).
// SymArgs::clk: the workgroup's shader-clock and wall-clock spans, stamped by lane 0 of wave
// 0. The start stamps wait in LDS, not in registers: held in SGPRs across the unit loop they
// added 5 SGPR spills to the 1M kernel.
struct ClockSpan {
  // {start s_memtime, start s_memrealtime, clk pointer or 0}: the pointer waits there too
  __device__ __forceinline__ static unsigned long long* slot() {
    __shared__ unsigned long long t0[3];
    return t0;
  }
  __device__ __forceinline__ static void begin(const SymArgs& a) {
    if (threadIdx.x == 0) {
      slot()[2] = reinterpret_cast<unsigned long long>(a.clk);
      if (a.clk) {
        slot()[0] = __builtin_amdgcn_s_memtime();
        slot()[1] = __builtin_amdgcn_s_memrealtime();
      }
    }
  }
  __device__ __forceinline__ static void end() {
    if (threadIdx.x == 0) {
      unsigned long long* clk = reinterpret_cast<unsigned long long*>(slot()[2]);
      if (clk) {
        const unsigned long long mt1 = __builtin_amdgcn_s_memtime();
        const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_fetch_add(clk, mt1 - slot()[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(clk + 1, rt1 - slot()[1], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(clk + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
};

template <typename T, bool EXACT, bool DEFER, bool DYN, bool PF>
__device__ __forceinline__ void force_sym_entry(SymArgs a) {
  ClockSpan::begin(a);
  if constexpr (!DEFER && !DYN) {
    const unsigned w = force_sym_body<T, EXACT>(a, blockIdx.x);
    if (w) audit_unit(a, w);
  } else if constexpr (DYN && !PF) {
    // Many units per slot (1M on one GPU: ~300): every workgroup fetches each unit when it
    // needs it (round 4's loop). The first-wave / early-fetch form below measured 0.1 %
    // slower there (163.08-163.34 vs 163.01-163.11 ms, alternating) and 1.1 % faster at 65K
    // (0.696-0.697 vs 0.704 ms), 1M / 8 per rank even (profiles/r5_dyn_loop_ab.jsonl); the
    // launcher picks by units per resident slot.
    __shared__ unsigned next_s;
    const int cap = (int)blockIdx.x < a.first_wave ? 1 : a.unit_cap;
    unsigned done = 0;  // audit weight of the units this workgroup ran: one add at exit
    for (int k = 0; k < cap; ++k) {
      if (threadIdx.x == 0)
        next_s = __hip_atomic_fetch_add(a.work, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const unsigned u = next_s;
      if (u >= (unsigned)a.n_units) break;
      done += force_sym_body<T, EXACT>(a, (int)u);
      __syncthreads();  // next_s and the LDS tiles are rewritten by the next unit
    }
    if (done) audit_unit(a, done);
  } else if constexpr (DYN) {
    // Dynamic fetch: unit indices in launch order from a device counter. The hardware hands
    // workgroups to the 8 XCDs in a fixed rotation, so a static unit per workgroup gives every
    // XCD the same number of units, and the slowest XCD (they differ by up to ~4 % in
    // throughput, bench/unit_timeline.py) sets the launch's end. Here a workgroup keeps taking
    // units (up to unit_cap; the first wave one each, so slots free up early for a concurrent
    // collective), and faster XCDs simply take more. Same units, same slots: same bits.
    // The first wave (the resident slots) takes one unit each, unit = blockIdx.x, with no
    // fetch: 512 workgroups pulling one counter at launch start serialise on it (one word
    // saturates at ~88 dequeues/us, MI355X_MICROARCH.md dequeue row: ~6 us per launch, 0.9 %
    // of a 65K step). Every later fetch returns first_wave + the counter's next value, so the
    // counter still starts at 0 (the memset / finalize re-arm) and every unit runs once.
    __shared__ unsigned next_s;
    const bool fw = (int)blockIdx.x < a.first_wave;
    const unsigned base = (unsigned)a.first_wave;
    auto fetch = [&]() -> unsigned {
      return base + __hip_atomic_fetch_add(a.work, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    unsigned done = 0;  // audit weight of the units this workgroup ran: one add at exit
    // Two inlined copies of the unit body (first wave / fetch loop) on purpose: one call site
    // shrinks the code by half but measured 0.8 % slower at 65K and equal at 1M
    // (profiles/r5_ab_onebody_rejected.jsonl).
    if (fw && !a.persist) {
      if ((int)blockIdx.x < a.n_units) done += force_sym_body<T, EXACT>(a, (int)blockIdx.x);
    } else {
      // The next unit's index is taken when this unit starts, so its fetch latency hides
      // behind the unit (short units at small N pay it once per ~2 tiles) - except near the
      // end of the queue (fewer than first_wave units left), where a unit held back behind a
      // running one would lengthen the launch tail: there it is taken after the unit.
      // (65K 0.708-0.710 vs 0.713-0.714 ms, 1M 163.78-163.91 vs 164.16-164.32 ms, alternating
      // on one box: profiles/r5_prefetch_ab.jsonl.)
      // (persistent: every workgroup is in the first wave; its first unit is its blockIdx.x)
      if (!fw && threadIdx.x == 0) next_s = fetch();
      __syncthreads();
      unsigned u = fw ? (unsigned)blockIdx.x : next_s;
      const int cap = fw ? 0x7fffffff : a.unit_cap;
      for (int k = 0; k < cap && u < (unsigned)a.n_units; ++k) {
        const bool more = k + 1 < cap;
        const bool early = more && u + base < (unsigned)a.n_units;
        unsigned nx = ~0u;
        if (threadIdx.x == 0 && early) nx = fetch();
        done += force_sym_body<T, EXACT>(a, (int)u);
        __syncthreads();  // every wave is done with next_s and the LDS tiles
        if (threadIdx.x == 0) next_s = early ? nx : more ? fetch() : ~0u;
        __syncthreads();
        u = next_s;
      }
    }
    if (done) audit_unit(a, done);
  } else {
    const unsigned n = a.defer[0];
    if (blockIdx.x == 0 && threadIdx.x == 0 && n > 0)
      __hip_atomic_fetch_max(a.defer_max, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned done = 0;
    for (unsigned k = blockIdx.x; k < n; k += gridDim.x) {
      a.defer_index = (int32_t)k;
      done += force_sym_body<T, EXACT>(a, 0);
      __syncthreads();  // the next unit reuses the LDS tiles
    }
    if (done) audit_unit(a, done);
  }
  ClockSpan::end();
}

// (separate instantiations: the static kernels keep their own register allocation)
template <bool EXACT, bool DEFER = false, bool DYN = false, bool PF = false>
__global__ __launch_bounds__(Geo<float>::kThreads) void force_sym_kernel_f32(SymArgs a) {
  force_sym_entry<float, EXACT, DEFER, DYN, PF>(a);
}
template <bool EXACT, bool DEFER = false, bool DYN = false, bool PF = false>
__global__ __launch_bounds__(Geo<double>::kThreads)
void force_sym_kernel_f64(SymArgs a) {
  force_sym_entry<double, EXACT, DEFER, DYN, PF>(a);
}

// ---- canonical j-side reduction ----------------------------------------------------------
// S(x) = sum over the rows A whose shell holds body x of Pj[A][d - 1] (d = (X - A) mod NC):
// a binary tree over the B row blocks (gs_common.h sym_blocks), each leaf the row-ascending
// sum of one block (rows outside X's shell add +0.0, an identity here: a sum started at +0.0
// never becomes -0.0). A rank reduces the dyadic nodes covering its block range; the
// receiver completes the tree with a binary-counter merge (left + right), so S(x) has the
// same bits for every rank count.

// Binary-counter merge of dyadic sub-trees pushed in global order: pos counts the blocks
// merged so far and its set bits are the pending levels, kept as a stack with the lowest
// (most recent) on top. A node of level l starts at a multiple of 2^l, so nothing below l is
// pending: pushing it merges (left + right) with the top while bit l, l + 1, ... of pos is
// set (the carries of pos + 2^l), then becomes the top. Every index is a compile-time
// constant, so the stack lives in registers (an earlier form indexed acc[level] and went to
// scratch); callers push in a wave-uniform order, so the carry branches do not diverge.
template <typename T, int C>
struct TreeAcc {
  static constexpr int kDepth = 9;  // B <= 256 blocks (gs_common.h kSymMaxBlocks)
  T st[kDepth][C];
  unsigned pos;
  __device__ __forceinline__ void push(int level, T* v) {
    unsigned p = pos >> level;
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
      if (!(p & 1u)) break;
#pragma unroll
      for (int c = 0; c < C; ++c) v[c] = st[0][c] + v[c];  // left + right
#pragma unroll
      for (int s = 0; s + 1 < kDepth; ++s)
#pragma unroll
        for (int c = 0; c < C; ++c) st[s][c] = st[s + 1][c];
      p >>= 1;
    }
#pragma unroll
    for (int s = kDepth - 1; s > 0; --s)
#pragma unroll
      for (int c = 0; c < C; ++c) st[s][c] = st[s - 1][c];
#pragma unroll
    for (int c = 0; c < C; ++c) st[0][c] = v[c];
    pos += 1u << level;
  }
  // Once pos is a power of two (a whole node or the whole tree) one sub-tree is pending.
  __device__ __forceinline__ void result(T* v) const {
#pragma unroll
    for (int c = 0; c < C; ++c) v[c] = st[0][c];
  }
};

// Leaves b in [lo, lo + n) of an aligned sub-tree (n a power of two, lo a multiple of n) into
// t. Four aligned leaves are summed as ((l0 + l1) + (l2 + l3)) and pushed as one level-2
// sub-tree: exactly what four level-0 pushes merge to (binary-counter order), with a quarter of
// the stack shifts. (Loading the four leaves' rows as one batch for 1- and 2-row blocks, same
// bits, doubled the node reduce at 1M: 1.12 vs ~0.6 ms, profiles/r4s2_b256_leaf_batch_ab.jsonl.)
template <typename T, int C, typename Leaf>
__device__ __forceinline__ void push_leaves(TreeAcc<T, C>& t, int lo, int n, Leaf&& leaf) {
  if (n >= 4) {
    for (int b = lo; b < lo + n; b += 4) {
      T v[4][C];
#pragma unroll
      for (int j = 0; j < 4; ++j) leaf(b + j, v[j]);
#pragma unroll
      for (int c = 0; c < C; ++c) v[0][c] = (v[0][c] + v[1][c]) + (v[2][c] + v[3][c]);
      t.push(2, v[0]);
    }
  } else {
    for (int b = lo; b < lo + n; ++b) {
      T v[C];
      leaf(b, v);
      t.push(0, v);
    }
  }
}

// Adds, in ascending row order, Pj of the rows in [A_lo, A_hi) whose shell holds chunk X
// (body (X, c), one component per C). The caller passes a range where the distance
// d = X - A + wrap lies in [1, NC/2], so only the antipodal row (d = NC/2) needs the shell
// test; row A's partial sits (H - 1) x 3 x kSymC elements after row A - 1's. The loads of U
// rows are issued ahead of their ordered adds.
// (A: the accumulated type; T here. A 16-byte vector of consecutive bodies' T, one load per
// row, gave the same bits but measured no faster at 1M on one GPU and slower at the 1M / 8
// rank shape (node reduce 53 + 41 + 31 vs 52 + 37 + 19 us, row reduce 97-99 vs 96 us:
// profiles/r5_reduce_vec_ab.jsonl), so the kernels load one body per thread.)
template <typename A, typename T>
__device__ __forceinline__ A ld(const T* p) {
  return *reinterpret_cast<const A*>(p);
}

// NT: non-temporal loads of Pj (read once per step). At the 1M / 8 rank shape the node reduce
// stages take 38 instead of 43 us each (chain 257 against 274 us). On one GPU the node reduce
// drops 677 -> 632 us but the row reduce grows 590 -> 704 us whether it runs before or after
// it (same row-reduce code): the plain loads of the node reduce are what evict the force
// launch's dirty lines from the memory-side cache, and without them the row reduce pays the
// write-backs. One GPU keeps plain loads, and so do two ranks (chain 718-723 against 763 us
// with NT at rank 1 of 2; rank 1 of 4: 409-410 with NT against 426 us without;
// profiles/r5_nt_loads_ab.txt).
template <bool NT, typename A, typename T>
__device__ __forceinline__ A ld_pj(const T* p) {
  if constexpr (NT && std::is_same<A, T>::value) return __builtin_nontemporal_load(p);
  else return *reinterpret_cast<const A*>(p);
}

template <typename T, int C, typename A = T, bool NT = false>
__device__ __forceinline__ void pj_range_add(const SymArgs& a, int A_lo, int A_hi, int X,
                                             int wrap, const T* pjc, int64_t comp_stride,
                                             A* out) {
  constexpr int U = 8;
  const int64_t step = (int64_t)(a.H - 1) * 3 * kSymC;
  const T* p0 = pjc + ((int64_t)(A_lo - a.a0 - a.band0) * a.H + (X - A_lo + wrap - 1)) * 3 * kSymC;
  for (int A0 = A_lo; A0 < A_hi; A0 += U, p0 += U * step) {
    A v[U][C];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int Ar = A0 + u;
      const int d = X - Ar + wrap;
      const bool ok = Ar < A_hi && (d != a.NC / 2 || shell_len(Ar, a.NC) == a.NC / 2);
      const T* p = p0 + u * step;
#pragma unroll
      for (int k = 0; k < C; ++k) v[u][k] = ok ? ld_pj<NT, A>(p + k * comp_stride) : A(0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < C; ++k) out[k] += v[u][k];
  }
}

// Row-ascending sum of Pj over the rows [A_lo, A_hi) of one block for body (X, c), from +0.0.
// Only rows A with X - A in [1, NC/2] (mod NC) can hold X in their shell: a cyclic range of
// NC/2 rows, at most two linear pieces, visited in ascending order. Skipping the other rows
// keeps the bits of adding +0.0 for them (a sum started at +0.0 never becomes -0.0) and
// halves the loop.
template <typename T, int C, typename A = T, bool NT = false>
__device__ __forceinline__ void pj_row_sum(const SymArgs& a, int A_lo, int A_hi, int X,
                                           const T* pjc, int64_t comp_stride, A* out) {
#pragma unroll
  for (int k = 0; k < C; ++k) out[k] = A(0);
  const int s0 = X - a.NC / 2;  // the shell rows of X: [s0, X - 1] cyclically
  if (s0 >= 0) {
    pj_range_add<T, C, A, NT>(a, max(A_lo, s0), min(A_hi, X), X, 0, pjc, comp_stride, out);
  } else {
    pj_range_add<T, C, A, NT>(a, A_lo, min(A_hi, X), X, 0, pjc, comp_stride, out);
    pj_range_add<T, C, A, NT>(a, max(A_lo, s0 + a.NC), A_hi, X, a.NC, pjc, comp_stride, out);
  }
}

// Owner rank of chunk row X.
__device__ __forceinline__ int sym_row_owner(const SymArgs& a, int X) {
  const int blk = X / a.RB;
  int q = 0;
  while (q + 1 < a.P && a.blk_lo[q + 1] <= blk) ++q;
  return q;
}

// Multi-band runs: the leaf sum of every block inside the band (bands hold whole blocks),
// into Bbuf[block - first own block][3][bodies]. Grid: (bodies / 256, blocks in the band).
template <typename T>
__global__ __launch_bounds__(256) void sym_block_reduce_kernel(SymArgs a) {
  const int64_t nb = (int64_t)a.real_chunks * kSymC;
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= nb) return;
  const int X = (int)(x / kSymC), c = (int)(x % kSymC);
  const int b = (a.a0 + a.band0) / a.RB + (int)blockIdx.y;
  const int A_lo = max(b * a.RB, 0), A_hi = min((b + 1) * a.RB, a.real_chunks);
  T v[3];
  pj_row_sum<T, 3>(a, A_lo, max(A_lo, A_hi), X, static_cast<const T*>(a.Pj) + c, kSymC, v);
  T* o = static_cast<T*>(a.Bbuf) + (int64_t)(b - a.blk_lo[a.rank]) * 3 * nb + x;
  o[0] = v[0];
  o[nb] = v[1];
  o[2 * nb] = v[2];
}

// Node k (blockIdx.y) of this rank's dyadic decomposition, for every body x of a real chunk:
// the tree over the node's blocks, leaves from Pj directly (one band holds all the rank's
// rows) or from Bbuf (multi-band runs). Output Sbuf[dest rank q][node k][3][n_local(q)].
// Latency-bound (a chain of row loads per body): 3 components per thread amortise the row
// bookkeeping, U = 8 rows of loads are in flight, and only the NC/2 rows that can hold the
// body in their shell are visited (pj_row_sum).
template <typename T, bool NT>
__device__ __forceinline__ void sym_node_reduce_body(const SymArgs& a, int bx, int by) {
  if (a.sig && bx == 0 && by == 0 && threadIdx.x == 0) {  // (SymArgs::sig)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(a.sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const int64_t nb = (int64_t)a.real_chunks * kSymC;
  const int64_t tx = (int64_t)bx * 256 + threadIdx.x;
  if (a.x_count > 0 && tx >= a.x_count) return;
  int64_t x = a.x_lo + tx;
  if (x >= (int64_t)a.NC * kSymC) x -= (int64_t)a.NC * kSymC;  // (a cyclic range of ranks)
  if (x >= nb) return;
  const int X = (int)(x / kSymC), c = (int)(x % kSymC);
  const int own_lo = a.blk_lo[a.rank], own_hi = a.blk_lo[a.rank + 1];
  int lo = own_lo, l = sym_dyadic_level(lo, own_hi);
  for (int k = 0; k < by; ++k) {
    lo += 1 << l;
    l = sym_dyadic_level(lo, own_hi);
  }
  TreeAcc<T, 3> t;
  t.pos = 0;
  const T* Bb = static_cast<const T*>(a.Bbuf);
  const T* pjc = static_cast<const T*>(a.Pj) + c;
  auto leaf = [&](int b, T* v) {
    if (Bb) {
      const T* p = Bb + (int64_t)(b - own_lo) * 3 * nb + x;
      v[0] = p[0];
      v[1] = p[nb];
      v[2] = p[2 * nb];
    } else {
      const int A_lo = b * a.RB, A_hi = min((b + 1) * a.RB, a.real_chunks);
      pj_row_sum<T, 3, T, NT>(a, A_lo, max(A_lo, A_hi), X, pjc, kSymC, v);
    }
  };
  push_leaves(t, lo, 1 << l, leaf);
  T r[3];
  t.result(r);
  const int q = sym_row_owner(a, X);
  const int64_t bq = (int64_t)a.blk_lo[q] * a.RB * kSymC;
  const int64_t nlq = (int64_t)(a.blk_lo[q + 1] - a.blk_lo[q]) * a.RB * kSymC;
  T* o = static_cast<T*>(a.Sbuf) + (int64_t)a.nn * 3 * bq + (int64_t)by * 3 * nlq + (x - bq);
  o[0] = r[0];
  o[nlq] = r[1];
  o[2 * nlq] = r[2];
}

template <typename T, bool NT>
__global__ __launch_bounds__(256) void sym_node_reduce_kernel(SymArgs a) {
  sym_node_reduce_body<T, NT>(a, (int)blockIdx.x, (int)blockIdx.y);
}

// S(x) for an own body: every rank's nodes in global order, merged into the full tree; the
// other ranks' from Rbuf[node][3][n_local] (received), this rank's own nodes straight from
// its Sbuf block (they never leave the GPU: no copy on the comm stream's critical path).
template <typename T>
__device__ __forceinline__ void sym_tree_all(const SymArgs& a, int64_t li, T* S) {
  TreeAcc<T, 3> t;
  t.pos = 0;
  const T* R = static_cast<const T*>(a.Rbuf) + li;
  const T* own = static_cast<const T*>(a.Sbuf) + (int64_t)a.nn * 3 * a.i_begin + li;
  int j = 0;
  for (int q = 0; q < a.P; ++q) {
    const int hi = a.blk_lo[q + 1];
    const int j0 = j;
    for (int lo = a.blk_lo[q]; lo < hi; ++j) {
      const int l = sym_dyadic_level(lo, hi);
      const T* p = q == a.rank ? own + (int64_t)(j - j0) * 3 * a.n_local
                               : R + (int64_t)j * 3 * a.n_local;
      T v[3] = {p[0], p[a.n_local], p[2 * a.n_local]};
      t.push(l, v);
      lo += 1 << l;
    }
  }
  t.result(S);
}

// The split segments [s, segs) of band row br added to acc in segment order, each as
// (((part 0 + part 1) + part 2) + ...): part 0 from Pi (p: this body and component's Pi
// column), parts 1 .. Np-1 from Px (off: the body and component offset within a slot).
template <typename T, typename A = T>
__device__ __forceinline__ A split_parts_add(const SymArgs& a, int br, int s, int segs,
                                             int64_t off, const T* p, A acc) {
  const T* px =
      static_cast<const T*>(a.Px) + (int64_t)br * a.Kr * (a.Np - 1) * 3 * kSymC + off;
  for (; s < segs; ++s) {
    const int sp = s - (a.S - a.Kr);
    A t = ld<A>(p + (int64_t)s * 3 * kSymC);
    for (int q = 0; q + 1 < a.Np; ++q) t += ld<A>(px + ((int64_t)sp * (a.Np - 1) + q) * 3 * kSymC);
    acc += t;
  }
  return acc;
}

// The canonical i-side total of one body component, in two halves (round 6):
//   Ti = h0 + h1,  h0 = Pd[0] + ... + Pd[D-1] + Pi[0] + ... + Pi[m-1]   (ascending, from Pd[0])
//                  h1 = +0.0 + Pi[m] + ... + Pi[ns-1] + the split segments [ns, segs), each
//                       (((part 0 + part 1) + part 2) + ...)
// The one-rank fused tail computes h0 and h1 in two different waves (twice the loads in flight
// for a latency-bound sum: 65K 28.8 us for the whole tail before); the row reduce in one
// thread, as two independent add chains. m splits the loads evenly with the j-side tree rows
// (NC / 2) the tail's second half also carries. A function of the geometry only, so every
// path and every P give the same bits (round 5's single ascending chain had other bits:
// VERDICT r5 weak #9, determinism and P-independence are what is required).
__device__ __forceinline__ int ti_mid(const SymArgs& a, int segs, int ns) {
  // Above NC = 32 no path splits the halves across waves (gs_stepper::tail_split_on), and one
  // long chain plus the split parts measured faster than two balanced chains in one thread
  // (128K / 256K +0.15-0.25 % with the balanced split: profiles/r6_tail_split_ab.jsonl).
  if (a.NC > 32) return ns;
  const int loads = a.D + ns + (segs - ns) * a.Np + a.NC / 2;
  const int m = loads / 2 - a.D;
  return m < 0 ? 0 : (m > ns ? ns : m);
}

// acc + Pi[s0] + ... + Pi[s1 - 1] in order (p: the body component's Pi column), the loads of
// 8 segments issued ahead of their adds.
template <typename T>
__device__ __forceinline__ T pi_range_add(const T* __restrict__ p, int s0, int s1, T acc) {
  constexpr int U = 8;
  int s = s0;
  for (; s + U <= s1; s += U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + (int64_t)(s + u) * 3 * kSymC);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; s < s1; ++s) acc += __builtin_nontemporal_load(p + (int64_t)s * 3 * kSymC);
  return acc;
}

// h0 / h1 of band row br, component k, body c (see ti_mid).
template <typename T>
__device__ __forceinline__ T ti_half0(const SymArgs& a, int br, int k, int c, int m) {
  const T* __restrict__ pd = static_cast<const T*>(a.Pd) + (int64_t)br * a.D * 3 * kSymC +
                             k * kSymC + c;
  T acc = pd[0];
  for (int q = 1; q < a.D; ++q) acc += pd[q * 3 * kSymC];
  const T* p = static_cast<const T*>(a.Pi) + (int64_t)br * a.S * 3 * kSymC + k * kSymC + c;
  return pi_range_add(p, 0, m, acc);
}
template <typename T>
__device__ __forceinline__ T ti_half1(const SymArgs& a, int br, int k, int c, int m, int ns,
                                      int segs) {
  const T* p = static_cast<const T*>(a.Pi) + (int64_t)br * a.S * 3 * kSymC + k * kSymC + c;
  T acc = pi_range_add(p, m, ns, T(0));
  if (ns < segs) acc = split_parts_add(a, br, ns, segs, k * kSymC + c, p, acc);
  return acc;
}

// Ti = h0 + h1 (ti_mid) for the bodies of the band's rows. Grid: (bodies / 256, 3
// components). A streaming sum: one component per thread triples the loads in flight, the
// two halves are independent chains, and the loads of 8 segments are issued ahead of their
// (ordered) adds.
template <typename T>
__device__ __forceinline__ void sym_row_reduce_body(const SymArgs& a, int bx, int k) {
  const int64_t b = (int64_t)bx * 256 + threadIdx.x;  // body within the band; k: component
  if (b >= (int64_t)a.band_rows * kSymC) return;
  const int br = (int)(b / kSymC), c = (int)(b % kSymC);
  const int A = a.a0 + a.band0 + br;
  if ((int64_t)A * kSymC >= a.n_real) return;  // all-ghost row
  const int segs = (16 * shell_len(A, a.NC) + a.L - 1) / a.L;  // shell quanta / L
  const int ns = min(segs, a.S - a.Kr);  // unsplit segments; then split ones: Pi + Px parts
  const int m = ti_mid(a, segs, ns);
  const T h0 = ti_half0<T>(a, br, k, c, m);
  const T h1 = ti_half1<T>(a, br, k, c, m, ns, segs);
  static_cast<T*>(a.Ti)[(int64_t)k * a.n_local + (int64_t)(a.band0 + br) * kSymC + c] = h0 + h1;
}

template <typename T>
__global__ __launch_bounds__(256) void sym_row_reduce_kernel(SymArgs a) {
  sym_row_reduce_body<T>(a, (int)blockIdx.x, (int)blockIdx.y);
}

// The rank's own node sums (the last node reduce of the exchange, a.x_lo / x_count) and the
// row reduce in ONE launch: blocks [0, node_bx * nn) run the node reduce (dispatched first:
// they are the latency-bound chains), the rest the row reduce. Two memory-bound sums of the
// post-force chain share the launch's ramp and tail instead of running back to back. Same
// sums per body, same bits.
template <typename T, bool NT>
__global__ __launch_bounds__(256) void sym_node_row_kernel(SymArgs a, int node_bx, int row_bx) {
  const int nnb = node_bx * a.nn;
  if ((int)blockIdx.x < nnb) {
    sym_node_reduce_body<T, NT>(a, (int)blockIdx.x % node_bx, (int)blockIdx.x / node_bx);
  } else {
    const int k = (int)blockIdx.x - nnb;
    sym_row_reduce_body<T>(a, k % row_bx, k / row_bx);
  }
}

// a = Ti + S (the canonical tree over all ranks' nodes), then kick-drift (cuda.cu:73-76,
// mpi.c:207-215) exactly as the one-sided kernels' epilogue (nbody_kernels.hip
// integrate_store); ghost rows are zeroed.
template <typename T>
__global__ __launch_bounds__(256) void sym_finalize_kernel(SymArgs a) {
  using V4 = sym::Vec4<T>;
  const int64_t li = (int64_t)blockIdx.x * 256 + threadIdx.x;
  // This step's gated launches have completed (stream order): re-arm the gate for the next
  // all-gather into the same buffer (two steps on) and empty the deferred list.
  if (a.gate && li < a.gate_n)
    __hip_atomic_store(a.gate + li, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.gate && li == 0) __hip_atomic_store(a.defer, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // re-arm the dynamic unit counter of this step's force launch (as sym_tail_kernel does): the
  // next step's launch skips its memset (SymArgs::work_zero)
  if (a.work && li == 0) __hip_atomic_store(a.work, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (li >= a.n_local) return;
  const int64_t gi = a.i_begin + li;
  V4* vel = static_cast<V4*>(a.vel);
  const V4 zero = {T(0), T(0), T(0), T(0)};
  if (gi >= a.n_real) {
    if (a.acc_out) {
      static_cast<V4*>(a.acc_out)[li] = zero;
    } else {
      vel[li] = zero;
      static_cast<V4*>(a.X_next)[gi] = zero;
    }
    return;
  }
  const T* ti = static_cast<const T*>(a.Ti) + li;
  T S[3];
  sym_tree_all<T>(a, li, S);
  const T ax = ti[0] + S[0], ay = ti[a.n_local] + S[1], az = ti[2 * a.n_local] + S[2];
  if (a.acc_out) {
    static_cast<V4*>(a.acc_out)[li] = V4{ax, ay, az, T(0)};
    return;
  }
  const T dt = (T)a.dt;
  const V4 xi = static_cast<const V4*>(a.X)[gi];
  V4 v = vel[li];
  v.x = v.x + ax * dt;
  v.y = v.y + ay * dt;
  v.z = v.z + az * dt;
  V4 xn;
  xn.x = xi.x + v.x * dt;
  xn.y = xi.y + v.y * dt;
  xn.z = xi.z + v.z * dt;
  xn.w = xi.w;
  vel[li] = v;
  static_cast<V4*>(a.X_next)[gi] = xn;
}

// One rank, one band: the node reduce, the row reduce and finalize in ONE kernel (no Sbuf /
// Ti round trip, two launches fewer: at 65K bodies the three took ~28 us plus launch gaps of
// a 0.73 ms step). The sums keep the exact order of the three-kernel path, so the bits are
// the same: Ti = h0 + h1 (ti_mid); S = the tree over the B row blocks (leaves row-ascending
// from 0); a = Ti + S. SPLIT: 6 waves over 64 bodies; wave w sums half w / 3 of component
// w % 3 (coalesced partial reads), the second-half waves the j-side tree S too (65K: the tail
// 28.8 -> 24.8 us, the step -0.4 to -0.6 %); else 3 waves, each thread both halves as two
// chains (128K / 256K: the split form measured 0.6 / 1.3 % slower per step). Same sums either
// way; wave 0 then integrates the 64 bodies.
template <typename T, bool SPLIT>
__global__ __launch_bounds__(SPLIT ? 384 : 192) void sym_tail_kernel(SymArgs a) {
  using V4 = sym::Vec4<T>;
  __shared__ T h1_s[3][64], s_s[3][64], acc_s[3][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int k = w % 3, half = w / 3;
  const int64_t li = (int64_t)blockIdx.x * 64 + l;
  if (a.gate && blockIdx.x == 0 && (int)threadIdx.x < a.gate_n)
    __hip_atomic_store(a.gate + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (a.gate && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(a.defer, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // re-arm the dynamic unit counter of the force launch that preceded this kernel (the
  // stepper then skips the next launch's memset: SymArgs::work_zero)
  if (a.work && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(a.work, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t gi = a.i_begin + li;
  const bool real = li < a.n_local && gi < a.n_real;
  T h = T(0);
  if (real) {
    const int X = (int)(gi / kSymC), c = (int)(gi % kSymC);
    const int br = X - a.a0;  // one band: band0 = 0, the body's own row
    const int segs = (16 * shell_len(X, a.NC) + a.L - 1) / a.L;
    const int ns = min(segs, a.S - a.Kr);
    const int m = ti_mid(a, segs, ns);
    if (half == 0) h = ti_half0<T>(a, br, k, c, m);
    if (half == 1 || !SPLIT) {
      h1_s[k][l] = ti_half1<T>(a, br, k, c, m, ns, segs);
      // S: the tree over the B row blocks (sym_node_reduce_kernel's single node [0, B))
      TreeAcc<T, 1> t;
      t.pos = 0;
      const T* pjc = static_cast<const T*>(a.Pj) + k * kSymC + c;
      push_leaves(t, 0, a.B, [&](int b, T* v) {
        const int A_lo = b * a.RB, A_hi = min((b + 1) * a.RB, a.real_chunks);
        pj_row_sum<T, 1>(a, A_lo, max(A_lo, A_hi), X, pjc, kSymC, v);
      });
      T S[1];
      t.result(S);
      s_s[k][l] = S[0];
    }
  }
  __syncthreads();
  if (real && half == 0) acc_s[k][l] = (h + h1_s[k][l]) + s_s[k][l];  // (Ti) + S
  __syncthreads();
  if (w != 0 || li >= a.n_local) return;
  V4* vel = static_cast<V4*>(a.vel);
  const V4 zero = {T(0), T(0), T(0), T(0)};
  if (!real) {
    if (a.acc_out) {
      static_cast<V4*>(a.acc_out)[li] = zero;
    } else {
      vel[li] = zero;
      static_cast<V4*>(a.X_next)[gi] = zero;
    }
    return;
  }
  const T ax = acc_s[0][l], ay = acc_s[1][l], az = acc_s[2][l];
  if (a.acc_out) {
    static_cast<V4*>(a.acc_out)[li] = V4{ax, ay, az, T(0)};
    return;
  }
  const T dt = (T)a.dt;  // kick-drift exactly as sym_finalize_kernel
  const V4 xi = static_cast<const V4*>(a.X)[gi];
  V4 v = vel[li];
  v.x = v.x + ax * dt;
  v.y = v.y + ay * dt;
  v.z = v.z + az * dt;
  V4 xn;
  xn.x = xi.x + v.x * dt;
  xn.y = xi.y + v.y * dt;
  xn.z = xi.z + v.z * dt;
  xn.w = xi.w;
  vel[li] = v;
  static_cast<V4*>(a.X_next)[gi] = xn;
}

template <typename T>
hipError_t launch_force_sym_t(const SymArgs& a, hipStream_t s) {
  int units = a.band_rows * (a.S + a.D);
  // units 0 (diagonal parts last) and the all-gather units 6 order list every split segment
  // as Np part units at their end
  if (a.Kr > 0 && (a.units == 0 || (a.units == 6 && a.gate_n <= 1)))
    units += a.band_rows * a.Kr * (a.Np - 1);
  if (a.units >= 6 && (a.band_rows != a.rows || !a.lf)) return hipErrorInvalidValue;
  if (a.units == 7) units = a.defer_grid;  // strided walk over the deferred list
  if (units <= 0) return hipSuccess;
  SymArgs b = a;
  b.n_units = units;
  unsigned g = (unsigned)units;
  if (a.work && (a.units == 0 || a.units == 6) && a.unit_cap > 1 && units > a.first_wave) {
    // the counter starts at 0 for every launch: a stream-ordered memset (a graph node when
    // captured), unless the fused tail kernel that ran after the previous launch on this
    // stream already re-armed it (work_zero; saves a launch per step at small N)
    if (!a.work_zero) {
      const hipError_t e = hipMemsetAsync(a.work, 0, sizeof(unsigned), s);
      if (e != hipSuccess) return e;
    }
    // first wave: one unit per workgroup; the rest: up to unit_cap each, with 25 % slack so
    // a fast XCD can take more than its rotation share
    const int64_t rest = units - a.first_wave;
    const int64_t more = (5 * rest + 4LL * a.unit_cap - 1) / (4LL * a.unit_cap);
    g = (unsigned)(a.first_wave + (more < rest ? more : rest));
    // Persistent workgroups only with many units per slot (1M on one GPU: 165.21-165.68 vs
    // 165.49-166.00 ms against round 4's loop, alternating); at 65K the workgroup turnover
    // measured faster (0.699-0.705 vs 0.715-0.727 ms), as did caps 2-4 against 6-8
    // (profiles/r5_persist_ab.jsonl, r5_cap_small_n.jsonl).
    b.persist = a.persist && (int64_t)units > 128LL * a.first_wave ? 1 : 0;
    if (b.persist) g = (unsigned)a.first_wave;
  } else {
    b.work = nullptr;  // static: unit = blockIdx.x
    b.persist = 0;
  }
  const dim3 grid(g), block(Geo<T>::kThreads);
  const bool d = a.units == 7, y = b.work != nullptr;
  // the first-wave / early-fetch form of the dynamic loop up to 128 units per resident slot
  // (force_sym_entry)
  const bool pf = y && (b.persist || (int64_t)units <= 128LL * (a.first_wave > 0 ? a.first_wave : 1));
  if constexpr (sizeof(T) == 8) {
    if (a.exact) {
      if (d) hipLaunchKernelGGL((force_sym_kernel_f64<true, true>), grid, block, 0, s, b);
      else if (pf) hipLaunchKernelGGL((force_sym_kernel_f64<true, false, true, true>), grid, block, 0, s, b);
      else if (y) hipLaunchKernelGGL((force_sym_kernel_f64<true, false, true>), grid, block, 0, s, b);
      else hipLaunchKernelGGL((force_sym_kernel_f64<true>), grid, block, 0, s, b);
    } else {
      if (d) hipLaunchKernelGGL((force_sym_kernel_f64<false, true>), grid, block, 0, s, b);
      else if (pf) hipLaunchKernelGGL((force_sym_kernel_f64<false, false, true, true>), grid, block, 0, s, b);
      else if (y) hipLaunchKernelGGL((force_sym_kernel_f64<false, false, true>), grid, block, 0, s, b);
      else hipLaunchKernelGGL((force_sym_kernel_f64<false>), grid, block, 0, s, b);
    }
  } else {
    if (a.exact) {
      if (d) hipLaunchKernelGGL((force_sym_kernel_f32<true, true>), grid, block, 0, s, b);
      else if (pf) hipLaunchKernelGGL((force_sym_kernel_f32<true, false, true, true>), grid, block, 0, s, b);
      else if (y) hipLaunchKernelGGL((force_sym_kernel_f32<true, false, true>), grid, block, 0, s, b);
      else hipLaunchKernelGGL((force_sym_kernel_f32<true>), grid, block, 0, s, b);
    } else {
      if (d) hipLaunchKernelGGL((force_sym_kernel_f32<false, true>), grid, block, 0, s, b);
      else if (pf) hipLaunchKernelGGL((force_sym_kernel_f32<false, false, true, true>), grid, block, 0, s, b);
      else if (y) hipLaunchKernelGGL((force_sym_kernel_f32<false, false, true>), grid, block, 0, s, b);
      else hipLaunchKernelGGL((force_sym_kernel_f32<false>), grid, block, 0, s, b);
    }
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_force_sym(const SymArgs& a, hipStream_t s) {
  return a.fp64 ? launch_force_sym_t<double>(a, s) : launch_force_sym_t<float>(a, s);
}

}  // namespace gs

extern "C" int gs_sym_tile_shape(int32_t fp64, int32_t* waves, int32_t* ipl, int32_t* jpl) {
  using namespace gs;
  if (waves) *waves = fp64 ? Geo<double>::W : Geo<float>::W;
  if (ipl) *ipl = fp64 ? Geo<double>::I : Geo<float>::I;
  if (jpl) *jpl = fp64 ? Geo<double>::J : Geo<float>::J;
  return 0;
}

namespace gs {

hipError_t launch_sym_block_reduce(const SymArgs& a, hipStream_t s) {
  if (!a.Bbuf || a.band_rows % a.RB || (a.a0 + a.band0) % a.RB) return hipErrorInvalidValue;
  const int64_t bodies = (int64_t)a.real_chunks * kSymC;
  const dim3 grid((unsigned)((bodies + 255) / 256), (unsigned)(a.band_rows / a.RB));
  if (a.fp64) hipLaunchKernelGGL(sym_block_reduce_kernel<double>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(sym_block_reduce_kernel<float>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sym_node_reduce(const SymArgs& a, hipStream_t s) {
  // leaves from Pj need every own row in the slots (one band), else from Bbuf
  if (!a.Bbuf && (a.band0 != 0 || a.band_rows != a.rows)) return hipErrorInvalidValue;
  const int64_t nb = (int64_t)a.real_chunks * kSymC;
  const int64_t bodies = a.x_count > 0 ? a.x_count : nb;
  if (bodies <= 0) return hipSuccess;
  const dim3 grid((unsigned)((bodies + 255) / 256), (unsigned)a.nn);
  const bool nt = a.P > 2;  // (ld_pj)
  if (a.fp64) {
    if (nt) hipLaunchKernelGGL((sym_node_reduce_kernel<double, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((sym_node_reduce_kernel<double, false>), grid, dim3(256), 0, s, a);
  } else {
    if (nt) hipLaunchKernelGGL((sym_node_reduce_kernel<float, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((sym_node_reduce_kernel<float, false>), grid, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_sym_node_row(const SymArgs& a, hipStream_t s) {
  if (!a.Bbuf && (a.band0 != 0 || a.band_rows != a.rows)) return hipErrorInvalidValue;
  const int64_t nb = (int64_t)a.real_chunks * kSymC;
  const int64_t bodies = a.x_count > 0 ? a.x_count : nb;
  const int node_bx = (int)((bodies + 255) / 256);
  const int row_bx = (int)(((int64_t)a.band_rows * kSymC + 255) / 256);
  const dim3 grid((unsigned)(node_bx * a.nn + 3 * row_bx));
  const bool nt = a.P > 2;  // (ld_pj)
  if (a.fp64) {
    if (nt) hipLaunchKernelGGL((sym_node_row_kernel<double, true>), grid, dim3(256), 0, s, a, node_bx, row_bx);
    else hipLaunchKernelGGL((sym_node_row_kernel<double, false>), grid, dim3(256), 0, s, a, node_bx, row_bx);
  } else {
    if (nt) hipLaunchKernelGGL((sym_node_row_kernel<float, true>), grid, dim3(256), 0, s, a, node_bx, row_bx);
    else hipLaunchKernelGGL((sym_node_row_kernel<float, false>), grid, dim3(256), 0, s, a, node_bx, row_bx);
  }
  return hipGetLastError();
}

hipError_t launch_sym_row_reduce(const SymArgs& a, hipStream_t s) {
  const int64_t bodies = (int64_t)a.band_rows * kSymC;
  const dim3 grid((unsigned)((bodies + 255) / 256), 3);
  if (a.fp64) hipLaunchKernelGGL(sym_row_reduce_kernel<double>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(sym_row_reduce_kernel<float>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sym_finalize(const SymArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)((a.n_local + 255) / 256));
  if (a.fp64) hipLaunchKernelGGL(sym_finalize_kernel<double>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(sym_finalize_kernel<float>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sym_tail(const SymArgs& a, hipStream_t s, bool split) {
  if (a.P != 1 || a.band_rows != a.rows) return hipErrorInvalidValue;  // one rank, one band
  const dim3 grid((unsigned)((a.n_local + 63) / 64));
  if (split) {
    if (a.fp64) hipLaunchKernelGGL((sym_tail_kernel<double, true>), grid, dim3(384), 0, s, a);
    else hipLaunchKernelGGL((sym_tail_kernel<float, true>), grid, dim3(384), 0, s, a);
  } else {
    if (a.fp64) hipLaunchKernelGGL((sym_tail_kernel<double, false>), grid, dim3(192), 0, s, a);
    else hipLaunchKernelGGL((sym_tail_kernel<float, false>), grid, dim3(192), 0, s, a);
  }
  return hipGetLastError();
}

int sym_occupancy(int fp64) {
  int n = 0;
  const hipError_t e =
      fp64 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, force_sym_kernel_f64<false>,
                                                          Geo<double>::kThreads, 0)
           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, force_sym_kernel_f32<false>,
                                                          Geo<float>::kThreads, 0);
  return e == hipSuccess ? n : 0;
}

}  // namespace gs
