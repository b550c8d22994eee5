// Probe-only pieces of the Newton-3 register tile (csrc/tools/sym_probe.hip): the round-1
// variant that holds the j positions in registers and rotates them lane to lane with DPP,
// and the DPP-folded subtraction whose issue cost the probe measures. Production reads the j
// positions from an LDS-staged tile instead (csrc/include/gs_sym_tile.h tile_lds_jp: one
// ds_read_b128 per j and step on the LDS pipe, 4 v_mov_dpp fewer per j and step); the results
// that decided it are in profiles/r1_sym_probe.jsonl and r1_sym_ab*.jsonl.
#pragma once
#include "gs_sym_tile.h"

namespace gs {
namespace sym {
namespace probe {

// a - b with `a` taken from lane l-O of the row, as one v_sub_f32_dpp. The compiler's DPP
// combiner folds a v_mov_b32_dpp only into a single use, so this is written out. A
// DPP-modified VALU op measured ~2.1 ns per wave-instruction against ~1.3 ns plain, so the
// tile fetches each j value once per step with v_mov_b32_dpp instead of folding DPP into its
// I consumers. The caller must not have written `a` with a VALU op in the two preceding
// instructions (DPP read hazard).
template <int O>
__device__ __forceinline__ float sub_from(float a, float b) {
  if constexpr (O % 16 == 0) {
    return a - b;
  } else {
    float d;
    asm("v_sub_f32_dpp %0, %1, %2 row_ror:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "=v"(d) : "v"(a), "v"(b), "i"(O));
    return d;
  }
}

template <int I>
using ISet = ISetT<float, I>;

template <int J>
struct JSet {
  float x[J], y[J], z[J], mu[J];
  float cx[J], cy[J], cz[J];  // carriers: j-side accumulators travelling with the j-bodies
};

// All I i-bodies of the lane against one j-body, i-pairs packed (two i-bodies per v_pk_*):
// i-side accumulators updated; with SYM the j side's sum over the lane's i-bodies is
// returned as t (two packed halves). 2 i-pairs per stage group, r^-3 = rsq(r^2)^3.
template <int I, bool SYM>
__device__ __forceinline__ void meet_j(ISet<I>& a, float xj, float yj, float zj, float mj,
                                       float eps2, f2& tx, f2& ty, f2& tz) {
  static_assert(I % 2 == 0, "i-bodies are processed in pairs");
  constexpr int U = (I / 2) % 2 == 0 ? 2 : 1;
#pragma unroll
  for (int i0 = 0; i0 < I; i0 += 2 * U) {
    f2 dx[U], dy[U], dz[U], r2[U], y[U], y3[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 2 * u;
      dx[u] = f2(xj) - f2{a.x[i], a.x[i + 1]};
      dy[u] = f2(yj) - f2{a.y[i], a.y[i + 1]};
      dz[u] = f2(zj) - f2{a.z[i], a.z[i + 1]};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) r2[u] = pk_fma(dx[u], dx[u], f2(eps2));
#pragma unroll
    for (int u = 0; u < U; ++u) r2[u] = pk_fma(dy[u], dy[u], r2[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) r2[u] = pk_fma(dz[u], dz[u], r2[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      y[u].x = __builtin_amdgcn_rsqf(r2[u].x);
      y[u].y = __builtin_amdgcn_rsqf(r2[u].y);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y[u] * y[u];
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y3[u] * y[u];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 2 * u;
      const f2 si = f2(mj) * y3[u];
      f2 ax = {a.ax[i], a.ax[i + 1]}, ay = {a.ay[i], a.ay[i + 1]}, az = {a.az[i], a.az[i + 1]};
      ax = pk_fma(si, dx[u], ax);
      ay = pk_fma(si, dy[u], ay);
      az = pk_fma(si, dz[u], az);
      a.ax[i] = ax.x; a.ax[i + 1] = ax.y;
      a.ay[i] = ay.x; a.ay[i + 1] = ay.y;
      a.az[i] = az.x; a.az[i + 1] = az.y;
    }
    if constexpr (SYM) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + 2 * u;
        const f2 sj = f2{a.mu[i], a.mu[i + 1]} * y3[u];
        if (i == 0) {
          tx = sj * dx[u]; ty = sj * dy[u]; tz = sj * dz[u];
        } else {
          tx = pk_fma(sj, dx[u], tx);
          ty = pk_fma(sj, dy[u], ty);
          tz = pk_fma(sj, dz[u], tz);
        }
      }
    }
  }
}

// One step: every lane meets the j-bodies of lane l-O of its row (v_mov_b32_dpp row_ror:O);
// the carrier of lane l-1 (the j this lane just met) moves here and takes -t.
template <int I, int J, bool SYM, int O>
__device__ __forceinline__ void step(ISet<I>& a, JSet<J>& b, float eps2) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    f2 tx, ty, tz;
    meet_j<I, SYM>(a, row_from<O>(b.x[j]), row_from<O>(b.y[j]), row_from<O>(b.z[j]),
                   row_from<O>(b.mu[j]), eps2, tx, ty, tz);
    if constexpr (SYM) {
      b.cx[j] = row_from<1>(b.cx[j]) - (tx.x + tx.y);
      b.cy[j] = row_from<1>(b.cy[j]) - (ty.x + ty.y);
      b.cz[j] = row_from<1>(b.cz[j]) - (tz.x + tz.y);
    }
  }
}

template <int I, int J, bool SYM, int... Os>
__device__ __forceinline__ void row_pass(ISet<I>& a, JSet<J>& b, float eps2,
                                         std::integer_sequence<int, Os...>) {
  (step<I, J, SYM, Os + 1>(a, b, eps2), ...);
}

template <int J, bool SYM>
__device__ __forceinline__ void next_row(JSet<J>& b, int addr) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    b.x[j] = wave_from_minus16(b.x[j], addr);
    b.y[j] = wave_from_minus16(b.y[j], addr);
    b.z[j] = wave_from_minus16(b.z[j], addr);
    b.mu[j] = wave_from_minus16(b.mu[j], addr);
    if constexpr (SYM) {
      b.cx[j] = wave_from_minus16(b.cx[j], addr);
      b.cy[j] = wave_from_minus16(b.cy[j], addr);
      b.cz[j] = wave_from_minus16(b.cz[j], addr);
    }
  }
}

// All (64 I) x (64 J) pairs of the wave's i-set and j-set. On return the j-set (positions
// and carriers) is back in its original lanes. Must be called by all 64 lanes (full exec).
template <int I, int J, bool SYM>
__device__ __forceinline__ void tile(ISet<I>& a, JSet<J>& b, float eps2) {
  const int addr = ((static_cast<int>(__lane_id()) + 48) & 63) << 2;
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    row_pass<I, J, SYM>(a, b, eps2, std::make_integer_sequence<int, 16>{});
    next_row<J, SYM>(b, addr);
  }
}

}  // namespace probe
}  // namespace sym
}  // namespace gs
