// Newton-3 (symmetric) register tile for the direct sum on gfx950 (fp32 and fp64).
//
// The reference's cuda.cu:53-60 visits each unordered pair once (j > i) and scatters the
// equal-and-opposite force into both bodies (cuda.cu:43-49), but does it with racy
// non-atomic global read-modify-writes. This tile keeps the "one pair,
// two interactions" saving without any scatter: each wave holds an i-set of 64*I bodies in
// registers, meets a j-tile of 64*J bodies and visits all (64 I) x (64 J) pairs, accumulating
//   * the i side in per-lane registers (as the one-sided kernels do), and
//   * the j side in per-lane "carrier" registers that travel with the j-bodies.
//
// Within a 16-lane row, at step k (k = 0..15) every lane meets the j-body of lane l-(k+1)
// (DPP row_ror:n reads lane l - n of the row; checked on gfx950). The carriers advance one
// lane per step with a single `v_sub_f32_dpp row_ror:1` that also subtracts the step's
// contribution, so the carrier of a j-body always sits in the lane currently meeting it.
// After 16 steps the carriers are home; they then move one row (16 lanes) with ds_bpermute,
// and after 4 such phases every lane has met every j of the tile. The j positions come
// either from an LDS-staged copy of the tile (`tile_lds`, the production path: one
// ds_read_b128 per j and step on the LDS pipe) or from registers rotated like the carriers
// (`tile`, `v_mov_b32_dpp row_ror:(k+1)`, fp32 only, kept as the GS_SYM_JLDS=0 A/B path).
//
// Cost per pair (two interactions), fp32: 3 sub + 3 FMA (r^2) + v_rsq_f32 + 2 mul (r^-3)
// + 2 mul (s_i, s_j) + 6 FMA/mul (both accumulators), all packed two pairs per v_pk_*
// instruction: 4 v_pk + 0.5 v_rsq per interaction, against 6 v_pk + 1 v_rsq for the
// one-sided loop (nbody_kernels.hip interact_pk). fp64: 20 f64 ops + 1 v_rsq_f64 per pair.
// fp32 ships the j-pair packed form (tile_lds_jp, below): the pair is the lane's two j-slots
// against one i-body, so the carriers need no fold of packed halves.
//
// Numerics: the pair term uses the fast-cutoff core (r^2 + eps2, nbody_kernels.hip FM_FAST)
// or, with EXACT, the reference hard cutoff as a select; r^-3 = (y*y)*y with y = rsq(r^2 +
// eps2) (fp64: the refined r^-3 of the one-sided fp64 path). The j-side term of a pair is the
// exact negation of what body j would compute for body i (x_i - x_j = -(x_j - x_i) in IEEE).
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <type_traits>
#include <utility>

namespace gs {
namespace sym {

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}

// Value of `v` held by lane (l - O) of the same 16-lane row (row_ror:O); O = 16 is identity.
template <int O>
__device__ __forceinline__ float row_from(float v) {
  if constexpr (O % 16 == 0) {
    return v;
  } else {
    return dpp<0x120 + O>(v);
  }
}

// a - b with `a` taken from lane l-O of the row, as one v_sub_f32_dpp. The compiler's DPP
// combiner folds a v_mov_b32_dpp only into a single use, so this is written out. Used by the
// DPP issue-cost probe (csrc/tools/sym_probe.hip): a DPP-modified VALU op measured ~2.1 ns
// per wave-instruction against ~1.3 ns plain, so the tile fetches each j value once per step
// with v_mov_b32_dpp instead of folding DPP into its I consumers. The caller must not have
// written `a` with a VALU op in the two preceding instructions (DPP read hazard).
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

// Value of `v` held by lane (l - 16) mod 64 (next row down, wave-wide).
__device__ __forceinline__ float wave_from_minus16(float v, int addr) {
  return __builtin_bit_cast(float,
                            __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, v)));
}

// fp64 counterparts of the cross-lane moves: one DPP / bpermute per 32-bit half.
template <int O>
__device__ __forceinline__ double row_from(double v) {
  if constexpr (O % 16 == 0) {
    return v;
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, 0x120 + O, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), 0x120 + O, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  }
}

__device__ __forceinline__ double wave_from_minus16(double v, int addr) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)u);
  const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

template <typename T, int I>
struct ISetT {
  T x[I], y[I], z[I], mu[I];
  T ax[I], ay[I], az[I];
};
template <int I>
using ISet = ISetT<float, I>;

template <int J>
struct JSet {
  float x[J], y[J], z[J], mu[J];
  float cx[J], cy[J], cz[J];  // carriers: j-side accumulators travelling with the j-bodies
};

// One step: every lane meets the j-bodies of lane l-O of its row. SYM = false is the
// one-sided variant (diagonal tiles: i-set == j-set, each ordered pair once on the i side).
using f2 = float __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// One step: every lane meets the j-bodies of lane l-O of its row. SYM = false is the
// one-sided variant (diagonal tiles: i-set == j-set, each ordered pair once on the i side).
//
// Arithmetic runs on pairs of i-bodies as 2-vectors, so everything but the rsq issues as
// v_pk_{add,mul,fma}_f32 (two interactions per instruction; a scalar VALU op costs the same
// issue slot as a packed one on gfx950, profiles/r1_sym_probe.jsonl). The j values are
// fetched once per step with v_mov_b32_dpp (DPP cannot modify VOP3P) and broadcast by op_sel.
// Per 2 pairs (4 interactions): 16 v_pk + 2 v_rsq_f32; per j and step: 4 v_mov_dpp +
// 3 v_add + 3 v_sub_dpp for the carriers.
#ifndef GS_SYM_U
#define GS_SYM_U 2
#endif
// r^-3 from rsq cubed (0) or rcp(r^2) * rsq(r^2) (1), fp32 tiles. 1 trades a v_pk_mul for a
// second transcendental and measured 7.9 % slower (1M 177.2 vs 164.3 ms, 65K 0.788 vs
// 0.726 ms, alternating runs, profiles/r2_rcp_ab.jsonl): the trans pipe is not free here,
// although an isolated stream hides 8 rsq behind 64 v_pk_fma (profiles/r2_trans_probe.jsonl).
#ifndef GS_SYM_RCP
#define GS_SYM_RCP 0
#endif
// All I i-bodies of the lane against one j-body (xj, yj, zj, mj): i-side accumulators updated;
// with SYM the j side's sum over the lane's i-bodies is returned as t (two packed halves).
// EXACT: the reference hard cutoff (cuda.cu:39, mpi.c:64), r^-3 := 0 when r^2 < cut2, so
// the pair contributes to neither side (also removes the self term of diagonal tiles).
template <int I, bool SYM, bool EXACT = false>
__device__ __forceinline__ void meet_j(ISet<I>& a, float xj, float yj, float zj, float mj,
                                       float eps2, f2& tx, f2& ty, f2& tz, float cut2 = 0.f) {
  static_assert(I % 2 == 0, "i-bodies are processed in pairs");
  // U i-pairs go through each stage together (stage-major source order), so consecutive
  // instructions are independent and the packed-result read hazard needs no s_nop.
  constexpr int U = (I / 2) % GS_SYM_U == 0 ? GS_SYM_U : 1;
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
#ifdef GS_SYM_PROBE_NO_RSQ  // timing probe only: what the transcendental costs in this loop
      y[u] = r2[u] * f2(0.5f);
#else
      y[u].x = __builtin_amdgcn_rsqf(r2[u].x);
      y[u].y = __builtin_amdgcn_rsqf(r2[u].y);
#endif
    }
#if GS_SYM_RCP
    // r^-3 = rcp(r^2) * rsq(r^2) (A/B variant, see GS_SYM_RCP)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      y3[u].x = __builtin_amdgcn_rcpf(r2[u].x);
      y3[u].y = __builtin_amdgcn_rcpf(r2[u].y);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y3[u] * y[u];
#else
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y[u] * y[u];
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y3[u] * y[u];
#endif
    if constexpr (EXACT) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        y3[u].x = r2[u].x >= cut2 ? y3[u].x : 0.f;
        y3[u].y = r2[u].y >= cut2 ? y3[u].y : 0.f;
      }
    }
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

template <int I, int J, bool SYM, int O>
__device__ __forceinline__ void step(ISet<I>& a, JSet<J>& b, float eps2) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    f2 tx, ty, tz;
    meet_j<I, SYM>(a, row_from<O>(b.x[j]), row_from<O>(b.y[j]), row_from<O>(b.z[j]),
                   row_from<O>(b.mu[j]), eps2, tx, ty, tz);
    if constexpr (SYM) {
      // carrier of lane l-1 (the j this lane just met) moves here and takes -t.
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

// ---------------------------------------------------------------------------------------
// LDS-position variant: the j positions are not held in registers and rotated with DPP;
// the workgroup stages each j-tile once into LDS and every lane reads the body it meets with
// one ds_read_b128 per j and step (the LDS pipe, not the VALU). Only the carriers rotate
// (DPP row_ror:1 each step, ds_bpermute by 16 lanes each phase), so per j and step the VALU
// overhead drops from 4 v_mov_dpp + 3 v_add + 3 v_sub_dpp to 3 v_add + 3 v_sub_dpp, and the
// 4*J position registers are freed.
//
// Staged layout, [J][4 row groups][32] float4: body (slot j, lane 16 g + c') is stored at
// entries 15 - c' and 31 - c' of (j, g). At phase p (row group data shifted by p) and step k,
// lane 16 R + c meets lane 16 ((R - p) & 3) + ((c - k - 1) & 15) (DPP row_ror:n reads lane
// l - n of the row; verified on gfx950), which sits at entry 16 - c + k in [1, 31]: a
// per-phase base address plus the immediate offset k.
template <typename T, int J>
struct CSetT {
  T cx[J], cy[J], cz[J];
};
template <int J>
using CSet = CSetT<float, J>;

template <typename T>
using Vec4 = typename std::conditional<sizeof(T) == 4, float4, double4>::type;

constexpr int kStagedRows = 128;  // V4 rows per j-slot in the staged layout

__device__ __forceinline__ int staged_entry(int lane_src, int copy) {
  const int g = lane_src >> 4, c = lane_src & 15;
  return g * 32 + (copy ? 31 - c : 15 - c);
}

// Scheduling regions of the fp64 hot block (GS_SYM_PIPE64, as GS_SYM_PIPE for fp32 below):
// 1 (default) reads the next step's j-body from LDS one step ahead and keeps LDS reads inside
// their step: 512K fp64 99.62-99.66 vs 100.09-100.19 ms, same bits; 2 also closes a region
// after every i-body (100.08-100.11 ms: the f64 chains then need s_nops); 0 neither
// (profiles/r3s2_sched_barrier_fp64_ab.jsonl).
#ifndef GS_SYM_PIPE64
#define GS_SYM_PIPE64 1
#endif
// (A/B) what may cross the fp64 step barrier: 0x0406 VALU, SALU, TRANS (default); 0 nothing
#ifndef GS_SYM_STEP_MASK64
#define GS_SYM_STEP_MASK64 0x0406
#endif
// fp64 pair arithmetic (no packed f64 VALU on gfx950): the integrator's own fp64 formula
// (nbody_kernels.hip interact, step path): y0 = v_rsq_f64(r^2), e = 1 - r^2 y0^2,
// r^-3 = y0^3 (1 + 3/2 e + 15/8 e^2) with |e| <= 1.1e-7, i.e. double-precision r^-3;
// w = r^-3 then feeds both sides: 20 f64 ops + 1 v_rsq_f64 per pair (two interactions)
// against 2 x (16 + 1) one-sided.
template <int I, bool SYM, bool EXACT = false>
__device__ __forceinline__ void meet_j(ISetT<double, I>& a, double xj, double yj, double zj,
                                       double mj, double eps2, double& tx, double& ty,
                                       double& tz, double cut2 = 0.0) {
  // Opaque constants (loop-invariant, eps2 finite): kept in VGPRs instead of being
  // re-materialised per pair (1.5 and 1.875 are not inline f64 constants).
  const double c15 = 1.5 + eps2 * 0.0, c1875 = 1.875 + eps2 * 0.0;
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const double dx = xj - a.x[i], dy = yj - a.y[i], dz = zj - a.z[i];
    const double r2 = __builtin_fma(dz, dz, __builtin_fma(dy, dy, __builtin_fma(dx, dx, eps2)));
    // EXACT (reference hard cutoff): the pair's r^-3 is 0 below the cutoff. One select on w
    // (as the fp32 tiles do): an inf/NaN formed below the cutoff (r = 0: rsq = inf, e = NaN)
    // never leaves it. Selecting the rsq input as well cost 2 more v_cndmask per pair.
    const double y0 = __builtin_amdgcn_rsq(r2);
    const double y2 = y0 * y0;
    const double e = __builtin_fma(-r2, y2, 1.0);
    const double corr = __builtin_fma(e, __builtin_fma(e, c1875, c15), 1.0);
    double w = (y2 * y0) * corr;
    if constexpr (EXACT) w = r2 >= cut2 ? w : 0.0;
    const double si = mj * w;
    a.ax[i] = __builtin_fma(si, dx, a.ax[i]);
    a.ay[i] = __builtin_fma(si, dy, a.ay[i]);
    a.az[i] = __builtin_fma(si, dz, a.az[i]);
    if constexpr (SYM) {
      const double sj = a.mu[i] * w;
      if (i == 0) {
        tx = sj * dx; ty = sj * dy; tz = sj * dz;
      } else {
        tx = __builtin_fma(sj, dx, tx);
        ty = __builtin_fma(sj, dy, ty);
        tz = __builtin_fma(sj, dz, tz);
      }
    }
#if GS_SYM_PIPE64 >= 2
    __builtin_amdgcn_sched_barrier(0);  // one i-body's temporaries in flight at a time
#endif
  }
}

template <typename T, int I, int J, bool SYM, bool EXACT, int K>
__device__ __forceinline__ void lds_step(ISetT<T, I>& a, CSetT<T, J>& c, const Vec4<T>* base,
                                         T eps2, T cut2) {
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const Vec4<T> q = base[j * kStagedRows + K];
    if constexpr (sizeof(T) == 4) {
      f2 tx, ty, tz;
      meet_j<I, SYM, EXACT>(a, q.x, q.y, q.z, q.w, eps2, tx, ty, tz, cut2);
      if constexpr (SYM) {
        c.cx[j] = row_from<1>(c.cx[j]) - (tx.x + tx.y);
        c.cy[j] = row_from<1>(c.cy[j]) - (ty.x + ty.y);
        c.cz[j] = row_from<1>(c.cz[j]) - (tz.x + tz.y);
      }
    } else {
      double tx, ty, tz;
      meet_j<I, SYM, EXACT>(a, q.x, q.y, q.z, q.w, eps2, tx, ty, tz, cut2);
      if constexpr (SYM) {
        c.cx[j] = row_from<1>(c.cx[j]) - tx;
        c.cy[j] = row_from<1>(c.cy[j]) - ty;
        c.cz[j] = row_from<1>(c.cz[j]) - tz;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// j-pair packed fp32 variant (J = 2): the two j-slots of a step form the packed pair and the
// lane's i-bodies are splat operands, instead of packing two i-bodies against one j. The
// pair arithmetic is the same 16 v_pk + 2 v_rsq per pair-pair, but the j-side sum of a step
// comes out as one packed value whose halves ARE the two carriers' increments: per step
// 6 v_sub_f32_dpp move the carriers, against 6 v_add (folding i-pair halves) + 6 v_sub_dpp.
// The i side accumulates packed (slot-0 and slot-1 halves) and is folded once per unit.
// Staged layout per entry (same entries as above): two float4, (x0, x1, y0, y1) and
// (z0, z1, mu0, mu1), so each ds_read_b128 lands packed pairs in register pairs. The 32-byte
// lane stride costs LDS bank conflicts (1.3e10 conflict cycles in 3 steps at 1M) but the LDS
// pipe has slack: two 16-byte planes remove them and measured 0.4 % slower (167.75 vs
// 167.07 ms, alternating runs, profiles/r1_sym_ab_jpack.jsonl).
template <int I>
struct ISetP {
  float x[I], y[I], z[I], mu[I];
  f2 ax[I], ay[I], az[I];
};

// i-bodies per stage group: each group's rsq burst is followed by an s_nop (trans-use
// hazard); 4 halves the groups. 1M: U 4 169.42 ms, U 2 170.6, U 8 170.2 (alternating runs,
// profiles/r1_sym_ab_jpack.jsonl).
// Scheduling regions of the hot block (GS_SYM_PIPE). LLVM's max-ILP scheduler, left alone
// with the unrolled 16-step block, hoists LDS reads of many steps to its top and interleaves
// the stage groups freely. 2 (default): each step reads the next step's j-pair from LDS and a
// barrier keeps LDS reads inside their step (ALU may cross it), and a full barrier closes every
// stage group, so one group's temporaries are in flight at a time: same instructions and bits,
// 1M 159.6-159.9 vs 162.4-162.5 ms (alternating runs, profiles/r3s2_sched_barrier_ab.jsonl).
// 1: the step barrier only (-0.8 %). 0: no barriers. A software pipeline that ran group n's
// geometry + rsq beside group n-1's accumulations in one region measured -0.5 % (not kept),
// groups of 2 i-bodies -0.6 %, and no form reaches 3 waves/SIMD without spilling.
#ifndef GS_SYM_PIPE
#define GS_SYM_PIPE 2
#endif
// Instruction kinds that may cross the group / step barriers (0: none; 0x0406: VALU, SALU,
// TRANS). Closing the step regions completely measured -1.0 % against letting ALU work cross
// them (1M 159.98-160.00 vs 161.48-161.66 ms, 65K 0.694 vs 0.700-0.702 ms, same bits;
// letting TRANS cross the group barriers instead: 159.7 vs 161.2 ms;
// profiles/r3s2_barrier_mask_ab.jsonl).
#ifndef GS_SYM_GROUP_MASK
#define GS_SYM_GROUP_MASK 0
#endif
#ifndef GS_SYM_STEP_MASK
#define GS_SYM_STEP_MASK 0
#endif
#ifndef GS_SYM_UP
#define GS_SYM_UP 4
#endif
template <int I, bool SYM, bool EXACT>
__device__ __forceinline__ void meet_jp(ISetP<I>& a, f2 xj, f2 yj, f2 zj, f2 mj, float eps2,
                                        f2& tx, f2& ty, f2& tz, float cut2) {
  constexpr int U = I % GS_SYM_UP == 0 ? GS_SYM_UP : 1;
#pragma unroll
  for (int i0 = 0; i0 < I; i0 += U) {
    f2 dx[U], dy[U], dz[U], r2[U], y[U], y3[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dx[u] = xj - f2(a.x[i0 + u]);
      dy[u] = yj - f2(a.y[i0 + u]);
      dz[u] = zj - f2(a.z[i0 + u]);
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
#if GS_SYM_RCP
    // r^-3 = rcp(r^2) * rsq(r^2) (A/B variant, see GS_SYM_RCP)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      y3[u].x = __builtin_amdgcn_rcpf(r2[u].x);
      y3[u].y = __builtin_amdgcn_rcpf(r2[u].y);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y3[u] * y[u];
#else
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y[u] * y[u];
#pragma unroll
    for (int u = 0; u < U; ++u) y3[u] = y3[u] * y[u];
#endif
    if constexpr (EXACT) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        y3[u].x = r2[u].x >= cut2 ? y3[u].x : 0.f;
        y3[u].y = r2[u].y >= cut2 ? y3[u].y : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u;
      const f2 si = mj * y3[u];
      a.ax[i] = pk_fma(si, dx[u], a.ax[i]);
      a.ay[i] = pk_fma(si, dy[u], a.ay[i]);
      a.az[i] = pk_fma(si, dz[u], a.az[i]);
    }
    if constexpr (SYM) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u;
        const f2 sj = f2(a.mu[i]) * y3[u];
        if (i == 0) {
          tx = sj * dx[u]; ty = sj * dy[u]; tz = sj * dz[u];
        } else {
          tx = pk_fma(sj, dx[u], tx);
          ty = pk_fma(sj, dy[u], ty);
          tz = pk_fma(sj, dz[u], tz);
        }
      }
    }
#if GS_SYM_PIPE >= 2
    __builtin_amdgcn_sched_barrier(GS_SYM_GROUP_MASK);  // one i-group's temporaries at a time
#endif
  }
}

template <int I, bool SYM, bool EXACT, int K>
__device__ __forceinline__ void lds_step_jp(ISetP<I>& a, CSetT<float, 2>& c, const float4* base,
                                            float eps2, float cut2) {
  const float4 p = base[2 * K], q = base[2 * K + 1];
  f2 tx, ty, tz;
  meet_jp<I, SYM, EXACT>(a, f2{p.x, p.y}, f2{p.z, p.w}, f2{q.x, q.y}, f2{q.z, q.w}, eps2, tx,
                         ty, tz, cut2);
  if constexpr (SYM) {
    c.cx[0] = row_from<1>(c.cx[0]) - tx.x;
    c.cx[1] = row_from<1>(c.cx[1]) - tx.y;
    c.cy[0] = row_from<1>(c.cy[0]) - ty.x;
    c.cy[1] = row_from<1>(c.cy[1]) - ty.y;
    c.cz[0] = row_from<1>(c.cz[0]) - tz.x;
    c.cz[1] = row_from<1>(c.cz[1]) - tz.y;
  }
}

// GS_SYM_PIPE >= 1: step K reads step K+1's j-pair from LDS before its own arithmetic, and a
// scheduling barrier closes the step (GS_SYM_STEP_MASK), so every ds_read stays inside it.
template <int I, bool SYM, bool EXACT, int K>
__device__ __forceinline__ void lds_step_jp_pipe(ISetP<I>& a, CSetT<float, 2>& c,
                                                 const float4* base, float4& p, float4& q,
                                                 float eps2, float cut2) {
  float4 pn, qn;
  if constexpr (K + 1 < 16) {
    pn = base[2 * (K + 1)];
    qn = base[2 * (K + 1) + 1];
  }
  f2 tx, ty, tz;
  meet_jp<I, SYM, EXACT>(a, f2{p.x, p.y}, f2{p.z, p.w}, f2{q.x, q.y}, f2{q.z, q.w}, eps2, tx,
                         ty, tz, cut2);
  if constexpr (SYM) {
    c.cx[0] = row_from<1>(c.cx[0]) - tx.x;
    c.cx[1] = row_from<1>(c.cx[1]) - tx.y;
    c.cy[0] = row_from<1>(c.cy[0]) - ty.x;
    c.cy[1] = row_from<1>(c.cy[1]) - ty.y;
    c.cz[0] = row_from<1>(c.cz[0]) - tz.x;
    c.cz[1] = row_from<1>(c.cz[1]) - tz.y;
  }
  if constexpr (K + 1 < 16) {
    p = pn;
    q = qn;
  }
  __builtin_amdgcn_sched_barrier(GS_SYM_STEP_MASK);  // closes the step (LDS reads stay in it)
}

template <int I, bool SYM, bool EXACT, int... Ks>
__device__ __forceinline__ void lds_row_pass_jp(ISetP<I>& a, CSetT<float, 2>& c,
                                                const float4* base, float eps2, float cut2,
                                                std::integer_sequence<int, Ks...>) {
#if GS_SYM_PIPE
  float4 p = base[0], q = base[1];
  (lds_step_jp_pipe<I, SYM, EXACT, Ks>(a, c, base, p, q, eps2, cut2), ...);
#else
  (lds_step_jp<I, SYM, EXACT, Ks>(a, c, base, eps2, cut2), ...);
#endif
}

// All (64 I) x 128 pairs against the pair-staged j-tile (LDS). Carriers return home.
template <int I, bool SYM, bool EXACT>
__device__ __forceinline__ void tile_lds_jp(ISetP<I>& a, CSetT<float, 2>& c, const float4* tile,
                                            float eps2, float cut2) {
  const int lane = static_cast<int>(__lane_id());
  const int R = lane >> 4, col = lane & 15;
  const int addr = ((lane + 48) & 63) << 2;
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    const float4* base = tile + 2 * (((R - p) & 3) * 32 + (16 - col));
    lds_row_pass_jp<I, SYM, EXACT>(a, c, base, eps2, cut2,
                                   std::make_integer_sequence<int, 16>{});
    if constexpr (SYM) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        c.cx[j] = wave_from_minus16(c.cx[j], addr);
        c.cy[j] = wave_from_minus16(c.cy[j], addr);
        c.cz[j] = wave_from_minus16(c.cz[j], addr);
      }
    }
  }
}

// fp64, J = 1, GS_SYM_PIPE64 >= 1: step K holds its j-body in q and reads step K + 1's.
template <typename T, int I, bool SYM, bool EXACT, int K>
__device__ __forceinline__ void lds_step_pipe(ISetT<T, I>& a, CSetT<T, 1>& c, const Vec4<T>* base,
                                              Vec4<T>& q, T eps2, T cut2) {
  Vec4<T> qn;
  if constexpr (K + 1 < 16) qn = base[K + 1];
  T tx, ty, tz;
  meet_j<I, SYM, EXACT>(a, q.x, q.y, q.z, q.w, eps2, tx, ty, tz, cut2);
  if constexpr (SYM) {
    c.cx[0] = row_from<1>(c.cx[0]) - tx;
    c.cy[0] = row_from<1>(c.cy[0]) - ty;
    c.cz[0] = row_from<1>(c.cz[0]) - tz;
  }
  if constexpr (K + 1 < 16) q = qn;
  __builtin_amdgcn_sched_barrier(GS_SYM_STEP_MASK64);  // LDS and VMEM stay in the step
}

template <typename T, int I, int J, bool SYM, bool EXACT, int... Ks>
__device__ __forceinline__ void lds_row_pass(ISetT<T, I>& a, CSetT<T, J>& c,
                                             const Vec4<T>* base, T eps2, T cut2,
                                             std::integer_sequence<int, Ks...>) {
#if GS_SYM_PIPE64
  if constexpr (sizeof(T) == 8 && J == 1) {
    Vec4<T> q = base[0];
    (lds_step_pipe<T, I, SYM, EXACT, Ks>(a, c, base, q, eps2, cut2), ...);
    return;
  }
#endif
  (lds_step<T, I, J, SYM, EXACT, Ks>(a, c, base, eps2, cut2), ...);
}

// All (64 I) x (64 J) pairs against the staged j-tile `tile` (LDS). Carriers return home.
template <typename T, int I, int J, bool SYM, bool EXACT>
__device__ __forceinline__ void tile_lds(ISetT<T, I>& a, CSetT<T, J>& c, const Vec4<T>* tile,
                                         T eps2, T cut2) {
  const int lane = static_cast<int>(__lane_id());
  const int R = lane >> 4, col = lane & 15;
  const int addr = ((lane + 48) & 63) << 2;
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    const Vec4<T>* base = tile + ((R - p) & 3) * 32 + (16 - col);
    lds_row_pass<T, I, J, SYM, EXACT>(a, c, base, eps2, cut2,
                                      std::make_integer_sequence<int, 16>{});
    if constexpr (SYM) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        c.cx[j] = wave_from_minus16(c.cx[j], addr);
        c.cy[j] = wave_from_minus16(c.cy[j], addr);
        c.cz[j] = wave_from_minus16(c.cz[j], addr);
      }
    }
  }
}

}  // namespace sym
}  // namespace gs
