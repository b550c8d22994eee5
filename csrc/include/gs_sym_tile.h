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
// and after 4 such phases every lane has met every j of the tile. The j positions come from
// an LDS-staged copy of the tile: one ds_read_b128 per j and step on the LDS pipe, not the
// VALU. (Round 1 held them in registers and rotated them like the carriers, 4 more
// v_mov_dpp per j and step; that variant lives on only in the DPP probe,
// csrc/tools/sym_probe_tile.h.)
//
// Cost per pair (two interactions), fp32: 3 sub + 3 FMA (r^2) + v_rsq_f32 + 2 mul (r^-3)
// + 2 mul (s_i, s_j) + 6 FMA/mul (both accumulators), all packed two pairs per v_pk_*
// instruction: 4 v_pk + 0.5 v_rsq per interaction, against 6 v_pk + 1 v_rsq for the
// one-sided loop (nbody_kernels.hip interact_pk). fp32 packs the lane's two j-slots against
// one i-body (tile_lds_jp), so the two carriers' increments come out as the halves of one
// packed value. fp64: 20 f64 ops + 1 v_rsq_f64 per pair (tile_lds).
//
// Numerics: the pair term uses the fast-cutoff core (r^2 + eps2, nbody_kernels.hip FM_FAST)
// or, with EXACT, the reference hard cutoff (fp32: a clamp mask on r^2, cutoff_mask_r2; fp64:
// a select); r^-3 = (y*y)*y with y = rsq(r^2 +
// eps2) (fp64: the refined r^-3 of the one-sided fp64 path). The j-side term of a pair is the
// exact negation of what body j would compute for body i (x_i - x_j = -(x_j - x_i) in IEEE).
//
// Measured and not kept (git history has the code; profiles/ the numbers): r^-3 as
// rcp(r^2) * rsq(r^2) (+7.9 % at 1M: the trans pipe is not free, r2_rcp_ab.jsonl); i-pair
// packing instead of j-pair packing (r1_sym_ab_jpack.jsonl); 2 or 8 i-bodies per stage group
// (+0.7 %); no scheduling regions, or ALU allowed across the step barriers (+1.7 % / +1.0 %,
// r3s2_sched_barrier_ab.jsonl, r3s2_barrier_mask_ab.jsonl); an fp64 barrier per i-body
// (+0.5 %, r3s2_sched_barrier_fp64_ab.jsonl); the j side accumulated in LDS by no-return
// ds_add_f32 (6 per step, conflict-free, instead of the 6 v_sub_f32_dpp carrier moves: VALU
// 150 -> 144 per step) is 6.3x slower, 1030 vs 162.4 ms at 1M: an LDS float atomic costs the
// CU ~150 cycles per wave-instruction (r4s2_lds_atomic_carriers_ab.jsonl); a software-
// pipelined rsq (group g's rsq read two regions later, after group g+1's separations; 2
// i-bodies per group to stay in 256 VGPRs) is 1.3 % slower, 165.1 vs 163.1 ms, same bits
// (r4s2_rsq_pipeline_u2_ab.jsonl): the rsq latency is not what the tile waits on; i-body
// splats by op_sel from the (x, y) / (z, mu) pairs as loaded (inline asm: 231 -> 189 VGPRs,
// the compiler otherwise duplicates each coordinate into a register pair) +0.6 % at 2 waves
// per SIMD and +1.2 % at 3 (168 VGPRs), same bits (r4s2_opsel_occupancy3_ab.jsonl): more
// waves per SIMD do not raise this tile's issue rate; the carriers rotated by ds_bpermute at
// the top of each step with the j-side FMA chain starting from them (no v_sub_f32_dpp) keep
// the same cycles per pair but lower the power-limited engine clock, 2.22 -> 2.17 GHz:
// +2.2 % at 1M, +1.4 % fp64 (r6_carry_bpermute_rejected_ab.jsonl).
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

using f2 = float __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

// Reference hard cutoff for the packed fp32 tile (EXACT), bit-identical to the select
// `r2 >= cut2 ? r^-3 : 0` in two packed ops instead of two compares and two v_cndmask:
//   m  = clamp(fma(r2, -K, K cut2), 0, 1)   (ck = {-K, K cut2}, K a power of two, K cut2 ~ 2^40:
//        the fma is exact before its rounding, so its sign is that of cut2 - r2, and any
//        nonzero difference is >= one ulp of cut2, i.e. >= 2^16 after scaling: m is exactly 1
//        below the cutoff and exactly 0 at or above it; the VOP3P clamp bit is not emitted
//        for an elementwise min/max, hence the asm)
//   r2 = fma(m, FLT_MAX, r2)                (unchanged when m = 0; FLT_MAX below the cutoff, so
//        rsq ~ 5.4e-20 and its cube underflows to +0: the pair's r^-3 is exactly the select's
//        +0, and r = 0 never reaches the rsq as an inf)
// The ops this replaces cost the exact path +12.6 % over the fast core at 1M
// (profiles/r4s2_bench1m_kernel_stats_final.csv: 185.9 vs 165.0 ms).
__device__ __forceinline__ f2 cutoff_mask_r2(f2 r2, f2 ck) {
  f2 m;
  asm("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1] clamp"
      : "=v"(m)
      : "v"(r2), "s"(ck));
  return pk_fma(m, f2(3.40282347e38f), r2);
}

// Carriers of a lane's j-slots: the j-side accumulators travelling with the j-bodies.
template <typename T, int J>
struct CSetT {
  T cx[J], cy[J], cz[J];
};

template <typename T>
using Vec4 = typename std::conditional<sizeof(T) == 4, float4, double4>::type;

// ---------------------------------------------------------------------------------------
// LDS-staged j positions: the workgroup stages each j-tile once into LDS and every lane reads
// the body it meets with one ds_read_b128 per j and step; only the carriers rotate (DPP
// row_ror:1 each step, ds_bpermute by 16 lanes each phase).
//
// Staged layout, [J][4 row groups][32] entries: body (slot j, lane 16 g + c') is stored at
// entries 15 - c' and 31 - c' of (j, g). At phase p (row group data shifted by p) and step k,
// lane 16 R + c meets lane 16 ((R - p) & 3) + ((c - k - 1) & 15) (DPP row_ror:n reads lane
// l - n of the row; verified on gfx950), which sits at entry 16 - c + k in [1, 31]: a
// per-phase base address plus the immediate offset k.
constexpr int kStagedRows = 128;  // entries per j-slot in the staged layout

__device__ __forceinline__ int staged_entry(int lane_src, int copy) {
  const int g = lane_src >> 4, c = lane_src & 15;
  return g * 32 + (copy ? 31 - c : 15 - c);
}

// Instruction kinds that may cross the fp64 step barrier: VALU, SALU and TRANS (0x0406);
// LDS and VMEM stay inside their step.
constexpr int kStepMask64 = 0x0406;

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
  }
}

// ---------------------------------------------------------------------------------------
// fp32, j-pair packed (J = 2): the two j-slots of a step form the packed pair and the lane's
// i-bodies are splat operands. The pair arithmetic is 16 v_pk + 2 v_rsq per pair-pair, and
// the j-side sum of a step comes out as one packed value whose halves ARE the two carriers'
// increments: per step 6 v_sub_f32_dpp move the carriers. The i side accumulates packed
// (slot-0 and slot-1 halves) and is folded once per unit. Staged layout per entry: two
// float4, (x0, x1, y0, y1) and (z0, z1, mu0, mu1), so each ds_read_b128 lands packed pairs in
// register pairs. The 32-byte lane stride costs LDS bank conflicts (1.3e10 conflict cycles in
// 3 steps at 1M) but the LDS pipe has slack: two 16-byte planes remove them and measured
// 0.4 % slower (167.75 vs 167.07 ms, alternating runs, profiles/r1_sym_ab_jpack.jsonl).
template <int I>
struct ISetP {
  float x[I], y[I], z[I], mu[I];
  f2 ax[I], ay[I], az[I];
};

// i-bodies per stage group: each group's rsq burst is followed by an s_nop (trans-use
// hazard); 4 halves the groups. 1M: 4 169.42 ms, 2 170.6, 8 170.2 (alternating runs,
// profiles/r1_sym_ab_jpack.jsonl).
constexpr int kGroupI = 4;

// Scheduling regions of the hot block. LLVM's max-ILP scheduler, left alone with the
// unrolled 16-step block, hoists LDS reads of many steps to its top and interleaves the stage
// groups freely. Here each step reads the next step's j-pair from LDS, a barrier closes every
// stage group (one group's temporaries in flight at a time) and a barrier that nothing may
// cross closes every step (its LDS reads stay inside it): same instructions and bits, 1M
// 159.98 vs 162.4 ms (profiles/r3s2_sched_barrier_ab.jsonl, r3s2_barrier_mask_ab.jsonl).
template <int I, bool SYM, bool EXACT>
__device__ __forceinline__ void meet_jp(ISetP<I>& a, f2 xj, f2 yj, f2 zj, f2 mj, float eps2,
                                        f2& tx, f2& ty, f2& tz, f2 ck) {
  constexpr int U = I % kGroupI == 0 ? kGroupI : 1;
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
    if constexpr (EXACT) {
#pragma unroll
      for (int u = 0; u < U; ++u) r2[u] = cutoff_mask_r2(r2[u], ck);
    }
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
    __builtin_amdgcn_sched_barrier(0);  // one i-group's temporaries at a time
  }
}

// Step K: read step K+1's j-pair from LDS before this step's arithmetic; a scheduling barrier
// closes the step, so every ds_read stays inside it.
template <int I, bool SYM, bool EXACT, int K>
__device__ __forceinline__ void lds_step_jp(ISetP<I>& a, CSetT<float, 2>& c, const float4* base,
                                            float4& p, float4& q, float eps2, f2 ck) {
  float4 pn, qn;
  if constexpr (K + 1 < 16) {
    pn = base[2 * (K + 1)];
    qn = base[2 * (K + 1) + 1];
  }
  f2 tx, ty, tz;
  meet_jp<I, SYM, EXACT>(a, f2{p.x, p.y}, f2{p.z, p.w}, f2{q.x, q.y}, f2{q.z, q.w}, eps2, tx,
                         ty, tz, ck);
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
  __builtin_amdgcn_sched_barrier(0);  // closes the step (LDS reads stay in it)
}

template <int I, bool SYM, bool EXACT, int... Ks>
__device__ __forceinline__ void lds_row_pass_jp(ISetP<I>& a, CSetT<float, 2>& c,
                                                const float4* base, float eps2, f2 ck,
                                                std::integer_sequence<int, Ks...>) {
  float4 p = base[0], q = base[1];
  (lds_step_jp<I, SYM, EXACT, Ks>(a, c, base, p, q, eps2, ck), ...);
}

// All (64 I) x 128 pairs against the pair-staged j-tile (LDS). Carriers return home.
template <int I, bool SYM, bool EXACT>
__device__ __forceinline__ void tile_lds_jp(ISetP<I>& a, CSetT<float, 2>& c, const float4* tile,
                                            float eps2, f2 ck) {
  const int lane = static_cast<int>(__lane_id());
  const int R = lane >> 4, col = lane & 15;
  const int addr = ((lane + 48) & 63) << 2;
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    const float4* base = tile + 2 * (((R - p) & 3) * 32 + (16 - col));
    lds_row_pass_jp<I, SYM, EXACT>(a, c, base, eps2, ck,
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

// ---------------------------------------------------------------------------------------
// fp64, J = 1: step K holds its j-body in q and reads step K + 1's (one step ahead, kept
// inside the step by the barrier): 512K fp64 99.62-99.66 vs 100.09-100.19 ms without the
// regions, same bits (profiles/r3s2_sched_barrier_fp64_ab.jsonl).
template <int I, bool SYM, bool EXACT, int K>
__device__ __forceinline__ void lds_step64(ISetT<double, I>& a, CSetT<double, 1>& c,
                                           const double4* base, double4& q, double eps2,
                                           double cut2) {
  double4 qn;
  if constexpr (K + 1 < 16) qn = base[K + 1];
  double tx, ty, tz;
  meet_j<I, SYM, EXACT>(a, q.x, q.y, q.z, q.w, eps2, tx, ty, tz, cut2);
  if constexpr (SYM) {
    c.cx[0] = row_from<1>(c.cx[0]) - tx;
    c.cy[0] = row_from<1>(c.cy[0]) - ty;
    c.cz[0] = row_from<1>(c.cz[0]) - tz;
  }
  if constexpr (K + 1 < 16) q = qn;
  __builtin_amdgcn_sched_barrier(kStepMask64);  // LDS and VMEM stay in the step
}

template <int I, bool SYM, bool EXACT, int... Ks>
__device__ __forceinline__ void lds_row_pass64(ISetT<double, I>& a, CSetT<double, 1>& c,
                                               const double4* base, double eps2, double cut2,
                                               std::integer_sequence<int, Ks...>) {
  double4 q = base[0];
  (lds_step64<I, SYM, EXACT, Ks>(a, c, base, q, eps2, cut2), ...);
}

// All (64 I) x 64 pairs against the staged fp64 j-tile `tile` (LDS). Carriers return home.
template <int I, bool SYM, bool EXACT>
__device__ __forceinline__ void tile_lds64(ISetT<double, I>& a, CSetT<double, 1>& c,
                                           const double4* tile, double eps2, double cut2) {
  const int lane = static_cast<int>(__lane_id());
  const int R = lane >> 4, col = lane & 15;
  const int addr = ((lane + 48) & 63) << 2;
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    const double4* base = tile + ((R - p) & 3) * 32 + (16 - col);
    lds_row_pass64<I, SYM, EXACT>(a, c, base, eps2, cut2,
                                  std::make_integer_sequence<int, 16>{});
    if constexpr (SYM) {
      c.cx[0] = wave_from_minus16(c.cx[0], addr);
      c.cy[0] = wave_from_minus16(c.cy[0], addr);
      c.cz[0] = wave_from_minus16(c.cz[0], addr);
    }
  }
}

}  // namespace sym
}  // namespace gs
