// Shared host/device helpers: canonical layout math and the counter-based IC generator.
//
// Both are world-size independent by construction, which is what makes a P-rank run
// bitwise-equal to a 1-rank run (fixes the reference's rank-count-dependent results,
// SURVEY.md §2.7 D6, and its unseeded RNGs, D11: cuda.cu:127, mpi.c:96, pyspark.py:146-148).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GS_HD __host__ __device__ __forceinline__
#else
#define GS_HD static inline
#endif

namespace gs {

// Physical constants and reference ICs (cuda.cu:11,81-96; mpi.c:9,75-95; pyspark.py:46,124-141).
constexpr double kG = 6.67430e-11;
constexpr double kPosLo = -3e11, kPosHi = 3e11;
constexpr double kVelLo = -3e4, kVelHi = 3e4;
constexpr double kMassLo = 1e23, kMassHi = 1e25;

GS_HD uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Uniform double in [0, 1) for (seed, body, stream). Streams: 0-2 position, 3-5 velocity, 6 mass.
GS_HD double uniform01(uint64_t seed, uint64_t body, uint32_t stream) {
  const uint64_t key = mix64(seed ^ 0xD1B54A32D192ED03ull);
  const uint64_t h = mix64(key ^ (body * 16ull + stream));
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);  // 2^-53
}

// lo + (hi - lo) * u evaluated as two separately rounded fp64 operations (no FMA), the
// same as the NumPy implementation in gravsim/models/initial_conditions.py.
GS_HD double affine(double lo, double hi, double u) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __dadd_rn(lo, __dmul_rn(hi - lo, u));
#else
  volatile double prod = (hi - lo) * u;
  return lo + prod;
#endif
}

// One body of an IC family. ic: 0 = solar+random, 1 = random.
GS_HD void ic_body(int ic, uint64_t seed, int64_t i, double p[3], double v[3], double* m) {
  if (ic == 0 && i < 3) {
    // Sun, Earth, Mars (cuda.cu:82-93; mpi.c:79-93)
    const double px[3] = {0.0, 1.496e11, 2.279e11};
    const double vy[3] = {0.0, 29.78e3, 24.077e3};
    const double mm[3] = {1.989e30, 5.972e24, 6.39e23};
    p[0] = px[i]; p[1] = 0.0; p[2] = 0.0;
    v[0] = 0.0; v[1] = vy[i]; v[2] = 0.0;
    *m = mm[i];
    return;
  }
  for (int d = 0; d < 3; ++d) p[d] = affine(kPosLo, kPosHi, uniform01(seed, (uint64_t)i, d));
  for (int d = 0; d < 3; ++d) v[d] = affine(kVelLo, kVelHi, uniform01(seed, (uint64_t)i, 3 + d));
  *m = affine(kMassLo, kMassHi, uniform01(seed, (uint64_t)i, 6));
}

// Canonical j-chunk length: a function of N only (never of the rank count).
GS_HD int32_t auto_chunk(int64_t n) {
  int64_t p = 1;
  while (p < n) p <<= 1;
  int64_t c = p / 64;
  if (c < 2048) c = 2048;
  if (c > 65536) c = 65536;
  return (int32_t)c;
}

GS_HD int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

// ---- Newton-3 (sym) schedule: row blocks, rank ownership, canonical reduction tree -------
// The NC chunk rows are cut into B row blocks (B = the largest power of two <= 256 dividing
// NC, a function of n_pad only). Rank r of P owns blocks [sym_blk_lo(r), sym_blk_lo(r + 1))
// by the reference's remainder rule (mpi.c:184-187: the first B mod P ranks hold one more),
// so every P from 1 to 8 gets a balanced share of whole blocks: at 1M (NC 512, B 256) the
// busiest of 7 ranks holds 37 blocks against a mean of 36.6 (1.2 %; 64 blocks gave 10 against
// 9.1, 9.4 %), while a P dividing 8 still owns one aligned node. The j-side sums reach a body
// as a binary tree over the B blocks (each leaf a row-ascending sum), so the bits depend on
// n_pad only: a rank sends the dyadic sub-trees covering its block range, and the receiver
// completes the same tree (binary-counter merge, left + right).
constexpr int32_t kSymMaxBlocks = 256;
GS_HD int32_t sym_blocks(int32_t NC) {
  int32_t b = kSymMaxBlocks;
  while (b > 1 && NC % b) b >>= 1;
  return b;
}
GS_HD int32_t sym_blk_lo(int32_t B, int32_t P, int32_t r) {
  const int32_t base = B / P, rem = B % P;
  return r * base + (r < rem ? r : rem);
}
// Level of the dyadic node that starts at block lo inside [lo, hi): the largest l with
// lo % 2^l == 0 and lo + 2^l <= hi (maximal nodes).
GS_HD int32_t sym_dyadic_level(int32_t lo, int32_t hi) {
  int32_t l = 0;
  while (((lo >> l) & 1) == 0 && lo + (2 << l) <= hi) ++l;
  return l;
}
// Dyadic nodes covering [lo, hi).
GS_HD int32_t sym_node_count(int32_t lo, int32_t hi) {
  int32_t n = 0;
  while (lo < hi) {
    lo += 1 << sym_dyadic_level(lo, hi);
    ++n;
  }
  return n;
}

// Unit-map entries of the gated sym launch (layout.cpp gs_sym_unit_map_*, nbody_sym.hip
// local_first_unit): unit (segment or diagonal part) in bits 0-11, row in bits 12-27, flags
// in bits 28-31 (31 remote; all-gather order: 30 part unit, 28-29 its part; ring: 28-30 stage).
constexpr int kUnitRowShift = 12;
constexpr int32_t kUnitMax = 0xfff;      // largest unit index (S + D - 1 < 4096)
constexpr int32_t kUnitRowMax = 0xffff;  // most rows a map can hold

// Threads per one-sided force-kernel workgroup (i-bodies per workgroup = kForceBlock * ipl):
// 4 waves (profiles/r1_block_sweep.jsonl).
constexpr int kForceBlock = 256;

}  // namespace gs
