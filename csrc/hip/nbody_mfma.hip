// Experimental MFMA-assisted fp32 force kernel (SURVEY.md §7.2 item 8, §2.2 "MFMA-assisted
// variant"): the pairwise squared distance is a small GEMM on the matrix cores,
//
//   r²_ij = |x_i|² + |x_j|² − 2 x_i·x_j  =  C_i + Σ_k A_ik B_kj     (K = 4)
//   A_i = (−2x_i, −2y_i, −2z_i, 1),  B_j = (x_j, y_j, z_j, |x_j|²),  C_i = |x_i|² + eps²
//
// one v_mfma_f32_16x16x4_f32 per 16 i × 16 j tile. rsqrt, the μ/r³ scaling and the
// accumulation stay on the VALU (they are not GEMM-shaped). Coordinates are re-centred on
// the workgroup's first i-body before the GEMM: with |x| ~ 3e11 m and a 24-bit mantissa the
// expanded form otherwise cancels catastrophically for close pairs. Re-centring fixes
// spatially clustered i-blocks only; for i-blocks spread over the whole domain the relative
// error of a pair's r² is ~ eps_f32 · (|x_i'| / r)², so this variant is NOT the default.
//
// Measured on MI355X it is slower than the VALU kernel (docs/DESIGN.md §2): it saves the 3
// FMAs of r² per pair but pays an MFMA (16.5 ns per 16x16x4, barely overlapped with VALU
// issue), a max() guarding the cancelled self term, and LDS operand traffic. It is kept as
// an opt-in (`--kernel mfma`, split schedule, fp32) so the comparison stays reproducible.
//
// Layout of v_mfma_f32_16x16x4_f32 on a wave64 (lane l = 16 q + t, q = l / 16, t = l % 16):
//   A[i][k] : lane (i + 16 k)       B[k][j] : lane (j + 16 k)
//   D[i][j] : lane (j + 16 (i / 4)), element i % 4
// so lane (q, t) receives r² for rows 4q .. 4q+3 of the row group and column t.
//
// Work decomposition: a 256-thread workgroup owns 256 i-bodies (4 waves × 4 row groups of
// 16). Per j tile of 256 bodies (LDS, re-centred on write), each wave runs 16 j-steps of
// 16 columns × 4 MFMAs. Per chunk, each lane sums its column subset (j ≡ t mod 16) in j
// order; a fixed xor-butterfly over the 16 lanes of a q-group then gives the chunk sum,
// stored as the same per-chunk partial the VALU split kernel writes, so the existing
// reduce/integrate kernel and the canonical chunk order are reused. Results are
// deterministic but not bit-identical to the VALU kernels (different in-chunk order).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gravsim.h"
#include "gs_kernels.h"

namespace gs {
namespace {

using f2 = float __attribute__((ext_vector_type(2)));
using f4 = float __attribute__((ext_vector_type(4)));

constexpr int kMBlock = 256;  // threads = i-bodies per workgroup
constexpr int kMTile = 256;   // j-bodies per LDS tile
constexpr int kGroups = 4;    // 16-row groups per wave

// FM: 0 = fast (eps² core, no select), 1 = exact hard cutoff.
template <int FM>
__global__ __launch_bounds__(kMBlock) void force_mfma_kernel(KArgs<float> a) {
  __shared__ f4 P[2][kMTile];  // (x', y', z', mu): accumulate operands
  __shared__ f4 Q[2][kMTile];  // (x', y', z', |x'|²): GEMM B operand, one component per lane

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, t = lane & 15;
  const int64_t ib = (int64_t)blockIdx.x * kMBlock;
  const f4* X = reinterpret_cast<const f4*>(a.X);
  const f4 cen = X[a.i_begin + ib];  // re-centring origin: the block's first body

  // Chunk range of this workgroup (same partition as force_split_kernel).
  const int sb = min(max(a.skip_begin, a.c_begin), a.c_end);
  const int se = min(max(a.skip_end, sb), a.c_end);
  const int skip_len = se - sb;
  const int span = (a.c_end - a.c_begin) - skip_len;
  const int per = (span + (int)gridDim.y - 1) / (int)gridDim.y;
  const int v0 = (int)blockIdx.y * per;
  const int v1 = min(v0 + per, span);
  if (v0 >= v1) return;

  // Per-wave constants: A operand and C (|x_i'|² + eps²) per row group, x_i' for the 4 rows
  // of each group this lane receives.
  float Aop[kGroups];
  f4 Cop[kGroups];
  float xi[kGroups][4], yi[kGroups][4], zi[kGroups][4];
#pragma unroll
  for (int g = 0; g < kGroups; ++g) {
    const int64_t row0 = a.i_begin + ib + wave * 64 + g * 16;
    const f4 pa = X[row0 + t];
    const float ax = pa.x - cen.x, ay = pa.y - cen.y, az = pa.z - cen.z;
    Aop[g] = q == 0 ? -2.0f * ax : q == 1 ? -2.0f * ay : q == 2 ? -2.0f * az : 1.0f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const f4 pr = X[row0 + 4 * q + v];
      xi[g][v] = pr.x - cen.x;
      yi[g][v] = pr.y - cen.y;
      zi[g][v] = pr.z - cen.z;
      Cop[g][v] = __builtin_fmaf(zi[g][v], zi[g][v],
                                 __builtin_fmaf(yi[g][v], yi[g][v],
                                                __builtin_fmaf(xi[g][v], xi[g][v], a.eps2)));
    }
  }

  f4* part = reinterpret_cast<f4*>(a.partial);
  const int tiles_per_chunk = (int)(a.chunk / kMTile);

  for (int vc = v0; vc < v1; ++vc) {
    const int c = a.c_begin + vc < sb ? a.c_begin + vc : a.c_begin + vc + skip_len;
    const f4* src = X + (int64_t)c * a.chunk;
    float sx[kGroups][4] = {}, sy[kGroups][4] = {}, sz[kGroups][4] = {};

    // Stage tile 0; later tiles are prefetched into registers during the previous tile.
    f4 nxt = src[threadIdx.x];
    for (int tl = 0; tl < tiles_per_chunk; ++tl) {
      const int buf = tl & 1;
      {
        f4 p, b;
        p.x = b.x = nxt.x - cen.x;
        p.y = b.y = nxt.y - cen.y;
        p.z = b.z = nxt.z - cen.z;
        p.w = nxt.w;
        b.w = __builtin_fmaf(b.z, b.z, __builtin_fmaf(b.y, b.y, b.x * b.x));
        P[buf][threadIdx.x] = p;
        Q[buf][threadIdx.x] = b;
      }
      __syncthreads();
      if (tl + 1 < tiles_per_chunk) nxt = src[(int64_t)(tl + 1) * kMTile + threadIdx.x];
      const float* Qf = reinterpret_cast<const float*>(Q[buf]);
#pragma unroll 2
      for (int js = 0; js < kMTile / 16; ++js) {
        const f4 pj = P[buf][js * 16 + t];
        const float bop = Qf[(js * 16 + t) * 4 + q];
#pragma unroll
        for (int g = 0; g < kGroups; ++g) {
          f4 r2 = __builtin_amdgcn_mfma_f32_16x16x4f32(Aop[g], bop, Cop[g], 0, 0, 0);
#pragma unroll
          for (int v = 0; v < 4; v += 2) {
            f2 inv;
            if constexpr (FM == 0) {
              // The expanded form can cancel below the core (self term, coincident bodies):
              // clamp to eps² so 1/r³ stays finite; dx = 0 then makes the term exactly 0.
              inv.x = __builtin_amdgcn_rsqf(fmaxf(r2[v], a.eps2));
              inv.y = __builtin_amdgcn_rsqf(fmaxf(r2[v + 1], a.eps2));
            } else {
              inv.x = r2[v] >= a.cut2 ? __builtin_amdgcn_rsqf(r2[v]) : 0.0f;
              inv.y = r2[v + 1] >= a.cut2 ? __builtin_amdgcn_rsqf(r2[v + 1]) : 0.0f;
            }
            const f2 mi = f2(pj.w) * inv;
            const f2 s = mi * (inv * inv);
            const f2 dx = f2(pj.x) - f2{xi[g][v], xi[g][v + 1]};
            const f2 dy = f2(pj.y) - f2{yi[g][v], yi[g][v + 1]};
            const f2 dz = f2(pj.z) - f2{zi[g][v], zi[g][v + 1]};
            f2 ax = {sx[g][v], sx[g][v + 1]}, ay = {sy[g][v], sy[g][v + 1]},
               az = {sz[g][v], sz[g][v + 1]};
            ax = __builtin_elementwise_fma(s, dx, ax);
            ay = __builtin_elementwise_fma(s, dy, ay);
            az = __builtin_elementwise_fma(s, dz, az);
            sx[g][v] = ax.x; sx[g][v + 1] = ax.y;
            sy[g][v] = ay.x; sy[g][v + 1] = ay.y;
            sz[g][v] = az.x; sz[g][v + 1] = az.y;
          }
        }
      }
      __syncthreads();  // buffer buf is rewritten two tiles later; all waves are done with it
    }

    // Chunk sum over the 16 columns of each q-group: fixed xor butterfly (deterministic).
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
          sx[g][v] += __shfl_xor(sx[g][v], m, 64);
          sy[g][v] += __shfl_xor(sy[g][v], m, 64);
          sz[g][v] += __shfl_xor(sz[g][v], m, 64);
        }
    // Lane (q, t) stores row (g = t / 4, v = t % 4) of its q-group.
    const int64_t li = ib + wave * 64 + (t >> 2) * 16 + 4 * q + (t & 3);
    f4 o = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int g = 0; g < kGroups; ++g)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if ((t >> 2) == g && (t & 3) == v) {
          o.x = sx[g][v];
          o.y = sy[g][v];
          o.z = sz[g][v];
        }
    part[(int64_t)c * a.n_local + li] = o;
  }
}

}  // namespace

// Split launch of the MFMA variant: grid (n_local / 256, groups), one chunk range per group.
hipError_t launch_force_mfma(const KArgs<float>& a, int groups, hipStream_t s) {
  const int span = split_span(a);
  if (span <= 0) return hipSuccess;
  if (a.phi || a.chunk % kMTile != 0 || a.n_local % kMBlock != 0) return hipErrorInvalidValue;
  if (groups < 1) groups = 1;
  if (groups > span) groups = span;
  const dim3 grid((unsigned)(a.n_local / kMBlock), (unsigned)groups);
  if (a.exact)
    hipLaunchKernelGGL((force_mfma_kernel<1>), grid, dim3(kMBlock), 0, s, a);
  else
    hipLaunchKernelGGL((force_mfma_kernel<0>), grid, dim3(kMBlock), 0, s, a);
  return hipGetLastError();
}

int mfma_occupancy(int fm) {
  int b = 0;
  const hipError_t e =
      fm == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, force_mfma_kernel<0>, kMBlock, 0)
              : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, force_mfma_kernel<1>, kMBlock, 0);
  return e == hipSuccess ? b : 0;
}

}  // namespace gs
