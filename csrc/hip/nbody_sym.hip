// Newton-3 (symmetric) fp32 force schedule for gfx950: every unordered pair is evaluated
// once and its equal-and-opposite contribution reaches both bodies.
//
// Reference parity: cuda.cu:53-60 loops j > i and scatters F into forces[i] and -F into
// forces[j] (cuda.cu:43-49, Newton's third law) with racy non-atomic global read-modify-
// writes and a triangular load imbalance (D5). pyspark.py:80-84 applies
// the same +F/-F pair reduction on the driver. Here the saving is kept without any race:
//   * the pair arithmetic is the DPP register tile of gs_sym_tile.h (i side in registers,
//     j side in carriers that travel lane to lane), 4 v_pk + 0.5 v_rsq per interaction
//     against 6 v_pk + 1 v_rsq for the one-sided kernels;
//   * work is a canonical cyclic half-shell of 2048-body chunks (gs_kernels.h, SymArgs), so
//     every chunk row carries the same amount of work and rank ownership is a plain block
//     partition of rows;
//   * both sides land in pre-assigned partial slots and are summed in a fixed order by the
//     group-reduce and finalize kernels: deterministic, and the same bits for every rank
//     count P dividing 8 (the group sums are what crosses ranks).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gravsim.h"
#include "gs_kernels.h"
#include "gs_sym_tile.h"

namespace gs {
namespace {

// Workgroup shape: W waves, I i-bodies and J j-bodies per lane; one workgroup holds one
// 2048-body chunk on its i side (W * 64 * I == kSymC). GS_SYM_SHAPE picks the A/B variant:
// 0 = (8 waves, I 4, J 4), 1 = (4 waves, I 8, J 2).
#ifndef GS_SYM_SHAPE
#define GS_SYM_SHAPE 1
#endif
#if GS_SYM_SHAPE == 1
constexpr int kW = 4, kI = 8, kJ = 2;
#else
constexpr int kW = 8, kI = 4, kJ = 4;
#endif
// Occupancy floor (waves per SIMD) as an A/B knob.
#ifdef GS_SYM_WAVES_PER_EU
#define GS_SYM_WPE __attribute__((amdgpu_waves_per_eu(GS_SYM_WAVES_PER_EU)))
#else
#define GS_SYM_WPE
#endif
constexpr int kTileI = 64 * kI;       // i bodies per wave
constexpr int kTileJ = 64 * kJ;       // j bodies per tile
constexpr int kThreads = 64 * kW;
constexpr int kTilesPerChunk = kSymC / kTileJ;
static_assert(kW * kTileI == kSymC, "one workgroup holds one chunk on its i side");

#ifndef GS_SYM_JLDS
#define GS_SYM_JLDS 1
#endif
// j positions: staged in LDS and read per step (1), or held in registers and rotated with
// DPP (0). See gs_sym_tile.h tile_lds / tile.
constexpr bool kJlds = GS_SYM_JLDS;

__device__ __forceinline__ int shell_len(int A, int NC) { return A < NC / 2 ? NC / 2 : NC / 2 - 1; }

// Unit (row a, segment s) -> the sequence of j-tiles it visits, in order, skipping all-ghost
// column chunks (mu = 0 there, and their rows are never read). s == S is the diagonal chunk.
struct TileSeq {
  int A, NC, real_chunks, d1, d, t;
  bool diag;
  __device__ __forceinline__ int valid(int dd) const {
    while (dd <= d1 && (A + dd) % NC >= real_chunks) ++dd;
    return dd;
  }
  __device__ __forceinline__ bool done() const { return d > d1; }
  __device__ __forceinline__ int64_t row0() const {
    const int B = diag ? A : (A + d) % NC;
    return (int64_t)B * kSymC + t * kTileJ;
  }
  __device__ __forceinline__ void next() {
    if (++t == kTilesPerChunk) {
      t = 0;
      d = diag ? d1 + 1 : valid(d + 1);
    }
  }
};

// Stage the j-tile at row0 into the tile_lds layout (64 * kJ bodies, each stored twice).
__device__ __forceinline__ void stage_store(float4* dst, int b, const float4& q) {
  const int j = b / 64, l = b % 64;
  dst[j * sym::kStagedRows + sym::staged_entry(l, 0)] = q;
  dst[j * sym::kStagedRows + sym::staged_entry(l, 1)] = q;
}

using SlotT = float[2][kW][3][kTileJ];
using JtT = float4[2][kJ * sym::kStagedRows];

// Visit the unit's j-tiles. SYM: pairs both ways, j-side partials to Pj (the diagonal chunk
// runs with SYM = false: every ordered pair once on the i side).
template <bool SYM>
__device__ __forceinline__ void run_tiles(const SymArgs& a, sym::ISet<kI>& is, TileSeq seq,
                                          int ar, SlotT& slot, JtT& jt) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float4* X4 = reinterpret_cast<const float4*>(a.X);
  int buf = 0, cur = 0;
  if constexpr (kJlds) {
    if (!seq.done() && threadIdx.x < kTileJ)
      stage_store(jt[0], threadIdx.x, X4[seq.row0() + threadIdx.x]);
    __syncthreads();
  }
  while (!seq.done()) {
    TileSeq nx = seq;
    nx.next();
    const int d = seq.d, t = seq.t;
    float4 q_next;
    const bool stage_next = kJlds && !nx.done() && threadIdx.x < kTileJ;
    if (stage_next) q_next = X4[nx.row0() + threadIdx.x];  // lands during the arithmetic
    float cx[kJ], cy[kJ], cz[kJ];
    if constexpr (kJlds) {
      sym::CSet<kJ> cs;
#pragma unroll
      for (int j = 0; j < kJ; ++j) cs.cx[j] = cs.cy[j] = cs.cz[j] = 0.f;
      sym::tile_lds<kI, kJ, SYM>(is, cs, jt[cur], a.eps2);
#pragma unroll
      for (int j = 0; j < kJ; ++j) { cx[j] = cs.cx[j]; cy[j] = cs.cy[j]; cz[j] = cs.cz[j]; }
    } else {
      sym::JSet<kJ> js;
      const int64_t row0 = seq.row0();
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        const float4 q = X4[row0 + j * 64 + lane];
        js.x[j] = q.x; js.y[j] = q.y; js.z[j] = q.z; js.mu[j] = q.w;
        js.cx[j] = js.cy[j] = js.cz[j] = 0.f;
      }
      sym::tile<kI, kJ, SYM>(is, js, a.eps2);
#pragma unroll
      for (int j = 0; j < kJ; ++j) { cx[j] = js.cx[j]; cy[j] = js.cy[j]; cz[j] = js.cz[j]; }
    }
    if constexpr (SYM) {
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        slot[buf][w][0][j * 64 + lane] = cx[j];
        slot[buf][w][1][j * 64 + lane] = cy[j];
        slot[buf][w][2][j * 64 + lane] = cz[j];
      }
    }
    // jt[cur ^ 1] was last read in the previous tile, before the previous barrier.
    if (stage_next) stage_store(jt[cur ^ 1], threadIdx.x, q_next);
    if (kJlds || SYM) __syncthreads();
    if constexpr (SYM) {
      // Sum the waves' carriers in wave order (fixed) and store the tile's j-side partial.
      float* pj = a.Pj + ((int64_t)ar * a.H + (d - 1)) * 3 * kSymC;
      for (int v = threadIdx.x; v < 3 * kTileJ; v += kThreads) {
        const int c = v / kTileJ, b = v % kTileJ;
        float acc = slot[buf][0][c][b];
#pragma unroll
        for (int u = 1; u < kW; ++u) acc += slot[buf][u][c][b];
        pj[(int64_t)c * kSymC + t * kTileJ + b] = acc;
      }
      buf ^= 1;  // the other buffer was last read before this tile's barrier
    }
    cur ^= 1;
    seq = nx;
  }
}

// One workgroup per unit (row a, segment s); s == S is the row's diagonal chunk.
__global__ __launch_bounds__(kThreads) GS_SYM_WPE void force_sym_kernel(SymArgs a) {
  __shared__ SlotT slot;  // j-side carriers of each wave, double-buffered
  __shared__ JtT jt;      // staged j-tiles (kJlds), double-buffered
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ar = blockIdx.x / (a.S + 1), s = blockIdx.x % (a.S + 1);
  const int A = a.a0 + ar;
  if ((int64_t)A * kSymC >= a.n_real) return;  // all-ghost row: never read
  const float4* X4 = reinterpret_cast<const float4*>(a.X);
  sym::ISet<kI> is;
  const int64_t i_row0 = (int64_t)A * kSymC + w * kTileI;
#pragma unroll
  for (int i = 0; i < kI; ++i) {
    const float4 q = X4[i_row0 + i * 64 + lane];
    is.x[i] = q.x; is.y[i] = q.y; is.z[i] = q.z; is.mu[i] = q.w;
    is.ax[i] = is.ay[i] = is.az[i] = 0.f;
  }
  const bool diag = s == a.S;
  TileSeq seq{A, a.NC, a.real_chunks, 0, 0, 0, diag};
  float* out;
  if (diag) {
    // One pseudo-shell step: the 2048-body diagonal chunk (self term 0 through the core).
    run_tiles<false>(a, is, seq, ar, slot, jt);
    out = a.Pd + (int64_t)ar * 3 * kSymC;
  } else {
    const int h = shell_len(A, a.NC);
    const int d0 = s * a.L + 1;
    if (d0 > h) return;
    seq.d1 = min(d0 + a.L - 1, h);
    seq.d = seq.valid(d0);
    run_tiles<true>(a, is, seq, ar, slot, jt);
    out = a.Pi + ((int64_t)ar * a.S + s) * 3 * kSymC;
  }
#pragma unroll
  for (int i = 0; i < kI; ++i) {
    const int b = w * kTileI + i * 64 + lane;
    out[b] = is.ax[i];
    out[kSymC + b] = is.ay[i];
    out[2 * kSymC + b] = is.az[i];
  }
}

// S_g(x) for this rank's groups and every body x of a real chunk: rows A of group g in
// ascending order, each contributing Pj[A][d - 1] with d = (X - A) mod NC when X lies in
// A's shell. Grid: (bodies / 256, groups per rank).
__global__ __launch_bounds__(256) void sym_group_reduce_kernel(SymArgs a) {
  const int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= (int64_t)a.real_chunks * kSymC) return;
  const int gpr = kSymGroups / a.P;  // groups per rank
  const int gl = blockIdx.y;
  const int R = a.NC / kSymGroups;
  const int g = (a.a0 / R) + gl;
  const int X = (int)(x / kSymC), c = (int)(x % kSymC);
  float sx = 0.f, sy = 0.f, sz = 0.f;
  for (int A = g * R; A < (g + 1) * R && A < a.real_chunks; ++A) {
    const int d = (X - A + a.NC) % a.NC;
    if (d == 0 || d > shell_len(A, a.NC)) continue;
    const float* p = a.Pj + ((int64_t)(A - a.a0) * a.H + (d - 1)) * 3 * kSymC + c;
    sx += p[0];
    sy += p[kSymC];
    sz += p[2 * kSymC];
  }
  const int q = (int)(x / a.n_local);
  const int64_t xl = x % a.n_local;
  float* o = a.Sbuf + ((int64_t)q * gpr + gl) * 3 * a.n_local + xl;
  o[0] = sx;
  o[a.n_local] = sy;
  o[2 * a.n_local] = sz;
}

// a = Pd + sum_s Pi[s] + sum_g S_g, then kick-drift (cuda.cu:73-76, mpi.c:207-215) exactly as
// the one-sided kernels' epilogue (nbody_kernels.hip integrate_store); ghost rows are zeroed.
__global__ __launch_bounds__(256) void sym_finalize_kernel(SymArgs a) {
  const int64_t li = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (li >= a.n_local) return;
  const int64_t gi = a.i_begin + li;
  float4* vel = reinterpret_cast<float4*>(a.vel);
  if (gi >= a.n_real) {
    if (a.acc_out) {
      reinterpret_cast<float4*>(a.acc_out)[li] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      vel[li] = make_float4(0.f, 0.f, 0.f, 0.f);
      reinterpret_cast<float4*>(a.X_next)[gi] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    return;
  }
  const int A = (int)(gi / kSymC), c = (int)(gi % kSymC);
  const int ar = A - a.a0;
  const float* pd = a.Pd + (int64_t)ar * 3 * kSymC + c;
  float ax = pd[0], ay = pd[kSymC], az = pd[2 * kSymC];
  const int h = shell_len(A, a.NC);
  const int segs = (h + a.L - 1) / a.L;
  for (int s = 0; s < segs; ++s) {
    const float* p = a.Pi + ((int64_t)ar * a.S + s) * 3 * kSymC + c;
    ax += p[0];
    ay += p[kSymC];
    az += p[2 * kSymC];
  }
  const int gpr = kSymGroups / a.P;
  for (int gg = 0; gg < kSymGroups; ++gg) {  // source rank gg / gpr, its local group gg % gpr
    const float* p = a.Rbuf + (int64_t)gg * 3 * a.n_local + li;
    ax += p[0];
    ay += p[a.n_local];
    az += p[2 * a.n_local];
  }
  (void)gpr;
  if (a.acc_out) {
    reinterpret_cast<float4*>(a.acc_out)[li] = make_float4(ax, ay, az, 0.f);
    return;
  }
  const float4 xi = reinterpret_cast<const float4*>(a.X)[gi];
  float4 v = vel[li];
  v.x = v.x + ax * a.dt;
  v.y = v.y + ay * a.dt;
  v.z = v.z + az * a.dt;
  float4 xn;
  xn.x = xi.x + v.x * a.dt;
  xn.y = xi.y + v.y * a.dt;
  xn.z = xi.z + v.z * a.dt;
  xn.w = xi.w;
  vel[li] = v;
  reinterpret_cast<float4*>(a.X_next)[gi] = xn;
}

}  // namespace

hipError_t launch_force_sym(const SymArgs& a, hipStream_t s) {
  const int units = a.rows * (a.S + 1);
  if (units <= 0) return hipSuccess;
  hipLaunchKernelGGL(force_sym_kernel, dim3(units), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sym_group_reduce(const SymArgs& a, hipStream_t s) {
  const int64_t bodies = (int64_t)a.real_chunks * kSymC;
  const int gpr = kSymGroups / a.P;
  hipLaunchKernelGGL(sym_group_reduce_kernel, dim3((unsigned)((bodies + 255) / 256), gpr),
                     dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sym_finalize(const SymArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(sym_finalize_kernel, dim3((unsigned)((a.n_local + 255) / 256)), dim3(256),
                     0, s, a);
  return hipGetLastError();
}

int sym_occupancy() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, force_sym_kernel, kThreads, 0) !=
      hipSuccess)
    return 0;
  return n;
}

}  // namespace gs
