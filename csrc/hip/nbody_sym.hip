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

constexpr int kW = 8;                 // waves per workgroup
constexpr int kI = 4, kJ = 4;         // i / j bodies per lane
constexpr int kTile = 64 * kI;        // 256-body wave tile
constexpr int kThreads = 64 * kW;     // 512
constexpr int kTilesPerChunk = kSymC / kTile;
static_assert(64 * kJ == kTile, "i and j tiles have the same size");
static_assert(kW * kTile == kSymC, "one workgroup holds one chunk on its i side");

__device__ __forceinline__ int shell_len(int A, int NC) { return A < NC / 2 ? NC / 2 : NC / 2 - 1; }

__device__ __forceinline__ void load_jset(const float4* __restrict__ X4, int64_t row0,
                                          sym::JSet<kJ>& b) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const float4 q = X4[row0 + j * 64 + lane];
    b.x[j] = q.x; b.y[j] = q.y; b.z[j] = q.z; b.mu[j] = q.w;
    b.cx[j] = b.cy[j] = b.cz[j] = 0.f;
  }
}

// One workgroup per unit (row a, segment s); s == S is the row's diagonal chunk.
__global__ __launch_bounds__(kThreads) void force_sym_kernel(SymArgs a) {
  __shared__ float slot[2][kW][3][kTile];  // j-side carriers of each wave, double-buffered
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ar = blockIdx.x / (a.S + 1), s = blockIdx.x % (a.S + 1);
  const int A = a.a0 + ar;
  if ((int64_t)A * kSymC >= a.n_real) return;  // all-ghost row: never read
  const float4* X4 = reinterpret_cast<const float4*>(a.X);
  sym::ISet<kI> is;
  const int64_t i_row0 = (int64_t)A * kSymC + w * kTile;
#pragma unroll
  for (int i = 0; i < kI; ++i) {
    const float4 q = X4[i_row0 + i * 64 + lane];
    is.x[i] = q.x; is.y[i] = q.y; is.z[i] = q.z; is.mu[i] = q.w;
    is.ax[i] = is.ay[i] = is.az[i] = 0.f;
  }
  float* out;
  if (s == a.S) {
    // Diagonal chunk: all ordered pairs on the i side (the self term is 0 through the core).
    for (int t = 0; t < kTilesPerChunk; ++t) {
      sym::JSet<kJ> js;
      load_jset(X4, (int64_t)A * kSymC + t * kTile, js);
      sym::tile<kI, kJ, false>(is, js, a.eps2);
    }
    out = a.Pd + (int64_t)ar * 3 * kSymC;
  } else {
    const int h = shell_len(A, a.NC);
    const int d0 = s * a.L + 1;
    if (d0 > h) return;
    const int d1 = min(d0 + a.L - 1, h);
    int buf = 0;
    for (int d = d0; d <= d1; ++d) {
      const int B = (A + d) % a.NC;
      if (B >= a.real_chunks) continue;  // all-ghost column chunk: mu = 0, never read
      float* pj = a.Pj + ((int64_t)ar * a.H + (d - 1)) * 3 * kSymC;
      for (int t = 0; t < kTilesPerChunk; ++t) {
        sym::JSet<kJ> js;
        load_jset(X4, (int64_t)B * kSymC + t * kTile, js);
        sym::tile<kI, kJ, true>(is, js, a.eps2);
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
          slot[buf][w][0][j * 64 + lane] = js.cx[j];
          slot[buf][w][1][j * 64 + lane] = js.cy[j];
          slot[buf][w][2][j * 64 + lane] = js.cz[j];
        }
        __syncthreads();
        // Sum the 8 waves' carriers in wave order (fixed) and store the tile's j-side partial.
        for (int v = threadIdx.x; v < 3 * kTile; v += kThreads) {
          const int c = v / kTile, b = v % kTile;
          float acc = slot[buf][0][c][b];
#pragma unroll
          for (int u = 1; u < kW; ++u) acc += slot[buf][u][c][b];
          pj[(int64_t)c * kSymC + t * kTile + b] = acc;
        }
        buf ^= 1;  // the other buffer was last read before this tile's barrier
      }
    }
    out = a.Pi + ((int64_t)ar * a.S + s) * 3 * kSymC;
  }
#pragma unroll
  for (int i = 0; i < kI; ++i) {
    const int b = w * kTile + i * 64 + lane;
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
