// gfx950 (MI355X / CDNA4) direct-sum N-body kernels.
//
// Replaces the reference's single CUDA kernel (cuda.cu:32-60, launched at :156) and its host
// integrator (cuda.cu:63-78). Design:
//   * SoA state: X = (x, y, z, mu = G*m) as one 16-B (fp32) / 32-B (fp64) vector per body, so
//     a j-body is one dwordx4 (fp32) load and no G*m_i*m_j product exists to overflow (D1).
//   * i-owned accumulation in registers: each lane owns IPL i-bodies and sums the full j row.
//     No Newton-3 scatter, no atomics, no race (D4), no triangular imbalance (D5).
//   * j-bodies arrive either as LDS tiles filled by LDS-DMA (global_load_lds_dwordx4, one
//     1-KiB wave-instruction per 64 fp32 bodies) and read as broadcast ds_read_b128, or as
//     wave-uniform SGPR operands through the scalar cache (s_load_dwordx16). Both variants
//     stream the same j range in the same order and give bitwise-identical results.
//   * Canonical chunked summation: the j range is cut into fixed chunks (length chosen from N
//     only); each chunk is summed from zero in j order and the chunk sums are added in chunk
//     order. The fused kernel (one workgroup sweeps every chunk, KD integrate in the
//     epilogue) and the split kernel (per-chunk partials + reduce/integrate kernel) therefore
//     produce the same bits, for any rank count.
//   * Kick-drift (symplectic Euler, "KD") integrate fused into the force epilogue:
//     v += a dt; x += v dt (cuda.cu:73-76, mpi.c:207-215, pyspark.py:97-99).
//   * Exact reference cutoff: zero force when r^2 < cutoff^2 (cuda.cu:39, mpi.c:64),
//     implemented as a select, which also removes the self term.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_common.h"
#include "gravsim.h"
#include "gs_kernels.h"

namespace gs {

template <typename T> struct VecT;
template <> struct VecT<float> { using type = float __attribute__((ext_vector_type(4))); };
template <> struct VecT<double> { using type = double __attribute__((ext_vector_type(4))); };
template <typename T> using V4 = typename VecT<T>::type;

constexpr int kBlock = kForceBlock;  // 256 = 4 waves of 64

__device__ __forceinline__ float rsqrt_dev(float x) { return __builtin_amdgcn_rsqf(x); }

// fp64: v_rsq_f64 seed (max relative error 5.2e-8, measured: profiles/r1_microbench_v3.jsonl)
// + one Halley step, cubically convergent: e = 1 - x y^2, y <- y + y e (1/2 + 3/8 e).
// (5.2e-8)^3 is far below 2^-53, so one step reaches double precision in 5 f64 ops where two
// Newton steps need 7 (512K fp64: profiles/r1_sweep_512k_fp64_halley.log vs _newton.log).
__device__ __forceinline__ double rsqrt_dev(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double e = __builtin_fma(-x * y, y, 1.0);
  const double p = __builtin_fma(e, 0.375, 0.5);
  return __builtin_fma(y * e, p, y);
}

__device__ __forceinline__ float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }

// Force modes (template FM):
//   FM_FAST  : r^2 + eps2 with eps2 >= a tiny overflow-safe core (set by the host), no select.
//              The self term and coincident bodies give s*0 = 0. Bit-identical to FM_EXACT
//              for every pair with r^2 >= 2^24 * eps2 (fp32: r >~ 4.5 mm at solar masses).
//   FM_EXACT : reference hard cutoff (cuda.cu:39, mpi.c:64): s = 0 when r^2 < cutoff^2.
//   FM_PHI   : FM_EXACT plus the potential sum (diagnostics / accel queries).
enum { FM_FAST = 0, FM_EXACT = 1, FM_PHI = 2 };

// One i-j interaction. 3 sub + 3 fma (r^2) + rsq + 3 mul + 3 fma; FM_EXACT adds cmp/select.
template <typename T, int FM>
__device__ __forceinline__ void interact(T xi, T yi, T zi, T xj, T yj, T zj, T muj, T cut2,
                                         T eps2, T& ax, T& ay, T& az, T& ph) {
  const T dx = xj - xi, dy = yj - yi, dz = zj - zi;
  const T r2 = fma_(dz, dz, fma_(dy, dy, fma_(dx, dx, eps2)));
  if constexpr (sizeof(T) == 8 && FM != FM_PHI) {
    // fp64 step path: refine r^-3 directly instead of r^-1. With y0 = v_rsq_f64(r2) and
    // e = 1 - r2 y0^2 (|e| <= 1.1e-7), r^-3 = y0^3 (1 - e)^(-3/2) = y0^3 (1 + 3/2 e + 15/8 e^2)
    // + O(e^3 ~ 1e-21): 7 f64 ops where a Halley-refined r^-1 followed by mu r^-1 r^-2 takes 8.
    // FM_EXACT: one select on s; an inf/NaN formed below the cutoff (r = 0: rsq = inf,
    // e = NaN) never leaves it (selecting the rsq input too cost 2 more v_cndmask).
    const T y0 = __builtin_amdgcn_rsq(r2);
    const T y2 = y0 * y0;
    const T e = fma_(-r2, y2, T(1));
    // 1.875 and 1.5 are not inline f64 constants: made opaque (loop-invariant, eps2 is a
    // finite kernel argument) so they live in VGPRs instead of being re-materialised by
    // v_mov_b32 pairs for a v_fmac in every interaction.
    const T c15 = T(1.5) + eps2 * T(0), c1875 = T(1.875) + eps2 * T(0);
    const T corr = fma_(e, fma_(e, c1875, c15), T(1));
    T s = (muj * (y2 * y0)) * corr;
    if constexpr (FM == FM_EXACT) s = r2 >= cut2 ? s : T(0);
    ax = fma_(s, dx, ax);
    ay = fma_(s, dy, ay);
    az = fma_(s, dz, az);
    return;
  }
  T inv;
  if constexpr (FM == FM_FAST) {
    inv = rsqrt_dev(r2);
  } else {
    const bool ok = r2 >= cut2;
    if constexpr (sizeof(T) == 8) {
      // Branch-free: the Newton sequence would otherwise be predicated behind exec-mask jumps.
      inv = rsqrt_dev(ok ? r2 : T(1));
      inv = ok ? inv : T(0);
    } else {
      inv = ok ? rsqrt_dev(r2) : T(0);
    }
  }
  const T mi = muj * inv;
  const T s = mi * (inv * inv);
  ax = fma_(s, dx, ax);
  ay = fma_(s, dy, ay);
  az = fma_(s, dz, az);
  if constexpr (FM == FM_PHI) ph += mi;
}

// fp32, pairs of i per lane as 2-vectors: every op but the rsq is one v_pk_* for two
// interactions, and the j scalar is broadcast by op_sel instead of SGPR-pair copies. Each
// element sees exactly the scalar interact() arithmetic, so results are bit-identical
// (+10 % over the compiler's own SLP packing: profiles/r1_ab_explicit_pk.jsonl).
using f2 = float __attribute__((ext_vector_type(2)));

template <int FM>
__device__ __forceinline__ void interact_pk(f2 xi, f2 yi, f2 zi, float xj, float yj, float zj,
                                            float muj, float cut2, float eps2, f2& ax, f2& ay,
                                            f2& az) {
  const f2 dx = f2(xj) - xi, dy = f2(yj) - yi, dz = f2(zj) - zi;
  const f2 r2 = __builtin_elementwise_fma(
      dz, dz, __builtin_elementwise_fma(dy, dy, __builtin_elementwise_fma(dx, dx, f2(eps2))));
  f2 inv;
  inv.x = rsqrt_dev(r2.x);
  inv.y = rsqrt_dev(r2.y);
  if constexpr (FM == FM_EXACT) {
    inv.x = r2.x >= cut2 ? inv.x : 0.0f;
    inv.y = r2.y >= cut2 ? inv.y : 0.0f;
  }
  const f2 mi = f2(muj) * inv;
  const f2 s = mi * (inv * inv);
  ax = __builtin_elementwise_fma(s, dx, ax);
  ay = __builtin_elementwise_fma(s, dy, ay);
  az = __builtin_elementwise_fma(s, dz, az);
}

template <typename T, int IPL>
struct IState {
  T x[IPL], y[IPL], z[IPL], mu[IPL];
  T ax[IPL], ay[IPL], az[IPL], ph[IPL];  // current chunk
  T tx[IPL], ty[IPL], tz[IPL], tp[IPL];  // canonical running total over chunks
};

template <typename T, int IPL>
__device__ __forceinline__ void zero_chunk(IState<T, IPL>& s) {
#pragma unroll
  for (int k = 0; k < IPL; ++k) s.ax[k] = s.ay[k] = s.az[k] = s.ph[k] = T(0);
}

template <typename T, int IPL, int FM>
__device__ __forceinline__ void interact_all(IState<T, IPL>& s, const V4<T>& q, T cut2, T eps2) {
  if constexpr (sizeof(T) == 4 && IPL % 2 == 0 && FM != FM_PHI) {
#pragma unroll
    for (int k = 0; k < IPL; k += 2) {
      f2 ax = {s.ax[k], s.ax[k + 1]}, ay = {s.ay[k], s.ay[k + 1]}, az = {s.az[k], s.az[k + 1]};
      interact_pk<FM>(f2{s.x[k], s.x[k + 1]}, f2{s.y[k], s.y[k + 1]}, f2{s.z[k], s.z[k + 1]},
                      q.x, q.y, q.z, q.w, cut2, eps2, ax, ay, az);
      s.ax[k] = ax.x; s.ax[k + 1] = ax.y;
      s.ay[k] = ay.x; s.ay[k + 1] = ay.y;
      s.az[k] = az.x; s.az[k + 1] = az.y;
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < IPL; ++k)
    interact<T, FM>(s.x[k], s.y[k], s.z[k], q.x, q.y, q.z, q.w, cut2, eps2, s.ax[k], s.ay[k],
                     s.az[k], s.ph[k]);
}


// LDS tile geometry: kTileBytes per tile buffer (4 KiB = 256 fp32 / 128 fp64 bodies),
// double-buffered. Each wave-instruction of the fill moves one 1-KiB piece.
constexpr int kTileBytes = 4096;
static_assert(kTileBytes % 1024 == 0, "tile must be whole 1 KiB wave pieces");
template <typename T> struct Tile { static constexpr int kBodies = kTileBytes / sizeof(V4<T>); };

// Issue the LDS-DMA fill of one tile: per round each of the 4 waves moves one 1-KiB piece
// (64 lanes x 16 B); the LDS destination is the wave-uniform base + lane*16.
template <typename T>
__device__ __forceinline__ void tile_fill(const V4<T>* __restrict__ src, V4<T>* dst) {
  constexpr int kRound = kBlock * 16;  // bytes one pass of the workgroup moves
  static_assert(kTileBytes % kRound == 0, "tile must be whole workgroup x 1 KiB-per-wave passes");
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < kTileBytes / kRound; ++r) {
    const char* g = reinterpret_cast<const char*>(src) + r * kRound + wave * 1024 + lane * 16;
    char* l = reinterpret_cast<char*>(dst) + r * kRound + wave * 1024;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                     (__attribute__((address_space(3))) void*)l, 16, 0, 0);
  }
}

// A contiguous run of virtual chunk indices [v0, v1) over the chunk sequence
// [c_begin, c_end) minus the skipped range [skip_begin, skip_end): chunk(v) maps back to the
// canonical chunk index, so per-chunk partial sums are the same bits whichever launch
// (rank-local overlap phase, remote phase, single-rank sweep) computes them.
struct ChunkSeq {
  int c_begin, skip_begin, skip_len;
  __device__ __forceinline__ int chunk(int v) const {
    const int c = c_begin + v;
    return c < skip_begin ? c : c + skip_len;
  }
};

// Sweep virtual chunks [v0, v1) through LDS tiles; on_chunk(c) after every finished chunk.
template <typename T, int IPL, int FM, typename OnChunk>
__device__ __forceinline__ void sweep_lds(const V4<T>* __restrict__ X, int64_t chunk,
                                          const ChunkSeq& seq, int v0, int v1, T cut2, T eps2,
                                          IState<T, IPL>& st, V4<T> (*tile)[Tile<T>::kBodies],
                                          OnChunk on_chunk) {
  constexpr int TB = Tile<T>::kBodies;
  const int tpc = (int)(chunk / TB);  // tiles per chunk
  const int ntiles = (v1 - v0) * tpc;
  if (ntiles <= 0) return;
  auto tile_src = [&](int t) {
    return X + (int64_t)seq.chunk(v0 + t / tpc) * chunk + (int64_t)(t % tpc) * TB;
  };
  tile_fill<T>(tile_src(0), tile[0]);
  zero_chunk<T, IPL>(st);
  for (int t = 0; t < ntiles; ++t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // tile t is in LDS for every wave; buffer (t+1)&1 is free
    if (t + 1 < ntiles) tile_fill<T>(tile_src(t + 1), tile[(t + 1) & 1]);
    const V4<T>* cur = tile[t & 1];
#pragma unroll 8
    for (int j = 0; j < TB; ++j) {
      const V4<T> q = cur[j];  // uniform address: one broadcast ds_read per wave
      interact_all<T, IPL, FM>(st, q, cut2, eps2);
    }
    if ((t + 1) % tpc == 0) {
      on_chunk(seq.chunk(v0 + t / tpc));
      zero_chunk<T, IPL>(st);
    }
  }
}

// Sweep virtual chunks [v0, v1) with wave-uniform j loaded into SGPRs via the scalar cache.
template <typename T, int IPL, int FM, typename OnChunk>
__device__ __forceinline__ void sweep_smem(const V4<T>* __restrict__ X, int64_t chunk,
                                           const ChunkSeq& seq, int v0, int v1, T cut2, T eps2,
                                           IState<T, IPL>& st, OnChunk on_chunk) {
  for (int v = v0; v < v1; ++v) {
    const int c = seq.chunk(v);
    zero_chunk<T, IPL>(st);
    // Constant address space: the j stream is read-only for the kernel's lifetime, and this
    // guarantees scalar (s_load) loads even where the compiler cannot prove no-clobber.
    using CV4 = const __attribute__((address_space(4))) V4<T>;
    CV4* p = (CV4*)(X + (int64_t)c * chunk);
    // Software pipeline: the next 4 j-bodies (one s_load_dwordx16 for fp32) are requested
    // before the current 4 are consumed, so scalar-cache / L2 latency overlaps the VALU work.
    V4<T> q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    // Scalar loads return out of order, so any wait is lgkmcnt(0). Drain the first batch
    // here; otherwise the wait for it lands inside the loop after the next prefetch is
    // issued and stalls on that prefetch every iteration.
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    for (int64_t j = 4; j < chunk; j += 4) {
      const V4<T> n0 = p[j], n1 = p[j + 1], n2 = p[j + 2], n3 = p[j + 3];
      __builtin_amdgcn_sched_barrier(0);  // keep the loads at the top of the iteration
      interact_all<T, IPL, FM>(st, q0, cut2, eps2);
      interact_all<T, IPL, FM>(st, q1, cut2, eps2);
      interact_all<T, IPL, FM>(st, q2, cut2, eps2);
      interact_all<T, IPL, FM>(st, q3, cut2, eps2);
      q0 = n0; q1 = n1; q2 = n2; q3 = n3;
    }
    interact_all<T, IPL, FM>(st, q0, cut2, eps2);
    interact_all<T, IPL, FM>(st, q1, cut2, eps2);
    interact_all<T, IPL, FM>(st, q2, cut2, eps2);
    interact_all<T, IPL, FM>(st, q3, cut2, eps2);
    on_chunk(c);
  }
}

template <typename T, int IPL>
__device__ __forceinline__ void load_i(const KArgs<T>& a, IState<T, IPL>& st, int64_t ib) {
#pragma unroll
  for (int k = 0; k < IPL; ++k) {
    const V4<T> p = reinterpret_cast<const V4<T>*>(a.X)[a.i_begin + ib + threadIdx.x + k * kBlock];
    st.x[k] = p.x; st.y[k] = p.y; st.z[k] = p.z; st.mu[k] = p.w;
    st.tx[k] = st.ty[k] = st.tz[k] = st.tp[k] = T(0);
  }
}

// Kick-drift epilogue for one lane's IPL bodies; ghost rows are pinned at the origin, massless.
template <typename T, int IPL>
__device__ __forceinline__ void integrate_store(const KArgs<T>& a, const IState<T, IPL>& st,
                                                int64_t ib) {
  V4<T>* vel = reinterpret_cast<V4<T>*>(a.vel);
  V4<T>* xn = reinterpret_cast<V4<T>*>(a.X_next);
#pragma unroll
  for (int k = 0; k < IPL; ++k) {
    const int64_t li = ib + threadIdx.x + k * kBlock;
    const int64_t gi = a.i_begin + li;
    if (gi < a.n_real) {
      V4<T> v = vel[li];
      v.x = v.x + st.tx[k] * a.dt;
      v.y = v.y + st.ty[k] * a.dt;
      v.z = v.z + st.tz[k] * a.dt;
      V4<T> x;
      x.x = st.x[k] + v.x * a.dt;
      x.y = st.y[k] + v.y * a.dt;
      x.z = st.z[k] + v.z * a.dt;
      x.w = st.mu[k];
      vel[li] = v;
      xn[gi] = x;
    } else {
      const V4<T> z = {T(0), T(0), T(0), T(0)};
      vel[li] = z;
      xn[gi] = z;
    }
  }
}

// ---------------------------------------------------------------------------------------
// SPLIT: grid (i_blocks, groups). Workgroup (b, g) sweeps chunks of group g and stores one
// partial (ax, ay, az, sum mu/r) per chunk: partial[c * n_local + i].
template <typename T, int IPL, int KV, int FM>
__global__ __launch_bounds__(kBlock) void force_split_kernel(KArgs<T> a) {
  __shared__ __attribute__((aligned(16))) V4<T> tile[2][Tile<T>::kBodies];
  const int64_t ib = (int64_t)blockIdx.x * (kBlock * IPL);
  const int sb = min(max(a.skip_begin, a.c_begin), a.c_end);
  const int se = min(max(a.skip_end, sb), a.c_end);
  const ChunkSeq seq{a.c_begin, sb, se - sb};
  const int span = (a.c_end - a.c_begin) - (se - sb);
  const int per = (span + (int)gridDim.y - 1) / (int)gridDim.y;
  const int v0 = (int)blockIdx.y * per;
  const int v1 = min(v0 + per, span);
  IState<T, IPL> st;
  load_i<T, IPL>(a, st, ib);
  V4<T>* part = reinterpret_cast<V4<T>*>(a.partial);
  auto store = [&](int c) {
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
      V4<T> o;
      o.x = st.ax[k]; o.y = st.ay[k]; o.z = st.az[k]; o.w = st.ph[k];
      part[(int64_t)c * a.n_local + ib + threadIdx.x + k * kBlock] = o;
    }
  };
  const V4<T>* X = reinterpret_cast<const V4<T>*>(a.X);
  if constexpr (KV == GS_KERNEL_LDS)
    sweep_lds<T, IPL, FM>(X, a.chunk, seq, v0, v1, a.cut2, a.eps2, st, tile, store);
  else
    sweep_smem<T, IPL, FM>(X, a.chunk, seq, v0, v1, a.cut2, a.eps2, st, store);
}

// FUSED: grid (i_blocks). One workgroup sweeps every chunk in canonical order and integrates
// in its epilogue (no partial buffer); used when the i-blocks alone fill the GPU.
template <typename T, int IPL, int KV, int FM>
__global__ __launch_bounds__(kBlock) void force_fused_kernel(KArgs<T> a) {
  __shared__ __attribute__((aligned(16))) V4<T> tile[2][Tile<T>::kBodies];
  const int64_t ib = (int64_t)blockIdx.x * (kBlock * IPL);
  IState<T, IPL> st;
  load_i<T, IPL>(a, st, ib);
  auto fold = [&](int) {
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
      st.tx[k] += st.ax[k]; st.ty[k] += st.ay[k]; st.tz[k] += st.az[k]; st.tp[k] += st.ph[k];
    }
  };
  const V4<T>* X = reinterpret_cast<const V4<T>*>(a.X);
  const ChunkSeq seq{0, a.n_chunks, 0};
  if constexpr (KV == GS_KERNEL_LDS)
    sweep_lds<T, IPL, FM>(X, a.chunk, seq, 0, a.n_chunks, a.cut2, a.eps2, st, tile, fold);
  else
    sweep_smem<T, IPL, FM>(X, a.chunk, seq, 0, a.n_chunks, a.cut2, a.eps2, st, fold);
  if (a.acc_out) {
    V4<T>* out = reinterpret_cast<V4<T>*>(a.acc_out);
#pragma unroll
    for (int k = 0; k < IPL; ++k) {
      V4<T> o;
      o.x = st.tx[k]; o.y = st.ty[k]; o.z = st.tz[k]; o.w = -st.tp[k];
      out[ib + threadIdx.x + k * kBlock] = o;
    }
  } else {
    integrate_store<T, IPL>(a, st, ib);
  }
}

// REDUCE: total = sum over chunks (canonical order) of partial[c][i]; integrate or emit acc.
template <typename T>
__global__ __launch_bounds__(kBlock) void reduce_integrate_kernel(KArgs<T> a) {
  const V4<T>* part = reinterpret_cast<const V4<T>*>(a.partial);
  const V4<T>* X = reinterpret_cast<const V4<T>*>(a.X);
  for (int64_t li = (int64_t)blockIdx.x * kBlock + threadIdx.x; li < a.n_local;
       li += (int64_t)gridDim.x * kBlock) {
    T tx = 0, ty = 0, tz = 0, tp = 0;
    for (int c = 0; c < a.n_chunks; ++c) {
      const V4<T> p = part[(int64_t)c * a.n_local + li];
      tx += p.x; ty += p.y; tz += p.z; tp += p.w;
    }
    if (a.acc_out) {
      V4<T> o;
      o.x = tx; o.y = ty; o.z = tz; o.w = -tp;
      reinterpret_cast<V4<T>*>(a.acc_out)[li] = o;
      continue;
    }
    const int64_t gi = a.i_begin + li;
    V4<T>* vel = reinterpret_cast<V4<T>*>(a.vel);
    V4<T>* xn = reinterpret_cast<V4<T>*>(a.X_next);
    if (gi < a.n_real) {
      const V4<T> xi = X[gi];
      V4<T> v = vel[li];
      v.x = v.x + tx * a.dt;
      v.y = v.y + ty * a.dt;
      v.z = v.z + tz * a.dt;
      V4<T> x;
      x.x = xi.x + v.x * a.dt;
      x.y = xi.y + v.y * a.dt;
      x.z = xi.z + v.z * a.dt;
      x.w = xi.w;
      vel[li] = v;
      xn[gi] = x;
    } else {
      const V4<T> z = {T(0), T(0), T(0), T(0)};
      vel[li] = z;
      xn[gi] = z;
    }
  }
}

// ICs on device: full positions (every rank) + this rank's velocities; masses to fp64 array.
template <typename T>
__global__ __launch_bounds__(kBlock) void init_ics_kernel(int ic, uint64_t seed, int64_t n,
                                                          int64_t n_pad, int64_t i_begin,
                                                          int64_t n_local, double G, T* X4,
                                                          T* vel4, double* mass) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n_pad;
       i += (int64_t)gridDim.x * kBlock) {
    double p[3] = {0, 0, 0}, v[3] = {0, 0, 0}, m = 0;
    if (i < n) ic_body(ic, seed, i, p, v, &m);
    X4[4 * i] = (T)p[0];
    X4[4 * i + 1] = (T)p[1];
    X4[4 * i + 2] = (T)p[2];
    X4[4 * i + 3] = (T)(G * m);
    if (mass) mass[i] = m;
    const int64_t li = i - i_begin;
    if (li >= 0 && li < n_local) {
      vel4[4 * li] = (T)v[0];
      vel4[4 * li + 1] = (T)v[1];
      vel4[4 * li + 2] = (T)v[2];
      vel4[4 * li + 3] = T(0);
    }
  }
}

// Count non-finite components in X4 rows [i0, i1) and vel4 rows [0, nl) (NaN/Inf guard).
template <typename T>
__global__ __launch_bounds__(kBlock) void count_nonfinite_kernel(const T* X4, int64_t i0,
                                                                 int64_t nl, const T* vel4,
                                                                 unsigned long long* out) {
  unsigned long long cnt = 0;
  for (int64_t li = (int64_t)blockIdx.x * kBlock + threadIdx.x; li < nl;
       li += (int64_t)gridDim.x * kBlock) {
    for (int d = 0; d < 3; ++d) {
      cnt += !isfinite(X4[4 * (i0 + li) + d]);
      cnt += !isfinite(vel4[4 * li + d]);
    }
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off, 64);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(out, cnt);
}

// ---------------------------------------------------------------------------------------
// Host launchers.

template <typename T, int IPL, int KV>
static hipError_t launch_split_t(const KArgs<T>& a, int groups, hipStream_t s) {
  const int64_t blocks = a.n_local / (kBlock * IPL);
  dim3 grid((unsigned)blocks, (unsigned)groups);
  if (a.phi)
    hipLaunchKernelGGL((force_split_kernel<T, IPL, KV, FM_PHI>), grid, dim3(kBlock), 0, s, a);
  else if (a.exact)
    hipLaunchKernelGGL((force_split_kernel<T, IPL, KV, FM_EXACT>), grid, dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((force_split_kernel<T, IPL, KV, FM_FAST>), grid, dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <typename T, int IPL, int KV>
static hipError_t launch_fused_t(const KArgs<T>& a, hipStream_t s) {
  const dim3 grid((unsigned)(a.n_local / (kBlock * IPL)));
  if (a.phi)
    hipLaunchKernelGGL((force_fused_kernel<T, IPL, KV, FM_PHI>), grid, dim3(kBlock), 0, s, a);
  else if (a.exact)
    hipLaunchKernelGGL((force_fused_kernel<T, IPL, KV, FM_EXACT>), grid, dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((force_fused_kernel<T, IPL, KV, FM_FAST>), grid, dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <typename T, int KV>
static hipError_t dispatch_ipl(const KArgs<T>& a, int ipl, bool fused, int groups,
                               hipStream_t s) {
  switch (ipl) {
    case 1: return fused ? launch_fused_t<T, 1, KV>(a, s) : launch_split_t<T, 1, KV>(a, groups, s);
    case 2: return fused ? launch_fused_t<T, 2, KV>(a, s) : launch_split_t<T, 2, KV>(a, groups, s);
    case 4: return fused ? launch_fused_t<T, 4, KV>(a, s) : launch_split_t<T, 4, KV>(a, groups, s);
    case 8:
      if constexpr (sizeof(T) == 4)
        return fused ? launch_fused_t<T, 8, KV>(a, s) : launch_split_t<T, 8, KV>(a, groups, s);
      return hipErrorInvalidValue;
    default: return hipErrorInvalidValue;
  }
}

template <typename T>
static hipError_t dispatch(const KArgs<T>& a, int kernel, int ipl, bool fused, int groups,
                           hipStream_t s) {
  if (kernel == GS_KERNEL_SMEM) return dispatch_ipl<T, GS_KERNEL_SMEM>(a, ipl, fused, groups, s);
  return dispatch_ipl<T, GS_KERNEL_LDS>(a, ipl, fused, groups, s);
}

template <typename T>
hipError_t launch_force_split(const KArgs<T>& a, int kernel, int ipl, int groups, hipStream_t s) {
  const int span = split_span(a);
  if (span <= 0) return hipSuccess;
  if (groups < 1) groups = 1;
  if (groups > span) groups = span;
  if (kernel == GS_KERNEL_MFMA) {
    if constexpr (sizeof(T) == 4) {
      // The MFMA variant does not form the potential sum: accel queries (phi) use the
      // SGPR-streaming VALU kernel on the same chunk range.
      if (!a.phi) return launch_force_mfma(a, groups, s);
      return dispatch<T>(a, GS_KERNEL_SMEM, ipl, false, groups, s);
    }
    return hipErrorInvalidValue;
  }
  return dispatch<T>(a, kernel, ipl, false, groups, s);
}

template <typename T>
hipError_t launch_force_fused(const KArgs<T>& a, int kernel, int ipl, hipStream_t s) {
  if (kernel == GS_KERNEL_MFMA) return hipErrorInvalidValue;  // split schedule only
  return dispatch<T>(a, kernel, ipl, true, 1, s);
}

template <typename T>
hipError_t launch_reduce_integrate(const KArgs<T>& a, hipStream_t s) {
  int64_t blocks = (a.n_local + kBlock - 1) / kBlock;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((reduce_integrate_kernel<T>), dim3((unsigned)blocks), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_init_ics(int ic, uint64_t seed, int64_t n, int64_t n_pad, int64_t i_begin,
                           int64_t n_local, double G, T* X4, T* vel4, double* mass,
                           hipStream_t s) {
  int64_t blocks = (n_pad + kBlock - 1) / kBlock;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL((init_ics_kernel<T>), dim3((unsigned)blocks), dim3(kBlock), 0, s, ic, seed,
                     n, n_pad, i_begin, n_local, G, X4, vel4, mass);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_count_nonfinite(const T* X4, int64_t i0, int64_t nl, const T* vel4,
                                  unsigned long long* out, hipStream_t s) {
  int64_t blocks = (nl + kBlock - 1) / kBlock;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((count_nonfinite_kernel<T>), dim3((unsigned)blocks), dim3(kBlock), 0, s, X4,
                     i0, nl, vel4, out);
  return hipGetLastError();
}

// Resident workgroups per CU of the split kernel actually launched for (kernel, ipl, mode).
template <typename T, int IPL, int KV>
static int occ_t(int fm) {
  int b = 0;
  hipError_t e;
  if (fm == FM_PHI)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, force_split_kernel<T, IPL, KV, FM_PHI>, kBlock, 0);
  else if (fm == FM_EXACT)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, force_split_kernel<T, IPL, KV, FM_EXACT>, kBlock, 0);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, force_split_kernel<T, IPL, KV, FM_FAST>, kBlock, 0);
  return e == hipSuccess ? b : 0;
}

template <typename T>
int split_occupancy(int kernel, int ipl, int fm) {
  if (kernel == GS_KERNEL_MFMA) {
    if (sizeof(T) != 4) return 0;
    if (fm != FM_PHI) return mfma_occupancy(fm);
    kernel = GS_KERNEL_SMEM;
  }
  const bool smem = kernel == GS_KERNEL_SMEM;
  switch (ipl) {
    case 1: return smem ? occ_t<T, 1, GS_KERNEL_SMEM>(fm) : occ_t<T, 1, GS_KERNEL_LDS>(fm);
    case 2: return smem ? occ_t<T, 2, GS_KERNEL_SMEM>(fm) : occ_t<T, 2, GS_KERNEL_LDS>(fm);
    case 4: return smem ? occ_t<T, 4, GS_KERNEL_SMEM>(fm) : occ_t<T, 4, GS_KERNEL_LDS>(fm);
    case 8:
      if constexpr (sizeof(T) == 4)
        return smem ? occ_t<T, 8, GS_KERNEL_SMEM>(fm) : occ_t<T, 8, GS_KERNEL_LDS>(fm);
      return 0;
    default: return 0;
  }
}

#define GS_INSTANTIATE(T)                                                                      \
  template int split_occupancy<T>(int, int, int);                                              \
  template hipError_t launch_force_split<T>(const KArgs<T>&, int, int, int, hipStream_t);      \
  template hipError_t launch_force_fused<T>(const KArgs<T>&, int, int, hipStream_t);           \
  template hipError_t launch_reduce_integrate<T>(const KArgs<T>&, hipStream_t);                \
  template hipError_t launch_init_ics<T>(int, uint64_t, int64_t, int64_t, int64_t, int64_t,    \
                                         double, T*, T*, double*, hipStream_t);                \
  template hipError_t launch_count_nonfinite<T>(const T*, int64_t, int64_t, const T*,          \
                                                unsigned long long*, hipStream_t);
GS_INSTANTIATE(float)
GS_INSTANTIATE(double)

}  // namespace gs
