// Throughput and correctness probe for the Newton-3 register tile (csrc/include/gs_sym_tile.h).
//
// Each wave owns a random i-set (64*I bodies) and j-set (64*J bodies) and runs the tile R
// times. Reports interactions/s (2 per pair for the symmetric tile, 1 for the one-sided one)
// so the number compares directly with the production one-sided kernel (4.6e12 /s at 1M,
// profiles/r1_pk_bench_default.log), and checks one wave against an fp64 host sum.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/include csrc/tools/sym_probe.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "sym_probe_tile.h"

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));     \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// xi, xj: per wave 64*I and 64*J bodies (x, y, z, mu). out_i: 64*I accelerations (x,y,z,0),
// out_j: 64*J carriers.
template <int I, int J, bool SYM, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void probe_kernel(const f4* __restrict__ xi,
                                                    const f4* __restrict__ xj,
                                                    f4* __restrict__ out_i, f4* __restrict__ out_j,
                                                    int reps, float eps2) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  gs::sym::probe::ISet<I> a;
  gs::sym::probe::JSet<J> b;
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const f4 q = xi[(size_t)wave * 64 * I + i * 64 + lane];
    a.x[i] = q.x; a.y[i] = q.y; a.z[i] = q.z; a.mu[i] = q.w;
    a.ax[i] = a.ay[i] = a.az[i] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const f4 q = xj[(size_t)wave * 64 * J + j * 64 + lane];
    b.x[j] = q.x; b.y[j] = q.y; b.z[j] = q.z; b.mu[j] = q.w;
    b.cx[j] = b.cy[j] = b.cz[j] = 0.f;
  }
  for (int r = 0; r < reps; ++r) gs::sym::probe::tile<I, J, SYM>(a, b, eps2);
#pragma unroll
  for (int i = 0; i < I; ++i)
    out_i[(size_t)wave * 64 * I + i * 64 + lane] = f4{a.ax[i], a.ay[i], a.az[i], 0.f};
#pragma unroll
  for (int j = 0; j < J; ++j)
    out_j[(size_t)wave * 64 * J + j * 64 + lane] = f4{b.cx[j], b.cy[j], b.cz[j], 0.f};
}

// Issue cost of a DPP-modified VALU op against the plain op: 8 independent chains of
// x = x(lane-1 of row) - c (MODE 1) or x = x - c (MODE 0), folded single-use DPP.
template <int MODE>
__global__ __launch_bounds__(256) void dpp_chain_kernel(float* out, int iters, float c) {
  float x[8];
  const float cv = c * threadIdx.x;  // VGPR operand
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = 1.0f + 0.001f * (threadIdx.x + u);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (MODE == 1) x[u] = gs::sym::probe::sub_from<1>(x[u], cv);
      else x[u] = x[u] - cv;
    }
  }
  float s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += x[u];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Does v_rsq_f32 overlap packed VALU work? Per iteration: MODE 0 = 16 v_pk_fma_f32 (8
// independent 2-vector chains), MODE 1 = 4 v_rsq_f32 (4 independent chains), MODE 2 = both,
// interleaved (rsq results consumed only in the next iteration). If MODE 2 ~ max(0, 1) the
// transcendental runs beside the VALU; if ~ 0 + 1 it serialises.
template <int MODE>
__global__ __launch_bounds__(256) void trans_overlap_kernel(float* out, int iters, float c) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 v[8];
  float r[4];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = f2{1.0f + 0.001f * (threadIdx.x + u), 1.5f};
#pragma unroll
  for (int u = 0; u < 4; ++u) r[u] = 1.0f + 0.01f * (threadIdx.x + u);
  const f2 cc = f2{c, c}, dd = f2{0.5f, 0.5f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (MODE != 1) {
        v[u] = __builtin_elementwise_fma(v[u], cc, dd);
        v[u] = __builtin_elementwise_fma(v[u], cc, dd);
      }
      if constexpr (MODE != 0) {
        if ((u & 1) == 0) r[u >> 1] = __builtin_amdgcn_rsqf(r[u >> 1]) + 1.0f;
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += v[u].x + v[u].y;
#pragma unroll
  for (int u = 0; u < 4; ++u) s += r[u];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int MODE>
static void run_trans_overlap() {
  float* d;
  const int blocks = 256 * 8, iters = 2048;
  CK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  trans_overlap_kernel<MODE><<<blocks, 256>>>(d, 16, 0.999f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  trans_overlap_kernel<MODE><<<blocks, 256>>>(d, iters, 0.999f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double wave_iters = (double)blocks * 4 * iters / 1024.0;  // per SIMD
  printf("{\"probe\": \"trans_overlap\", \"mode\": \"%s\", \"ns_per_iter_per_simd\": %.3f}\n",
         MODE == 0 ? "16 v_pk_fma" : MODE == 1 ? "4 v_rsq" : "16 v_pk_fma + 4 v_rsq",
         ms * 1e6 / wave_iters);
  fflush(stdout);
  CK(hipFree(d));
}

template <int MODE>
static void run_dpp_chain() {
  float* d;
  const int blocks = 256 * 8, iters = 4096;
  CK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  dpp_chain_kernel<MODE><<<blocks, 256>>>(d, 16, 1e-7f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  dpp_chain_kernel<MODE><<<blocks, 256>>>(d, iters, 1e-7f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double winstr = (double)blocks * 4 * iters * 8;  // wave-instructions
  printf("{\"probe\": \"dpp_chain\", \"mode\": \"%s\", \"ns_per_wave_instr_per_simd\": %.3f}\n",
         MODE ? "v_sub_f32_dpp row_ror:1" : "v_sub_f32", ms * 1e6 / (winstr / 1024.0));
  fflush(stdout);
  CK(hipFree(d));
}

template <int I, int J, bool SYM, int WPE = 1>
static void run(int waves, int reps) {
  const size_t ni = (size_t)waves * 64 * I, nj = (size_t)waves * 64 * J;
  std::vector<f4> hi(ni), hj(nj);
  std::mt19937_64 rng(1234);
  std::uniform_real_distribution<double> up(-3e11, 3e11), um(1e23, 1e25);
  const double G = 6.67430e-11;
  for (auto& q : hi) q = f4{(float)up(rng), (float)up(rng), (float)up(rng), (float)(G * um(rng))};
  for (auto& q : hj) q = f4{(float)up(rng), (float)up(rng), (float)up(rng), (float)(G * um(rng))};
  if (!SYM) hj = std::vector<f4>(hi.begin(), hi.begin() + nj);  // diagonal: j-set == i-set
  const float eps2 = 3.39e-12f;
  f4 *di, *dj, *oi, *oj;
  CK(hipMalloc(&di, ni * 16)); CK(hipMalloc(&dj, nj * 16));
  CK(hipMalloc(&oi, ni * 16)); CK(hipMalloc(&oj, nj * 16));
  CK(hipMemcpy(di, hi.data(), ni * 16, hipMemcpyHostToDevice));
  CK(hipMemcpy(dj, hj.data(), nj * 16, hipMemcpyHostToDevice));
  const int blocks = waves / 4;
  // correctness: one rep, wave 0
  probe_kernel<I, J, SYM, WPE><<<blocks, 256>>>(di, dj, oi, oj, 1, eps2);
  CK(hipDeviceSynchronize());
  std::vector<f4> ri(ni), rj(nj);
  CK(hipMemcpy(ri.data(), oi, ni * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rj.data(), oj, nj * 16, hipMemcpyDeviceToHost));
  double worst = 0;
  for (int w = 0; w < 2; ++w) {
    for (int ii = 0; ii < 64 * I; ++ii) {
      const f4 p = hi[(size_t)w * 64 * I + ii];
      double ax = 0, ay = 0, az = 0;
      for (int jj = 0; jj < 64 * J; ++jj) {
        const f4 q = hj[(size_t)w * 64 * J + jj];
        double dx = (double)q.x - p.x, dy = (double)q.y - p.y, dz = (double)q.z - p.z;
        double r2 = dx * dx + dy * dy + dz * dz + eps2;
        double s = q.w / (r2 * sqrt(r2));
        ax += s * dx; ay += s * dy; az += s * dz;
      }
      const f4 g = ri[(size_t)w * 64 * I + ii];
      const double n = sqrt(ax * ax + ay * ay + az * az);
      const double e = sqrt(pow(g.x - ax, 2) + pow(g.y - ay, 2) + pow(g.z - az, 2)) / n;
      if (e > worst) worst = e;
    }
    if (SYM) {
      for (int jj = 0; jj < 64 * J; ++jj) {
        const f4 q = hj[(size_t)w * 64 * J + jj];
        double ax = 0, ay = 0, az = 0;
        for (int ii = 0; ii < 64 * I; ++ii) {
          const f4 p = hi[(size_t)w * 64 * I + ii];
          double dx = (double)p.x - q.x, dy = (double)p.y - q.y, dz = (double)p.z - q.z;
          double r2 = dx * dx + dy * dy + dz * dz + eps2;
          double s = p.w / (r2 * sqrt(r2));
          ax += s * dx; ay += s * dy; az += s * dz;
        }
        const f4 g = rj[(size_t)w * 64 * J + jj];
        const double n = sqrt(ax * ax + ay * ay + az * az);
        const double e = sqrt(pow(g.x - ax, 2) + pow(g.y - ay, 2) + pow(g.z - az, 2)) / n;
        if (e > worst) worst = e;
      }
    }
  }
  // throughput
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto launch = [&]() {
    probe_kernel<I, J, SYM, WPE><<<blocks, 256>>>(di, dj, oi, oj, reps, eps2);
  };
  launch();
  CK(hipEventRecord(e0));
  const int launches = 3;
  for (int l = 0; l < launches; ++l) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double pairs = (double)waves * reps * (64.0 * I) * (64.0 * J) * launches;
  const double inter = pairs * (SYM ? 2.0 : 1.0);
  printf("{\"probe\": \"%s\", \"I\": %d, \"J\": %d, \"sym\": %s, \"wpe\": %d, \"waves\": %d, \"reps\": %d, "
         "\"ms\": %.3f, \"interactions_per_s\": %.4e, \"max_rel_err\": %.3e}\n",
         "sym_tile_dpp", I, J, SYM ? "true" : "false", WPE, waves, reps, ms / launches, inter / (ms * 1e-3), worst);
  fflush(stdout);
  CK(hipFree(di)); CK(hipFree(dj)); CK(hipFree(oi)); CK(hipFree(oj));
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 256 * 4 * 8;
  const int reps = argc > 2 ? atoi(argv[2]) : 40;
  run_dpp_chain<0>();
  run_dpp_chain<1>();
  run_trans_overlap<0>();
  run_trans_overlap<1>();
  run_trans_overlap<2>();
  if (argc > 3) return 0;  // overlap probes only
  run<4, 4, true>(waves, reps);
  run<4, 2, true>(waves, reps);
  run<8, 1, true>(waves, reps / 2);
  run<8, 2, true>(waves, reps / 2);
  run<16, 1, true>(waves, reps / 4);
  run<4, 2, true, 6>(waves, reps);
  run<4, 4, false>(waves, reps);
  return 0;
}
