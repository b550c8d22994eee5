// gfx950 microbenchmarks that size the N-body kernel design:
//   1. issue throughput of v_fma_f32 / v_rsq_f32 / v_pk_fma_f32 and of an rsq+fma mix
//      (does the transcendental overlap with plain VALU under multi-wave load?)
//   2. throughput of v_mfma_f32_16x16x4_f32 and v_mfma_f32_4x4x1_16b_f32, alone and beside
//      VALU work (separate pipes?)
//   3. the operand/result lane layout of v_mfma_f32_4x4x1_16b_f32 (exact integer data)
// Build: hipcc -O3 --offload-arch=gfx950 csrc/tools/microbench.hip -o microbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));           \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

// OPS: 0 fma, 1 rsq, 2 mix(1 rsq + 7 fma), 3 pk_fma, 4 mix(1 rsq + 14 fma)
template <int OPS>
__global__ __launch_bounds__(256) void valu_kernel(float* out, int iters, float a, float b) {
  float x[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = 1.0f + 0.001f * (threadIdx.x + u);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (OPS == 0) {
        x[u] = __builtin_fmaf(x[u], a, b);
      } else if constexpr (OPS == 1) {
        x[u] = __builtin_amdgcn_rsqf(x[u]);
      } else if constexpr (OPS == 2) {
        float y = __builtin_amdgcn_rsqf(x[u]);
#pragma unroll
        for (int k = 0; k < 7; ++k) y = __builtin_fmaf(y, a, b);
        x[u] = y;
      } else if constexpr (OPS == 4) {
        float y = __builtin_amdgcn_rsqf(x[u]);
#pragma unroll
        for (int k = 0; k < 14; ++k) y = __builtin_fmaf(y, a, b);
        x[u] = y;
      }
    }
    if constexpr (OPS == 3) {
      typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        f2 v = {x[u], x[u + 1]};
        f2 aa = {a, a}, bb = {b, b};
        v = __builtin_elementwise_fma(v, aa, bb);
        x[u] = v.x;
        x[u + 1] = v.y;
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += x[u];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// MFMA throughput; VALU_TOO adds 8 independent fma chains per MFMA.
template <int SHAPE, bool VALU_TOO>
__global__ __launch_bounds__(256) void mfma_kernel(float* out, int iters, float a, float b) {
  f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  float av = 0.001f * threadIdx.x, bv = 0.002f * threadIdx.x;
  float x[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = 1.0f + u;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (SHAPE == 16)
        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[q], 0, 0, 0);
      else
        acc[q] = __builtin_amdgcn_mfma_f32_4x4x1f32(av, bv, acc[q], 0, 0, 0);
      if constexpr (VALU_TOO) {
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = __builtin_fmaf(x[u], a, b);
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) s += acc[q].x + acc[q].y + acc[q].z + acc[q].w;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += x[u];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// 16 independent chains, x4 unrolled: VALU peak without dependency or loop-overhead limits.
template <bool PK>
__global__ __launch_bounds__(256) void valu16_kernel(float* out, int iters, float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 x[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = f2{1.0f + 0.001f * threadIdx.x, 1.0f + u};
  const f2 aa = {a, a}, bb = {b, b};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int rep = 0; rep < 4; ++rep)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if constexpr (PK) {
          x[u] = __builtin_elementwise_fma(x[u], aa, bb);
        } else {
          x[u].x = __builtin_fmaf(x[u].x, a, b);
          x[u].y = __builtin_fmaf(x[u].y, a, b);
        }
      }
  }
  float s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += x[u].x + x[u].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Role split: waves 0,2 of each workgroup run an MFMA loop, waves 1,3 run a VALU loop.
// MODE 0: both roles, 1: MFMA role only (VALU waves exit), 2: VALU role only.
template <int MODE>
__global__ __launch_bounds__(256) void split_kernel(float* out, int iters, float a, float b) {
  const int w = threadIdx.x >> 6;
  float s = 0;
  if ((w & 1) == 0) {
    if (MODE == 2) return;
    f4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
    float av = 0.001f * threadIdx.x, bv = 0.002f * threadIdx.x;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[q], 0, 0, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) s += acc[q].x + acc[q].y + acc[q].z + acc[q].w;
  } else {
    if (MODE == 1) return;
    float x[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) x[u] = 1.0f + u;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int rep = 0; rep < 2; ++rep)
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = __builtin_fmaf(x[u], a, b);
#pragma unroll
    for (int u = 0; u < 16; ++u) s += x[u];
  }
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Accuracy of the raw v_rsq_f64 / v_rsq_f32 seeds vs a correctly rounded 1/sqrt (relative).
__global__ void rsq_accuracy_kernel(double* out, int n) {
  double worst64 = 0, worst32 = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    // log-uniform inputs over [1e-20, 1e30]
    const double u = (double)((i * 2654435761u) & 0xFFFFFF) / 16777216.0;
    const double x = pow(10.0, -20.0 + 50.0 * u) * (1.0 + 1e-3 * (i & 1023));
    const double ref = 1.0 / sqrt(x);
    const double y64 = __builtin_amdgcn_rsq(x);
    worst64 = fmax(worst64, fabs(y64 - ref) / ref);
    const float xf = (float)x;
    const double reff = 1.0 / sqrt((double)xf);
    worst32 = fmax(worst32, fabs((double)__builtin_amdgcn_rsqf(xf) - reff) / reff);
  }
  for (int off = 32; off > 0; off >>= 1) {
    worst64 = fmax(worst64, __shfl_down(worst64, off, 64));
    worst32 = fmax(worst32, __shfl_down(worst32, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    out[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = worst64;
    out[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) + 1] = worst32;
  }
}

template <int OPS>
__global__ __launch_bounds__(256) void f64_kernel(float* out, int iters, float a, float b) {
  double x[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = 1.0 + 0.001 * (threadIdx.x + u);
  const double da = a, db = b;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if constexpr (OPS == 0) x[u] = __builtin_fma(x[u], da, db);
      else x[u] = __builtin_amdgcn_rsq(x[u]);
    }
  }
  double s = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += x[u];
  out[blockIdx.x * 256 + threadIdx.x] = (float)s;
}

__global__ void layout_kernel(float* out, int mode) {
  const int l = threadIdx.x;
  float a = 1.f, b = 1.f;
  if (mode == 0) a = (float)(l + 1);
  if (mode == 1) b = (float)(l + 1);
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

template <typename K>
static float time_kernel(K kern, float* out, int iters, int blocks, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 0.0001f);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0001f, 0.0001f);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int clk_khz = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const int blocks = cus * 8;  // 8 workgroups of 4 waves per CU -> 8 waves per SIMD
  float* out;
  CK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
  const int iters = 2048;
  const double waves_per_simd = (double)blocks * 4 / (cus * 4);
  printf("{\"cus\": %d, \"clock_mhz\": %.0f}\n", cus, clk_khz / 1e3);
  struct { const char* name; float ms; double instr_per_iter; } r[5];
  r[0] = {"v_fma_f32 x8", time_kernel(valu_kernel<0>, out, iters, blocks, 5), 8};
  r[1] = {"v_rsq_f32 x8", time_kernel(valu_kernel<1>, out, iters, blocks, 5), 8};
  r[2] = {"(rsq + 7 fma) x8", time_kernel(valu_kernel<2>, out, iters, blocks, 5), 64};
  r[3] = {"v_pk_fma_f32 x4", time_kernel(valu_kernel<3>, out, iters, blocks, 5), 4};
  r[4] = {"(rsq + 14 fma) x8", time_kernel(valu_kernel<4>, out, iters, blocks, 5), 120};
  for (auto& x : r) {
    // wave-instructions per SIMD = waves_per_simd * iters * instr_per_iter
    const double wi = waves_per_simd * iters * x.instr_per_iter;
    const double ns_per_wi = x.ms * 1e6 / wi;
    printf("{\"test\": \"%s\", \"ms\": %.4f, \"ns_per_wave_instr_per_simd\": %.4f, "
           "\"cycles_at_2.4GHz\": %.3f}\n", x.name, x.ms, ns_per_wi, ns_per_wi * 2.4);
  }
  struct { const char* name; float ms; } m[4];
  m[0] = {"mfma 16x16x4 f32", time_kernel(mfma_kernel<16, false>, out, iters, blocks, 5)};
  m[1] = {"mfma 4x4x1_16b f32", time_kernel(mfma_kernel<4, false>, out, iters, blocks, 5)};
  m[2] = {"mfma 16x16x4 + 8 fma", time_kernel(mfma_kernel<16, true>, out, iters, blocks, 5)};
  m[3] = {"mfma 4x4x1 + 8 fma", time_kernel(mfma_kernel<4, true>, out, iters, blocks, 5)};
  for (auto& x : m) {
    const double mi = waves_per_simd * iters * 4;
    const double ns = x.ms * 1e6 / mi;
    printf("{\"test\": \"%s\", \"ms\": %.4f, \"ns_per_mfma_per_simd\": %.4f, "
           "\"cycles_at_2.4GHz\": %.3f}\n", x.name, x.ms, ns, ns * 2.4);
  }
  {
    // 64 fma (or 32 pk_fma) per iteration per lane
    const float t0 = time_kernel(valu16_kernel<false>, out, iters, blocks, 5);
    const float t1 = time_kernel(valu16_kernel<true>, out, iters, blocks, 5);
    const double wi0 = waves_per_simd * iters * 64, wi1 = waves_per_simd * iters * 32;
    printf("{\"test\": \"v_fma_f32 16 chains\", \"ms\": %.4f, \"ns_per_wave_instr_per_simd\": %.4f, \"lane_flops_per_clk_per_simd_at_2.4\": %.2f}\n",
           t0, t0 * 1e6 / wi0, 128.0 / (t0 * 1e6 / wi0 * 2.4));
    printf("{\"test\": \"v_pk_fma_f32 16 chains\", \"ms\": %.4f, \"ns_per_wave_instr_per_simd\": %.4f, \"lane_flops_per_clk_per_simd_at_2.4\": %.2f}\n",
           t1, t1 * 1e6 / wi1, 256.0 / (t1 * 1e6 / wi1 * 2.4));
    const float s0 = time_kernel(split_kernel<0>, out, iters, blocks, 5);
    const float s1 = time_kernel(split_kernel<1>, out, iters, blocks, 5);
    const float s2 = time_kernel(split_kernel<2>, out, iters, blocks, 5);
    printf("{\"test\": \"role split mfma-waves + valu-waves\", \"both_ms\": %.4f, \"mfma_only_ms\": %.4f, \"valu_only_ms\": %.4f, \"overlap\": %.3f}\n",
           s0, s1, s2, (s1 + s2 - s0) / (s1 < s2 ? s1 : s2));
  }
  {
    const float f0 = time_kernel(f64_kernel<0>, out, iters, blocks, 5);
    const float f1 = time_kernel(f64_kernel<1>, out, iters, blocks, 5);
    const double wi = waves_per_simd * iters * 8;
    printf("{\"test\": \"v_fma_f64 x8\", \"ns_per_wave_instr_per_simd\": %.4f}\n", f0 * 1e6 / wi);
    printf("{\"test\": \"v_rsq_f64 x8\", \"ns_per_wave_instr_per_simd\": %.4f}\n", f1 * 1e6 / wi);
    double* acc;
    const int nb = 1024;
    CK(hipMalloc(&acc, (size_t)nb * 4 * 2 * sizeof(double)));
    hipLaunchKernelGGL(rsq_accuracy_kernel, dim3(nb), dim3(256), 0, 0, acc, 1 << 24);
    std::vector<double> h(nb * 4 * 2);
    CK(hipMemcpy(h.data(), acc, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    double w64 = 0, w32 = 0;
    for (int i = 0; i < nb * 4; ++i) { w64 = fmax(w64, h[2 * i]); w32 = fmax(w32, h[2 * i + 1]); }
    printf("{\"test\": \"rsq seed accuracy\", \"v_rsq_f64_max_rel_err\": %.3e, \"v_rsq_f32_max_rel_err\": %.3e}\n", w64, w32);
    CK(hipFree(acc));
  }
  float h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, out, mode);
    CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
    printf("{\"layout_4x4x1\": \"%s\", \"D\": [", mode == 0 ? "A=lane+1,B=1" : "A=1,B=lane+1");
    for (int i = 0; i < 256; ++i) printf("%s%.0f", i ? "," : "", h[i]);
    printf("]}\n");
  }
  CK(hipFree(out));
  return 0;
}
