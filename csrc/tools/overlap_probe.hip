// Concurrency probe for the progressive reduce (docs/DESIGN.md §12): can a streaming reduction
// run beside a VALU-bound launch that holds 2 workgroups of 4 waves x ~232 VGPRs per CU (the
// sym force kernel's shape) without taking its slots or its issue cycles?
//   F: VALU-bound stand-in for the force launch (4 waves, 232 VGPRs, 2 workgroups per CU).
//   R: streaming sum of a large buffer (3 GB, the 1M one-GPU partial slots), two shapes:
//      "wide"  - one thread per 4 floats, default register allocation, a large grid;
//      "slim"  - 48 VGPRs at most (amdgpu_num_vgpr(48)): fits beside two F waves per SIMD,
//                a persistent grid of one workgroup per CU.
// Prints one JSON line per case: F alone, R alone, and F with R launched on a second stream right
// after it (R's end and the pair's end), in ms.
//   overlap_probe [f_iters] [r_gb]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int kF = 154;  // accumulators per lane (F's register footprint)

__global__ __launch_bounds__(256)
void f_kernel(float* out, int iters, float s) {
  float a[kF];
#pragma unroll
  for (int k = 0; k < kF; ++k) a[k] = s * (float)(threadIdx.x + k);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < kF; ++k) a[k] = __builtin_fmaf(a[k], 0.999999f, a[(k + 1) % kF] * 1e-7f);
  }
  float t = 0.f;
#pragma unroll
  for (int k = 0; k < kF; ++k) t += a[k];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

// one float4 per thread per step, grid-stride; 8 loads in flight
__global__ __launch_bounds__(256) void r_wide(const float4* __restrict__ p, int64_t n4,
                                              float* out) {
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n4; i += 8 * stride) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  for (; i < n4; i += stride) {
    const float4 v = p[i];
    acc += (v.x + v.y) + (v.z + v.w);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(40)))
void r_slim(const float4* __restrict__ p, int64_t n4, float* out) {
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 7 * stride < n4; i += 8 * stride) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
  }
  for (; i < n4; i += stride) {
    const float4 v = p[i];
    acc += (v.x + v.y) + (v.z + v.w);
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  const double gb = argc > 2 ? atof(argv[2]) : 3.0;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int64_t n4 = (int64_t)(gb * 1e9) / 16;
  float4* buf;
  float *fo, *ro;
  CK(hipMalloc(&buf, n4 * 16));
  CK(hipMemset(buf, 0, n4 * 16));
  CK(hipMalloc(&fo, (size_t)2 * cus * 256 * 4));
  CK(hipMalloc(&ro, (size_t)64 * cus * 256 * 4));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, ef, er;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&ef));
  CK(hipEventCreate(&er));
  const int fgrid = 2 * cus;
  auto launch_r = [&](int shape, hipStream_t s) {
    if (shape == 0) hipLaunchKernelGGL(r_wide, dim3(16 * cus), dim3(256), 0, s, buf, n4, ro);
    else hipLaunchKernelGGL(r_slim, dim3(cus * shape), dim3(256), 0, s, buf, n4, ro);
  };
  auto ms = [&](hipEvent_t a, hipEvent_t b) {
    float t = 0.f;
    CK(hipEventElapsedTime(&t, a, b));
    return (double)t;
  };
  // warm-up
  hipLaunchKernelGGL(f_kernel, dim3(fgrid), dim3(256), 0, s1, fo, 10, 1.f);
  launch_r(0, s1);
  launch_r(1, s1);
  CK(hipStreamSynchronize(s1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, s1));
    hipLaunchKernelGGL(f_kernel, dim3(fgrid), dim3(256), 0, s1, fo, iters, 1.f);
    CK(hipEventRecord(ef, s1));
    CK(hipEventSynchronize(ef));
    const double f_alone = ms(e0, ef);
    const int shapes[3] = {0, 1, 2};
    for (int shape : shapes) {
      CK(hipEventRecord(e0, s1));
      launch_r(shape, s1);
      CK(hipEventRecord(er, s1));
      CK(hipEventSynchronize(er));
      const double r_alone = ms(e0, er);
      CK(hipEventRecord(e0, s1));
      hipLaunchKernelGGL(f_kernel, dim3(fgrid), dim3(256), 0, s1, fo, iters, 1.f);
      CK(hipEventRecord(ef, s1));
      CK(hipStreamWaitEvent(s2, e0, 0));
      launch_r(shape, s2);
      CK(hipEventRecord(er, s2));
      CK(hipEventSynchronize(ef));
      CK(hipEventSynchronize(er));
      printf("{\"rep\": %d, \"r_shape\": \"%s\", \"f_alone_ms\": %.3f, \"r_alone_ms\": %.3f, "
             "\"f_with_r_ms\": %.3f, \"r_end_with_f_ms\": %.3f, \"r_gb\": %.2f}\n",
             rep, shape == 0 ? "wide16" : shape == 1 ? "slim1" : "slim2", f_alone, r_alone,
             ms(e0, ef), ms(e0, er), gb);
      fflush(stdout);
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
