// Probe: does v_rsq_f32 overlap with packed-f32 VALU work on gfx950, and does the answer
// depend on where the rsq sits in the stream (burst vs spaced) and on waves per SIMD?
// The sym force tile issues 2 v_rsq_f32 per 16 v_pk_* (gs_sym_tile.h::meet_jp) in bursts
// of 8; this measures the same mix with exact instruction order (inline asm, so the
// compiler cannot re-schedule it) at 1, 2 and 4 waves per SIMD.
//   mode 0: 64 v_pk_fma_f32 only
//   mode 1: 8 v_rsq_f32 only
//   mode 2: 8 rsq burst, then 64 pk_fma          (today's shape)
//   mode 3: (1 rsq + 8 pk_fma) x 8               (spaced)
//   mode 4: (2 rsq + 16 pk_fma) x 4              (pairs spaced)
//   mode 5: 120 v_fma_f32 (24 chains): the same lane-FMA count unpacked
//   mode 6: (fma r; rsq r; 7 pk_fma) x 8      (rsq input produced by the op before it)
//   mode 7: (rsq r; fma r; 7 pk_fma) x 8      (rsq output read by the op after it)
//   mode 8: (fma r; 7 pk_fma) x 8             (control of 6 / 7 without the rsq)
//   mode 9: (fma r; rsq r; fma r; 7 pk_fma) x 8 (both, as in the force tile)
//   mode 10: (fma r; fma r; 7 pk_fma) x 8     (control of 9)
// Output: one JSON line per (mode, waves/SIMD): ns per wave-iteration per SIMD.
// Result (profiles/r2_trans_probe.jsonl, 2 waves/SIMD): 64 pk_fma 136 ns, + 8 rsq in any
// placement 140-143 ns, 120 fma 191 ns. In the sym tile a second transcendental per pair
// (GS_SYM_RCP) still cost 7.9 %: there the trans results feed the next instructions.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define PK(k) "v_pk_fma_f32 %" #k ", %" #k ", %[m], %[c]\n"
#define RSQ(k) "v_rsq_f32 %" #k ", %" #k "\n"
#define PK8A PK(0) PK(1) PK(2) PK(3) PK(4) PK(5) PK(6) PK(7)
#define PK8B PK(8) PK(9) PK(10) PK(11) PK(12) PK(13) PK(14) PK(15)
#define PK16 PK8A PK8B
#define OPS                                                                                  \
  "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+v"(a8), \
      "+v"(a9), "+v"(a10), "+v"(a11), "+v"(a12), "+v"(a13), "+v"(a14), "+v"(a15), "+v"(r0), \
      "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
#define INS [m] "v"(m), [c] "v"(c), [ms] "v"(ms), [cs] "v"(cs)
#define FR(k) "v_fma_f32 %" #k ", %" #k ", %[ms], %[cs]\n"
#define PK7A PK(0) PK(1) PK(2) PK(3) PK(4) PK(5) PK(6)
#define PK7B PK(8) PK(9) PK(10) PK(11) PK(12) PK(13) PK(14)
#define DEP6(k, P7) FR(k) RSQ(k) P7
#define DEP7(k, P7) RSQ(k) FR(k) P7
#define DEP8(k, P7) FR(k) P7
#define DEP9(k, P7) FR(k) RSQ(k) FR(k) P7
#define DEP10(k, P7) FR(k) FR(k) P7
#define X8(D) D(16, PK7A) D(17, PK7B) D(18, PK7A) D(19, PK7B) D(20, PK7A) D(21, PK7B) \
  D(22, PK7A) D(23, PK7B)

template <int MODE>
__global__ __launch_bounds__(256) void probe(float* out, int iters, float s) {
  f2 a0 = s + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
     a6 = a0 + 6, a7 = a0 + 7, a8 = a0 + 8, a9 = a0 + 9, a10 = a0 + 10, a11 = a0 + 11,
     a12 = a0 + 12, a13 = a0 + 13, a14 = a0 + 14, a15 = a0 + 15;
  float r0 = s + 1, r1 = s + 2, r2 = s + 3, r3 = s + 4, r4 = s + 5, r5 = s + 6, r6 = s + 7,
        r7 = s + 8;
  const f2 m = f2(0.999f), c = f2(1e-3f);
  const float ms = 0.999f, cs = 1e-3f;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 6) {
      asm volatile(X8(DEP6) : OPS : INS);
    } else if constexpr (MODE == 7) {
      asm volatile(X8(DEP7) : OPS : INS);
    } else if constexpr (MODE == 8) {
      asm volatile(X8(DEP8) : OPS : INS);
    } else if constexpr (MODE == 9) {
      asm volatile(X8(DEP9) : OPS : INS);
    } else if constexpr (MODE == 10) {
      asm volatile(X8(DEP10) : OPS : INS);
    } else if constexpr (MODE == 0) {
      asm volatile(PK16 PK16 PK16 PK16 : OPS : INS);
    } else if constexpr (MODE == 1) {
      asm volatile(RSQ(16) RSQ(17) RSQ(18) RSQ(19) RSQ(20) RSQ(21) RSQ(22) RSQ(23) : OPS : INS);
    } else if constexpr (MODE == 2) {
      asm volatile(RSQ(16) RSQ(17) RSQ(18) RSQ(19) RSQ(20) RSQ(21) RSQ(22) RSQ(23)
                   PK16 PK16 PK16 PK16 : OPS : INS);
    } else if constexpr (MODE == 3) {
      asm volatile(RSQ(16) PK8A RSQ(17) PK8B RSQ(18) PK8A RSQ(19) PK8B RSQ(20) PK8A RSQ(21)
                   PK8B RSQ(22) PK8A RSQ(23) PK8B : OPS : INS);
    } else {
      asm volatile(RSQ(16) RSQ(17) PK16 RSQ(18) RSQ(19) PK16 RSQ(20) RSQ(21) PK16 RSQ(22)
                   RSQ(23) PK16 : OPS : INS);
    }
  }
  f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + a8 + a9 + a10 + a11 + a12 + a13 + a14 + a15;
  out[blockIdx.x * blockDim.x + threadIdx.x] = t.x + t.y + r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}

#define F(k) "v_fma_f32 %" #k ", %" #k ", %[m], %[c]\n"
#define F24                                                                                  \
  F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(8) F(9) F(10) F(11) F(12) F(13) F(14) F(15) F(16) \
      F(17) F(18) F(19) F(20) F(21) F(22) F(23)

__global__ __launch_bounds__(256) void probe_fma(float* out, int iters, float s) {
  float v[24];
#pragma unroll
  for (int k = 0; k < 24; ++k) v[k] = s + k + threadIdx.x;
  const float m = 0.999f, c = 1e-3f;
  for (int it = 0; it < iters; ++it) {
    asm volatile(F24 F24 F24 F24 F24
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                   "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]),
                   "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15]), "+v"(v[16]),
                   "+v"(v[17]), "+v"(v[18]), "+v"(v[19]), "+v"(v[20]), "+v"(v[21]),
                   "+v"(v[22]), "+v"(v[23])
                 : [m] "v"(m), [c] "v"(c));
  }
  float t = 0;
#pragma unroll
  for (int k = 0; k < 24; ++k) t += v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int MODE>
static void launch(int blocks, float* out, int iters) {
  if constexpr (MODE == 5)
    probe_fma<<<blocks, 256>>>(out, iters, 1.0f);
  else
    probe<MODE><<<blocks, 256>>>(out, iters, 1.0f);
}

template <int MODE>
static void run(const char* name, float* out, int cus, int iters) {
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int blocks = cus * wps;  // 256 threads = one wave per SIMD per block
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    launch<MODE>(blocks, out, iters);  // warm-up at full length (clock settles)
    CHECK(hipGetLastError());
    CHECK(hipEventRecord(e0));
    launch<MODE>(blocks, out, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    // ns per wave-iteration per SIMD: every SIMD runs wps waves x iters iterations.
    const double ns = ms * 1e6 / (double(iters) * wps);
    printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_iter\": %.3f}\n",
           name, wps, ms, ns);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
  }
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  float* out;
  CHECK(hipMalloc(&out, sizeof(float) * cus * 4 * 256));
  for (int rep = 0; rep < 2; ++rep) {  // two passes: the second is on a warm clock
    run<0>("64 pk_fma", out, cus, iters);
    run<5>("120 fma", out, cus, iters);
    run<1>("8 rsq", out, cus, iters);
    run<2>("8 rsq burst + 64 pk_fma", out, cus, iters);
    run<3>("(rsq + 8 pk_fma) x8", out, cus, iters);
    run<4>("(2 rsq + 16 pk_fma) x4", out, cus, iters);
    run<6>("(fma; rsq; 7 pk) x8 [rsq input dependent]", out, cus, iters);
    run<7>("(rsq; fma; 7 pk) x8 [rsq output dependent]", out, cus, iters);
    run<8>("(fma; 7 pk) x8 [control]", out, cus, iters);
    run<9>("(fma; rsq; fma; 7 pk) x8 [both dependent]", out, cus, iters);
    run<10>("(fma; fma; 7 pk) x8 [control of 9]", out, cus, iters);
  }
  CHECK(hipFree(out));
  return 0;
}
