// Native CPU direct-sum engine (fp64 and fp32), OpenMP over i.
//
// Replaces the per-rank CPU loop of mpi.c:196-216 (and the pair map of pyspark.py:59-86)
// with the intended physics: accelerations for step k use only step-k positions (Jacobi),
// never the in-place Gauss-Seidel update of mpi.c. The j sum follows the
// canonical chunk order shared with the GPU kernels so that results do not depend on the
// number of ranks. Serves BASELINE config #1 ("1,024 bodies on CPU") and as a fast oracle.
#include <math.h>

#include <cmath>
#include <type_traits>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#if defined(__AVX2__) && defined(__FMA__)
#include <immintrin.h>
#define GS_CPU_SIMD 1
#endif

#include "gravsim.h"

void gs_set_error(const char* msg);

namespace {

template <typename T>
inline T rsqrt_ref(T r2) { return T(1) / std::sqrt(r2); }

template <typename T>
inline void accel_one(const T* X4, int64_t n_real, int64_t i, int32_t chunk, T cut2, T eps2,
                      T out[4]) {
  const T xi = X4[4 * i], yi = X4[4 * i + 1], zi = X4[4 * i + 2];
  const int64_t n_chunks = (n_real + chunk - 1) / chunk;
  T tx = 0, ty = 0, tz = 0, tp = 0;
  for (int64_t c = 0; c < n_chunks; ++c) {
    T ax = 0, ay = 0, az = 0, ph = 0;
    // Rows in [n_real, n_pad) are massless ghosts: their terms are exact zeros (the GPU
    // kernels sweep them anyway), so the CPU stops at n_real.
    const int64_t j0 = c * chunk, j1 = j0 + chunk < n_real ? j0 + chunk : n_real;
    for (int64_t j = j0; j < j1; ++j) {
      const T dx = X4[4 * j] - xi, dy = X4[4 * j + 1] - yi, dz = X4[4 * j + 2] - zi;
      const T mu = X4[4 * j + 3];
      const T r2 = std::fma(dz, dz, std::fma(dy, dy, std::fma(dx, dx, eps2)));
      const T inv = (r2 >= cut2) ? rsqrt_ref(r2) : T(0);
      const T mi = mu * inv;
      const T s = mi * (inv * inv);
      ax = std::fma(s, dx, ax);
      ay = std::fma(s, dy, ay);
      az = std::fma(s, dz, az);
      ph += mi;
    }
    tx += ax; ty += ay; tz += az; tp += ph;
  }
  out[0] = tx; out[1] = ty; out[2] = tz; out[3] = -tp;
}

#ifdef GS_CPU_SIMD
// AVX2 lanes over i (4 fp64 / 8 fp32 bodies per vector). Every lane runs exactly the scalar
// accel_one() sequence (same fma nesting, correctly rounded sqrt and divide, same chunk
// order), so the vector and scalar paths agree bit for bit; only independent i are batched.
template <typename T> struct Simd;
template <> struct Simd<double> {
  using V = __m256d;
  static constexpr int L = 4;
  static V set1(double a) { return _mm256_set1_pd(a); }
  static V zero() { return _mm256_setzero_pd(); }
  static V sub(V a, V b) { return _mm256_sub_pd(a, b); }
  static V add(V a, V b) { return _mm256_add_pd(a, b); }
  static V mul(V a, V b) { return _mm256_mul_pd(a, b); }
  static V fma(V a, V b, V c) { return _mm256_fmadd_pd(a, b, c); }
  static V inv_sqrt_masked(V r2, V cut2) {
    const V inv = _mm256_div_pd(_mm256_set1_pd(1.0), _mm256_sqrt_pd(r2));
    return _mm256_and_pd(inv, _mm256_cmp_pd(r2, cut2, _CMP_GE_OQ));
  }
  static void store(double* p, V a) { _mm256_storeu_pd(p, a); }
};
template <> struct Simd<float> {
  using V = __m256;
  static constexpr int L = 8;
  static V set1(float a) { return _mm256_set1_ps(a); }
  static V zero() { return _mm256_setzero_ps(); }
  static V sub(V a, V b) { return _mm256_sub_ps(a, b); }
  static V add(V a, V b) { return _mm256_add_ps(a, b); }
  static V mul(V a, V b) { return _mm256_mul_ps(a, b); }
  static V fma(V a, V b, V c) { return _mm256_fmadd_ps(a, b, c); }
  static V inv_sqrt_masked(V r2, V cut2) {
    const V inv = _mm256_div_ps(_mm256_set1_ps(1.0f), _mm256_sqrt_ps(r2));
    return _mm256_and_ps(inv, _mm256_cmp_ps(r2, cut2, _CMP_GE_OQ));
  }
  static void store(float* p, V a) { _mm256_storeu_ps(p, a); }
};

// Accelerations of bodies [i, i + L); out[d * L + l] = component d of body i + l.
template <typename T, bool PHI>
inline void accel_block(const T* X4, int64_t n_real, int64_t i, int32_t chunk, T cut2, T eps2,
                        T* out) {
  using S = Simd<T>;
  using V = typename S::V;
  constexpr int L = S::L;
  alignas(32) T bx[L], by[L], bz[L];
  for (int l = 0; l < L; ++l) {
    bx[l] = X4[4 * (i + l)];
    by[l] = X4[4 * (i + l) + 1];
    bz[l] = X4[4 * (i + l) + 2];
  }
  V xi, yi, zi;
  memcpy(&xi, bx, sizeof(V));
  memcpy(&yi, by, sizeof(V));
  memcpy(&zi, bz, sizeof(V));
  const V e2 = S::set1(eps2), c2 = S::set1(cut2);
  const int64_t n_chunks = (n_real + chunk - 1) / chunk;
  V tx = S::zero(), ty = S::zero(), tz = S::zero(), tp = S::zero();
  for (int64_t c = 0; c < n_chunks; ++c) {
    V ax = S::zero(), ay = S::zero(), az = S::zero(), ph = S::zero();
    const T* q = X4 + 4 * c * (int64_t)chunk;
    const int64_t len = n_real - c * (int64_t)chunk < chunk ? n_real - c * (int64_t)chunk : chunk;
    for (int64_t j = 0; j < len; ++j, q += 4) {
      const V dx = S::sub(S::set1(q[0]), xi), dy = S::sub(S::set1(q[1]), yi),
              dz = S::sub(S::set1(q[2]), zi);
      const V r2 = S::fma(dz, dz, S::fma(dy, dy, S::fma(dx, dx, e2)));
      const V inv = S::inv_sqrt_masked(r2, c2);
      const V mi = S::mul(S::set1(q[3]), inv);
      const V s = S::mul(mi, S::mul(inv, inv));
      ax = S::fma(s, dx, ax);
      ay = S::fma(s, dy, ay);
      az = S::fma(s, dz, az);
      if (PHI) ph = S::add(ph, mi);
    }
    tx = S::add(tx, ax); ty = S::add(ty, ay); tz = S::add(tz, az);
    if (PHI) tp = S::add(tp, ph);
  }
  S::store(out, tx);
  S::store(out + L, ty);
  S::store(out + 2 * L, tz);
  S::store(out + 3 * L, tp);
  if (PHI)
    for (int l = 0; l < L; ++l) out[3 * L + l] = -out[3 * L + l];
}
#endif

template <typename T>
int accel_range(const T* X4, int64_t n_real, int64_t i0, int64_t i1, int32_t chunk, T cut2,
                T eps2, T* acc4) {
  if (chunk <= 0 || i1 < i0) { gs_set_error("cpu_accel: bad arguments"); return -1; }
  int64_t i_vec = i0;
#ifdef GS_CPU_SIMD
  constexpr int L = Simd<T>::L;
  const int64_t nblk = (i1 - i0) / L;
  i_vec = i0 + nblk * L;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nblk; ++b) {
    T out[4 * L];
    const int64_t i = i0 + b * L;
    accel_block<T, true>(X4, n_real, i, chunk, cut2, eps2, out);
    for (int l = 0; l < L; ++l)
      for (int d = 0; d < 4; ++d) acc4[4 * (i + l - i0) + d] = out[d * L + l];
  }
#endif
#pragma omp parallel for schedule(static)
  for (int64_t i = i_vec; i < i1; ++i) {
    T out[4];
    accel_one<T>(X4, n_real, i, chunk, cut2, eps2, out);
    for (int d = 0; d < 4; ++d) acc4[4 * (i - i0) + d] = out[d];
  }
  return 0;
}

template <typename T>
inline void kick_drift(const T* X4, T* Xn4, T* vel4, int64_t i0, int64_t i, const T a[3], T dt) {
  T* v = vel4 + 4 * (i - i0);
  T* xo = Xn4 + 4 * i;
  // Kick then drift (cuda.cu:73-76, mpi.c:207-215, pyspark.py:97-99).
  for (int d = 0; d < 3; ++d) {
    v[d] = v[d] + a[d] * dt;
    xo[d] = X4[4 * i + d] + v[d] * dt;
  }
  xo[3] = X4[4 * i + 3];
}

template <typename T>
int step_range(const T* X4, T* Xn4, T* vel4, int64_t n_real, int64_t i0, int64_t i1,
               int32_t chunk, T dt, T cut2, T eps2) {
  if (chunk <= 0 || i1 < i0) { gs_set_error("cpu_step: bad arguments"); return -1; }
  const int64_t i_real = i1 < n_real ? i1 : (i0 > n_real ? i0 : n_real);  // [i0, i_real) real
  int64_t i_vec = i0;
#ifdef GS_CPU_SIMD
  constexpr int L = Simd<T>::L;
  const int64_t nblk = (i_real - i0) / L;
  i_vec = i0 + nblk * L;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < nblk; ++b) {
    T out[4 * L];
    const int64_t i = i0 + b * L;
    accel_block<T, false>(X4, n_real, i, chunk, cut2, eps2, out);
    for (int l = 0; l < L; ++l) {
      const T a[3] = {out[l], out[L + l], out[2 * L + l]};
      kick_drift<T>(X4, Xn4, vel4, i0, i + l, a, dt);
    }
  }
#endif
#pragma omp parallel for schedule(static)
  for (int64_t i = i_vec; i < i1; ++i) {
    if (i >= n_real) {
      T* v = vel4 + 4 * (i - i0);
      T* xo = Xn4 + 4 * i;
      xo[0] = xo[1] = xo[2] = xo[3] = 0;
      v[0] = v[1] = v[2] = v[3] = 0;
      continue;
    }
    T a[4];
    accel_one<T>(X4, n_real, i, chunk, cut2, eps2, a);
    kick_drift<T>(X4, Xn4, vel4, i0, i, a, dt);
  }
  return 0;
}

// fp64 accelerations of bodies [i0, i1) with, per component, the sum of the terms' absolute
// values: out8[8 * (i - i0) + d] = a_d, out8[8 * (i - i0) + 4 + d] = sum_j |term_ij,d|
// (d < 3; entries 3 and 7 are 0). A floating-point sum of the terms is judged against that
// scale: |a_gpu - a| <= c * eps * sum |terms| (the accuracy gates of bench.py and the 1M test).
// A = double (the fp32 gates) or long double (x87 extended, 64-bit significand: the fp64 gates,
// where an fp64 reference's own rounding is of the fp64 kernel's order).
template <typename A>
int accel_abs_range(const double* X4, int64_t n_real, int64_t i0, int64_t i1, double cut2,
                    double eps2, double* out8) {
  if (i1 < i0) { gs_set_error("cpu_accel_abs: bad arguments"); return -1; }
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = i0; i < i1; ++i) {
    const A xi = X4[4 * i], yi = X4[4 * i + 1], zi = X4[4 * i + 2];
    A a[3] = {0, 0, 0}, s_abs[3] = {0, 0, 0};
    for (int64_t j = 0; j < n_real; ++j) {
      const A dx = (A)X4[4 * j] - xi, dy = (A)X4[4 * j + 1] - yi, dz = (A)X4[4 * j + 2] - zi;
      A r2;
      if constexpr (std::is_same<A, double>::value)
        r2 = std::fma(dz, dz, std::fma(dy, dy, std::fma(dx, dx, eps2)));
      else
        r2 = dx * dx + dy * dy + dz * dz + (A)eps2;  // (fmal is a libm software call)
      if (!(r2 >= (A)cut2)) continue;
      const A inv = (A)1 / std::sqrt(r2);
      const A s = (A)X4[4 * j + 3] * inv * inv * inv;
      const A t[3] = {s * dx, s * dy, s * dz};
      for (int d = 0; d < 3; ++d) {
        a[d] += t[d];
        s_abs[d] += std::fabs(t[d]);
      }
    }
    double* o = out8 + 8 * (i - i0);
    for (int d = 0; d < 3; ++d) {
      o[d] = (double)a[d];
      o[4 + d] = (double)s_abs[d];
    }
    o[3] = o[7] = 0.0;
  }
  return 0;
}

}  // namespace

extern "C" {

int gs_cpu_accel_abs_f64(const double* X4, int64_t n_real, int64_t i0, int64_t i1, double cut2,
                         double eps2, double* out8) {
  return accel_abs_range<double>(X4, n_real, i0, i1, cut2, eps2, out8);
}
int gs_cpu_accel_abs_ld(const double* X4, int64_t n_real, int64_t i0, int64_t i1, double cut2,
                        double eps2, double* out8) {
  return accel_abs_range<long double>(X4, n_real, i0, i1, cut2, eps2, out8);
}

int gs_cpu_accel_f64(const double* X4, int64_t n_real, int64_t i0, int64_t i1, int32_t chunk,
                     double cut2, double eps2, double* acc4) {
  return accel_range<double>(X4, n_real, i0, i1, chunk, cut2, eps2, acc4);
}
int gs_cpu_accel_f32(const float* X4, int64_t n_real, int64_t i0, int64_t i1, int32_t chunk,
                     float cut2, float eps2, float* acc4) {
  return accel_range<float>(X4, n_real, i0, i1, chunk, cut2, eps2, acc4);
}
int gs_cpu_step_f64(const double* X4, double* Xn4, double* vel4, int64_t n_real, int64_t i0,
                    int64_t i1, int32_t chunk, double dt, double cut2, double eps2) {
  return step_range<double>(X4, Xn4, vel4, n_real, i0, i1, chunk, dt, cut2, eps2);
}
int gs_cpu_step_f32(const float* X4, float* Xn4, float* vel4, int64_t n_real, int64_t i0,
                    int64_t i1, int32_t chunk, float dt, float cut2, float eps2) {
  return step_range<float>(X4, Xn4, vel4, n_real, i0, i1, chunk, dt, cut2, eps2);
}
int gs_cpu_set_threads(int32_t n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}

int gs_cpu_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

}  // extern "C"
