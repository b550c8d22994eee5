// Native CPU direct-sum engine (fp64 and fp32), OpenMP over i.
//
// Replaces the per-rank CPU loop of mpi.c:196-216 (and the pair map of pyspark.py:59-86)
// with the intended physics: accelerations for step k use only step-k positions (Jacobi),
// never the in-place Gauss-Seidel update of mpi.c. The j sum follows the
// canonical chunk order shared with the GPU kernels so that results do not depend on the
// number of ranks. Serves BASELINE config #1 ("1,024 bodies on CPU") and as a fast oracle.
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
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
    const int64_t j0 = c * chunk, j1 = j0 + chunk;
    for (int64_t j = j0; j < j1; ++j) {
      // Rows in [n_real, n_pad) are massless ghosts; every chunk is swept whole, exactly as
      // the GPU kernels do, so ghost terms contribute exact zeros in both engines.
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

template <typename T>
int accel_range(const T* X4, int64_t n_real, int64_t i0, int64_t i1, int32_t chunk, T cut2,
                T eps2, T* acc4) {
  if (chunk <= 0 || i1 < i0) { gs_set_error("cpu_accel: bad arguments"); return -1; }
#pragma omp parallel for schedule(static)
  for (int64_t i = i0; i < i1; ++i) {
    T out[4];
    accel_one<T>(X4, n_real, i, chunk, cut2, eps2, out);
    for (int d = 0; d < 4; ++d) acc4[4 * (i - i0) + d] = out[d];
  }
  return 0;
}

template <typename T>
int step_range(const T* X4, T* Xn4, T* vel4, int64_t n_real, int64_t i0, int64_t i1,
               int32_t chunk, T dt, T cut2, T eps2) {
  if (chunk <= 0 || i1 < i0) { gs_set_error("cpu_step: bad arguments"); return -1; }
#pragma omp parallel for schedule(static)
  for (int64_t i = i0; i < i1; ++i) {
    T* v = vel4 + 4 * (i - i0);
    T* xo = Xn4 + 4 * i;
    if (i >= n_real) {
      xo[0] = xo[1] = xo[2] = xo[3] = 0;
      v[0] = v[1] = v[2] = v[3] = 0;
      continue;
    }
    T a[4];
    accel_one<T>(X4, n_real, i, chunk, cut2, eps2, a);
    // Kick then drift (cuda.cu:73-76, mpi.c:207-215, pyspark.py:97-99).
    for (int d = 0; d < 3; ++d) {
      v[d] = v[d] + a[d] * dt;
      xo[d] = X4[4 * i + d] + v[d] * dt;
    }
    xo[3] = X4[4 * i + 3];
  }
  return 0;
}

}  // namespace

extern "C" {

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
