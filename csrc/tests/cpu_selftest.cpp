// Host-side self-test of the native CPU engine, layout math and IC generator, built with
// -fsanitize=address,undefined by tests/test_sanitizers.py (GPU sanitizers are not available
// on the target pool; SURVEY.md §5 "race detection / sanitizers"). Exit code 0 = pass.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "gravsim.h"

static int fails = 0;
#define EXPECT(c, ...)                        \
  do {                                        \
    if (!(c)) {                               \
      fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);           \
      fprintf(stderr, "\n");                  \
      ++fails;                                \
    }                                         \
  } while (0)

int main() {
  // layout: every (n, P) partitions the padded range exactly, chunk independent of P
  for (int64_t n : {1, 3, 1000, 2048, 2049, 100003}) {
    int32_t chunk0 = -1;
    for (int P : {1, 2, 3, 7, 8}) {
      int64_t covered = 0, n_pad = 0;
      for (int r = 0; r < P; ++r) {
        gs_config c{};
        c.n = n; c.rank = r; c.nranks = P;
        gs_layout L{};
        EXPECT(gs_layout_compute(&c, &L) == 0, "layout n=%lld P=%d", (long long)n, P);
        EXPECT(L.local_begin == covered, "slice order");
        covered += L.n_local;
        n_pad = L.n_pad;
        if (chunk0 < 0) chunk0 = L.chunk;
        EXPECT(L.chunk == chunk0, "chunk depends on P");
        // one-sided schedules: equal slices; sym: whole 2048-row blocks, possibly uneven
        if (L.mode == GS_MODE_SYM)
          EXPECT(L.n_pad % 16384 == 0 && L.n_local % 2048 == 0, "sym padding");
        else
          EXPECT(L.n_pad % ((int64_t)P * L.chunk) == 0, "padding");
      }
      EXPECT(covered == n_pad, "slices tile the padded range");
    }
  }
  gs_config bad{};
  bad.n = 0; bad.nranks = 1;
  gs_layout L{};
  EXPECT(gs_layout_compute(&bad, &L) != 0, "n=0 accepted");

  // ICs + CPU engine vs a naive fp64 loop
  const int64_t n = 777;
  std::vector<double> pos(3 * n), vel(3 * n), mass(n);
  gs_ic_fill_host(GS_IC_SOLAR_RANDOM, 42, n, 0, n, pos.data(), vel.data(), mass.data());
  EXPECT(mass[0] == 1.989e30 && pos[3] == 1.496e11, "solar bodies");
  gs_config c{};
  c.n = n; c.nranks = 1;
  EXPECT(gs_layout_compute(&c, &L) == 0, "layout");
  const double G = 6.67430e-11;
  std::vector<double> X(4 * L.n_pad, 0.0), acc(4 * n);
  for (int64_t i = 0; i < n; ++i) {
    for (int d = 0; d < 3; ++d) X[4 * i + d] = pos[3 * i + d];
    X[4 * i + 3] = G * mass[i];
  }
  EXPECT(gs_cpu_accel_f64(X.data(), n, 0, n, L.chunk, 1e-20, 0.0, acc.data()) == 0, "accel");
  double worst = 0;
  for (int64_t i = 0; i < n; ++i) {
    double a[3] = {0, 0, 0}, sabs = 0;
    for (int64_t j = 0; j < n; ++j) {
      const double dx = pos[3 * j] - pos[3 * i], dy = pos[3 * j + 1] - pos[3 * i + 1],
                   dz = pos[3 * j + 2] - pos[3 * i + 2];
      const double r2 = dx * dx + dy * dy + dz * dz;
      if (r2 < 1e-20) continue;
      const double s = G * mass[j] / (r2 * sqrt(r2));
      a[0] += s * dx; a[1] += s * dy; a[2] += s * dz;
      sabs += s * (fabs(dx) + fabs(dy) + fabs(dz));
    }
    for (int d = 0; d < 3; ++d) worst = fmax(worst, fabs(acc[4 * i + d] - a[d]) / sabs);
  }
  EXPECT(worst < 1e-13, "accel error %g", worst);

  // one step on a padded array, ghost rows zeroed
  std::vector<double> Xn(4 * L.n_pad, -1.0), V(4 * L.n_local, 0.0);
  for (int64_t i = 0; i < n; ++i)
    for (int d = 0; d < 3; ++d) V[4 * i + d] = vel[3 * i + d];
  EXPECT(gs_cpu_step_f64(X.data(), Xn.data(), V.data(), n, 0, L.n_local, L.chunk, 3600.0, 1e-20,
                         0.0) == 0, "step");
  for (int64_t i = n; i < L.n_local; ++i) EXPECT(Xn[4 * i] == 0.0 && Xn[4 * i + 3] == 0.0, "ghost");
  for (int64_t i = 0; i < n; ++i) EXPECT(isfinite(Xn[4 * i]) && Xn[4 * i + 3] == X[4 * i + 3], "row");
  EXPECT(gs_cpu_step_f64(X.data(), Xn.data(), V.data(), n, 5, 2, L.chunk, 1.0, 0, 0) != 0,
         "bad range accepted");

  // fp32 engine on the same data stays finite (no G*m*m overflow)
  std::vector<float> Xf(X.begin(), X.end()), accf(4 * n);
  EXPECT(gs_cpu_accel_f32(Xf.data(), n, 0, n, L.chunk, 1e-20f, 0.f, accf.data()) == 0, "f32");
  for (float v : accf) EXPECT(isfinite(v), "f32 non-finite");

  if (fails) {
    fprintf(stderr, "%d failures\n", fails);
    return 1;
  }
  printf("cpu_selftest ok\n");
  return 0;
}
