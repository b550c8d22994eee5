// gravsim_bench: standalone native driver (no Python), the counterpart of the reference's
// three `main`s (cuda.cu:120-178, mpi.c:140-268). Same Stepper, kernels and RCCL path as the
// Python package; writes the mpi.c log layout and one JSON metrics line.
//
//   gravsim_bench --n 65536 --steps 100 [--dt 3600] [--dtype fp32|fp64] [--kernel lds|smem]
//                 [--mode fused|split] [--ipl 2] [--seed S] [--init solar+random|random]
//                 [--log-dir DIR] [--dump FILE] [--progress-every 100] [--no-graph]
//                 [--strategy allgather|ring] [--cutoff-mode auto|exact|fast]
// Multi-GPU (one process per GPU): set RANK / WORLD_SIZE / LOCAL_RANK and pass
// --rendezvous FILE on a shared filesystem; rank 0 publishes the RCCL unique id there.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "gravsim.h"

namespace {

struct Args {
  gs_config cfg{};
  int steps = 100;
  uint64_t seed = 20250307;
  int ic = GS_IC_SOLAR_RANDOM;
  std::string log_dir, dump, rendezvous;
  int progress_every = 100;
};

[[noreturn]] void die(const char* what) {
  fprintf(stderr, "gravsim_bench: %s: %s\n", what, gs_last_error());
  exit(1);
}

Args parse(int argc, char** argv) {
  Args a;
  a.cfg.n = 65536;
  a.cfg.dtype = GS_FP32;
  a.cfg.nranks = 1;
  a.cfg.use_graph = 1;
  a.cfg.dt = 3600.0;
  a.cfg.G = 6.67430e-11;
  a.cfg.cutoff = 1e-10;
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) { fprintf(stderr, "missing value for %s\n", k.c_str()); exit(2); }
      return argv[++i];
    };
    if (k == "--n") a.cfg.n = atoll(val());
    else if (k == "--steps") a.steps = atoi(val());
    else if (k == "--dt") a.cfg.dt = atof(val());
    else if (k == "--dtype") a.cfg.dtype = strcmp(val(), "fp64") == 0 ? GS_FP64 : GS_FP32;
    else if (k == "--kernel") { const char* v = val(); a.cfg.kernel = !strcmp(v, "smem") ? GS_KERNEL_SMEM : GS_KERNEL_LDS; }
    else if (k == "--mode") { const char* v = val(); a.cfg.mode = !strcmp(v, "split") ? GS_MODE_SPLIT : GS_MODE_FUSED; }
    else if (k == "--ipl") a.cfg.ipl = atoi(val());
    else if (k == "--chunk") a.cfg.chunk = atoi(val());
    else if (k == "--seed") a.seed = strtoull(val(), nullptr, 10);
    else if (k == "--init") a.ic = strcmp(val(), "random") == 0 ? GS_IC_RANDOM : GS_IC_SOLAR_RANDOM;
    else if (k == "--cutoff") a.cfg.cutoff = atof(val());
    else if (k == "--softening") a.cfg.softening = atof(val());
    else if (k == "--log-dir") a.log_dir = val();
    else if (k == "--dump") a.dump = val();
    else if (k == "--rendezvous") a.rendezvous = val();
    else if (k == "--progress-every") a.progress_every = atoi(val());
    else if (k == "--no-graph") a.cfg.use_graph = 0;
    else if (k == "--strategy") a.cfg.strategy = strcmp(val(), "ring") == 0 ? GS_STRATEGY_RING : GS_STRATEGY_ALLGATHER;
    else if (k == "--cutoff-mode") { const char* v = val(); a.cfg.cutoff_mode = !strcmp(v, "exact") ? 1 : !strcmp(v, "fast") ? 2 : 0; }
    else if (k == "--help" || k == "-h") {
      printf("usage: gravsim_bench --n N --steps S [--dt DT] [--dtype fp32|fp64] ...\n");
      exit(0);
    } else {
      fprintf(stderr, "unknown argument %s\n", k.c_str());
      exit(2);
    }
  }
  const char* r = getenv("RANK");
  const char* w = getenv("WORLD_SIZE");
  const char* lr = getenv("LOCAL_RANK");
  a.cfg.rank = r ? atoi(r) : 0;
  a.cfg.nranks = w ? atoi(w) : 1;
  a.cfg.device = lr ? atoi(lr) : a.cfg.rank;
  return a;
}

// File rendezvous for the 128-byte RCCL unique id (bounded wait).
void share_unique_id(const Args& a, char id[128]) {
  if (a.cfg.rank == 0) {
    if (gs_rccl_unique_id(id)) die("rccl unique id");
    std::string tmp = a.rendezvous + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(id, 1, 128, f) != 128) die("write rendezvous");
    fclose(f);
    rename(tmp.c_str(), a.rendezvous.c_str());
    return;
  }
  for (int t = 0; t < 6000; ++t) {
    FILE* f = fopen(a.rendezvous.c_str(), "rb");
    if (f) {
      size_t got = fread(id, 1, 128, f);
      fclose(f);
      if (got == 128) return;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  fprintf(stderr, "gravsim_bench: rendezvous timeout on %s\n", a.rendezvous.c_str());
  exit(1);
}

}  // namespace

int main(int argc, char** argv) {
  Args a = parse(argc, argv);
  gs_stepper* s = nullptr;
  if (gs_stepper_create(&a.cfg, &s)) die("stepper_create");
  if (a.cfg.nranks > 1) {
    if (a.rendezvous.empty()) {
      fprintf(stderr, "gravsim_bench: WORLD_SIZE > 1 needs --rendezvous FILE\n");
      return 2;
    }
    char id[128];
    share_unique_id(a, id);
    if (gs_stepper_comm_init(s, id, a.cfg.rank, a.cfg.nranks)) die("comm_init");
    int32_t cnt = 0, ur = -1, dev = -1;  // (comm_init has checked them against the layout)
    gs_stepper_comm_info(s, &cnt, &ur, &dev);
    fprintf(stderr, "gravsim_bench: rank %d: RCCL communicator of %d ranks, rank %d on device %d\n",
            a.cfg.rank, cnt, ur, dev);
  }
  if (gs_stepper_init_ics(s, a.ic, a.seed)) die("init_ics");
  gs_layout L;
  gs_stepper_layout(s, &L);
  const bool root = a.cfg.rank == 0;

  char stamp[64];
  time_t tt = time(nullptr);
  strftime(stamp, sizeof(stamp), "%Y%m%d_%H%M%S", localtime(&tt));
  FILE* log = nullptr;
  if (root && !a.log_dir.empty()) {
    std::string d = a.log_dir + "/gravity_logs_mpi";
    mkdir(a.log_dir.c_str(), 0755);
    mkdir(d.c_str(), 0700);
    std::string path = d + "/mpi_c_simulation_" + stamp + ".txt";
    log = fopen(path.c_str(), "w");
    if (log)
      fprintf(log,
              "Starting MPI C gravity simulation at %s\nNumber of processes: %d\n"
              "Number of particles: %lld\nSteps: %d\nTimestep: %f seconds\n\n",
              stamp, a.cfg.nranks, (long long)a.cfg.n, a.steps, a.cfg.dt);
  }

  double clk[4];
  gs_stepper_clock(s, clk);  // (reset: the engine-clock record covers the timed loop only)
  const auto t0 = std::chrono::steady_clock::now();
  for (int done = 0; done < a.steps;) {
    if (root && a.progress_every > 0 && done % a.progress_every == 0)
      printf("Step %d/%d\n", done, a.steps);
    int k = a.progress_every > 0 ? a.progress_every - done % a.progress_every : a.steps;
    if (k > a.steps - done) k = a.steps - done;
    if (gs_stepper_step(s, k)) die("step");
    done += k;
  }
  if (gs_stepper_sync(s)) die("sync");
  const double wall =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (gs_stepper_clock(s, clk)) die("clock");  // {GHz, workgroup cycles, wg-seconds, wgs}
  const int64_t bad = gs_stepper_count_nonfinite(s);

  std::vector<double> pos((size_t)a.cfg.n * 3);
  if (gs_stepper_get_state(s, pos.data(), nullptr, nullptr)) die("get_state");
  if (root) {
    if (log) {
      fprintf(log, "\nPerformance Statistics:\nTotal execution time: %.2f seconds\n"
                   "Average time per step: %.4f seconds\n\nFinal positions:\n",
              wall, a.steps ? wall / a.steps : 0.0);
      for (int64_t i = 0; i < a.cfg.n; ++i)
        fprintf(log, "Particle %lld: (%e, %e, %e)\n", (long long)i, pos[3 * i], pos[3 * i + 1],
                pos[3 * i + 2]);
      fprintf(log, "\nSimulation completed successfully\n");
      fclose(log);
    }
    if (!a.dump.empty()) {
      FILE* f = fopen(a.dump.c_str(), "w");
      for (int64_t i = 0; f && i < a.cfg.n; ++i)
        fprintf(f, "Particle %lld: (%e, %e, %e)\n", (long long)i, pos[3 * i], pos[3 * i + 1],
                pos[3 * i + 2]);
      if (f) fclose(f);
    }
    const double n = (double)a.cfg.n;
    printf("{\"n\": %lld, \"steps\": %d, \"nranks\": %d, \"dtype\": \"%s\", \"wall_s\": %.6f, "
           "\"ms_per_step\": %.4f, \"body_updates_per_s\": %.6e, \"interactions_per_s\": %.6e, "
           "\"kernel\": %d, \"mode\": %d, \"ipl\": %d, \"chunk\": %d, \"nonfinite\": %lld, "
           "\"engine_clock_ghz\": %.4f}\n",
           (long long)a.cfg.n, a.steps, a.cfg.nranks, a.cfg.dtype == GS_FP64 ? "fp64" : "fp32",
           wall, a.steps ? 1e3 * wall / a.steps : 0.0, a.steps ? n * a.steps / wall : 0.0,
           a.steps ? n * n * a.steps / wall : 0.0, L.kernel, L.mode, L.ipl, L.chunk,
           (long long)bad, clk[0]);
  }
  gs_stepper_destroy(s);
  return bad ? 3 : 0;
}
