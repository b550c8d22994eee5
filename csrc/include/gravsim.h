// gravsim native C ABI — MI355X (gfx950) N-body runtime.
//
// One header for both native libraries:
//   libgravsim_hip.so  (hipcc, gfx950): device kernels + the GPU Stepper (streams, events,
//                      hipGraph replay, RCCL all-gather over xGMI).
//   libgravsim_cpu.so  (g++ -fopenmp): fp64/fp32 direct-sum CPU engine (mpi.c world_size=1
//                      analogue and fast native oracle).
// Python binds these with ctypes (gravsim/ops/_native.py); there is no torch ABI coupling,
// so the libraries also serve the standalone C++ driver in csrc/tools/.
//
// Reference parity (what these replace, /root/reference):
//   cuda.cu:32-60   calculate_force_between + calculate_forces_kernel  -> gs force kernels
//   cuda.cu:63-78   host update()                                      -> fused KD epilogue
//   cuda.cu:145-160 cudaMalloc/Memcpy/DeviceSynchronize per step       -> device-resident Stepper
//   mpi.c:160-236   MPI_Bcast / MPI_Allgatherv / MPI_Barrier           -> RCCL in-place all-gather
//   mpi.c:196-216   per-rank O(N^2/P) loop + in-place integrate       -> gs_cpu_step (Jacobi)
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum gs_dtype { GS_FP32 = 0, GS_FP64 = 1 };

// Force kernel variants (the j-body source).
enum gs_kernel {
  GS_KERNEL_AUTO = 0,
  GS_KERNEL_LDS = 1,   // j-tiles staged into LDS by global_load_lds (LDS-DMA), broadcast ds_read_b128
  GS_KERNEL_SMEM = 2,  // wave-uniform j read through the scalar cache into SGPRs (s_load_dwordx16)
  GS_KERNEL_MFMA = 3,  // experimental fp32: r^2 as a 16x16x4 f32 MFMA GEMM, re-centred tiles
};

// Step schedule.
enum gs_mode {
  GS_MODE_AUTO = 0,
  GS_MODE_FUSED = 1,   // one workgroup per i-block sweeps every j-chunk, KD integrate in the epilogue
  GS_MODE_SPLIT = 2,   // i-block x chunk-group grid writes per-chunk partials; reduce+integrate kernel
  GS_MODE_SYM = 3,     // fp32 Newton-3: each unordered pair once, both sides (nbody_sym.hip)
};

// Initial-condition families (models). Same formulas in gravsim/models/initial_conditions.py.
// Multi-rank exchange strategies.
enum gs_strategy {
  GS_STRATEGY_ALLGATHER = 0,  // one in-place ncclAllGather, overlapped with the local chunks
  GS_STRATEGY_RING = 1,       // P-1 neighbour ncclSend/ncclRecv, each slice computed on arrival
};

enum gs_ic {
  GS_IC_SOLAR_RANDOM = 0,  // Sun/Earth/Mars + uniform cube bodies (cuda.cu:81-96,129-131)
  GS_IC_RANDOM = 1,        // uniform cube bodies only
};

typedef struct gs_config {
  int64_t n;          // real (global) body count
  int32_t dtype;      // gs_dtype
  int32_t kernel;     // gs_kernel
  int32_t mode;       // gs_mode
  int32_t ipl;        // i-bodies per lane (0 = auto)
  int32_t chunk;      // canonical j-chunk length (0 = auto, from n only)
  int32_t rank;       // this process' rank
  int32_t nranks;     // world size (bodies are block-partitioned over ranks)
  int32_t device;     // HIP device ordinal
  int32_t use_graph;  // capture the step loop into a hipGraph and replay it
  int32_t split_groups;  // SPLIT mode: chunk groups per i-block (0 = auto)
  int32_t cutoff_mode;   // 0 auto, 1 exact hard cutoff (select), 2 fast (overflow-safe core)
  int32_t strategy;      // 0 all-gather (default), 1 ring pass (neighbour send/recv, pipelined)
  double dt;          // time step [s]
  double G;           // gravitational constant
  double cutoff;      // hard cutoff radius [m]: zero force below it (mpi.c:64)
  double softening;   // Plummer softening length [m] (0 = reference semantics)
} gs_config;

typedef struct gs_layout {
  int64_t n;            // real bodies
  int64_t n_pad;        // padded global length (multiple of nranks*chunk)
  int64_t n_local;      // bodies per rank (padded)
  int64_t local_begin;  // global index of this rank's slice
  int32_t chunk;        // canonical j-chunk length
  int32_t n_chunks;     // chunks that contain at least one real body
  int32_t ipl;          // resolved i-bodies per lane
  int32_t kernel;       // resolved kernel variant
  int32_t mode;         // resolved schedule
  int32_t split_groups; // resolved chunk groups (SPLIT)
} gs_layout;

// ---------------------------------------------------------------- layout (host-only math)
// Canonical, world-size-independent decomposition (shared by CPU and GPU engines).
int gs_layout_compute(const gs_config* cfg, gs_layout* out);
int32_t gs_auto_chunk(int64_t n);
// Symmetric (Newton-3) schedule geometry for a padded body count, and its partial-buffer
// bytes per rank (GS_MODE_SYM).
int gs_sym_geometry(int64_t n_pad, int32_t* NC, int32_t* H, int32_t* L, int32_t* S,
                    int32_t* D);
int64_t gs_sym_bytes(int64_t n_pad, int32_t nranks, int32_t esz);
// Rows [a0, a0 + rows) of one rank (whole row blocks, mpi.c's remainder rule) and the
// reduction-tree nodes: B blocks of RB rows, nn nodes sent by this rank, nb by lower ranks,
// NN in all (gs_common.h).
int gs_sym_rank_rows(int64_t n_pad, int32_t nranks, int32_t rank, int32_t* a0, int32_t* rows);
int gs_sym_nodes(int64_t n_pad, int32_t nranks, int32_t rank, int32_t* B, int32_t* RB,
                 int32_t* nn, int32_t* nb, int32_t* NN);
// Busiest rank's work over the mean of the sym schedule's whole-row-block ownership
// (ceil(B / P) * P / B); mode auto picks sym only up to 1.25.
double gs_sym_imbalance(int64_t n_pad, int32_t nranks);
// Shell length of chunk row A (the antipodal pairs split between rows by parity).
int32_t gs_sym_shell_len(int32_t A, int32_t NC);
// Unit order of the gated sym launch for one rank (see layout.cpp); returns the entry count.
// 1 if rank src's node sums for rank dst's bodies can be nonzero, 0 if the geometry makes
// them +0.0 for every body (the exchange skips that send), -1 on bad arguments.
int32_t gs_sym_pair_live(int64_t n_pad, int32_t nranks, int32_t src, int32_t dst);
int64_t gs_sym_unit_map(int64_t n_pad, int32_t rank, int32_t nranks, int64_t fill,
                        int32_t* out, int64_t cap);
// ... with the last kr shell segments of every row split into np part units at the end (bit
// 30, part in bits 28-29; rows < 4096); the _kr form is np = 2.
int64_t gs_sym_unit_map_kr(int64_t n_pad, int32_t rank, int32_t nranks, int64_t fill,
                           int32_t kr, int32_t* out, int64_t cap);
int64_t gs_sym_unit_map_parts(int64_t n_pad, int32_t rank, int32_t nranks, int64_t fill,
                              int32_t kr, int32_t np, int32_t* out, int64_t cap);
// Split shell segments per row (SymArgs::Kr) for a geometry: S / 16 when a segment has at
// least 2 tiles of 128 bodies (L >= 2), else 0; and the parts each is split into (SymArgs::Np:
// 4 when L >= 4, else 2).
int32_t gs_sym_split_segments(int64_t n_pad);
int32_t gs_sym_split_parts(int64_t n_pad);
// The same for the ring strategy: entries carry the ring stage (bits 28-30) at which the last
// slice a unit reads arrives, and units are ordered by stage (rows < 4096, nranks <= 8).
int64_t gs_sym_unit_map_ring(int64_t n_pad, int32_t rank, int32_t nranks, int64_t fill,
                             int32_t* out, int64_t cap);

// ---------------------------------------------------------------- counter-based RNG / ICs (host)
// Fill bodies [begin, end) of the IC family into fp64 arrays (pos/vel: 3 per body, mass: 1).
void gs_ic_fill_host(int32_t ic, uint64_t seed, int64_t n, int64_t begin, int64_t end,
                     double* pos, double* vel, double* mass);

// ---------------------------------------------------------------- CPU engine (libgravsim_cpu)
// Accelerations for global bodies [i0, i1) against all j (positions X4 = x,y,z,mu; n_pad rows),
// summed in the canonical chunk order. acc4 gets (ax, ay, az, phi) per body. fp64 or fp32 (X4 type).
int gs_cpu_accel_f64(const double* X4, int64_t n_real, int64_t i0, int64_t i1, int32_t chunk,
                     double cut2, double eps2, double* acc4);
int gs_cpu_accel_f32(const float* X4, int64_t n_real, int64_t i0, int64_t i1, int32_t chunk,
                     float cut2, float eps2, float* acc4);
// One KD step for global bodies [i0, i1): reads X4 (full), vel4 (local, i0-based), writes
// Xnext4 rows [i0, i1) and vel4. Ghost rows (>= n_real) are zeroed.
// fp64 accelerations of rows [i0, i1) plus, per component, sum_j |term_ij| (8 doubles per
// row: a_x, a_y, a_z, 0, |.|_x, |.|_y, |.|_z, 0): the scale of a rounding-error bound.
int gs_cpu_accel_abs_f64(const double* X4, int64_t n_real, int64_t i0, int64_t i1, double cut2,
                         double eps2, double* out8);
// The same in long double (x87 extended): the reference of the fp64 accuracy gates.
int gs_cpu_accel_abs_ld(const double* X4, int64_t n_real, int64_t i0, int64_t i1, double cut2,
                        double eps2, double* out8);
int gs_cpu_step_f64(const double* X4, double* Xnext4, double* vel4, int64_t n_real, int64_t i0,
                    int64_t i1, int32_t chunk, double dt, double cut2, double eps2);
int gs_cpu_step_f32(const float* X4, float* Xnext4, float* vel4, int64_t n_real, int64_t i0,
                    int64_t i1, int32_t chunk, float dt, float cut2, float eps2);
int gs_cpu_num_threads(void);
int gs_cpu_set_threads(int32_t n);  // OpenMP threads for the CPU engine (returns the new max)

// ---------------------------------------------------------------- GPU Stepper (libgravsim_hip)
typedef struct gs_stepper gs_stepper;

int gs_stepper_create(const gs_config* cfg, gs_stepper** out);
int gs_stepper_destroy(gs_stepper* s);
int gs_stepper_layout(gs_stepper* s, gs_layout* out);
// Generate ICs on device (every rank generates the full position set and its own velocities).
int gs_stepper_init_ics(gs_stepper* s, int32_t ic, uint64_t seed);
// Upload a global fp64 state (pos n*3, vel n*3, mass n). Every rank passes the full arrays.
int gs_stepper_set_state(gs_stepper* s, const double* pos, const double* vel, const double* mass);
// Download: full gathered positions (n*3), this rank's velocities (global layout n*3: only the
// rank's own rows are written), masses (n). Any pointer may be NULL.
int gs_stepper_get_state(gs_stepper* s, double* pos, double* vel, double* mass);
// Enqueue n steps (asynchronous w.r.t. the host).
int gs_stepper_step(gs_stepper* s, int32_t nsteps);
int gs_stepper_sync(gs_stepper* s);
// Bounded wait (timeout_s <= 0: unbounded) polling RCCL async errors; aborts the communicator
// when no enqueued step completes for timeout_s (the deadline bounds progress, not the run).
int gs_stepper_wait(gs_stepper* s, double timeout_s);
// Accelerations (+potential) of this rank's bodies for the current positions: acc4 = n_local*4.
int gs_stepper_accel(gs_stepper* s, double* acc4);
// Accelerations through the step's own force path (configured kernel and cutoff mode, no
// potential): what the integrator sees. acc4[:, 3] is 0.
int gs_stepper_accel_step_path(gs_stepper* s, double* acc4);
// Non-finite guard: returns number of non-finite position/velocity components on this rank.
int64_t gs_stepper_count_nonfinite(gs_stepper* s);
int64_t gs_stepper_steps_done(gs_stepper* s);
// 1 if the next step starts a replayable two-step period (an even step whose buffer still
// needs its gather, multi-rank): steps from here run from the graph / segmented plan.
int32_t gs_stepper_period_start(gs_stepper* s);
// Per-step phase timing of the last step (ms): up to the local/force phase, the step's
// collectives (all-gather + node-sum exchange spans on the comm stream), and the whole step.
int gs_stepper_phase_ms(gs_stepper* s, float* local_ms, float* comm_ms, float* total_ms);
// Eager steps record per-step phase events while on (hipGraph replay is off meanwhile).
int gs_stepper_set_timing(gs_stepper* s, int32_t on);
// Averages over the timed steps since the last call: out[0] steps, [1] step ms, [2] gather
// ms, [3] exchange ms, [4] exposed gather ms, [5] exposed exchange ms (compute-stream stalls),
// [6] the most force units a step deferred past the gather (overlap 3), [7] reserved.
int gs_stepper_phase_stats(gs_stepper* s, double* out8);
// Sym schedule work beside the all-gather: 0 wait then one launch, 3 one local-first launch
// whose remote units run once the gather is published or are deferred to a second launch
// behind it (the default for nranks > 1; GRAVSIM_SYM_OVERLAP sets another initial value).
int gs_stepper_set_overlap(gs_stepper* s, int32_t mode);
int32_t gs_stepper_get_overlap(gs_stepper* s);
// Units a dynamic-fetch workgroup may take after the first wave (<= 1: static units).
int32_t gs_stepper_get_dyn_cap(gs_stepper* s);
// Schedule knobs for an independent re-run (bench.py's replay audit): use_graph 0 eager,
// 1 single-rank graphs, 2 multi-rank capture too; dyn_cap <= 1 static units (one per
// workgroup), > 1 dynamic fetch with that many units per workgroup, < 0 unchanged.
int gs_stepper_set_schedule(gs_stepper* s, int32_t use_graph, int32_t dyn_cap);
// Test / A-B tuning of the sym schedule (< 0 or 0: unchanged): first_wave = workgroups of
// the dynamic launch that take one unit each (default: the resident slots; tests shrink it so
// small runs fetch dynamically too); fused_tail 1 / 0 forces the one-rank fused reduction
// tail / the three-kernel tail (default: fused up to 256K bodies). Same bits either way.
int gs_stepper_set_tuning(gs_stepper* s, int32_t first_wave, int32_t fused_tail);
// One-rank sym launches with persistent workgroups (1, the default) or round 4's workgroup
// turnover (0): same units and slots, same bits.
int gs_stepper_set_persist(gs_stepper* s, int32_t on);
// Re-resolve the force path with a new cutoff mode (0 auto, 1 exact select, 2 fast core).
int gs_stepper_set_cutoff_mode(gs_stepper* s, int32_t mode);
// Work audit of the sym schedule: force units completed since the last reset (waits for the
// compute stream) and the units one step must run on this rank (rows x (S + D + (Np - 1) Kr):
// a split segment counts as its Np parts, whichever way it runs); both 0 for the one-sided
// schedules.
int gs_stepper_audit(gs_stepper* s, uint64_t* units_done, uint64_t* units_per_step);
int gs_stepper_audit_reset(gs_stepper* s);
// Engine clock of the sym force launches since the last call (then reset; waits for the
// compute stream): out4[0] the duration-weighted shader clock (GHz, s_memtime against
// s_memrealtime per workgroup), [1] workgroup shader-cycles, [2] workgroup-seconds, [3]
// workgroups. All 0 for the one-sided schedules.
int gs_stepper_clock(gs_stepper* s, double* out4);
// Compiled force-tile shape of the sym kernels for fp64 (0) or fp32: *waves per workgroup,
// *ipl i-bodies and *jpl j-bodies per lane (bench.py builds its kernel label from this).
int gs_sym_tile_shape(int32_t fp64, int32_t* waves, int32_t* ipl, int32_t* jpl);
// What the last replayed steps ran from: *mode 0 eager, 1 one hipGraph per two steps, 2 a
// segmented plan (multi-rank: compute segments as graphs, collectives eager between them);
// *segments = graph segments per two steps (mode 2).
int gs_stepper_graph_info(gs_stepper* s, int32_t* mode, int32_t* segments);
// Steps per replayed one-rank graph launch (GRAVSIM_GRAPH_STEPS; 2 = one ping-pong period).
int gs_stepper_graph_steps(gs_stepper* s);
// Device memory ledger: entry i (name, bytes) of the HBM buffers this stepper owns; returns
// the entry count (i out of range: only the count).
int32_t gs_stepper_mem_entry(gs_stepper* s, int32_t i, const char** tag, uint64_t* bytes);
// Unit timeline of the last sym force launch (stepper created with GRAVSIM_UNIT_TRACE set):
// copies up to `cap` entries of 4 words {start, end (100 MHz ticks), HW_ID | XCC_ID << 32,
// row << 32 | segment} (all zero: the slot ran no unit) and clears them. Returns the count;
// out = nullptr returns the capacity; 0 when tracing is off.
int64_t gs_stepper_unit_trace(gs_stepper* s, uint64_t* out, int64_t cap);
// Bound on the host waiting for the oldest of the enqueued steps when it runs far ahead.
int gs_stepper_set_timeout(gs_stepper* s, double step_timeout_s);
// Resolved force path: *exact = 1 for the hard-cutoff select, *eps2 = r^2 offset in use.
int gs_stepper_force_mode(gs_stepper* s, int32_t* exact, double* eps2);
void* gs_stepper_compute_stream(gs_stepper* s);

// Virtual ranks on one device: shards[r] created with rank r of P; steps all of them in
// lockstep with the all-gather done by device copies (the RCCL schedule without RCCL).
int gs_group_step(gs_stepper** shards, int32_t P, int32_t nsteps);

// RCCL: 128-byte unique id (rank 0 creates it; the launcher broadcasts it), then init.
int gs_rccl_unique_id(void* out128);
int gs_stepper_comm_init(gs_stepper* s, const void* id128, int32_t rank, int32_t nranks);
// Poll RCCL async errors; aborts the communicator on error. Returns 0 if healthy.
int gs_stepper_comm_check(gs_stepper* s);
// How far gs_stepper_comm_init got (safe to call from another thread, e.g. a watchdog):
// 0 not started, 1 in ncclCommInitRank, 2 warm-up all-gather, 3 warm-up ring send/recv,
// 4 warm-up peer send/recv, 5 waiting for the warm-up, 6 done, -1 aborted.
int32_t gs_stepper_comm_stage(gs_stepper* s);
// What the communicator is (ncclCommCount, ncclCommUserRank, ncclCommCuDevice, read at init
// and checked there against nranks / rank / the stepper's device): count 0 before comm_init
// or when none was kept (one rank).
int gs_stepper_comm_info(gs_stepper* s, int32_t* count, int32_t* user_rank, int32_t* cu_device);
// Abort the live RCCL communicator once (ncclCommAbort; callable from another thread to
// unblock collectives that will never complete). Returns 1 if it aborted, 0 if there was none.
int32_t gs_stepper_abort(gs_stepper* s);

int gs_hip_device_count(void);
const char* gs_hip_kernel_info(void);

// ---------------------------------------------------------------- HIP IPC (ipc.hip)
// Cross-process sharing of device memory and events on one node: what RCCL's intra-node P2P
// transport builds on (tests/test_ipc_gpu.py). Handles are HIP_IPC_HANDLE_SIZE (64) bytes.
int gs_dev_alloc(int32_t device, uint64_t bytes, void** out);
int gs_dev_free(void* p);
int gs_dev_copy(void* dst, const void* src, uint64_t bytes, int32_t to_device);
int gs_ipc_mem_handle(void* p, void* out64);
int gs_ipc_mem_open(int32_t device, const void* h64, void** out);
int gs_ipc_mem_close(void* p);
int gs_ipc_event_create(int32_t device, void** ev, void* out64);
int gs_ipc_event_open(int32_t device, const void* h64, void** ev);
int gs_event_record_sync(void* ev);
int gs_event_wait_sync(void* ev);
int gs_event_destroy(void* ev);

// ---------------------------------------------------------------- errors
const char* gs_last_error(void);

#ifdef __cplusplus
}
#endif
