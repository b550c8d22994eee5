// Internal to the native runtime (stepper.hip, stepper_comm.hip, stepper_plan.hip): the
// Stepper's state and the helpers its translation units share. Not part of the C API
// (gravsim.h).
#pragma once
#include <dlfcn.h>
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <unistd.h>
#include <math.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "gravsim.h"
#include "gs_common.h"
#include "gs_kernels.h"

void gs_set_error(const char* msg);

#define GS_HIP(call)                                                                \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      char b_[384];                                                                 \
      snprintf(b_, sizeof(b_), "%s:%d %s: %s", __FILE__, __LINE__, #call,           \
               hipGetErrorString(e_));                                              \
      gs_set_error(b_);                                                             \
      return -1;                                                                    \
    }                                                                               \
  } while (0)

#define GS_NCCL(call)                                                               \
  do {                                                                              \
    ncclResult_t r_ = (call);                                                       \
    if (r_ != ncclSuccess) {                                                        \
      char b_[384];                                                                 \
      snprintf(b_, sizeof(b_), "%s:%d %s: %s", __FILE__, __LINE__, #call,           \
               ncclGetErrorString(r_));                                             \
      gs_set_error(b_);                                                             \
      return -1;                                                                    \
    }                                                                               \
  } while (0)

struct gs_stepper {
  gs_config cfg;
  gs_layout L;
  size_t esz = 4;  // element size
  hipStream_t s_comp = nullptr, s_comm = nullptr;
  hipStream_t s_rem = nullptr;  // second compute stream: remote chunks beside the local ones
  hipStream_t s_rem2 = nullptr;  // third compute stream: ring sub-steps alternate rem/rem2
  hipEvent_t ev_rem2 = nullptr;
  std::vector<hipEvent_t> ev_recv;  // ring: per sub-step "slice arrived" events
  hipEvent_t ev_ready = nullptr, ev_gathered = nullptr, ev_remote = nullptr, ev_fork = nullptr;
  hipEvent_t ev_t0 = nullptr, ev_local = nullptr, ev_end = nullptr;
  void* X[2] = {nullptr, nullptr};
  void* vel = nullptr;
  void* partial = nullptr;
  void* acc = nullptr;
  double* mass_dev = nullptr;
  unsigned long long* nonfinite = nullptr;
  std::vector<double> mass_host;
  int64_t k = 0;  // steps done; current positions live in X[k & 1]
  bool full[2] = {true, false};
  ncclComm_t comm = nullptr;
  bool have_comm = false;
  // Watchdog view of the communicator (gs_stepper_comm_stage / gs_stepper_abort may run on
  // another thread): the handle once ncclCommInitRank returned it, and the init stage.
  std::atomic<ncclComm_t> comm_live{nullptr};
  std::atomic<int> comm_stage{0};
  // What RCCL formed (ncclCommCount / ncclCommUserRank / ncclCommCuDevice after init): checked
  // against the layout's nranks / rank and the stepper's device there, reported by
  // gs_stepper_comm_info (bench.py enforces one distinct GPU per rank on top of it).
  int32_t comm_count = 0, comm_user_rank = -1, comm_cu_device = -1;
  bool virt = false;  // member of a virtual-rank group (gather = device copies, gs_group_step)
  bool emulate = false;  // GRAVSIM_EMULATE_RANK: run one rank's launch shapes, no exchange
  // sym work beside a pending gather (GRAVSIM_SYM_OVERLAP, gs_stepper_set_overlap): 0 none
  // (wait, then one launch), 3 one launch with the rank-local units first and the remote ones
  // gated on the gather in-kernel (the multi-rank default).
  int sym_overlap = 0;
  hipGraphExec_t graph = nullptr;
  // One-rank runs also replay a graph of graph_steps steps (graph_steps / 2 ping-pong periods)
  // whenever that many are left: each graph launch costs an idle gap on the GPU (~14 us at
  // 65K under the profiler, against 0 between the kernels inside a graph), paid once per
  // launch instead of once per period. 32 up to 256K bodies, 8 up to 2M, else 2 (create);
  // GRAVSIM_GRAPH_STEPS overrides (even; <= 2: periods only).
  hipGraphExec_t graph_long = nullptr;
  int graph_steps = 2;
  bool timed = false;  // eager steps record phase events
  int own_c0 = 0, own_c1 = 0;  // this rank's chunks clipped to [0, n_chunks)
  bool exact = true;           // hard-cutoff select vs fast core-softened path
  double eps2 = 0.0;           // r^2 offset used by the kernels
  int cus = 256;               // compute units
  int occ[3] = {0, 0, 0};      // split-kernel workgroups per CU by force mode
  // Newton-3 symmetric schedule (GS_MODE_SYM): partial slots, node sums, geometry.
  char* sym_Pi = nullptr;  // element type: float or double (esz)
  char* sym_Pj = nullptr;
  char* sym_Pd = nullptr;
  char* sym_Px = nullptr;  // parts 1 .. Np-1 of the split segments [band][Kr][Np-1][3][kSymC]
  char* sym_S = nullptr;  // node sums by destination rank
  char* sym_R = nullptr;  // node sums of every rank, global node order (== sym_S, one rank)
  char* sym_Ti = nullptr;  // per-body i-side totals [3][n_local]
  char* sym_Bb = nullptr;  // multi-band runs: per-block leaf sums [own blocks][3][bodies]
  int32_t sym_NC = 0, sym_H = 0, sym_L = 0, sym_S_n = 0, sym_D = 1;
  int32_t sym_Kr = 0;    // split shell segments per row (gs_sym_split_segments)
  int32_t sym_Np = 2;    // parts per split segment (gs_sym_split_parts)
  // extra units per row from the split segments: a step runs rows x (S + D + kx) units
  int32_t sym_kx() const { return sym_Kr * (sym_Np - 1); }
  int32_t sym_band = 0;  // rows per band (Pi/Pj/Pd hold one band; a multiple of sym_RB)
  // Row blocks and reduction-tree nodes (gs_sym_nodes): rank q owns blocks
  // [blk_lo[q], blk_lo[q + 1]) = bodies [rbeg[q], rbeg[q] + rcnt[q]); it sends nn(q) nodes,
  // the first of them global node nbase[q].
  int32_t sym_B = 8, sym_RB = 1, sym_NN = 1;
  int32_t blk_lo[9] = {0};
  std::vector<int64_t> rbeg, rcnt;
  std::vector<int32_t> nn, nbase;
  bool uniform = true;  // every rank owns the same body count (P | B: ncclAllGather)
  // live[src * P + dst]: rank src's node sums for rank dst's bodies can be nonzero
  // (gs_sym_pair_live); the exchange skips the other pairs (their sums are +0.0)
  std::vector<char> live;
  bool pair_live(int src, int dst) const {
    return live.empty() || live[(size_t)src * cfg.nranks + dst] != 0;
  }
  hipEvent_t ev_sym = nullptr;
  hipEvent_t ev_stage[2] = {nullptr, nullptr};  // node sums of an exchange stage reduced
  // Per-rank emulation with modeled collectives (GRAVSIM_EMU_COMM GB/s > 0): every all-gather
  // and node-sum exchange becomes a comm_model_kernel of the same byte count on s_comm.
  double emu_gbps = 0.0, emu_lat_us = 15.0;
  int emu_wgs = 16;
  // GRAVSIM_EMU_LINKS=1: price the node-sum exchange per xGMI link (each source peer's bytes
  // at emu_gbps, the peers of a stage in parallel: the time of the largest) instead of all of
  // a rank's bytes through one emu_gbps pipe. The all-gather keeps the one-pipe price (a ring
  // is per-link bound).
  bool emu_links = false;
  void* emu_buf = nullptr;
  unsigned long long* utrace = nullptr;  // GRAVSIM_UNIT_TRACE: per force workgroup timeline
  // Dynamic unit fetch of the sym force launch (gs_stepper_set_schedule; <= 1: static units):
  // units per workgroup after the first wave, and the first wave's size (resident slots).
  // Round 3 took 2 (shorter-lived workgroups shorten the launch tail; against 4: 1M / 8 per
  // rank -1.0 %, 1M one GPU -0.2 %, 65K -1.4 %, profiles/r3s2_dyn_cap_ab.jsonl). With the
  // final units in quarter parts (round 4) the tail no longer needs that: 3 against 2, paired
  // per round, 1M one GPU -0.14 % (4 of 4 rounds), 65K -0.5 %, 1M / 8 per rank even
  // (profiles/r4s2_dyn_cap_quarter_parts_ab.jsonl). Same units and slots: same bits. fp64
  // keeps 4 (no gain from 2: profiles/r4s2_fp64_i8_dyncap_ab.jsonl).
  int dyn_cap = 3;
  int sym_first_wave = 0;
  bool sym_persist = true;  // one-rank dynamic launches: persistent workgroups (SymArgs::persist)
  int64_t utrace_main = 0;               // entries of the main launch (deferred ones follow)
  size_t emu_cap = 0;
  double clk_khz = 100000.0;  // device wall clock (wall_clock64) rate
  // Gather gates (sym_overlap 3): [0], [1] gate of X[0] / X[1]; [3] the most units one step
  // deferred past the gather (since the last phase_stats call). defer: count + unit list.
  unsigned* gate_buf = nullptr;
  unsigned* defer = nullptr;
  int32_t* sym_lf = nullptr;  // units-6 order: unit -> row, segment (bit 31 remote)
  // Ring strategy of the sym schedule: P-1 neighbour stages instead of one all-gather; the
  // gated launch waits per stage (ring_gate[8 * buffer + stage], set after each stage's
  // receive) and its unit map orders the remote units by stage.
  bool sym_ring = false;
  unsigned* ring_gate = nullptr;
  int fuse_tail = -1;         // -1 by size (<= 256K), 0 off, 1 on (gs_stepper_set_tuning)
  // fused tail: Ti's two halves in separate waves (1) or in one thread (0); -1 by size
  // (GRAVSIM_TAIL_SPLIT overrides, an A/B knob: same bits either way)
  // The split pays only where the grid is small: 65K (NC 32) 0.6875-0.6879 against
  // 0.6886-0.6904 ms one-thread; 128K (NC 64) 2.638 against 2.622 ms and 256K 10.44-10.46
  // against 10.31 ms, slower (profiles/r6_tail_split_ab.jsonl).
  int tail_split = -1;
  bool tail_split_on() const { return tail_split >= 0 ? tail_split != 0 : sym_NC <= 32; }
  // Phase timing of eager steps (timed): one event set per step, summed by phase_stats.
  struct PhaseEv {
    hipEvent_t t0, end, g0, g1, w0, w1, x0, x1, j0, j1;
    bool g, w, x, j;
    int nsteps;  // steps t0 .. end spans: 1, or 2 for a one-rank graph period
  };
  std::vector<PhaseEv> pev;
  int pev_used = 0;
  PhaseEv* pe = nullptr;  // the step being enqueued
  // Progress events (one per enqueued step or graph period) for the bounded wait: its
  // deadline restarts whenever one more completes, so it bounds progress, not the run.
  std::vector<hipEvent_t> prog;
  int64_t prog_rec = 0, prog_done = 0;
  double step_timeout_s = 0.0;  // 0: unbounded
  bool graph_failed = false;    // multi-rank capture refused: eager fallback
  bool work_zero = true;        // sym dynamic unit counter (gate_buf[4]) known to be 0
  // Work audit of the sym force launches (nbody_sym.hip: one batched add per workgroup of the
  // units it ran); a step runs rows x (S + D + (Np - 1) Kr) units on this rank (each split
  // segment counts as its Np parts) whatever the launch split or fetch order.
  unsigned long long* audit = nullptr;
  // Engine-clock record of the sym force launches (SymArgs::clk): {shader cycles, 100 MHz
  // ticks, workgroups} summed since the last gs_stepper_clock read.
  unsigned long long* clk = nullptr;
  // Fault injection for the audit's own test (GRAVSIM_FAULT_SKIP_UNITS=k): every dynamic
  // force launch starts its unit counter at k instead of 0, so units 0 .. k-1 never run,
  // exactly the failure class of a stale re-armed counter (a memset node when captured).
  unsigned fault_skip = 0;
  // Segmented step graph of multi-rank runs (use_graph 1): the compute stream's work between
  // two cross-stream points is captured as one graph segment; the collectives (RCCL, or the
  // emulation's modeled ones) and the event record/wait that order them against the compute
  // stream are issued eagerly between the segments on replay. RCCL is never captured, so the
  // socket-transport capture crash (profiles/r2_graph_comm_root_cause.txt) cannot occur.
  // Phase timing of a replayed plan (gs_stepper_set_timing): every op carries the step of
  // the period it belongs to (0 / 1) and a kWait op the stall it measures (mark: kMarkGather
  // = exposed gather, kMarkExchange = exposed node exchange); run_plan records the step's
  // t0 / end and the stall's events eagerly between the segments, and points `pe` at the
  // step's event set while the eager collectives run (their spans on s_comm).
  struct PlanOp {
    enum Kind { kGraph, kRecord, kWait, kHost } kind;
    hipGraphExec_t g;
    hipEvent_t ev;
    std::function<int()> fn;
    int step = 0;
    int mark = 0;
  };
  std::vector<PlanOp> plan;  // one ping-pong period (two steps)
  bool rec = false;          // recording a plan: s_comp is capturing a segment
  int rec_step = 0;          // recording: the step of the period being enqueued
  int seg_step = 0;          // recording: the step in which the open segment began
  int plan_graphs = 0;       // graph segments per period (diagnostics)
  int pev_plan = 0;          // timed steps that ran from a replayed plan (phase_stats)
  // Device memory ledger: every HBM buffer the stepper owns, by name (gs_stepper_mem_entry);
  // destroy frees exactly these. All of them are allocated before the first step, sized from
  // the layout (the sym bands from the free HBM), so nothing is allocated inside the loop.
  struct MemEntry {
    void* p;
    size_t bytes;
    const char* tag;
  };
  std::vector<MemEntry> mem;
  // Flag sync (fsync(): the multi-rank all-gather sym schedule): the cross-stream ordering
  // points are device counters with signal / wait kernels (comm_model.hip) instead of hipEvent
  // record / wait, so a replayed period is ONE compute graph plus the comm stream's eager ops,
  // no cut points. sync_buf[2 id] = signals of point id, [2 id + 1] = waits taken (kSync*);
  // sync_stats[3 k] = {stall ticks, waits, timeouts} of the compute stream's gather (k 0) and
  // exchange (k 1) waits, k 2 the comm stream's waits. GRAVSIM_SYNC=events keeps the events.
  // sync_stats[9]: the wait kernels' give-up bound in s_memrealtime ticks (a device word,
  // written by gs_stepper_set_timeout: captured graphs read the current value). sync_fail: a
  // sticky host-mapped word (hipHostMalloc, coherent) a wait that gave up sets, and the host
  // sets when it aborts the communicator; nonzero fails sync / wait / state reads
  // (sync_failed) and makes every later wait kernel fall through. [0] host view, device
  // pointer in sync_fail_dev.
  unsigned* sync_buf = nullptr;
  unsigned long long* sync_stats = nullptr;
  volatile unsigned* sync_fail = nullptr;
  unsigned* sync_fail_dev = nullptr;
  bool sync_events = false;  // GRAVSIM_SYNC=events
  bool plan_fsync = false;   // the recorded plan is one graph (flag sync) + comm host ops
};

#define GS_MARK(field, flag, stream)                             \
  do {                                                           \
    if (s->pe) {                                                 \
      GS_HIP(hipEventRecord(s->pe->field, (stream)));            \
      s->pe->flag = true;                                        \
    }                                                            \
  } while (0)

namespace gs::rt {

// What a compute-stream wait on another stream's event stands for, in the phase timing.
enum : int { kMarkNone = 0, kMarkGather = 1, kMarkExchange = 2 };
// Flag-sync points (gs_stepper::sync_buf): own slice of X written (compute -> comm, the
// all-gather's input), node sums of exchange stage 0 / 1 reduced (compute -> comm), exchange
// received (comm -> compute). The gather itself is published by the gate flag (level).
enum : int { kSyncReady = 0, kSyncStage0 = 1, kSyncStage1 = 2, kSyncExch = 3, kSyncCount = 4 };

inline size_t row_bytes(const gs_stepper* s) { return 4 * s->esz; }

// hipMalloc through the ledger; on failure the error names the buffer, its size and the
// free HBM (a 16M-body rank needs ~110 GB of partial slots).
template <typename T>
inline int dev_alloc(gs_stepper* s, T** p, size_t bytes, const char* tag) {
  void* v = nullptr;
  const hipError_t e = hipMalloc(&v, bytes ? bytes : 16);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    size_t free_b = 0, total_b = 0;
    (void)hipMemGetInfo(&free_b, &total_b);
    char b[320];
    snprintf(b, sizeof(b), "device allocation of %s (%.3f GB) failed: %s (free %.3f of %.3f GB)",
             tag, bytes / 1e9, hipGetErrorString(e), free_b / 1e9, total_b / 1e9);
    gs_set_error(b);
    return -1;
  }
  *p = static_cast<T*>(v);
  s->mem.push_back({v, bytes, tag});
  return 0;
}

// A multi-rank exchange is active: a real communicator, or the per-rank emulation.
inline bool xcomm(const gs_stepper* s) { return s->have_comm || s->emulate; }
// Remote slices must be brought in before they are read (RCCL, emulation, virtual ranks).
inline bool multi(const gs_stepper* s) { return s->have_comm || s->emulate || s->virt; }
// The sym kernels implement both cutoff paths (fast core and exact select).
inline bool use_sym(const gs_stepper* s) { return s->L.mode == GS_MODE_SYM; }
// Cross-stream ordering by device counters (flag sync) rather than events: the multi-rank
// sym schedule with the all-gather (the ring keeps its per-stage events).
// (--graph-comm captures the collectives into the step graph: that capture follows the comm
// stream through event edges, so it keeps the events.)
inline bool fsync(const gs_stepper* s) {
  return !s->sync_events && s->sync_buf && use_sym(s) && xcomm(s) && !s->sym_ring &&
         s->cfg.use_graph <= 1;
}

// ---- shared by the runtime's translation units -----------------------------------------
// stepper_plan.hip: compute-stream ordering points (eager, or cut points of a recorded
// segmented plan), step graphs, the progress-bounded wait.
int seg_cut(gs_stepper* s);
int seg_open(gs_stepper* s);
int comp_record(gs_stepper* s, hipEvent_t ev);
int comp_wait(gs_stepper* s, hipEvent_t ev, int mark = kMarkNone);
int comm_do(gs_stepper* s, std::function<int()> fn);
// Cross-stream points that switch between events and flag sync (fsync): compute -> comm
// (comp_signal on s_comp now, comm_wait_comp inside the comm op), comm -> compute
// (comm_signal_comp inside the comm op, comp_wait_comm on s_comp now). `ev` is the event of
// the event path; `id` the kSync point; `flag` a level flag for comp_wait_comm (the gate)
// instead of a counter.
int comp_signal(gs_stepper* s, hipEvent_t ev, int id, unsigned* clear = nullptr);
int comm_wait_comp(gs_stepper* s, hipEvent_t ev, int id);
int comm_signal_comp(gs_stepper* s, hipEvent_t ev, int id);
int comp_wait_comm(gs_stepper* s, hipEvent_t ev, int mark, int id, const unsigned* flag = nullptr);
void drop_graphs(gs_stepper* s);
int build_graph(gs_stepper* s, int steps = 2);
bool plan_ok(const gs_stepper* s);
int build_plan(gs_stepper* s);
int run_plan(gs_stepper* s);
int wait_until(gs_stepper* s, int64_t target, double timeout_s);
int note_progress(gs_stepper* s);

// stepper_comm.hip: the collectives (RCCL, the per-rank emulation's modeled ones).
int comm_model(gs_stepper* s, const void* src, size_t bytes, size_t src_cap,
               size_t time_bytes = SIZE_MAX);
void rank_slice(const gs_stepper* s, int q, int64_t* b0, int64_t* cnt);
int gather(gs_stepper* s, int cur, bool gate = false);
int ring_src(const gs_stepper* s, int sub);
void rank_chunks(const gs_stepper* s, int src, int* c0, int* c1);
int ring_xfer_rccl(gs_stepper* s, int cur, int sub);
int sym_reduce_exchange(gs_stepper* s, const gs::SymArgs& a0, bool* exchanged, bool* row_done);
// The flag-sync wait bound in s_memrealtime ticks: above the host's own progress bound
// (2 x the step timeout + 10 s, 600 s if unbounded; GRAVSIM_SYNC_LIMIT_S overrides, a test
// knob), so the host's abort wins a stall.
uint64_t sync_limit_ticks(const gs_stepper* s);
// Write it to the device word the wait kernels read (sync_stats[9]).
int write_sync_limit(gs_stepper* s);
// A flag-sync wait gave up (or the host aborted the communicator under one): sets the error,
// aborts a live communicator, returns true. Every host-side completion point checks it.
bool sync_failed(gs_stepper* s);
void maybe_install_crash_trace();
// ncclCommAbort once (the watchdog thread, a timeout or an async error may all ask for it).
bool abort_comm(gs_stepper* s);
// The communicator was aborted (comm_live null while have_comm): sets the error, true.
bool comm_dead(gs_stepper* s);

// stepper.hip: buffers, step enqueue, phase events.
gs_stepper::PhaseEv* phase_begin(gs_stepper* s);
size_t gather_bytes(const gs_stepper* s);
size_t exchange_bytes(const gs_stepper* s);
int ensure_partial(gs_stepper* s);
int enqueue_step_any(gs_stepper* s, bool capturing, bool gathered_externally = false);

}  // namespace gs::rt
