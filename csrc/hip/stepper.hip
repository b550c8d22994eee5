// GPU Stepper: device-resident N-body state and the per-step schedule.
//
// Reference parity:
//   cuda.cu:145-160  cudaMalloc / H2D once / per-step kernel + cudaDeviceSynchronize + D2H
//                    of forces + host update   -> everything stays on device; host transfers
//                    only at init, dump and checkpoint; no sync inside the step loop.
//   mpi.c:142-182    MPI_Init/Bcast/Type_create_struct -> RCCL communicator bootstrapped from a
//                    128-byte unique id; ICs are generated per rank (no broadcast needed).
//   mpi.c:227-236    MPI_Allgatherv (aliased buffers) + MPI_Barrier every step
//                    -> in-place ncclAllGather of (x, y, z, mu) rows on a high-priority comm
//                    stream, overlapped with the rank-local j-chunks on the compute stream;
//                    ordering by events, no barrier.
// One-sided split schedule, step k (P ranks, ping-pong buffers X[0], X[1]):
//   s_comm : wait(own slice of X[k&1] written) -> ncclAllGather in place -> record gathered
//   s_comp : split kernel over own chunks (reads only the own slice)     -> partials
//   s_rem  : wait(gathered) -> ONE split launch over every remote chunk  -> partials
//   s_comp : wait(remote) -> reduce in canonical chunk order + KD integrate
//            -> own slice of X[(k+1)&1]
// With one rank the step is a single fused launch (KD integrate in its epilogue) or split +
// reduce.
//
// Newton-3 sym schedule (GS_MODE_SYM, the default from 16K bodies fp32 / 32K fp64, any P up
// to 8; nbody_sym.hip):
//   s_comm : all-gather in place (ncclAllGather, or grouped ncclBroadcast for uneven slices),
//            then gate_set_kernel opens the gather gate
//   s_comp : ONE force launch, rank-local units first; a remote unit that finds the gate
//            closed defers itself; the deferred units run in a small launch behind the gather
//            event (sym_overlap 3, the multi-rank default) -> node reduce (this rank's dyadic
//            sub-trees of the row-block tree, per destination rank)
//   s_comm : node exchange: ncclSend/ncclRecv of every destination's node sums (one group)
//   s_comp : row reduce (i-side totals), then wait(exchange) -> finalize (the tree merge in
//            global node order + KD integrate) -> own slice of X[(k+1)&1]
// The partial slots and every summation order depend on n_pad only, so any P from 1 to 8
// gives the same bits.
//
// Replay: one rank captures two steps (one ping-pong period) as one hipGraph; multi-rank
// steps replay a segmented plan (compute segments as graphs, collectives eager between them,
// build_plan); use_graph >= 2 captures the collectives too (opt-in, --graph-comm).
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
  bool virt = false;  // member of a virtual-rank group (gather = device copies, gs_group_step)
  bool emulate = false;  // GRAVSIM_EMULATE_RANK: run one rank's launch shapes, no exchange
  // sym work beside a pending gather (GRAVSIM_SYM_OVERLAP): 0 none (wait, then one launch),
  // 1 the diagonal units first on the compute stream, 2 diagonal + rank-local shell units
  // concurrently with the rest on a second stream.
  int sym_overlap = 0;
  hipGraphExec_t graph = nullptr;
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
  char* sym_S = nullptr;  // node sums by destination rank
  char* sym_R = nullptr;  // node sums of every rank, global node order (== sym_S, one rank)
  char* sym_Ti = nullptr;  // per-body i-side totals [3][n_local]
  char* sym_Bb = nullptr;  // multi-band runs: per-block leaf sums [own blocks][3][bodies]
  int32_t sym_NC = 0, sym_H = 0, sym_L = 0, sym_S_n = 0, sym_D = 1;
  int32_t sym_band = 0;  // rows per band (Pi/Pj/Pd hold one band; a multiple of sym_RB)
  // Row blocks and reduction-tree nodes (gs_sym_nodes): rank q owns blocks
  // [blk_lo[q], blk_lo[q + 1]) = bodies [rbeg[q], rbeg[q] + rcnt[q]); it sends nn(q) nodes,
  // the first of them global node nbase[q].
  int32_t sym_B = 8, sym_RB = 1, sym_NN = 1;
  int32_t blk_lo[9] = {0};
  std::vector<int64_t> rbeg, rcnt;
  std::vector<int32_t> nn, nbase;
  bool uniform = true;  // every rank owns the same body count (P | B: ncclAllGather)
  hipEvent_t ev_sym = nullptr;
  // Per-rank emulation with modeled collectives (GRAVSIM_EMU_COMM_GBPS > 0): every all-gather
  // and node-sum exchange becomes a comm_model_kernel of the same byte count on s_comm.
  double emu_gbps = 0.0, emu_lat_us = 15.0;
  int emu_wgs = 16;
  void* emu_buf = nullptr;
  unsigned long long* utrace = nullptr;  // GRAVSIM_UNIT_TRACE: per force workgroup timeline
  // Dynamic unit fetch of the sym force launch (GRAVSIM_SYM_DYN_CAP; <= 1: static units):
  // units per workgroup after the first wave, and the first wave's size (resident slots).
  int dyn_cap = 4;
  int sym_first_wave = 0;
  int64_t utrace_main = 0;               // entries of the main launch (deferred ones follow)
  size_t emu_cap = 0;
  double clk_khz = 100000.0;  // device wall clock (wall_clock64) rate
  // Gather gates (sym_overlap 3): [0], [1] gate of X[0] / X[1]; [3] the most units one step
  // deferred past the gather (since the last phase_stats call). defer: count + unit list.
  unsigned* gate_buf = nullptr;
  unsigned* defer = nullptr;
  int32_t* sym_lf = nullptr;  // units-6 order: unit -> row << 16 | segment (bit 31 remote)
  // Ring strategy of the sym schedule: P-1 neighbour stages instead of one all-gather; the
  // gated launch waits per stage (ring_gate[8 * buffer + stage], set after each stage's
  // receive) and its unit map orders the remote units by stage.
  bool sym_ring = false;
  unsigned* ring_gate = nullptr;
  int gate_probe = 0;         // GRAVSIM_GATE_PROBE (emulation timing probes only)
  int diag_last = 1;          // GRAVSIM_SYM_DIAG_LAST=0: row-by-row unit order (A/B only)
  int fuse_tail = -1;         // GRAVSIM_SYM_FUSED_TAIL: -1 by size (<= 256K), 0 off, 1 on
  int parity = 1;             // GRAVSIM_SYM_PARITY=0: round-1 antipodal rule (A/B only)
  // Phase timing of eager steps (timed): one event set per step, summed by phase_stats.
  struct PhaseEv {
    hipEvent_t t0, end, g0, g1, w0, w1, x0, x1, j0, j1;
    bool g, w, x, j;
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
  // Work audit of the sym force launches: +1 per unit run (nbody_sym.hip audit_unit); a step
  // runs rows x (S + D) units on this rank whatever the launch split or fetch order.
  unsigned long long* audit = nullptr;
  // Fault injection for the audit's own test (GRAVSIM_FAULT_SKIP_UNITS=k): every dynamic
  // force launch starts its unit counter at k instead of 0, so units 0 .. k-1 never run,
  // exactly the failure class of a stale re-armed counter (a memset node when captured).
  unsigned fault_skip = 0;
  bool rearm_lastwg = false;  // GRAVSIM_SYM_REARM=lastwg: round 2's in-kernel counter re-arm
  // GRAVSIM_SYM_FORK_ROW=1 (A/B only): the row reduce on a second stream beside the node
  // reduce. Measured slower: the two streaming sums contend (reduce phase at 1M 1533-1592 us
  // per step against 1342-1381 in sequence; profiles/r3_reduce_fork_split_ab.txt).
  bool fork_row = false;
  // Segmented step graph of multi-rank runs (use_graph 1): the compute stream's work between
  // two cross-stream points is captured as one graph segment; the collectives (RCCL, or the
  // emulation's modeled ones) and the event record/wait that order them against the compute
  // stream are issued eagerly between the segments on replay. RCCL is never captured, so the
  // socket-transport capture crash (profiles/r2_graph_comm_root_cause.txt) cannot occur.
  struct PlanOp {
    enum Kind { kGraph, kRecord, kWait, kHost } kind;
    hipGraphExec_t g;
    hipEvent_t ev;
    std::function<int()> fn;
  };
  std::vector<PlanOp> plan;  // one ping-pong period (two steps)
  bool rec = false;          // recording a plan: s_comp is capturing a segment
  int plan_graphs = 0;       // graph segments per period (diagnostics)
  // Device memory ledger: every HBM buffer the stepper owns, by name (gs_stepper_mem_entry);
  // destroy frees exactly these. All of them are allocated before the first step, sized from
  // the layout (the sym bands from the free HBM), so nothing is allocated inside the loop.
  struct MemEntry {
    void* p;
    size_t bytes;
    const char* tag;
  };
  std::vector<MemEntry> mem;
};

namespace {

// Optional roctx ranges (GRAVSIM_ROCTX=1): resolved with dlopen so the library never links a
// profiler; under `rocprofv3 --marker-trace` the step phases show up on the timeline.
struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  Roctx() {
    if (!getenv("GRAVSIM_ROCTX")) return;
    for (const char* name : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                             "libroctx64.so"}) {
      void* h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
      pop = (int (*)())dlsym(h, "roctxRangePop");
      if (push && pop) return;
      push = nullptr;
      pop = nullptr;
    }
  }
};
Roctx& roctx() {
  static Roctx r;
  return r;
}
struct Range {
  bool on;
  explicit Range(const char* n) : on(roctx().push != nullptr) {
    if (on) roctx().push(n);
  }
  ~Range() {
    if (on) roctx().pop();
  }
};

size_t row_bytes(const gs_stepper* s) { return 4 * s->esz; }

// hipMalloc through the ledger; on failure the error names the buffer, its size and the
// free HBM (a 16M-body rank needs ~110 GB of partial slots).
template <typename T>
int dev_alloc(gs_stepper* s, T** p, size_t bytes, const char* tag) {
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

// ---- compute-stream ordering points (eager, or cut points of a recorded plan) ----------
// End the open capture segment and keep it as a graph if it holds any node.
int seg_cut(gs_stepper* s) {
  hipGraph_t g = nullptr;
  GS_HIP(hipStreamEndCapture(s->s_comp, &g));
  size_t nodes = 0;
  hipError_t e = hipGraphGetNodes(g, nullptr, &nodes);
  if (e == hipSuccess && nodes > 0) {
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (e == hipSuccess) {
      s->plan.push_back({gs_stepper::PlanOp::kGraph, x, nullptr, {}});
      ++s->plan_graphs;
    }
  }
  (void)hipGraphDestroy(g);
  GS_HIP(e);
  return 0;
}

int seg_open(gs_stepper* s) {
  GS_HIP(hipStreamBeginCapture(s->s_comp, hipStreamCaptureModeThreadLocal));
  return 0;
}

// hipEventRecord(ev, s_comp) for another stream to wait on.
int comp_record(gs_stepper* s, hipEvent_t ev) {
  if (!s->rec) {
    GS_HIP(hipEventRecord(ev, s->s_comp));
    return 0;
  }
  if (seg_cut(s)) return -1;
  s->plan.push_back({gs_stepper::PlanOp::kRecord, nullptr, ev, {}});
  return seg_open(s);
}

// hipStreamWaitEvent(s_comp, ev) on an event another stream records.
int comp_wait(gs_stepper* s, hipEvent_t ev) {
  if (!s->rec) {
    GS_HIP(hipStreamWaitEvent(s->s_comp, ev, 0));
    return 0;
  }
  if (seg_cut(s)) return -1;
  s->plan.push_back({gs_stepper::PlanOp::kWait, nullptr, ev, {}});
  return seg_open(s);
}

// Work on the comm stream (a collective and its event bookkeeping): run now, or replayed
// eagerly at this point of the plan.
int comm_do(gs_stepper* s, std::function<int()> fn) {
  if (!s->rec) return fn();
  if (seg_cut(s)) return -1;
  s->plan.push_back({gs_stepper::PlanOp::kHost, nullptr, nullptr, std::move(fn)});
  return seg_open(s);
}

void drop_graphs(gs_stepper* s) {
  if (s->graph) {
    (void)hipGraphExecDestroy(s->graph);
    s->graph = nullptr;
  }
  for (auto& op : s->plan)
    if (op.g) (void)hipGraphExecDestroy(op.g);
  s->plan.clear();
  s->plan_graphs = 0;
}

// A multi-rank exchange is active: a real communicator, or the per-rank emulation.
bool xcomm(const gs_stepper* s) { return s->have_comm || s->emulate; }
// Remote slices must be brought in before they are read (RCCL, emulation, virtual ranks).
bool multi(const gs_stepper* s) { return s->have_comm || s->emulate || s->virt; }

// Bytes one rank receives per step: the all-gather's remote slices, and the node sums the
// other ranks send it (sym schedule).
size_t gather_bytes(const gs_stepper* s) {
  return (size_t)(s->L.n_pad - s->L.n_local) * row_bytes(s);
}
size_t exchange_bytes(const gs_stepper* s) {
  return (size_t)(s->sym_NN - s->nn[s->cfg.rank]) * 3 * s->L.n_local * s->esz;
}

// Emulated collective on s_comm (GRAVSIM_EMU_COMM_GBPS > 0): the byte count moved through HBM
// by emu_wgs workgroups that stay resident for latency + bytes / rate (comm_model.hip). The
// kernel copies min(bytes, src_cap, emu_cap) bytes (src_cap: what the source buffer holds);
// the modeled time always uses the full byte count.
int comm_model(gs_stepper* s, const void* src, size_t bytes, size_t src_cap) {
  if (s->emu_gbps <= 0.0 || bytes == 0) return 0;
  const double us = s->emu_lat_us + (double)bytes / (s->emu_gbps * 1e3);
  if (bytes > s->emu_cap) bytes = s->emu_cap;  // (sized at create for the larger collective)
  if (bytes > src_cap) bytes = src_cap;
  const uint64_t ticks = (uint64_t)(us * s->clk_khz / 1e3);
  GS_HIP(gs::launch_comm_model(src, s->emu_buf, bytes, ticks, s->emu_wgs, s->s_comm));
  return 0;
}

// Phase events of the step being enqueued (timed eager steps; at most 256 per phase_stats).
gs_stepper::PhaseEv* phase_begin(gs_stepper* s) {
  if (s->pev_used >= (int)s->pev.size()) {
    if (s->pev.size() >= 256) return nullptr;
    gs_stepper::PhaseEv e{};
    for (hipEvent_t* p : {&e.t0, &e.end, &e.g0, &e.g1, &e.w0, &e.w1, &e.x0, &e.x1, &e.j0, &e.j1})
      if (hipEventCreate(p) != hipSuccess) return nullptr;
    s->pev.push_back(e);
  }
  gs_stepper::PhaseEv* p = &s->pev[s->pev_used++];
  p->g = p->w = p->x = p->j = false;
  return p;
}
#define GS_MARK(field, flag, stream)                             \
  do {                                                           \
    if (s->pe) {                                                 \
      GS_HIP(hipEventRecord(s->pe->field, (stream)));            \
      s->pe->flag = true;                                        \
    }                                                            \
  } while (0)

template <typename T>
gs::KArgs<T> base_args(gs_stepper* s, int cur) {
  gs::KArgs<T> a;
  memset(&a, 0, sizeof(a));
  a.X = static_cast<const T*>(s->X[cur]);
  a.X_next = static_cast<T*>(s->X[cur ^ 1]);
  a.vel = static_cast<T*>(s->vel);
  a.partial = static_cast<T*>(s->partial);
  a.acc_out = nullptr;
  a.i_begin = s->L.local_begin;
  a.n_local = s->L.n_local;
  a.n_real = s->L.n;
  a.chunk = s->L.chunk;
  a.n_chunks = s->L.n_chunks;
  a.c_begin = 0;
  a.c_end = s->L.n_chunks;
  a.phi = 0;
  a.exact = s->exact ? 1 : 0;
  a.dt = (T)s->cfg.dt;
  a.cut2 = (T)(s->cfg.cutoff * s->cfg.cutoff);
  a.eps2 = (T)s->eps2;
  return a;
}

// The sym kernels implement both cutoff paths (fast core and exact select).
bool use_sym(const gs_stepper* s) { return s->L.mode == GS_MODE_SYM; }

gs::SymArgs sym_args(gs_stepper* s, int cur) {
  gs::SymArgs a;
  memset(&a, 0, sizeof(a));
  a.X = s->X[cur];
  a.X_next = s->X[cur ^ 1];
  a.vel = s->vel;
  a.fp64 = s->esz == 8;
  a.Pi = s->sym_Pi;
  a.Pj = s->sym_Pj;
  a.Pd = s->sym_Pd;
  a.Sbuf = s->sym_S;
  a.Rbuf = s->sym_R;
  a.Ti = s->sym_Ti;
  a.n_real = s->L.n;
  a.n_local = s->L.n_local;
  a.i_begin = s->L.local_begin;
  a.NC = s->sym_NC;
  a.P = s->cfg.nranks;
  a.rows = (int32_t)(s->L.n_local / gs::kSymC);
  a.a0 = (int32_t)(s->L.local_begin / gs::kSymC);
  a.B = s->sym_B;
  a.RB = s->sym_RB;
  a.rank = s->cfg.rank;
  a.nn = s->nn[s->cfg.rank];
  a.node_maxl = gs_sym_node_maxl(s->sym_B, s->cfg.nranks);
  for (int q = 0; q <= s->cfg.nranks && q < 9; ++q) a.blk_lo[q] = s->blk_lo[q];
  a.Bbuf = s->sym_Bb;
  a.S = s->sym_S_n;
  a.L = s->sym_L;
  a.D = s->sym_D;
  a.H = s->sym_H;
  a.real_chunks = (int32_t)((s->L.n + gs::kSymC - 1) / gs::kSymC);
  a.dt = s->cfg.dt;
  a.eps2 = s->eps2;
  a.exact = s->exact ? 1 : 0;
  a.cut2 = s->cfg.cutoff * s->cfg.cutoff;
  a.band0 = 0;
  a.band_rows = a.rows;
  a.gate = nullptr;
  a.defer = s->defer;
  a.defer_max = s->gate_buf + 3;
  a.lf = s->sym_lf;
  a.defer_grid = 2 * s->cus;  // resident force workgroups: 2 per CU
  a.defer_index = 0;
  a.gate_probe = s->emulate ? s->gate_probe : 0;
  a.utrace = s->utrace;
  if (s->dyn_cap > 1) {
    a.work = s->gate_buf + 4;
    a.unit_cap = s->dyn_cap;
    a.first_wave = s->sym_first_wave;
  }
  a.trace_defer0 = (int32_t)s->utrace_main;
  a.diag_last = s->diag_last;
  a.parity = s->parity;
  a.audit = s->audit;
  return a;
}

// Group-sum exchange of the symmetric schedule: rank r sends S_g(x) of its groups for the
// bodies of rank q to q (ncclSend/ncclRecv pairs, one group call) and keeps its own block.
// With join = false the compute stream does not wait for it yet (the caller joins with
// hipStreamWaitEvent(s_comp, ev_sym) after work that does not read Rbuf).
int sym_exchange_rccl(gs_stepper* s, bool join = true) {
  if (comp_record(s, s->ev_ready)) return -1;
  if (comm_do(s, [s]() -> int {
        // To rank q: this rank's nn node sums of q's bodies (Sbuf block q); from rank q: its
        // nn(q) node sums of this rank's bodies, at its global node offset in Rbuf.
        const int P = s->cfg.nranks, r = s->cfg.rank;
        const size_t e = s->esz, nl = (size_t)s->L.n_local, my = (size_t)s->nn[r];
        const ncclDataType_t dt = s->esz == 8 ? ncclFloat64 : ncclFloat32;
        GS_HIP(hipStreamWaitEvent(s->s_comm, s->ev_ready, 0));
        GS_MARK(x0, x, s->s_comm);
        GS_HIP(hipMemcpyAsync(s->sym_R + (size_t)s->nbase[r] * 3 * nl * e,
                              s->sym_S + my * 3 * (size_t)s->rbeg[r] * e, my * 3 * nl * e,
                              hipMemcpyDeviceToDevice, s->s_comm));
        if (s->emulate) {
          // (the bytes this rank receives, read from its receive buffer: NN x 3 per own body)
          if (comm_model(s, s->sym_R, exchange_bytes(s),
                         (size_t)s->sym_NN * 3 * (size_t)s->L.n_local * s->esz))
            return -1;
        } else if (P > 1) {
          GS_NCCL(ncclGroupStart());
          for (int q = 0; q < P; ++q) {
            if (q == r) continue;
            GS_NCCL(ncclSend(s->sym_S + my * 3 * (size_t)s->rbeg[q] * e, my * 3 * s->rcnt[q], dt,
                             q, s->comm, s->s_comm));
            GS_NCCL(ncclRecv(s->sym_R + (size_t)s->nbase[q] * 3 * nl * e, (size_t)s->nn[q] * 3 * nl,
                             dt, q, s->comm, s->s_comm));
          }
          GS_NCCL(ncclGroupEnd());
        }
        GS_MARK(x1, x, s->s_comm);
        GS_HIP(hipEventRecord(s->ev_sym, s->s_comm));
        return 0;
      }))
    return -1;
  if (join) {
    GS_MARK(j0, j, s->s_comp);
    if (comp_wait(s, s->ev_sym)) return -1;
    GS_MARK(j1, j, s->s_comp);
  }
  return 0;
}

int ensure_sym(gs_stepper* s) {
  if (s->L.mode != GS_MODE_SYM || s->sym_Pi) return 0;
  if (gs_sym_geometry(s->L.n_pad, &s->sym_NC, &s->sym_H, &s->sym_L, &s->sym_S_n, &s->sym_D))
    return -1;
  const int P = s->cfg.nranks;
  s->rbeg.assign(P, 0);
  s->rcnt.assign(P, 0);
  s->nn.assign(P, 0);
  s->nbase.assign(P, 0);
  for (int q = 0; q < P; ++q) {
    int32_t a0 = 0, rw = 0, nb = 0, nnq = 0;
    if (gs_sym_rank_rows(s->L.n_pad, P, q, &a0, &rw) ||
        gs_sym_nodes(s->L.n_pad, P, q, &s->sym_B, &s->sym_RB, &nnq, &nb, &s->sym_NN))
      return -1;
    s->rbeg[q] = (int64_t)a0 * gs::kSymC;
    s->rcnt[q] = (int64_t)rw * gs::kSymC;
    s->nn[q] = nnq;
    s->nbase[q] = nb;
    s->uniform = s->uniform && s->rcnt[q] == s->rcnt[0];
  }
  for (int q = 0; q <= P && q < 9; ++q) s->blk_lo[q] = gs::sym_blk_lo(s->sym_B, P, q);
  const size_t nl = (size_t)s->L.n_local, rows = nl / gs::kSymC;
  const size_t e = s->esz;
  // Rows per band: the partial slots of one band stay within the budget: half of the free
  // HBM at creation (an MI355X has 288 GB; at least 32 GiB), GRAVSIM_SYM_BAND_MB overrides
  // (tests use a tiny budget to force many bands). 1M bodies need 6.4 GB for all rows; 16M
  // on 8 ranks needs 109 GB per rank, one band on an otherwise empty MI355X.
  const size_t per_row = (size_t)(s->sym_S_n + s->sym_H + s->sym_D) * 3 * gs::kSymC * e;
  size_t budget = (size_t)32 << 30;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b / 2 > budget) budget = free_b / 2;
  if (const char* mb = getenv("GRAVSIM_SYM_BAND_MB")) budget = (size_t)atoll(mb) << 20;
  // Bands hold whole row blocks, so each band's block leaves are complete (Bbuf).
  const size_t rb = (size_t)s->sym_RB;
  size_t band = budget / per_row / rb * rb;
  if (band < rb) band = rb;
  if (band > rows) band = rows;
  s->sym_band = (int32_t)band;
  if (dev_alloc(s, &s->sym_Pi, band * s->sym_S_n * 3 * gs::kSymC * e, "sym_Pi")) return -1;
  if (dev_alloc(s, &s->sym_Pj, band * s->sym_H * 3 * gs::kSymC * e, "sym_Pj")) return -1;
  if (dev_alloc(s, &s->sym_Pd, band * s->sym_D * 3 * gs::kSymC * e, "sym_Pd")) return -1;
  if (dev_alloc(s, &s->sym_Ti, 3 * nl * e, "sym_Ti")) return -1;
  const size_t nb = (size_t)((s->L.n + gs::kSymC - 1) / gs::kSymC) * gs::kSymC;  // real chunks
  if (band < rows && dev_alloc(s, &s->sym_Bb, rows / rb * 3 * nb * e, "sym_Bbuf")) return -1;
  const int r = s->cfg.rank;
  if (dev_alloc(s, &s->sym_S, (size_t)s->nn[r] * 3 * (size_t)s->L.n_pad * e, "sym_S")) return -1;
  // (zeroed once: the per-rank emulation never receives the other ranks' nodes)
  GS_HIP(hipMemsetAsync(s->sym_S, 0, (size_t)s->nn[r] * 3 * (size_t)s->L.n_pad * e, s->s_comp));
  if (P > 1) {
    if (dev_alloc(s, &s->sym_R, (size_t)s->sym_NN * 3 * nl * e, "sym_R")) return -1;
    GS_HIP(hipMemsetAsync(s->sym_R, 0, (size_t)s->sym_NN * 3 * nl * e, s->s_comp));
  } else {
    s->sym_R = s->sym_S;  // [node 0][3][n_pad] either way
  }
  return 0;
}

// Choose the fast or exact force path once the masses are known. The fast path adds a core
// c^2 to r^2 instead of selecting on the cutoff; c^2 is the smallest value that keeps
// mu_max * c^-3 (the self term's s) finite, so s * dx = 0 for the self term. It is used only
// when the requested cutoff lies inside that core (the default 1e-10 m does).
int ensure_partial(gs_stepper* s) {
  if (s->partial) return 0;
  return dev_alloc(s, &s->partial, (size_t)s->L.n_chunks * s->L.n_local * row_bytes(s), "partial");
}

void resolve_force_mode(gs_stepper* s) {
  double mu_max = 0.0;
  for (double m : s->mass_host) mu_max = fmax(mu_max, s->cfg.G * m);
  const double big = s->esz == 4 ? 3.4028234663852886e38 / 16.0 : 1.7976931348623157e308 / 16.0;
  const double floor2 = s->esz == 4 ? 1e-30 : 1e-290;
  const double core2 = fmax(pow(mu_max / big, 2.0 / 3.0), floor2);
  const double soft2 = s->cfg.softening * s->cfg.softening;
  const double cut2 = s->cfg.cutoff * s->cfg.cutoff;
  // fp64: the core is ~1e-190 m^2, far inside the cutoff, so the fast path softens at the
  // cutoff scale instead (eps2 = cut^2): r^2 + eps2 rounds to r^2 for every pair with
  // r^2 >= 2^53 eps2, i.e. r >= ~1 cm at the reference's 1e-10 m, the same guarantee fp32's
  // core gives. auto takes it while that radius is <= 1 cm (the select costs 7 % at 512K
  // fp64: 106.9 vs 99.2 ms, profiles/r2_fp64_fast_cutoff.txt).
  const double fast_eps2 = s->esz == 8 ? fmax(fmax(soft2, core2), cut2) : fmax(soft2, core2);
  bool exact;
  if (s->cfg.cutoff_mode == 1) exact = true;
  else if (s->cfg.cutoff_mode == 2) exact = false;
  else if (s->esz == 8) exact = fast_eps2 * 0x1p53 > 1e-4;
  else exact = cut2 > fast_eps2;
  s->exact = exact;
  s->eps2 = exact ? soft2 : fast_eps2;
}

// Chunk groups for one split launch of `span` chunks over the i-blocks: minimise
// rounds(g) * chunks_per_group(g) with rounds = ceil(i_blocks * g / resident).
int choose_groups(gs_stepper* s, int span, bool phi, bool concurrent = false) {
  if (span <= 0) return 1;
  if (s->cfg.split_groups > 0) return s->cfg.split_groups < span ? s->cfg.split_groups : span;
  // Local and remote launches share the GPU (two compute streams): one chunk per workgroup
  // lets the dispatcher balance both launches dynamically (multi-chunk workgroups of the
  // later launch would start behind the earlier one's and set a long tail).
  if (concurrent) return span;
  const int fm = phi ? 2 : (s->exact ? 1 : 0);
  const int64_t resident = (int64_t)(s->occ[fm] > 0 ? s->occ[fm] : 4) * s->cus;
  const int64_t ib = s->L.n_local / (GS_BLOCK * s->L.ipl);
  int best = 1;
  double best_cost = 1e300;
  for (int g = 1; g <= span; ++g) {
    const int64_t per = (span + g - 1) / g;
    if (g > 1 && (int64_t)(g - 1) * per >= span) continue;  // an empty trailing group
    const int64_t rounds = (ib * g + resident - 1) / resident;
    const double cost = (double)rounds * (double)per;
    // ties: prefer more workgroups (dynamic balance) while they fit in a few rounds
    const bool better = cost < best_cost * (1 - 1e-9) ||
                        (cost <= best_cost * (1 + 1e-9) && rounds <= 4 && g > best);
    if (better) {
      best = g;
      best_cost = cost;
    }
  }
  return best;
}

int ring_xfer_rccl(gs_stepper* s, int cur, int sub);
int ring_src(const gs_stepper* s, int sub);

// Bodies [*b0, *b0 + *cnt) of rank q's slice: the sym schedule's row blocks (uneven when P
// does not divide the block count), else equal slices.
void rank_slice(const gs_stepper* s, int q, int64_t* b0, int64_t* cnt) {
  if (!s->rbeg.empty()) {
    *b0 = s->rbeg[q];
    *cnt = s->rcnt[q];
  } else {
    *b0 = (int64_t)q * s->L.n_local;
    *cnt = s->L.n_local;
  }
}

// In-place all-gather of X[cur] on s_comm (ev_gathered marks completion). With `gate` the
// comm stream also publishes completion to a force launch already running (units 6). The sym
// schedule's ring strategy moves the slices in P-1 neighbour stages instead and, gated,
// publishes each stage as it lands (ring_gate[8 * cur + k]), so the units that read only
// slices already received can start.
int gather(gs_stepper* s, int cur, bool gate = false) {
  if (!xcomm(s) || s->full[cur]) return 0;
  if (comp_record(s, s->ev_ready)) return -1;
  s->full[cur] = true;
  return comm_do(s, [s, cur, gate]() -> int {
    char* buf = static_cast<char*>(s->X[cur]);
    const size_t count = (size_t)s->L.n_local * 4;
    GS_HIP(hipStreamWaitEvent(s->s_comm, s->ev_ready, 0));
    GS_MARK(g0, g, s->s_comm);
    const ncclDataType_t dt = s->esz == 4 ? ncclFloat32 : ncclFloat64;
    if (s->sym_ring && use_sym(s)) {
      for (int k = 1; k < s->cfg.nranks; ++k) {
        if (s->emulate) {
          const size_t sl = (size_t)s->rcnt[ring_src(s, k)] * row_bytes(s);
          if (comm_model(s, buf, sl, (size_t)s->L.n_pad * row_bytes(s))) return -1;
        } else if (ring_xfer_rccl(s, cur, k)) {
          return -1;
        }
        if (gate) GS_HIP(gs::launch_gate_set(s->ring_gate + 8 * cur + k, s->s_comm));
      }
    } else if (s->emulate) {
      if (comm_model(s, buf, gather_bytes(s), (size_t)s->L.n_pad * row_bytes(s))) return -1;
    } else if (!use_sym(s) || s->uniform) {
      GS_NCCL(ncclAllGather(buf + (size_t)s->L.local_begin * row_bytes(s), buf, count, dt,
                            s->comm, s->s_comm));
    } else {
      // Uneven row blocks (P not dividing the block count): every rank broadcasts its own
      // slice in place, all P in one group call (the Allgatherv of mpi.c:227-231).
      GS_NCCL(ncclGroupStart());
      for (int q = 0; q < s->cfg.nranks; ++q) {
        char* sl = buf + (size_t)s->rbeg[q] * row_bytes(s);
        GS_NCCL(ncclBroadcast(sl, sl, (size_t)s->rcnt[q] * 4, dt, q, s->comm, s->s_comm));
      }
      GS_NCCL(ncclGroupEnd());
    }
    GS_MARK(g1, g, s->s_comm);
    if (gate && !(s->sym_ring && use_sym(s)))
      GS_HIP(gs::launch_gate_set(s->gate_buf + cur, s->s_comm));
    GS_HIP(hipEventRecord(s->ev_gathered, s->s_comm));
    return 0;
  });
}

// ---- ring pass (strategy 1) ------------------------------------------------------------
// Rank r computes its own chunks first (sub-step 0), then at sub-step s the slice of rank
// (r - s) mod P, which arrives from the left neighbour while sub-step s-1 computes; it is
// forwarded to the right neighbour in the next sub-step. Each slice lands at its own offset
// of X[cur], so no buffer is reused within a step; per-chunk partials + the canonical reduce
// keep the result bit-identical to the all-gather schedule.
int ring_src(const gs_stepper* s, int sub) {
  const int P = s->cfg.nranks;
  return ((s->cfg.rank - sub) % P + P) % P;
}

void rank_chunks(const gs_stepper* s, int src, int* c0, int* c1) {
  const int64_t per = s->L.n_local / s->L.chunk;
  int64_t a = (int64_t)src * per, b = a + per;
  if (a > s->L.n_chunks) a = s->L.n_chunks;
  if (b > s->L.n_chunks) b = s->L.n_chunks;
  *c0 = (int)a;
  *c1 = (int)b;
}

// Enqueue the transfer of ring sub-step `sub` (1..P-1) on the comm stream: send the slice
// received at sub-step sub-1 (own slice for sub = 1) right, receive slice ring_src(sub) left.
int ring_xfer_rccl(gs_stepper* s, int cur, int sub) {
  const int P = s->cfg.nranks, r = s->cfg.rank;
  char* buf = static_cast<char*>(s->X[cur]);
  const ncclDataType_t dt = s->esz == 4 ? ncclFloat32 : ncclFloat64;
  int64_t sb, sc, rb, rc;
  rank_slice(s, ring_src(s, sub - 1), &sb, &sc);
  rank_slice(s, ring_src(s, sub), &rb, &rc);
  GS_NCCL(ncclGroupStart());
  GS_NCCL(ncclSend(buf + (size_t)sb * row_bytes(s), (size_t)sc * 4, dt, (r + 1) % P, s->comm,
                   s->s_comm));
  GS_NCCL(ncclRecv(buf + (size_t)rb * row_bytes(s), (size_t)rc * 4, dt, (r - 1 + P) % P, s->comm,
                   s->s_comm));
  GS_NCCL(ncclGroupEnd());
  return 0;
}

template <typename T>
int ring_compute(gs_stepper* s, const gs::KArgs<T>& a, int sub, hipEvent_t ready) {
  int c0, c1;
  rank_chunks(s, ring_src(s, sub), &c0, &c1);
  gs::KArgs<T> k = a;
  k.c_begin = c0;
  k.c_end = c1;
  hipStream_t st = sub == 0 ? s->s_comp : ((sub & 1) ? s->s_rem : s->s_rem2);
  if (ready) GS_HIP(hipStreamWaitEvent(st, ready, 0));
  GS_HIP(gs::launch_force_split<T>(k, s->L.kernel, s->L.ipl, choose_groups(s, c1 - c0, false, true),
                                   st));
  return 0;
}

template <typename T>
int ring_finish(gs_stepper* s, const gs::KArgs<T>& a) {
  GS_HIP(hipEventRecord(s->ev_remote, s->s_rem));
  GS_HIP(hipEventRecord(s->ev_rem2, s->s_rem2));
  GS_HIP(hipStreamWaitEvent(s->s_comp, s->ev_remote, 0));
  GS_HIP(hipStreamWaitEvent(s->s_comp, s->ev_rem2, 0));
  GS_HIP(gs::launch_reduce_integrate<T>(a, s->s_comp));
  return 0;
}

// Symmetric schedule, parts: 1 = force + node reduce (+ RCCL node-sum exchange),
// 2 = finalize (sum + integrate), 3 = both. Virtual-rank groups run part 1 on every shard,
// exchange by device copies, then part 2 (gs_group_step).
// Force + reductions over the rank's rows, band by band: the force units, the block / node
// reduce (multi-band runs: block leaves into Bbuf, the node reduce after the last band) and
// the row reduce (Ti). With one band
// and a pending all-gather (sym_overlap: the multi-rank default is 3, GRAVSIM_SYM_OVERLAP or
// gs_stepper_set_overlap choose another):
//   3: ONE launch whose grid lists the rank-local units first; a remote unit runs if the
//     gather has been published (gate flag set on the comm stream), else it defers itself to
//     a second small launch queued behind the gather event. No launch boundary and no
//     waiting workgroup: per-rank emulation of 1M / 8 with the collectives modeled at
//     64 GB/s + 15 us, 22.42-22.59 ms against 22.74-22.87 ms for 0 (docs/DESIGN.md §7,
//     profiles/r2_overlap_fill_ab.jsonl);
//   0: wait for the gather, then one launch of every unit;
//   1: the diagonal-chunk units (own rows only) run beside the gather, then the shell units
//     after it;
//   2: the diagonal units and the shell segments whose j-chunks are all own rows (1M, P = 8:
//     2080 of 16448 units) run on s_comp beside the gather and the other shell units on
//     s_rem after it, concurrently.
// Modes 1 and 2 pay a launch boundary (a unit is ~0.6 ms of work at 1M) to hide a ~0.1 ms
// gather and lost to 0 in round 1's emulation with free collectives (0: 21.0-21.2 ms,
// 1: 21.4-21.6, 2: 22.4-22.6; profiles/r1_sym_overlap_ab.txt); they are kept for A/B runs.
// With `exchange` the RCCL node-sum exchange starts right
// after the node reduce and runs beside the last row reduce; the compute stream joins
// it afterwards.
// One rank (no exchange, no virtual shards), one band, up to 256K bodies: the tree over the
// row blocks, the row reduce and finalize run as one sym_tail_kernel (same bits). Interleaved A/B
// (profiles/r2_fused_tail_ab.jsonl): 65K 0.707 vs 0.708 ms, 256K 10.51 vs 10.57 ms, but 1M
// 166.8 vs 166.1 ms, where the fused kernel's fewer threads for the j-side sums lose.
// GRAVSIM_SYM_FUSED_TAIL=0 / 1 forces the three-kernel / fused tail at any size.
// Every sym force launch goes through here: it tells the launcher whether the dynamic unit
// counter is known to be 0 (re-armed by the fused tail kernel enqueued after the previous
// launch on this stream), then marks it dirty until the next fused tail.
hipError_t force_sym_launch(gs_stepper* s, gs::SymArgs a, hipStream_t st) {
  a.work_zero = s->work_zero || s->rearm_lastwg ? 1 : 0;
  a.rearm_lastwg = s->rearm_lastwg ? 1 : 0;
  s->work_zero = false;
  if (s->fault_skip && a.work && (a.units == 0 || a.units == 6)) {
    const hipError_t e = hipMemsetD32Async(a.work, (int)s->fault_skip, 1, st);
    if (e != hipSuccess) return e;
    a.work_zero = 1;  // the launcher must not re-zero it
  }
  return gs::launch_force_sym(a, st);
}

bool fused_tail(const gs_stepper* s) {
  const bool size_ok = s->fuse_tail > 0 || (s->fuse_tail < 0 && s->sym_NC <= 128);
  return size_ok && s->cfg.nranks == 1 && !multi(s) && s->sym_band >= s->sym_NC;
}

int sym_force(gs_stepper* s, gs::SymArgs a, bool overlap_gather, bool exchange = false) {
  for (int b0 = 0; b0 < a.rows; b0 += s->sym_band) {
    a.band0 = b0;
    a.band_rows = s->sym_band < a.rows - b0 ? s->sym_band : a.rows - b0;
    a.units = 0;
    const bool one_band = a.band_rows == a.rows;
    const int ov = s->sym_overlap;
    if (overlap_gather && b0 == 0 && one_band && a.gate) {
      // 3: one launch with the local units first; remote units run in it once the gather is
      // published, or are deferred to a second launch queued behind the gather event.
      a.units = 6;
      GS_HIP(force_sym_launch(s, a, s->s_comp));
      GS_MARK(w0, w, s->s_comp);
      if (comp_wait(s, s->ev_gathered)) return -1;
      GS_MARK(w1, w, s->s_comp);
      a.units = 7;
      GS_HIP(force_sym_launch(s, a, s->s_comp));
      a.units = 0;
    } else if (overlap_gather && b0 == 0 && one_band && ov == 1) {
      gs::SymArgs d = a;
      d.units = 1;  // diagonal chunks beside the gather
      GS_HIP(force_sym_launch(s, d, s->s_comp));
      if (comp_wait(s, s->ev_gathered)) return -1;
      a.units = 2;
      GS_HIP(force_sym_launch(s, a, s->s_comp));
    } else if (overlap_gather && b0 == 0 && one_band && ov == 2) {
      // fork: s_rem starts after everything already on s_comp (X[cur] written) and the gather
      GS_HIP(hipEventRecord(s->ev_fork, s->s_comp));
      GS_HIP(hipStreamWaitEvent(s->s_rem, s->ev_fork, 0));
      GS_HIP(hipStreamWaitEvent(s->s_rem, s->ev_gathered, 0));
      gs::SymArgs r = a;
      r.units = 4;  // shell segments that read gathered rows
      GS_HIP(force_sym_launch(s, r, s->s_rem));
      GS_HIP(hipEventRecord(s->ev_remote, s->s_rem));
      a.units = 5;  // diagonal + rank-local shell units, beside the gather
      GS_HIP(force_sym_launch(s, a, s->s_comp));
      GS_HIP(hipStreamWaitEvent(s->s_comp, s->ev_remote, 0));  // join
    } else {
      if (overlap_gather && b0 == 0) {
        GS_MARK(w0, w, s->s_comp);
        if (comp_wait(s, s->ev_gathered)) return -1;
        GS_MARK(w1, w, s->s_comp);
      }
      GS_HIP(force_sym_launch(s, a, s->s_comp));
    }
    if (fused_tail(s)) continue;  // reductions + integrate in sym_tail_kernel (one band)
    const bool last = b0 + a.band_rows >= a.rows;
    // Without an exchange the row reduce (Pi, Pd -> Ti) and the block / node reduce (Pj) are
    // independent: fork_row (A/B knob) runs the row reduce on s_rem beside them (a fork /
    // join inside a captured step graph). In sequence is faster (see fork_row).
    const bool fork = !xcomm(s) && s->fork_row;
    if (fork) {
      GS_HIP(hipEventRecord(s->ev_fork, s->s_comp));
      GS_HIP(hipStreamWaitEvent(s->s_rem, s->ev_fork, 0));
      GS_HIP(gs::launch_sym_row_reduce(a, s->s_rem));
    }
    if (a.Bbuf) GS_HIP(gs::launch_sym_block_reduce(a, s->s_comp));  // the band's leaves
    if (last) GS_HIP(gs::launch_sym_node_reduce(a, s->s_comp));
    if (exchange && last && sym_exchange_rccl(s, false)) return -1;
    if (fork) {
      GS_HIP(hipEventRecord(s->ev_remote, s->s_rem));
      GS_HIP(hipStreamWaitEvent(s->s_comp, s->ev_remote, 0));
    } else {
      GS_HIP(gs::launch_sym_row_reduce(a, s->s_comp));
    }
    if (exchange && last) {
      GS_MARK(j0, j, s->s_comp);
      if (comp_wait(s, s->ev_sym)) return -1;
      GS_MARK(j1, j, s->s_comp);
    }
  }
  return 0;
}

int enqueue_sym(gs_stepper* s, int cur, bool need_gather, bool gathered_externally, int part,
                bool timed) {
  gs::SymArgs a = sym_args(s, cur);  // (emulation: the other ranks' nodes in Rbuf stay 0)
  // Gate the remote units on the gather in-kernel (GRAVSIM_SYM_OVERLAP=3): a collective of
  // this stepper (RCCL or modeled) and one band (the gated launch covers every unit).
  const bool gated = part == 3 && need_gather && !gathered_externally && xcomm(s) &&
                     s->sym_overlap == 3 && s->sym_band >= a.rows && s->sym_lf;
  if (gated) {
    a.gate = s->sym_ring ? s->ring_gate + 8 * cur : s->gate_buf + cur;
    a.gate_n = s->sym_ring ? 8 : 1;
  }
  if (part & 1) {
    if (need_gather) {
      if (gathered_externally) s->full[cur] = true;
      else if (gather(s, cur, gated)) return -1;
    }
    if (sym_force(s, a, need_gather, xcomm(s))) return -1;
    if (timed) GS_HIP(hipEventRecord(s->ev_local, s->s_comp));
  }
  if (part & 2) {
    if (fused_tail(s)) {
      GS_HIP(gs::launch_sym_tail(a, s->s_comp));
      s->work_zero = true;  // the tail re-armed the unit counter
    } else {
      GS_HIP(gs::launch_sym_finalize(a, s->s_comp));
    }
  }
  return 0;
}

// Clears the phase-event pointer on every exit path of an enqueue (an error return included),
// so gather() from download_state / accel_impl never records into a stale PhaseEv (pev may
// reallocate on the next phase_begin).
struct PhaseScope {
  gs_stepper* s;
  ~PhaseScope() { s->pe = nullptr; }
};

// Enqueue one step. `capturing` disables timing events.
template <typename T>
int enqueue_step(gs_stepper* s, bool capturing, bool gathered_externally) {
  Range range("gs.step");
  PhaseScope pscope{s};
  const int cur = (int)(s->k & 1);
  gs::KArgs<T> a = base_args<T>(s, cur);
  const int kernel = s->L.kernel, ipl = s->L.ipl;
  const bool fused = s->L.mode == GS_MODE_FUSED;
  const bool timed = s->timed && !capturing;
  s->pe = timed ? phase_begin(s) : nullptr;
  if (timed) GS_HIP(hipEventRecord(s->ev_t0, s->s_comp));
  if (s->pe) GS_HIP(hipEventRecord(s->pe->t0, s->s_comp));
  const bool need_gather = multi(s) && !s->full[cur];
  if (use_sym(s)) {
    if (enqueue_sym(s, cur, need_gather, gathered_externally, 3, timed)) return -1;
    if (timed) GS_HIP(hipEventRecord(s->ev_end, s->s_comp));
    if (s->pe) GS_HIP(hipEventRecord(s->pe->end, s->s_comp));
    s->pe = nullptr;
    s->full[cur ^ 1] = !multi(s);
    s->k += 1;
    return 0;
  }
  const bool ring = s->cfg.strategy == GS_STRATEGY_RING;
  if (need_gather && ring && !gathered_externally) {
    // Ring pass with RCCL (or timing emulation: no transfer, slices treated as present).
    GS_HIP(hipEventRecord(s->ev_fork, s->s_comp));
    GS_HIP(hipStreamWaitEvent(s->s_rem, s->ev_fork, 0));
    GS_HIP(hipStreamWaitEvent(s->s_rem2, s->ev_fork, 0));
    if (s->have_comm) {
      GS_HIP(hipStreamWaitEvent(s->s_comm, s->ev_fork, 0));
      GS_MARK(g0, g, s->s_comm);  // the ring's P-1 transfers are the step's gather span
    }
    if (ring_compute<T>(s, a, 0, nullptr)) return -1;
    for (int sub = 1; sub < s->cfg.nranks; ++sub) {
      hipEvent_t ready = nullptr;
      if (s->have_comm) {
        if (ring_xfer_rccl(s, cur, sub)) return -1;
        GS_HIP(hipEventRecord(s->ev_recv[sub], s->s_comm));
        ready = s->ev_recv[sub];
      }
      if (ring_compute<T>(s, a, sub, ready)) return -1;
    }
    if (s->have_comm) GS_MARK(g1, g, s->s_comm);
    if (ring_finish<T>(s, a)) return -1;
    if (timed) GS_HIP(hipEventRecord(s->ev_end, s->s_comp));
    if (s->pe) GS_HIP(hipEventRecord(s->pe->end, s->s_comp));
    s->pe = nullptr;
    s->full[cur] = true;
    s->full[cur ^ 1] = false;
    s->k += 1;
    return 0;
  }
  if (need_gather) {
    if (gathered_externally) s->full[cur] = true;
    else if (gather(s, cur)) return -1;
    // Rank-local chunks overlap the all-gather: they read only the own slice of X[cur].
    // The remote chunks run on a second compute stream gated only by the gather, so the two
    // launches share the GPU instead of serialising (the local launch alone holds only
    // n_local/(256*ipl) x own-chunk workgroups). The reduce/integrate waits for both.
    GS_HIP(hipEventRecord(s->ev_fork, s->s_comp));
    GS_HIP(hipStreamWaitEvent(s->s_rem, s->ev_fork, 0));
    gs::KArgs<T> loc = a;
    loc.c_begin = s->own_c0;
    loc.c_end = s->own_c1;
    GS_HIP(gs::launch_force_split<T>(loc, kernel, ipl,
                                     choose_groups(s, s->own_c1 - s->own_c0, false, true),
                                     s->s_comp));
    if (timed) GS_HIP(hipEventRecord(s->ev_local, s->s_comp));
    GS_HIP(hipStreamWaitEvent(s->s_rem, s->ev_gathered, 0));
    // One launch for every remote chunk: [0, n_chunks) minus the own range.
    gs::KArgs<T> r = a;
    r.skip_begin = s->own_c0;
    r.skip_end = s->own_c1;
    GS_HIP(gs::launch_force_split<T>(
        r, kernel, ipl, choose_groups(s, s->L.n_chunks - (s->own_c1 - s->own_c0), false, true),
        s->s_rem));
    GS_HIP(hipEventRecord(s->ev_remote, s->s_rem));
    GS_HIP(hipStreamWaitEvent(s->s_comp, s->ev_remote, 0));
    GS_HIP(gs::launch_reduce_integrate<T>(a, s->s_comp));
  } else {
    if (timed) GS_HIP(hipEventRecord(s->ev_local, s->s_comp));
    if (fused) {
      GS_HIP(gs::launch_force_fused<T>(a, kernel, ipl, s->s_comp));
    } else {
      GS_HIP(gs::launch_force_split<T>(a, kernel, ipl, choose_groups(s, s->L.n_chunks, false),
                                       s->s_comp));
      GS_HIP(gs::launch_reduce_integrate<T>(a, s->s_comp));
    }
  }
  if (timed) GS_HIP(hipEventRecord(s->ev_end, s->s_comp));
  if (s->pe) GS_HIP(hipEventRecord(s->pe->end, s->s_comp));
  s->pe = nullptr;
  s->full[cur ^ 1] = !multi(s);  // only the own slice of X[next] is fresh
  s->k += 1;
  return 0;
}

int enqueue_step_any(gs_stepper* s, bool capturing, bool gathered_externally = false) {
  return s->esz == 4 ? enqueue_step<float>(s, capturing, gathered_externally)
                     : enqueue_step<double>(s, capturing, gathered_externally);
}

int build_graph(gs_stepper* s) {
  // One ping-pong period (two steps) starting from an even step with a gathered buffer.
  const int64_t k0 = s->k;
  const bool f0 = s->full[0], f1 = s->full[1];
  hipGraph_t g = nullptr;
  // A replayed graph cannot rely on the counter state at capture time: its first sym force
  // launch always re-zeroes the unit counter (a later one may skip it after a fused tail
  // inside the graph; the flag left by the capture then matches every replay's end state).
  s->work_zero = false;
  GS_HIP(hipStreamBeginCapture(s->s_comp, hipStreamCaptureModeThreadLocal));
  int rc = enqueue_step_any(s, true);
  if (rc == 0) rc = enqueue_step_any(s, true);
  hipError_t e = hipStreamEndCapture(s->s_comp, &g);
  s->k = k0;
  s->full[0] = f0;
  s->full[1] = f1;
  if (rc) return rc;
  GS_HIP(e);
  GS_HIP(hipGraphInstantiate(&s->graph, g, nullptr, nullptr, 0));
  GS_HIP(hipGraphDestroy(g));
  return 0;
}

// Multi-rank steps whose cross-stream points all go through comp_record / comp_wait /
// comm_do: the sym schedule except overlap 2 (a second compute stream forked per step).
bool plan_ok(const gs_stepper* s) {
  return xcomm(s) && use_sym(s) && s->sym_overlap != 2 && s->cfg.use_graph == 1 && !s->timed;
}

// Record one ping-pong period (two steps, from an even step whose buffer needs its gather)
// as a plan: compute segments captured on s_comp, the collectives kept as eager host ops.
int build_plan(gs_stepper* s) {
  const int64_t k0 = s->k;
  const bool f0 = s->full[0], f1 = s->full[1];
  drop_graphs(s);
  s->work_zero = false;  // (as build_graph: a replay re-zeroes the dynamic unit counter)
  if (seg_open(s)) return -1;
  s->rec = true;
  int rc = enqueue_step_any(s, true);
  if (rc == 0) rc = enqueue_step_any(s, true);
  s->rec = false;
  const int cut = rc == 0 ? seg_cut(s) : 0;
  if (rc != 0) {  // abandon the open capture
    hipGraph_t g = nullptr;
    if (hipStreamEndCapture(s->s_comp, &g) == hipSuccess && g) (void)hipGraphDestroy(g);
  }
  s->k = k0;
  s->full[0] = f0;
  s->full[1] = f1;
  if (rc || cut) {
    drop_graphs(s);
    return -1;
  }
  return 0;
}

int run_plan(gs_stepper* s) {
  for (auto& op : s->plan) {
    switch (op.kind) {
      case gs_stepper::PlanOp::kGraph: GS_HIP(hipGraphLaunch(op.g, s->s_comp)); break;
      case gs_stepper::PlanOp::kRecord: GS_HIP(hipEventRecord(op.ev, s->s_comp)); break;
      case gs_stepper::PlanOp::kWait: GS_HIP(hipStreamWaitEvent(s->s_comp, op.ev, 0)); break;
      case gs_stepper::PlanOp::kHost:
        if (op.fn()) return -1;
        break;
    }
  }
  return 0;
}

template <typename T>
int upload_state(gs_stepper* s, const double* pos, const double* vel, const double* mass) {
  const int64_t n = s->L.n, np = s->L.n_pad, nl = s->L.n_local, b = s->L.local_begin;
  std::vector<T> X((size_t)np * 4, T(0));
  std::vector<T> V((size_t)nl * 4, T(0));
  for (int64_t i = 0; i < n; ++i) {
    X[4 * i] = (T)pos[3 * i];
    X[4 * i + 1] = (T)pos[3 * i + 1];
    X[4 * i + 2] = (T)pos[3 * i + 2];
    X[4 * i + 3] = (T)(s->cfg.G * mass[i]);
  }
  for (int64_t li = 0; li < nl; ++li) {
    const int64_t gi = b + li;
    if (gi >= n) break;
    V[4 * li] = (T)vel[3 * gi];
    V[4 * li + 1] = (T)vel[3 * gi + 1];
    V[4 * li + 2] = (T)vel[3 * gi + 2];
  }
  s->mass_host.assign(mass, mass + n);
  resolve_force_mode(s);
  GS_HIP(hipMemcpyAsync(s->X[0], X.data(), X.size() * sizeof(T), hipMemcpyHostToDevice,
                        s->s_comp));
  GS_HIP(hipMemcpyAsync(s->vel, V.data(), V.size() * sizeof(T), hipMemcpyHostToDevice,
                        s->s_comp));
  if (s->emulate)  // (see gs_stepper_init_ics)
    GS_HIP(hipMemcpyAsync(s->X[1], s->X[0], (size_t)np * 4 * sizeof(T), hipMemcpyDeviceToDevice,
                          s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  s->k = 0;
  s->full[0] = true;
  s->full[1] = false;
  return 0;
}

template <typename T>
int download_state(gs_stepper* s, double* pos, double* vel, double* mass) {
  const int cur = (int)(s->k & 1);
  if (pos && gather(s, cur)) return -1;
  if (pos && xcomm(s)) GS_HIP(hipStreamWaitEvent(s->s_comp, s->ev_gathered, 0));
  // A virtual-rank shard between steps holds only its own slice: return just those rows.
  const bool own_only = s->virt && !s->full[cur];
  GS_HIP(hipStreamSynchronize(s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comm));
  const int64_t n = s->L.n, nl = s->L.n_local, b = s->L.local_begin;
  if (pos) {
    std::vector<T> X((size_t)s->L.n_pad * 4);
    GS_HIP(hipMemcpy(X.data(), s->X[cur], X.size() * sizeof(T), hipMemcpyDeviceToHost));
    const int64_t i0 = own_only ? b : 0;
    const int64_t i1 = own_only ? (b + nl < n ? b + nl : n) : n;
    for (int64_t i = i0; i < i1; ++i)
      for (int d = 0; d < 3; ++d) pos[3 * i + d] = (double)X[4 * i + d];
  }
  if (vel) {
    std::vector<T> V((size_t)nl * 4);
    GS_HIP(hipMemcpy(V.data(), s->vel, V.size() * sizeof(T), hipMemcpyDeviceToHost));
    for (int64_t li = 0; li < nl && b + li < n; ++li)
      for (int d = 0; d < 3; ++d) vel[3 * (b + li) + d] = (double)V[4 * li + d];
  }
  if (mass)
    for (int64_t i = 0; i < n; ++i) mass[i] = s->mass_host[i];
  return 0;
}

template <typename T>
int accel_impl(gs_stepper* s, double* acc4, bool step_path) {
  // The one-sided split partials (n_chunks x n_local rows; 8.6 GB per rank at 16M / 8) are
  // allocated only when the query runs the split kernels, not for the sym step path.
  if (!(step_path && use_sym(s)) && ensure_partial(s)) return -1;
  const int cur = (int)(s->k & 1);
  if (s->virt && !s->full[cur]) {
    gs_set_error("accel: virtual-rank shard is not gathered (use the group API)");
    return -1;
  }
  if (gather(s, cur)) return -1;
  if (xcomm(s)) GS_HIP(hipStreamWaitEvent(s->s_comp, s->ev_gathered, 0));
  {
    if (step_path && use_sym(s)) {
      if (s->virt && s->cfg.nranks > 1) {
        gs_set_error("accel: the sym step path of a virtual-rank shard needs the group");
        return -1;
      }
      gs::SymArgs sa = sym_args(s, cur);
      sa.acc_out = s->acc;
      if (sym_force(s, sa, false)) return -1;
      if (xcomm(s) && sym_exchange_rccl(s)) return -1;
      if (fused_tail(s)) {
        GS_HIP(gs::launch_sym_tail(sa, s->s_comp));
        s->work_zero = true;
      } else {
        GS_HIP(gs::launch_sym_finalize(sa, s->s_comp));
      }
      GS_HIP(hipStreamSynchronize(s->s_comp));
      std::vector<T> A((size_t)s->L.n_local * 4);
      GS_HIP(hipMemcpy(A.data(), s->acc, A.size() * sizeof(T), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < A.size(); ++i) acc4[i] = (double)A[i];
      return 0;
    }
  }
  gs::KArgs<T> a = base_args<T>(s, cur);
  if (!step_path) {  // diagnostics: exact cutoff + potential
    a.phi = 1;
    a.exact = 1;
    a.eps2 = (T)(s->cfg.softening * s->cfg.softening);
  }
  a.acc_out = static_cast<T*>(s->acc);
  GS_HIP(gs::launch_force_split<T>(a, s->L.kernel, s->L.ipl,
                                   choose_groups(s, s->L.n_chunks, !step_path), s->s_comp));
  GS_HIP(gs::launch_reduce_integrate<T>(a, s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  std::vector<T> A((size_t)s->L.n_local * 4);
  GS_HIP(hipMemcpy(A.data(), s->acc, A.size() * sizeof(T), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < A.size(); ++i) acc4[i] = (double)A[i];
  return 0;
}

// Wait until progress event `target` - 1 has completed (target == prog_rec: every stream is
// idle). The deadline restarts whenever one more progress event completes.
int wait_until(gs_stepper* s, int64_t target, double timeout_s) {
  const int64_t R = (int64_t)s->prog.size();
  const bool all = target >= s->prog_rec;
  auto last = std::chrono::steady_clock::now();
  for (;;) {
    while (s->prog_done < s->prog_rec) {
      const hipError_t q = hipEventQuery(s->prog[s->prog_done % R]);
      if (q == hipErrorNotReady) break;
      if (q != hipSuccess) {
        char m[256];
        snprintf(m, sizeof(m), "stream error: %s", hipGetErrorString(q));
        gs_set_error(m);
        return -1;
      }
      ++s->prog_done;
      last = std::chrono::steady_clock::now();
    }
    bool done = s->prog_done >= target;
    if (all) {
      hipError_t a = hipStreamQuery(s->s_comp);
      if (a == hipSuccess) a = hipStreamQuery(s->s_rem);
      if (a == hipSuccess) a = hipStreamQuery(s->s_rem2);
      const hipError_t b = hipStreamQuery(s->s_comm);
      if ((a != hipSuccess && a != hipErrorNotReady) || (b != hipSuccess && b != hipErrorNotReady)) {
        char m[256];
        snprintf(m, sizeof(m), "stream error: %s / %s", hipGetErrorString(a), hipGetErrorString(b));
        gs_set_error(m);
        return -1;
      }
      done = a == hipSuccess && b == hipSuccess;
    }
    if (done) {
      if (all) s->prog_done = s->prog_rec;
      return 0;
    }
    if (s->have_comm && gs_stepper_comm_check(s)) return -1;
    const double el =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - last).count();
    if (timeout_s > 0 && el > timeout_s) {
      char m[256];
      snprintf(m, sizeof(m),
               "step timeout: no step completed for %.1f s (rank %d, step %lld of %lld "
               "enqueued); communicator aborted",
               el, s->cfg.rank, (long long)s->prog_done, (long long)s->prog_rec);
      if (s->have_comm) {
        (void)ncclCommAbort(s->comm);
        s->have_comm = false;
      }
      gs_set_error(m);
      return -1;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

// One progress event per enqueued step / graph period. At most prog.size() are outstanding:
// past that the host waits (bounded by step_timeout_s) for the oldest before enqueuing more.
int note_progress(gs_stepper* s) {
  const int64_t R = (int64_t)s->prog.size();
  if (R == 0) return 0;
  if (s->prog_rec - s->prog_done >= R && wait_until(s, s->prog_rec - R + 1, s->step_timeout_s))
    return -1;
  GS_HIP(hipEventRecord(s->prog[s->prog_rec % R], s->s_comp));
  ++s->prog_rec;
  return 0;
}

}  // namespace

extern "C" {

int gs_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* gs_hip_kernel_info(void) {
  return "gfx950 direct-sum: packed-fp32 SGPR j-stream (s_load_dwordx16) | LDS-DMA tiles "
         "(global_load_lds_dwordx4) | experimental MFMA r^2; fused KD epilogue; canonical "
         "chunk order; RCCL in-place all-gather or ring send/recv";
}

int gs_stepper_create(const gs_config* cfg, gs_stepper** out) {
  if (!cfg || !out) { gs_set_error("stepper_create: null argument"); return -1; }
  *out = nullptr;
  gs_stepper* s = new gs_stepper();
  s->cfg = *cfg;
  if (gs_layout_compute(cfg, &s->L)) { delete s; return -1; }
  s->esz = cfg->dtype == GS_FP64 ? 8 : 4;
  s->timed = getenv("GRAVSIM_PHASE_TIMING") != nullptr;
  s->emulate = getenv("GRAVSIM_EMULATE_RANK") != nullptr && cfg->nranks > 1;
  // Multi-rank sym steps default to the gated local-first launch (3): remote units start as
  // soon as the gather lands, nothing waits on it (see sym_force).
  s->sym_overlap = cfg->nranks > 1 ? 3 : 0;
  if (const char* ov = getenv("GRAVSIM_SYM_OVERLAP")) s->sym_overlap = atoi(ov);
  if (const char* v = getenv("GRAVSIM_EMU_COMM_GBPS")) s->emu_gbps = atof(v);
  if (const char* v = getenv("GRAVSIM_EMU_COMM_US")) s->emu_lat_us = atof(v);
  if (const char* v = getenv("GRAVSIM_EMU_COMM_WGS")) s->emu_wgs = atoi(v);
  if (const char* v = getenv("GRAVSIM_GATE_PROBE")) s->gate_probe = atoi(v);
  if (const char* v = getenv("GRAVSIM_SYM_DYN_CAP")) s->dyn_cap = atoi(v);
  if (const char* v = getenv("GRAVSIM_SYM_DIAG_LAST")) s->diag_last = atoi(v);
  if (const char* v = getenv("GRAVSIM_SYM_FUSED_TAIL")) s->fuse_tail = atoi(v) != 0 ? 1 : 0;
  if (const char* v = getenv("GRAVSIM_SYM_PARITY")) s->parity = atoi(v) != 0 ? 1 : 0;
  if (const char* v = getenv("GRAVSIM_FAULT_SKIP_UNITS")) s->fault_skip = (unsigned)atoi(v);
  if (const char* v = getenv("GRAVSIM_SYM_REARM")) s->rearm_lastwg = strcmp(v, "lastwg") == 0;
  if (const char* v = getenv("GRAVSIM_SYM_FORK_ROW")) s->fork_row = atoi(v) != 0;  // (A/B)
  const int64_t own_first = s->L.local_begin / s->L.chunk;
  const int64_t own_last = (s->L.local_begin + s->L.n_local) / s->L.chunk;
  s->own_c0 = (int)(own_first < s->L.n_chunks ? own_first : s->L.n_chunks);
  s->own_c1 = (int)(own_last < s->L.n_chunks ? own_last : s->L.n_chunks);
#define FAIL_CLEAN(call)          \
  do {                            \
    if ((call) != hipSuccess) {   \
      char b_[256];               \
      snprintf(b_, sizeof(b_), "stepper_create: %s failed: %s", #call, hipGetErrorString(hipGetLastError())); \
      gs_set_error(b_);           \
      gs_stepper_destroy(s);      \
      return -1;                  \
    }                             \
  } while (0)
#define ALLOC_CLEAN(ptr, bytes, tag)     \
  do {                                   \
    if (dev_alloc(s, ptr, bytes, tag)) { \
      gs_stepper_destroy(s);             \
      return -1;                         \
    }                                    \
  } while (0)
  FAIL_CLEAN(hipSetDevice(cfg->device));
  FAIL_CLEAN(hipDeviceGetAttribute(&s->cus, hipDeviceAttributeMultiprocessorCount, cfg->device));
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg->device) == hipSuccess &&
        khz > 0)
      s->clk_khz = khz;
  }
  {
    const int occ = gs::sym_occupancy(s->esz == 8);
    s->sym_first_wave = (occ > 0 ? occ : 2) * s->cus;
    // (tests shrink it so that small runs take the dynamic path too)
    if (const char* v = getenv("GRAVSIM_SYM_FIRST_WAVE")) s->sym_first_wave = atoi(v);
  }
  for (int fm = 0; fm < 3; ++fm)
    s->occ[fm] = s->esz == 4 ? gs::split_occupancy<float>(s->L.kernel, s->L.ipl, fm)
                             : gs::split_occupancy<double>(s->L.kernel, s->L.ipl, fm);
  resolve_force_mode(s);
  int lo = 0, hi = 0;
  FAIL_CLEAN(hipDeviceGetStreamPriorityRange(&lo, &hi));
  FAIL_CLEAN(hipStreamCreateWithFlags(&s->s_comp, hipStreamNonBlocking));
  FAIL_CLEAN(hipStreamCreateWithPriority(&s->s_comm, hipStreamNonBlocking, hi));
  FAIL_CLEAN(hipStreamCreateWithFlags(&s->s_rem, hipStreamNonBlocking));
  FAIL_CLEAN(hipStreamCreateWithFlags(&s->s_rem2, hipStreamNonBlocking));
  FAIL_CLEAN(hipEventCreateWithFlags(&s->ev_rem2, hipEventDisableTiming));
  s->ev_recv.assign((size_t)cfg->nranks, nullptr);
  for (auto& e : s->ev_recv) FAIL_CLEAN(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  FAIL_CLEAN(hipEventCreateWithFlags(&s->ev_remote, hipEventDisableTiming));
  FAIL_CLEAN(hipEventCreateWithFlags(&s->ev_sym, hipEventDisableTiming));
  FAIL_CLEAN(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
  FAIL_CLEAN(hipEventCreateWithFlags(&s->ev_ready, hipEventDisableTiming));
  FAIL_CLEAN(hipEventCreateWithFlags(&s->ev_gathered, hipEventDisableTiming));
  FAIL_CLEAN(hipEventCreate(&s->ev_t0));
  FAIL_CLEAN(hipEventCreate(&s->ev_local));
  FAIL_CLEAN(hipEventCreate(&s->ev_end));
  s->prog.assign(64, nullptr);
  for (auto& e : s->prog) FAIL_CLEAN(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const size_t rb = row_bytes(s);
  ALLOC_CLEAN(&s->X[0], (size_t)s->L.n_pad * rb, "X0");
  ALLOC_CLEAN(&s->X[1], (size_t)s->L.n_pad * rb, "X1");
  ALLOC_CLEAN(&s->vel, (size_t)s->L.n_local * rb, "vel");
  ALLOC_CLEAN(&s->acc, (size_t)s->L.n_local * rb, "acc");
  // Per-chunk partials (n_chunks x n_local rows) only for the split schedule; a single-rank
  // fused run never touches them (16M bodies: 64 GB saved), and allocates on demand.
  if ((s->L.mode == GS_MODE_SPLIT || (cfg->nranks > 1 && s->L.mode != GS_MODE_SYM)) &&
      ensure_partial(s)) {
    gs_stepper_destroy(s);
    return -1;
  }
  if (ensure_sym(s)) {
    gs_stepper_destroy(s);
    return -1;
  }
  ALLOC_CLEAN(&s->mass_dev, (size_t)s->L.n_pad * sizeof(double), "mass");
  ALLOC_CLEAN(&s->nonfinite, sizeof(unsigned long long), "nonfinite");
  ALLOC_CLEAN(&s->ring_gate, 16 * sizeof(unsigned), "ring_gate");
  FAIL_CLEAN(hipMemsetAsync(s->ring_gate, 0, 16 * sizeof(unsigned), s->s_comp));
  // [0..1] gather gates, [2..3] deferral stats, [4] dynamic unit-fetch counter
  ALLOC_CLEAN(&s->gate_buf, 8 * sizeof(unsigned), "gate");
  FAIL_CLEAN(hipMemsetAsync(s->gate_buf, 0, 8 * sizeof(unsigned), s->s_comp));
  if (s->L.mode == GS_MODE_SYM && !(getenv("GRAVSIM_AUDIT") && atoi(getenv("GRAVSIM_AUDIT")) == 0)) {
    // (GRAVSIM_AUDIT=0: no unit counter, for A/B timing of its cost only)
    ALLOC_CLEAN(&s->audit, sizeof(unsigned long long), "audit");
    FAIL_CLEAN(hipMemsetAsync(s->audit, 0, sizeof(unsigned long long), s->s_comp));
  }
  if (s->L.mode == GS_MODE_SYM) {
    // Deferred-unit list of the gated launch (one band's units) and the local-first order.
    const int rows = (int)(s->L.n_local / gs::kSymC);
    const size_t units = (size_t)rows * (s->sym_S_n + s->sym_D) + 1;
    ALLOC_CLEAN(&s->defer, units * sizeof(unsigned), "defer");
    FAIL_CLEAN(hipMemsetAsync(s->defer, 0, units * sizeof(unsigned), s->s_comp));
    // unit -> row << 16 | segment (bit 31: remote), local units first (layout.cpp).
    long fill = 4L * s->cus;  // two dispatch waves of 2 workgroups per CU
    if (const char* v = getenv("GRAVSIM_SYM_LF_FILL")) fill = atol(v);
    std::vector<int32_t> lf(units - 1);
    s->sym_ring = cfg->strategy == GS_STRATEGY_RING && cfg->nranks > 1;
    const int64_t got =
        s->sym_ring ? gs_sym_unit_map_ring(s->L.n_pad, cfg->rank, cfg->nranks, s->parity, fill,
                                           lf.data(), (int64_t)lf.size())
                    : gs_sym_unit_map(s->L.n_pad, cfg->rank, cfg->nranks, s->parity, fill,
                                      lf.data(), (int64_t)lf.size());
    lf.resize(got > 0 ? (size_t)got : 0);  // 0: geometry too large for the 16-bit fields
    if (!lf.empty()) {
      ALLOC_CLEAN(&s->sym_lf, lf.size() * sizeof(int32_t), "unit_map");
      FAIL_CLEAN(hipMemcpy(s->sym_lf, lf.data(), lf.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice));
    }
  }
  if (s->L.mode == GS_MODE_SYM && getenv("GRAVSIM_UNIT_TRACE")) {
    // One entry per unit of a band-wide launch plus as many deferred ones (units 7).
    s->utrace_main = (int64_t)s->sym_band * (s->sym_S_n + s->sym_D);
    ALLOC_CLEAN(&s->utrace, (size_t)(2 * s->utrace_main) * 4 * sizeof(unsigned long long), "unit_trace");
    FAIL_CLEAN(hipMemsetAsync(s->utrace, 0, (size_t)(2 * s->utrace_main) * 4 * 8, s->s_comp));
  }
  if (s->emulate && s->emu_gbps > 0.0) {
    // Scratch destination of the modeled collectives (the larger of the two per step).
    s->emu_cap = gather_bytes(s);
    if (s->L.mode == GS_MODE_SYM && exchange_bytes(s) > s->emu_cap) s->emu_cap = exchange_bytes(s);
    s->emu_cap &= ~(size_t)15;
    ALLOC_CLEAN(&s->emu_buf, s->emu_cap, "emu_comm");
  }
  // Zero on the compute stream itself: it is non-blocking, so a legacy-stream hipMemset
  // would NOT be ordered before later work on it (it could land after the IC kernel).
  FAIL_CLEAN(hipMemsetAsync(s->X[0], 0, (size_t)s->L.n_pad * rb, s->s_comp));
  FAIL_CLEAN(hipMemsetAsync(s->X[1], 0, (size_t)s->L.n_pad * rb, s->s_comp));
  FAIL_CLEAN(hipMemsetAsync(s->vel, 0, (size_t)s->L.n_local * rb, s->s_comp));
  FAIL_CLEAN(hipStreamSynchronize(s->s_comp));
#undef FAIL_CLEAN
#undef ALLOC_CLEAN
  *out = s;
  return 0;
}

int gs_stepper_destroy(gs_stepper* s) {
  if (!s) return 0;
  if (s->s_comp) (void)hipStreamSynchronize(s->s_comp);
  if (s->s_comm) (void)hipStreamSynchronize(s->s_comm);
  if (s->s_rem) (void)hipStreamSynchronize(s->s_rem);
  if (s->s_rem2) (void)hipStreamSynchronize(s->s_rem2);
  drop_graphs(s);
  if (s->have_comm) (void)ncclCommDestroy(s->comm);
  for (const auto& m : s->mem) (void)hipFree(m.p);
  s->mem.clear();
  for (hipEvent_t e : {s->ev_ready, s->ev_gathered, s->ev_t0, s->ev_local, s->ev_end,
                       s->ev_remote, s->ev_fork, s->ev_rem2, s->ev_sym})
    if (e) (void)hipEventDestroy(e);
  if (s->s_comp) (void)hipStreamDestroy(s->s_comp);
  if (s->s_comm) (void)hipStreamDestroy(s->s_comm);
  if (s->s_rem) (void)hipStreamDestroy(s->s_rem);
  if (s->s_rem2) (void)hipStreamDestroy(s->s_rem2);
  for (hipEvent_t e : s->ev_recv)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : s->prog)
    if (e) (void)hipEventDestroy(e);
  for (auto& p : s->pev)
    for (hipEvent_t e : {p.t0, p.end, p.g0, p.g1, p.w0, p.w1, p.x0, p.x1, p.j0, p.j1})
      if (e) (void)hipEventDestroy(e);
  delete s;
  return 0;
}

int gs_stepper_layout(gs_stepper* s, gs_layout* out) {
  if (!s || !out) return -1;
  *out = s->L;
  return 0;
}

int gs_stepper_init_ics(gs_stepper* s, int32_t ic, uint64_t seed) {
  GS_HIP(hipSetDevice(s->cfg.device));
  hipError_t e;
  if (s->esz == 4)
    e = gs::launch_init_ics<float>(ic, seed, s->L.n, s->L.n_pad, s->L.local_begin, s->L.n_local,
                                   s->cfg.G, static_cast<float*>(s->X[0]),
                                   static_cast<float*>(s->vel), s->mass_dev, s->s_comp);
  else
    e = gs::launch_init_ics<double>(ic, seed, s->L.n, s->L.n_pad, s->L.local_begin,
                                    s->L.n_local, s->cfg.G, static_cast<double*>(s->X[0]),
                                    static_cast<double*>(s->vel), s->mass_dev, s->s_comp);
  GS_HIP(e);
  s->mass_host.resize((size_t)s->L.n);
  GS_HIP(hipMemcpyAsync(s->mass_host.data(), s->mass_dev, (size_t)s->L.n * sizeof(double),
                        hipMemcpyDeviceToHost, s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  resolve_force_mode(s);
  s->k = 0;
  s->full[0] = true;
  s->full[1] = false;
  if (s->emulate) {
    // The emulated rank never receives remote rows: give X[1] the same realistic positions as
    // X[0] so odd steps do not run on all-zero remote rows (lower power, higher clocks: the
    // force kernel measured 5 % faster on them, profiles/r2_trace_steps_parity.txt).
    GS_HIP(hipMemcpyAsync(s->X[1], s->X[0], (size_t)s->L.n_pad * row_bytes(s),
                          hipMemcpyDeviceToDevice, s->s_comp));
    GS_HIP(hipStreamSynchronize(s->s_comp));
  }
  drop_graphs(s);
  return 0;
}

int gs_stepper_set_state(gs_stepper* s, const double* pos, const double* vel, const double* mass) {
  GS_HIP(hipSetDevice(s->cfg.device));
  drop_graphs(s);
  return s->esz == 4 ? upload_state<float>(s, pos, vel, mass)
                     : upload_state<double>(s, pos, vel, mass);
}

int gs_stepper_get_state(gs_stepper* s, double* pos, double* vel, double* mass) {
  GS_HIP(hipSetDevice(s->cfg.device));
  return s->esz == 4 ? download_state<float>(s, pos, vel, mass)
                     : download_state<double>(s, pos, vel, mass);
}

int gs_stepper_step(gs_stepper* s, int32_t nsteps) {
  GS_HIP(hipSetDevice(s->cfg.device));
  if (s->cfg.nranks > 1 && !s->have_comm && !s->emulate) {
    gs_set_error("step: nranks > 1 but no RCCL communicator (call gs_stepper_comm_init)");
    return -1;
  }
  // GRAVSIM_EMULATE_RANK runs one rank's launch shapes of a P-rank run on one GPU with the
  // collectives modeled (GRAVSIM_EMU_COMM_GBPS > 0) or free; remote slices hold stale data,
  // so the numbers are timings, not physics.
  // hipGraph replay of a two-step ping-pong period. Multi-rank (RCCL or emulated) steps are
  // captured collectives included only when use_graph >= 2 (opt-in: --graph-comm). Over
  // RCCL's socket transport that capture crashes inside hipStreamEndCapture
  // (profiles/r2_graph_comm_root_cause.txt), which no fallback here can catch; a capture
  // the runtime refuses with an error code falls back to eager steps.
  // Multi-rank runs with use_graph 1 (the default) replay a segmented plan instead: compute
  // segments as graphs, collectives eager between them (plan_ok, build_plan).
  const bool seg = plan_ok(s);
  const bool graph_ok = seg || (s->cfg.use_graph >= (xcomm(s) ? 2 : 1) && !s->timed &&
                                !(xcomm(s) && s->graph_failed));
  int32_t left = nsteps;
  while (left > 0) {
    const bool period_start = (s->k & 1) == 0 && (xcomm(s) ? !s->full[0] : true);
    if (graph_ok && left >= 2 && period_start && !s->graph_failed) {
      if (seg) {
        if (s->plan.empty() && build_plan(s)) {
          s->graph_failed = true;  // eager from here on (the error text is kept)
          continue;
        }
        if (run_plan(s)) return -1;
      } else {
        if (!s->graph && build_graph(s)) {
          if (!xcomm(s)) return -1;
          s->graph_failed = true;  // eager from here on (the error text is kept for inspection)
          continue;
        }
        GS_HIP(hipGraphLaunch(s->graph, s->s_comp));
      }
      s->k += 2;
      // After one period: X[1] was gathered in the second step, X[0] holds only the own slice.
      s->full[0] = !xcomm(s);
      s->full[1] = true;
      left -= 2;
      if (note_progress(s)) return -1;
      continue;
    }
    if (enqueue_step_any(s, false)) return -1;
    left -= 1;
    if (note_progress(s)) return -1;
  }
  return 0;
}

int gs_stepper_set_timing(gs_stepper* s, int32_t on) {
  s->timed = on != 0;
  s->pev_used = 0;
  return 0;
}

int gs_stepper_set_overlap(gs_stepper* s, int32_t mode) {
  if (mode < 0 || mode > 3) { gs_set_error("set_overlap: mode must be 0..3"); return -1; }
  s->sym_overlap = mode;
  drop_graphs(s);
  return 0;
}

int gs_stepper_set_schedule(gs_stepper* s, int32_t use_graph, int32_t dyn_cap) {
  if (use_graph < 0 || use_graph > 2) { gs_set_error("set_schedule: use_graph must be 0..2"); return -1; }
  s->cfg.use_graph = use_graph;
  if (dyn_cap >= 0) s->dyn_cap = dyn_cap;
  s->graph_failed = false;
  s->work_zero = false;  // (a dynamic launch after a static one re-zeroes its counter)
  drop_graphs(s);
  return 0;
}

int gs_stepper_set_cutoff_mode(gs_stepper* s, int32_t mode) {
  if (mode < 0 || mode > 2) { gs_set_error("set_cutoff_mode: mode must be 0..2"); return -1; }
  s->cfg.cutoff_mode = mode;
  resolve_force_mode(s);
  drop_graphs(s);
  return 0;
}

int32_t gs_stepper_get_overlap(gs_stepper* s) { return s->sym_overlap; }

int32_t gs_stepper_mem_entry(gs_stepper* s, int32_t i, const char** tag, uint64_t* bytes) {
  if (!s) return -1;
  if (i >= 0 && i < (int32_t)s->mem.size()) {
    if (tag) *tag = s->mem[i].tag;
    if (bytes) *bytes = s->mem[i].bytes;
  }
  return (int32_t)s->mem.size();
}

int gs_stepper_graph_info(gs_stepper* s, int32_t* mode, int32_t* segments) {
  if (mode) *mode = !s->plan.empty() ? 2 : (s->graph ? 1 : 0);
  if (segments) *segments = s->plan_graphs;
  return 0;
}

int gs_stepper_audit(gs_stepper* s, uint64_t* units_done, uint64_t* units_per_step) {
  if (units_done) *units_done = 0;
  if (units_per_step) *units_per_step = 0;
  if (!s->audit) return 0;  // one-sided schedules: no unit audit
  GS_HIP(hipSetDevice(s->cfg.device));
  const uint64_t rows = (uint64_t)(s->L.n_local / gs::kSymC);
  if (units_per_step) *units_per_step = rows * (uint64_t)(s->sym_S_n + s->sym_D);
  if (units_done) {
    GS_HIP(hipStreamSynchronize(s->s_comp));
    unsigned long long h = 0;
    GS_HIP(hipMemcpy(&h, s->audit, sizeof(h), hipMemcpyDeviceToHost));
    *units_done = h;
  }
  return 0;
}

int gs_stepper_audit_reset(gs_stepper* s) {
  if (!s->audit) return 0;
  GS_HIP(hipSetDevice(s->cfg.device));
  GS_HIP(hipMemsetAsync(s->audit, 0, sizeof(unsigned long long), s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  return 0;
}

int64_t gs_stepper_unit_trace(gs_stepper* s, uint64_t* out, int64_t cap) {
  if (!s->utrace) return 0;
  const int64_t n = 2 * s->utrace_main;
  if (!out) return n;
  GS_HIP(hipSetDevice(s->cfg.device));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  const int64_t m = cap < n ? cap : n;
  GS_HIP(hipMemcpy(out, s->utrace, (size_t)m * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  GS_HIP(hipMemsetAsync(s->utrace, 0, (size_t)n * 4 * sizeof(uint64_t), s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  return m;
}

int gs_stepper_set_timeout(gs_stepper* s, double step_timeout_s) {
  s->step_timeout_s = step_timeout_s > 0 ? step_timeout_s : 0.0;
  return 0;
}

int gs_stepper_sync(gs_stepper* s) {
  GS_HIP(hipStreamSynchronize(s->s_comm));
  GS_HIP(hipStreamSynchronize(s->s_rem));
  GS_HIP(hipStreamSynchronize(s->s_rem2));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  s->prog_done = s->prog_rec;
  return 0;
}

// Bounded wait for every stream, polling RCCL async errors. The deadline bounds PROGRESS: it
// restarts whenever one more enqueued step (or graph period) completes, so a long healthy
// run never trips it while a hang (a dead peer, a stuck collective) or an RCCL error aborts
// the communicator and returns -1 instead of blocking forever (the reference's
// MPI_ERRORS_ARE_FATAL / silent CUDA errors: SURVEY.md §5).
int gs_stepper_wait(gs_stepper* s, double timeout_s) {
  return wait_until(s, s->prog_rec, timeout_s);
}

// Phase timing of the eager steps enqueued since gs_stepper_set_timing(s, 1) / the previous
// call (at most 256), averaged per step. out[0] steps, [1] total ms, [2] all-gather ms and
// [3] node-sum exchange ms (spans on the comm stream), [4] exposed gather ms and [5]
// exposed exchange ms (compute-stream stalls on them: exposed comm = [4] + [5]), [6] the
// most force units one step deferred past the gather (overlap 3), [7] reserved (0).
int gs_stepper_phase_stats(gs_stepper* s, double* out8) {
  for (int i = 0; i < 8; ++i) out8[i] = 0.0;
  for (hipStream_t st : {s->s_comm, s->s_rem, s->s_rem2, s->s_comp})
    GS_HIP(hipStreamSynchronize(st));
  s->prog_done = s->prog_rec;
  const int n = s->pev_used;
  for (int i = 0; i < n; ++i) {
    const gs_stepper::PhaseEv& p = s->pev[i];
    float v = 0.f;
    GS_HIP(hipEventElapsedTime(&v, p.t0, p.end));
    out8[1] += v;
    if (p.g) { GS_HIP(hipEventElapsedTime(&v, p.g0, p.g1)); out8[2] += v; }
    if (p.x) { GS_HIP(hipEventElapsedTime(&v, p.x0, p.x1)); out8[3] += v; }
    if (p.w) { GS_HIP(hipEventElapsedTime(&v, p.w0, p.w1)); out8[4] += v; }
    if (p.j) { GS_HIP(hipEventElapsedTime(&v, p.j0, p.j1)); out8[5] += v; }
  }
  if (n > 0)
    for (int i = 1; i < 6; ++i) out8[i] /= n;
  out8[0] = n;
  unsigned d[2] = {0, 0};
  GS_HIP(hipMemcpy(d, s->gate_buf + 2, sizeof(d), hipMemcpyDeviceToHost));
  out8[6] = d[1];
  out8[7] = 0.0;
  // (on s_comp: a legacy-stream memset is not ordered against the non-blocking compute
  // stream, so the next gated launch could race it)
  GS_HIP(hipMemsetAsync(s->gate_buf + 2, 0, sizeof(d), s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  s->pev_used = 0;
  return 0;
}

int gs_stepper_accel(gs_stepper* s, double* acc4) {
  GS_HIP(hipSetDevice(s->cfg.device));
  return s->esz == 4 ? accel_impl<float>(s, acc4, false) : accel_impl<double>(s, acc4, false);
}

int gs_stepper_accel_step_path(gs_stepper* s, double* acc4) {
  GS_HIP(hipSetDevice(s->cfg.device));
  return s->esz == 4 ? accel_impl<float>(s, acc4, true) : accel_impl<double>(s, acc4, true);
}

int64_t gs_stepper_count_nonfinite(gs_stepper* s) {
  if (hipSetDevice(s->cfg.device) != hipSuccess) return -1;
  const int cur = (int)(s->k & 1);
  if (hipMemsetAsync(s->nonfinite, 0, sizeof(unsigned long long), s->s_comp) != hipSuccess)
    return -1;
  hipError_t e;
  if (s->esz == 4)
    e = gs::launch_count_nonfinite<float>(static_cast<const float*>(s->X[cur]),
                                          s->L.local_begin, s->L.n_local,
                                          static_cast<const float*>(s->vel), s->nonfinite,
                                          s->s_comp);
  else
    e = gs::launch_count_nonfinite<double>(static_cast<const double*>(s->X[cur]),
                                           s->L.local_begin, s->L.n_local,
                                           static_cast<const double*>(s->vel), s->nonfinite,
                                           s->s_comp);
  if (e != hipSuccess) return -1;
  unsigned long long h = 0;
  if (hipMemcpyAsync(&h, s->nonfinite, sizeof(h), hipMemcpyDeviceToHost, s->s_comp) !=
          hipSuccess ||
      hipStreamSynchronize(s->s_comp) != hipSuccess)
    return -1;
  return (int64_t)h;
}

int64_t gs_stepper_steps_done(gs_stepper* s) { return s->k; }

int gs_stepper_phase_ms(gs_stepper* s, float* local_ms, float* comm_ms, float* total_ms) {
  if (!s->timed) { gs_set_error("phase timing disabled (set GRAVSIM_PHASE_TIMING=1)"); return -1; }
  GS_HIP(hipEventSynchronize(s->ev_end));
  float a = 0, b = 0, c = 0;
  GS_HIP(hipEventElapsedTime(&a, s->ev_t0, s->ev_local));
  GS_HIP(hipEventElapsedTime(&b, s->ev_t0, s->ev_end));
  if (s->pev_used > 0) {  // the last step's collectives (all-gather + exchange spans)
    const gs_stepper::PhaseEv& p = s->pev[s->pev_used - 1];
    float v = 0.f;
    if (p.g && hipEventElapsedTime(&v, p.g0, p.g1) == hipSuccess) c += v;
    if (p.x && hipEventElapsedTime(&v, p.x0, p.x1) == hipSuccess) c += v;
  }
  if (local_ms) *local_ms = a;
  if (comm_ms) *comm_ms = c;
  if (total_ms) *total_ms = b;
  return 0;
}

void* gs_stepper_compute_stream(gs_stepper* s) { return (void*)s->s_comp; }

int gs_stepper_force_mode(gs_stepper* s, int32_t* exact, double* eps2) {
  if (exact) *exact = s->exact ? 1 : 0;
  if (eps2) *eps2 = s->eps2;
  return 0;
}

// Virtual ranks: P shards (rank r of P) in one process on one device. The all-gather is
// P*(P-1) device-to-device copies on shard 0's comm stream, fenced against every shard's
// compute stream by events: the same kernels, arguments and chunk order as the RCCL path, so
// a P-shard run must match the 1-rank run bit for bit (SURVEY.md §4.2 "virtual-rank mode").
int gs_group_step(gs_stepper** sh, int32_t P, int32_t nsteps) {
  if (!sh || P < 1) { gs_set_error("group_step: bad arguments"); return -1; }
  for (int r = 0; r < P; ++r) {
    if (sh[r]->cfg.nranks != P || sh[r]->cfg.rank != r || sh[r]->have_comm ||
        sh[r]->cfg.device != sh[0]->cfg.device || sh[r]->esz != sh[0]->esz ||
        sh[r]->L.n_pad != sh[0]->L.n_pad || sh[r]->k != sh[0]->k) {
      gs_set_error("group_step: shards must be ranks 0..P-1 of one layout, in step");
      return -1;
    }
  }
  GS_HIP(hipSetDevice(sh[0]->cfg.device));
  for (int r = 0; r < P; ++r) sh[r]->virt = P > 1;
  hipStream_t gsm = sh[0]->s_comm;
  const int64_t rbytes = (int64_t)row_bytes(sh[0]);
  for (int32_t it = 0; it < nsteps; ++it) {
    const int cur = (int)(sh[0]->k & 1);
    const bool need = P > 1 && !sh[0]->full[cur];
    if (need && sh[0]->cfg.strategy == GS_STRATEGY_RING) {
      // Ring pass with device copies: at sub-step s shard r receives slice (r - s) mod P
      // from shard r-1 (which holds it since sub-step s-1), on shard 0's comm stream.
      for (int r = 0; r < P; ++r) GS_HIP(hipEventRecord(sh[r]->ev_ready, sh[r]->s_comp));
      for (int r = 0; r < P; ++r) GS_HIP(hipStreamWaitEvent(gsm, sh[r]->ev_ready, 0));
      for (int r = 0; r < P; ++r) {
        GS_HIP(hipStreamWaitEvent(sh[r]->s_rem, sh[r]->ev_ready, 0));
        GS_HIP(hipStreamWaitEvent(sh[r]->s_rem2, sh[r]->ev_ready, 0));
      }
      for (int r = 0; r < P; ++r) {
        int rc = sh[r]->esz == 4
                     ? ring_compute<float>(sh[r], base_args<float>(sh[r], cur), 0, nullptr)
                     : ring_compute<double>(sh[r], base_args<double>(sh[r], cur), 0, nullptr);
        if (rc) return -1;
      }
      for (int sub = 1; sub < P; ++sub) {
        for (int r = 0; r < P; ++r) {
          const int left = (r - 1 + P) % P, src = ring_src(sh[r], sub);
          int64_t b0, cnt;
          rank_slice(sh[0], src, &b0, &cnt);
          GS_HIP(hipMemcpyAsync(static_cast<char*>(sh[r]->X[cur]) + b0 * rbytes,
                                static_cast<char*>(sh[left]->X[cur]) + b0 * rbytes, cnt * rbytes,
                                hipMemcpyDeviceToDevice, gsm));
        }
        for (int r = 0; r < P; ++r) GS_HIP(hipEventRecord(sh[r]->ev_recv[sub], gsm));
        for (int r = 0; r < P; ++r) {
          int rc = sh[r]->esz == 4
                       ? ring_compute<float>(sh[r], base_args<float>(sh[r], cur), sub,
                                             sh[r]->ev_recv[sub])
                       : ring_compute<double>(sh[r], base_args<double>(sh[r], cur), sub,
                                              sh[r]->ev_recv[sub]);
          if (rc) return -1;
        }
      }
      for (int r = 0; r < P; ++r) {
        int rc = sh[r]->esz == 4 ? ring_finish<float>(sh[r], base_args<float>(sh[r], cur))
                                 : ring_finish<double>(sh[r], base_args<double>(sh[r], cur));
        if (rc) return -1;
        sh[r]->full[cur] = true;
        sh[r]->full[cur ^ 1] = false;
        sh[r]->k += 1;
      }
      continue;
    }
    if (need) {
      for (int r = 0; r < P; ++r) GS_HIP(hipEventRecord(sh[r]->ev_ready, sh[r]->s_comp));
      for (int r = 0; r < P; ++r) GS_HIP(hipStreamWaitEvent(gsm, sh[r]->ev_ready, 0));
      for (int dst = 0; dst < P; ++dst)
        for (int src = 0; src < P; ++src) {
          if (src == dst) continue;
          int64_t b0, cnt;
          rank_slice(sh[0], src, &b0, &cnt);
          GS_HIP(hipMemcpyAsync(static_cast<char*>(sh[dst]->X[cur]) + b0 * rbytes,
                                static_cast<char*>(sh[src]->X[cur]) + b0 * rbytes, cnt * rbytes,
                                hipMemcpyDeviceToDevice, gsm));
        }
      for (int r = 0; r < P; ++r) GS_HIP(hipEventRecord(sh[r]->ev_gathered, gsm));
    }
    if (use_sym(sh[0]) && P > 1) {
      // Symmetric schedule: force + node reduce on every shard, then the node-sum exchange
      // as device copies (shard r's block for q -> shard q's slots of r's nodes), then
      // finalize.
      const size_t e = sh[0]->esz;
      for (int r = 0; r < P; ++r)
        if (enqueue_sym(sh[r], cur, need, true, 1, false)) return -1;
      for (int r = 0; r < P; ++r) GS_HIP(hipEventRecord(sh[r]->ev_ready, sh[r]->s_comp));
      for (int r = 0; r < P; ++r) GS_HIP(hipStreamWaitEvent(gsm, sh[r]->ev_ready, 0));
      for (int q = 0; q < P; ++q)
        for (int r = 0; r < P; ++r) {
          const size_t nr = (size_t)sh[0]->nn[r], nlq = (size_t)sh[0]->rcnt[q];
          GS_HIP(hipMemcpyAsync(sh[q]->sym_R + (size_t)sh[0]->nbase[r] * 3 * nlq * e,
                                sh[r]->sym_S + nr * 3 * (size_t)sh[0]->rbeg[q] * e,
                                nr * 3 * nlq * e, hipMemcpyDeviceToDevice, gsm));
        }
      GS_HIP(hipEventRecord(sh[0]->ev_sym, gsm));
      for (int r = 0; r < P; ++r) {
        GS_HIP(hipStreamWaitEvent(sh[r]->s_comp, sh[0]->ev_sym, 0));
        if (enqueue_sym(sh[r], cur, false, true, 2, false)) return -1;
        sh[r]->full[cur ^ 1] = false;
        sh[r]->k += 1;
      }
      continue;
    }
    for (int r = 0; r < P; ++r)
      if (enqueue_step_any(sh[r], false, need)) return -1;
  }
  return 0;
}

int gs_rccl_unique_id(void* out128) {
  ncclUniqueId id;
  GS_NCCL(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "unexpected ncclUniqueId size");
  memcpy(out128, &id, sizeof(id));
  return 0;
}

}  // extern "C"

namespace {
// GRAVSIM_CRASH_TRACE=1: a fatal signal in any thread of a rank (ours, HIP's or RCCL's
// proxy/socket threads) prints that thread's native stack to stderr before the default
// action runs. Host-side diagnosis only; it was added to locate the multi-process
// graph-capture crash over RCCL sockets (profiles/r2_graph_comm_multiprocess.txt).
constexpr int kTraceSigs[] = {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT};
struct sigaction g_prev_action[sizeof(kTraceSigs) / sizeof(int)];

void crash_trace_handler(int sig, siginfo_t* info, void*) {
  char head[160];
  const int len = snprintf(head, sizeof(head),
                           "gravsim: signal %d (addr %p) in pid %d tid %ld, native stack:\n", sig,
                           info ? info->si_addr : nullptr, (int)getpid(), (long)gettid());
  if (len > 0) (void)!write(2, head, (size_t)len);
  // Deep enough for a runaway recursion: print the innermost 8 and the outermost 40 frames.
  static void* frames[1 << 18];
  const int n = backtrace(frames, 1 << 18);
  if (n <= 48) {
    backtrace_symbols_fd(frames, n, 2);
  } else {
    backtrace_symbols_fd(frames, 8, 2);
    const int skipped = snprintf(head, sizeof(head), "  ... %d frames ...\n", n - 48);
    if (skipped > 0) (void)!write(2, head, (size_t)skipped);
    backtrace_symbols_fd(frames + n - 40, 40, 2);
  }
  // Chain to whatever was installed before (Python's faulthandler prints every thread's
  // Python stack), then the default action.
  for (size_t k = 0; k < sizeof(kTraceSigs) / sizeof(int); ++k)
    if (kTraceSigs[k] == sig) sigaction(sig, &g_prev_action[k], nullptr);
  raise(sig);
}

void maybe_install_crash_trace() {
  static bool done = false;
  if (done || !getenv("GRAVSIM_CRASH_TRACE")) return;
  done = true;
  void* warm[1];
  (void)backtrace(warm, 1);  // loads libgcc's unwinder now, not inside the handler
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = crash_trace_handler;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND | SA_ONSTACK;
  // An alternate stack for this (the host's main) thread, so a stack overflow still reports.
  static char alt[1 << 16];
  stack_t ss;
  memset(&ss, 0, sizeof(ss));
  ss.ss_sp = alt;
  ss.ss_size = sizeof(alt);
  (void)sigaltstack(&ss, nullptr);
  sigemptyset(&sa.sa_mask);
  for (size_t k = 0; k < sizeof(kTraceSigs) / sizeof(int); ++k)
    sigaction(kTraceSigs[k], &sa, &g_prev_action[k]);
}
}  // namespace

extern "C" {

int gs_stepper_comm_init(gs_stepper* s, const void* id128, int32_t rank, int32_t nranks) {
  maybe_install_crash_trace();
  if (rank != s->cfg.rank || nranks != s->cfg.nranks) {
    gs_set_error("comm_init: rank/nranks differ from the stepper's layout");
    return -1;
  }
  GS_HIP(hipSetDevice(s->cfg.device));
  ncclUniqueId id;
  memcpy(&id, id128, sizeof(id));
  // The one-sided multi-rank schedule is always split (the sym schedule has its own slots).
  if (s->L.mode != GS_MODE_SYM && ensure_partial(s)) return -1;
  GS_NCCL(ncclCommInitRank(&s->comm, nranks, id, rank));
  // GRAVSIM_FORCE_COMM keeps a 1-rank communicator live so the full multi-rank schedule
  // (in-place ncclAllGather, local/remote split on two streams, events) runs on one GPU.
  s->have_comm = nranks > 1 || getenv("GRAVSIM_FORCE_COMM") != nullptr;
  if (!s->have_comm) {
    (void)ncclCommDestroy(s->comm);
    s->comm = nullptr;
  }
  drop_graphs(s);
  if (s->have_comm) {
    // Warm-up: RCCL builds its transports lazily on the first collective and on the first
    // send/recv to each peer. Do both here on scratch memory (the accel buffer holds
    // n_local * 4 >= P elements) so that no timed or captured step pays for it.
    char* buf = static_cast<char*>(s->acc);
    const ncclDataType_t dt = s->esz == 4 ? ncclFloat32 : ncclFloat64;
    GS_NCCL(ncclAllGather(buf + (size_t)rank * s->esz, buf, 1, dt, s->comm, s->s_comm));
    if (nranks > 1 && s->cfg.strategy == GS_STRATEGY_RING) {
      GS_NCCL(ncclGroupStart());
      GS_NCCL(ncclSend(buf, 1, dt, (rank + 1) % nranks, s->comm, s->s_comm));
      GS_NCCL(ncclRecv(buf + (size_t)nranks * s->esz, 1, dt, (rank - 1 + nranks) % nranks,
                       s->comm, s->s_comm));
      GS_NCCL(ncclGroupEnd());
    }
    if (nranks > 1 && s->L.mode == GS_MODE_SYM) {
      // The sym schedule's node-sum exchange talks to every peer: connect them all now.
      GS_NCCL(ncclGroupStart());
      for (int q = 0; q < nranks; ++q) {
        if (q == rank) continue;
        GS_NCCL(ncclSend(buf + (size_t)q * s->esz, 1, dt, q, s->comm, s->s_comm));
        GS_NCCL(ncclRecv(buf + (size_t)(nranks + q) * s->esz, 1, dt, q, s->comm, s->s_comm));
      }
      GS_NCCL(ncclGroupEnd());
    }
    GS_HIP(hipStreamSynchronize(s->s_comm));
  }
  return 0;
}

int gs_stepper_comm_check(gs_stepper* s) {
  if (!s->have_comm) return 0;
  ncclResult_t async = ncclSuccess;
  GS_NCCL(ncclCommGetAsyncError(s->comm, &async));
  if (async != ncclSuccess && async != ncclInProgress) {
    char b[256];
    snprintf(b, sizeof(b), "RCCL async error: %s; communicator aborted", ncclGetErrorString(async));
    (void)ncclCommAbort(s->comm);
    s->have_comm = false;
    gs_set_error(b);
    return -1;
  }
  return 0;
}

}  // extern "C"
