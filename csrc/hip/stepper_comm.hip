// Collectives of the native Stepper: the per-step all-gather of positions (in-place
// ncclAllGather, or a group of in-place ncclBroadcasts for uneven slices), the ring pass,
// the sym schedule's node-sum exchange, the per-rank emulation's modeled collectives, and
// the RCCL communicator's bootstrap, warm-up and failure checks.
//
// Reference parity:
//   mpi.c:142-182  MPI_Init / Bcast / Type_create_struct -> ncclCommInitRank from a 128-byte
//                  unique id (the launcher broadcasts it over the gloo control plane)
//   mpi.c:227-236  MPI_Allgatherv (aliased buffers) + MPI_Barrier every step -> gather():
//                  in place on the comm stream, ordered by events, no barrier
#include "gs_stepper.h"

namespace gs::rt {

// Emulated collective on s_comm (GRAVSIM_EMU_COMM_GBPS > 0): the byte count moved through HBM
// by emu_wgs workgroups that stay resident for latency + bytes / rate (comm_model.hip). The
// kernel copies min(bytes, src_cap, emu_cap) bytes (src_cap: what the source buffer holds);
// the modeled time always uses the full byte count.
// time_bytes: the bytes that set the modeled duration (default: all of them); the kernel
// still moves `bytes` (clamped to the buffers).
int comm_model(gs_stepper* s, const void* src, size_t bytes, size_t src_cap, size_t time_bytes) {
  if (s->emu_gbps <= 0.0 || bytes == 0) return 0;
  if (time_bytes > bytes) time_bytes = bytes;
  const double us = s->emu_lat_us + (double)time_bytes / (s->emu_gbps * 1e3);
  if (bytes > s->emu_cap) bytes = s->emu_cap;  // (sized at create for the larger collective)
  if (bytes > src_cap) bytes = src_cap;
  const uint64_t ticks = (uint64_t)(us * s->clk_khz / 1e3);
  GS_HIP(gs::launch_comm_model(src, s->emu_buf, bytes, ticks, s->emu_wgs, s->s_comm));
  return 0;
}

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
int gather(gs_stepper* s, int cur, bool gate) {
  if (!xcomm(s) || s->full[cur]) return 0;
  // Flag sync publishes every gather through the gate flag of its buffer, gated launch or
  // not: the compute stream's wait on the gather polls it. The READY signal re-arms it first,
  // on the compute stream, so no wait behind this point can see a gate left set by an earlier
  // gather of the buffer (a state read's, before init reset the step count).
  if (comp_signal(s, s->ev_ready, kSyncReady,
                  fsync(s) && !s->sym_ring ? s->gate_buf + cur : nullptr))
    return -1;
  s->full[cur] = true;
  if (fsync(s)) gate = true;
  return comm_do(s, [s, cur, gate]() -> int {
    if (comm_dead(s)) return -1;
    char* buf = static_cast<char*>(s->X[cur]);
    const size_t count = (size_t)s->L.n_local * 4;
    if (comm_wait_comp(s, s->ev_ready, kSyncReady)) return -1;
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
bool abort_comm(gs_stepper* s) {
  ncclComm_t c = s->comm_live.exchange(nullptr);
  if (!c) return false;
  s->comm_stage.store(-1);
  // flag-sync waits still spinning on this communicator's collectives fall through (a wait
  // that gave up first keeps its own code, 1)
  if (s->sync_fail && s->sync_fail[0] == 0u) s->sync_fail[0] = 2u;
  (void)ncclCommAbort(c);
  return true;
}

// A communicator the watchdog thread (or a timeout / async error) aborted must not be used
// again: have_comm stays true on the main thread until it notices, but s->comm is freed once
// comm_live is null. Every RCCL call site checks this first.
bool comm_dead(gs_stepper* s) {
  if (!s->have_comm || s->emulate || s->comm_live.load() != nullptr) return false;
  gs_set_error("RCCL communicator aborted (watchdog, timeout or async error)");
  return true;
}

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
  if (comm_dead(s)) return -1;
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

// Node reduce for the bodies of destination ranks r + kb .. r + ke - 1 (mod P): consecutive
// ranks own consecutive rows, so that is one cyclic body range and one launch (their sums
// land in the Sbuf blocks of those ranks).
// `sig`: a flag-sync counter to raise before this work (SymArgs::sig; raised by a signal
// kernel instead when there is no launch to carry it).
// `with_row`: the row reduce goes into the same launch (launch_sym_node_row).
static int node_reduce_dests(gs_stepper* s, const gs::SymArgs& a0, int kb, int ke,
                             unsigned* sig = nullptr, bool with_row = false) {
  const int P = s->cfg.nranks, r = s->cfg.rank;
  // (destinations whose sums are +0.0 by the geometry at either end of the range are left out:
  // their node sums are never sent)
  while (kb < ke && !s->pair_live(r, (r + kb) % P)) ++kb;
  while (ke > kb && !s->pair_live(r, (r + ke - 1) % P)) --ke;
  gs::SymArgs a = a0;
  a.x_lo = kb < ke ? s->rbeg[(r + kb) % P] : 0;
  a.x_count = 0;
  for (int k = kb; k < ke; ++k) a.x_count += s->rcnt[(r + k) % P];
  if (a.x_count == 0) {
    if (sig) GS_HIP(gs::launch_sync_signal(sig, nullptr, s->s_comp));
    if (with_row) GS_HIP(gs::launch_sym_row_reduce(a0, s->s_comp));
    return 0;
  }
  a.sig = sig;
  if (with_row) GS_HIP(gs::launch_sym_node_row(a, s->s_comp));
  else GS_HIP(gs::launch_sym_node_reduce(a, s->s_comp));
  return 0;
}

// Node reduce + node-sum exchange of the symmetric schedule: rank r sends the sums of its
// reduction-tree nodes for the bodies of rank q to q and receives q's nodes for its own
// bodies (ncclSend/ncclRecv). Pipelined as a ring shift: at shift k rank r reduces the sums
// for rank r + k, and the sends of shift k pair with the receives of shift k on the peer
// (rank r + k receives from (r + k) - k = r), so every group of send/recv pairs is complete
// on both sides. The shifts go out in two stages: stage 1's messages travel while stage 2's
// destinations, the rank's own sums (they never leave the GPU) and the row reduce are
// computed, instead of the whole exchange waiting for the whole node reduce (1M / 8 ranks:
// a 190 us exchange behind a 100 us node reduce). Same kernels and sums per body: same bits.
// The compute stream joins the exchange later (comp_wait on ev_sym before finalize).
int sym_reduce_exchange(gs_stepper* s, const gs::SymArgs& a0, bool* exchanged, bool* row_done) {
  const int P = s->cfg.nranks, r = s->cfg.rank;
  // stage g: shifts [k_lo[g], k_lo[g + 1]). Stage 1 is the smaller one (a third of the
  // shifts): its reduce is short, so the messages start early, and the larger stage 2 reduce
  // plus the own sums and the row reduce hide behind its transfer.
  const int stages = P - 1 < 2 ? P - 1 : 2;
  const int k1 = (P - 1) / 3 > 1 ? (P - 1) / 3 : 1;
  const int k_lo[3] = {1, stages == 2 ? 1 + k1 : P, P};
  // With flag sync a stage's signal rides on the next node reduce launch (SymArgs::sig).
  unsigned* pending = nullptr;
  for (int g = 0; g < stages; ++g) {
    if (node_reduce_dests(s, a0, k_lo[g], k_lo[g + 1], pending)) return -1;
    pending = nullptr;
    if (fsync(s)) pending = s->sync_buf + 2 * (kSyncStage0 + g);
    else if (comp_signal(s, s->ev_stage[g], kSyncStage0 + g)) return -1;
    const int kb = k_lo[g], ke = k_lo[g + 1];
    const bool first = g == 0, last = g + 1 == stages;
    if (comm_do(s, [s, g, kb, ke, first, last]() -> int {
          const int P = s->cfg.nranks, r = s->cfg.rank;
          const size_t e = s->esz, nl = (size_t)s->L.n_local, my = (size_t)s->nn[r];
          if (comm_dead(s)) return -1;
          if (comm_wait_comp(s, s->ev_stage[g], kSyncStage0 + g)) return -1;
          if (first) GS_MARK(x0, x, s->s_comm);
          // Pairs whose node sums are +0.0 by the geometry (gs_sym_pair_live) are neither sent
          // nor received: the receiver's slots keep the +0.0 they were zeroed to (both sides
          // evaluate the same table, so every send still meets its receive).
          if (s->emulate) {
            // the bytes this rank receives in this stage, read from its receive buffer
            size_t bytes = 0, peak = 0;
            for (int k = kb; k < ke; ++k) {
              const int src = (r - k + P) % P;
              if (!s->pair_live(src, r)) continue;
              const size_t b = (size_t)s->nn[src] * 3 * nl * e;
              bytes += b;
              peak = b > peak ? b : peak;
            }
            if (comm_model(s, s->sym_R, bytes, (size_t)s->sym_NN * 3 * nl * e,
                           s->emu_links ? peak : bytes))
              return -1;
          } else {
            const ncclDataType_t dt = s->esz == 8 ? ncclFloat64 : ncclFloat32;
            GS_NCCL(ncclGroupStart());
            for (int k = kb; k < ke; ++k) {
              const int q = (r + k) % P, src = (r - k + P) % P;
              if (s->pair_live(r, q))
                GS_NCCL(ncclSend(s->sym_S + my * 3 * (size_t)s->rbeg[q] * e,
                                 my * 3 * s->rcnt[q], dt, q, s->comm, s->s_comm));
              if (s->pair_live(src, r))
                GS_NCCL(ncclRecv(s->sym_R + (size_t)s->nbase[src] * 3 * nl * e,
                                 (size_t)s->nn[src] * 3 * nl, dt, src, s->comm, s->s_comm));
            }
            GS_NCCL(ncclGroupEnd());
          }
          if (last) {
            GS_MARK(x1, x, s->s_comm);
            if (comm_signal_comp(s, s->ev_sym, kSyncExch)) return -1;
          }
          return 0;
        }))
      return -1;
  }
  // the own sums, last, with the row reduce in the same launch (one band: Pi, Pd, Px hold
  // every row; multi-band runs reduce their rows band by band)
  const bool with_row = a0.Bbuf == nullptr && a0.band0 == 0 && a0.band_rows == a0.rows;
  if (node_reduce_dests(s, a0, 0, 1, pending, with_row)) return -1;
  *row_done = with_row;
  // (a live 1-rank communicator: nothing to exchange, and nothing for finalize to wait for)
  *exchanged = stages > 0;
  return 0;
}

}  // namespace gs::rt

extern "C" {

int gs_rccl_unique_id(void* out128) {
  ncclUniqueId id;
  GS_NCCL(ncclGetUniqueId(&id));
  static_assert(sizeof(id) == 128, "unexpected ncclUniqueId size");
  memcpy(out128, &id, sizeof(id));
  return 0;
}

}  // extern "C"

namespace gs::rt {
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
}  // namespace gs::rt

using namespace gs::rt;

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
  // Stages for a watchdog on another thread (gs_stepper_comm_stage): a rank stuck here is
  // reported as "in ncclCommInitRank" / "in the warm-up", not just "in comm_init".
  s->comm_stage.store(1);
  GS_NCCL(ncclCommInitRank(&s->comm, nranks, id, rank));
  s->comm_live.store(s->comm);
  // What RCCL actually formed: the rank count, this rank's place in it and the
  // device its kernels run on must be the ones the layout and the stepper were built for.
  {
    int cnt = 0, ur = -1, dev = -1;
    GS_NCCL(ncclCommCount(s->comm, &cnt));
    GS_NCCL(ncclCommUserRank(s->comm, &ur));
    GS_NCCL(ncclCommCuDevice(s->comm, &dev));
    s->comm_count = cnt;
    s->comm_user_rank = ur;
    s->comm_cu_device = dev;
    if (cnt != nranks || ur != rank || dev != s->cfg.device) {
      char b[256];
      snprintf(b, sizeof(b),
               "comm_init: RCCL formed %d rank(s), this one rank %d on device %d; expected %d "
               "rank(s), rank %d on device %d",
               cnt, ur, dev, nranks, rank, s->cfg.device);
      abort_comm(s);
      gs_set_error(b);
      return -1;
    }
  }
  // GRAVSIM_FORCE_COMM keeps a 1-rank communicator live so the full multi-rank schedule
  // (in-place ncclAllGather, local/remote split on two streams, events) runs on one GPU.
  s->have_comm = nranks > 1 || getenv("GRAVSIM_FORCE_COMM") != nullptr;
  if (!s->have_comm) {
    s->comm_live.store(nullptr);
    (void)ncclCommDestroy(s->comm);
    s->comm = nullptr;
    s->comm_count = 0;  // (none kept)
  }
  drop_graphs(s);
  if (s->have_comm) {
    // Warm-up: RCCL builds its transports lazily on the first collective and on the first
    // send/recv to each peer. Do both here on scratch memory (the accel buffer holds
    // n_local * 4 >= P elements) so that no timed or captured step pays for it.
    char* buf = static_cast<char*>(s->acc);
    const ncclDataType_t dt = s->esz == 4 ? ncclFloat32 : ncclFloat64;
    s->comm_stage.store(2);
    GS_NCCL(ncclAllGather(buf + (size_t)rank * s->esz, buf, 1, dt, s->comm, s->s_comm));
    if (nranks > 1 && s->cfg.strategy == GS_STRATEGY_RING) {
      s->comm_stage.store(3);
      GS_NCCL(ncclGroupStart());
      GS_NCCL(ncclSend(buf, 1, dt, (rank + 1) % nranks, s->comm, s->s_comm));
      GS_NCCL(ncclRecv(buf + (size_t)nranks * s->esz, 1, dt, (rank - 1 + nranks) % nranks,
                       s->comm, s->s_comm));
      GS_NCCL(ncclGroupEnd());
    }
    if (nranks > 1 && s->L.mode == GS_MODE_SYM) {
      // The sym schedule's node-sum exchange talks to every peer: connect them all now.
      s->comm_stage.store(4);
      GS_NCCL(ncclGroupStart());
      for (int q = 0; q < nranks; ++q) {
        if (q == rank) continue;
        GS_NCCL(ncclSend(buf + (size_t)q * s->esz, 1, dt, q, s->comm, s->s_comm));
        GS_NCCL(ncclRecv(buf + (size_t)(nranks + q) * s->esz, 1, dt, q, s->comm, s->s_comm));
      }
      GS_NCCL(ncclGroupEnd());
    }
    // Bounded like a step: a peer that never joins the warm-up aborts the communicator after
    // the step timeout instead of blocking here forever.
    s->comm_stage.store(5);
    const int64_t rec = s->prog_rec;
    if (note_progress(s) || wait_until(s, rec + 1, s->step_timeout_s)) return -1;
  }
  s->comm_stage.store(6);
  return 0;
}

int32_t gs_stepper_comm_stage(gs_stepper* s) { return s ? s->comm_stage.load() : 0; }

int gs_stepper_comm_info(gs_stepper* s, int32_t* count, int32_t* user_rank, int32_t* cu_device) {
  if (!s) return -1;
  if (count) *count = s->comm_count;
  if (user_rank) *user_rank = s->comm_user_rank;
  if (cu_device) *cu_device = s->comm_cu_device;
  return 0;
}

int32_t gs_stepper_abort(gs_stepper* s) { return s && abort_comm(s) ? 1 : 0; }

int gs_stepper_comm_check(gs_stepper* s) {
  if (!s->have_comm) return 0;
  if (comm_dead(s)) {  // aborted from another thread: the handle is gone
    s->have_comm = false;
    return -1;
  }
  ncclResult_t async = ncclSuccess;
  GS_NCCL(ncclCommGetAsyncError(s->comm, &async));
  if (async != ncclSuccess && async != ncclInProgress) {
    char b[256];
    snprintf(b, sizeof(b), "RCCL async error: %s; communicator aborted", ncclGetErrorString(async));
    abort_comm(s);
    s->have_comm = false;
    gs_set_error(b);
    return -1;
  }
  return 0;
}

}  // extern "C"
