// Step graphs and segmented plans of the native Stepper, and its progress-bounded wait.
//
// One rank replays two steps (one ping-pong period) from one hipGraph (build_graph). A
// multi-rank step replays a *plan* (build_plan / run_plan): the compute stream's work between
// two cross-stream points is captured as one graph segment, and the collectives plus the
// event record / wait that order them against the compute stream are issued eagerly between
// the segments, so RCCL is never captured (profiles/r2_graph_comm_root_cause.txt). The step
// code marks those points through comp_record / comp_wait / comm_do, which act immediately
// when no plan is being recorded.
//
// Reference parity: cuda.cu:154-167 / mpi.c:189-237 run the step loop with a blocking
// device sync (cudaDeviceSynchronize) or MPI_Barrier per step; here the host runs ahead of
// the GPU (up to 64 steps) and waits on progress events with a deadline (wait_until).
#include "gs_stepper.h"

namespace gs::rt {

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
      gs_stepper::PlanOp op{gs_stepper::PlanOp::kGraph, x, nullptr, {}};
      op.step = s->seg_step;  // the segment holds work of the step it began in
      s->plan.push_back(std::move(op));
      ++s->plan_graphs;
    }
  }
  (void)hipGraphDestroy(g);
  GS_HIP(e);
  return 0;
}

int seg_open(gs_stepper* s) {
  s->seg_step = s->rec_step;
  GS_HIP(hipStreamBeginCapture(s->s_comp, hipStreamCaptureModeThreadLocal));
  return 0;
}

namespace {
int plan_push(gs_stepper* s, gs_stepper::PlanOp op) {
  if (seg_cut(s)) return -1;
  op.step = s->rec_step;
  s->plan.push_back(std::move(op));
  return seg_open(s);
}

// The events of a measured stall on s_comp (exposed gather w0/w1, exposed exchange j0/j1).
struct MarkEv {
  hipEvent_t gs_stepper::PhaseEv::*a;
  hipEvent_t gs_stepper::PhaseEv::*b;
  bool gs_stepper::PhaseEv::*flag;
};
MarkEv mark_events(int mark) {
  return mark == kMarkExchange
             ? MarkEv{&gs_stepper::PhaseEv::j0, &gs_stepper::PhaseEv::j1, &gs_stepper::PhaseEv::j}
             : MarkEv{&gs_stepper::PhaseEv::w0, &gs_stepper::PhaseEv::w1, &gs_stepper::PhaseEv::w};
}

// hipStreamWaitEvent(s_comp, ev), bracketed by the stall's phase events of `pe` (if any).
int timed_wait(gs_stepper* s, hipEvent_t ev, int mark, gs_stepper::PhaseEv* pe) {
  const MarkEv m = mark_events(mark);
  if (pe && mark != kMarkNone) GS_HIP(hipEventRecord(pe->*m.a, s->s_comp));
  GS_HIP(hipStreamWaitEvent(s->s_comp, ev, 0));
  if (pe && mark != kMarkNone) {
    GS_HIP(hipEventRecord(pe->*m.b, s->s_comp));
    pe->*m.flag = true;
  }
  return 0;
}
}  // namespace

// hipEventRecord(ev, s_comp) for another stream to wait on.
int comp_record(gs_stepper* s, hipEvent_t ev) {
  if (!s->rec) {
    GS_HIP(hipEventRecord(ev, s->s_comp));
    return 0;
  }
  return plan_push(s, {gs_stepper::PlanOp::kRecord, nullptr, ev, {}});
}

// hipStreamWaitEvent(s_comp, ev) on an event another stream records. `mark` names the stall
// for the phase timing (eager timed steps, or a replayed plan with timing on).
int comp_wait(gs_stepper* s, hipEvent_t ev, int mark) {
  if (!s->rec) return timed_wait(s, ev, mark, s->pe);
  gs_stepper::PlanOp op{gs_stepper::PlanOp::kWait, nullptr, ev, {}};
  op.mark = mark;
  return plan_push(s, std::move(op));
}

// Work on the comm stream (a collective and its event bookkeeping): run now, or replayed
// eagerly at this point of the plan. With flag sync the comm stream never waits on a host-
// visible point of the compute stream, so the op is kept without cutting the open segment
// (a replay issues a period's comm ops, then its one compute graph).
int comm_do(gs_stepper* s, std::function<int()> fn) {
  if (!s->rec) return fn();
  if (fsync(s)) {
    gs_stepper::PlanOp op{gs_stepper::PlanOp::kHost, nullptr, nullptr, std::move(fn)};
    op.step = s->rec_step;
    s->plan.push_back(std::move(op));
    return 0;
  }
  return plan_push(s, {gs_stepper::PlanOp::kHost, nullptr, nullptr, std::move(fn)});
}

// ---- cross-stream points: events, or device counters (flag sync) ------------------------
uint64_t sync_limit_ticks(const gs_stepper* s) {
  double t = s->step_timeout_s > 0 ? 2.0 * s->step_timeout_s + 10.0 : 600.0;
  if (const char* v = getenv("GRAVSIM_SYNC_LIMIT_S")) t = atof(v);
  return (uint64_t)(t * s->clk_khz * 1e3);
}

int write_sync_limit(gs_stepper* s) {
  if (!s->sync_stats) return 0;
  const unsigned long long v = sync_limit_ticks(s);
  // (a blocking copy from pageable memory: the word is current before any later enqueue; the
  // streams are non-blocking, so nothing in flight is waited for)
  GS_HIP(hipMemcpy(s->sync_stats + 9, &v, sizeof(v), hipMemcpyHostToDevice));
  return 0;
}

bool sync_failed(gs_stepper* s) {
  if (!s->sync_fail || s->sync_fail[0] == 0u) return false;
  if (s->have_comm) {
    abort_comm(s);
    s->have_comm = false;
  }
  gs_set_error(s->sync_fail[0] == 1u
                   ? "flag sync: a cross-stream wait gave up (a collective or a peer stalled "
                     "past the device bound); the step's results are invalid"
                   : "flag sync: the communicator was aborted while a step waited on it; the "
                     "step's results are invalid");
  return true;
}

int comp_signal(gs_stepper* s, hipEvent_t ev, int id, unsigned* clear) {
  if (!fsync(s)) return comp_record(s, ev);
  GS_HIP(gs::launch_sync_signal(s->sync_buf + 2 * id, clear, s->s_comp));
  return 0;
}

int comm_wait_comp(gs_stepper* s, hipEvent_t ev, int id) {
  if (!fsync(s)) {
    GS_HIP(hipStreamWaitEvent(s->s_comm, ev, 0));
    return 0;
  }
  GS_HIP(gs::launch_sync_wait(s->sync_buf + 2 * id, s->sync_buf + 2 * id + 1, s->sync_stats + 6,
                              s->sync_stats + 9, s->sync_fail_dev, s->s_comm));
  return 0;
}

int comm_signal_comp(gs_stepper* s, hipEvent_t ev, int id) {
  GS_HIP(hipEventRecord(ev, s->s_comm));  // (eager users: download / accel queries)
  if (fsync(s)) GS_HIP(gs::launch_sync_signal(s->sync_buf + 2 * id, nullptr, s->s_comm));
  return 0;
}

int comp_wait_comm(gs_stepper* s, hipEvent_t ev, int mark, int id, const unsigned* flag) {
  if (!fsync(s)) return comp_wait(s, ev, mark);
  unsigned long long* st = s->sync_stats + (mark == kMarkExchange ? 3 : 0);
  if (flag) {
    GS_HIP(gs::launch_sync_wait(flag, nullptr, st, s->sync_stats + 9, s->sync_fail_dev,
                                s->s_comp));
  } else {
    GS_HIP(gs::launch_sync_wait(s->sync_buf + 2 * id, s->sync_buf + 2 * id + 1, st,
                                s->sync_stats + 9, s->sync_fail_dev, s->s_comp));
  }
  return 0;
}

void drop_graphs(gs_stepper* s) {
  for (hipGraphExec_t* g : {&s->graph, &s->graph_long}) {
    if (*g) {
      (void)hipGraphExecDestroy(*g);
      *g = nullptr;
    }
  }
  for (auto& op : s->plan)
    if (op.g) (void)hipGraphExecDestroy(op.g);
  s->plan.clear();
  s->plan_graphs = 0;
  s->plan_fsync = false;
}

int build_graph(gs_stepper* s, int steps) {
  // `steps` / 2 ping-pong periods (s->graph: one, two steps; s->graph_long: graph_steps)
  // starting from an even step with a gathered buffer.
  const int64_t k0 = s->k;
  const bool f0 = s->full[0], f1 = s->full[1];
  hipGraph_t g = nullptr;
  // The dynamic unit counter is 0 between steps in every reachable state: zeroed at creation,
  // and every step's last kernel (finalize or the fused tail) re-arms it after the step's force
  // launches, so a replay may start without a memset. (Round 2's graphs assumed this while
  // only the fused tail re-armed the counter, and replays after a non-fused step skipped
  // units; tests/test_gpu_sym.py test_sym_graph_replays_rezero_unit_counter and the work audit
  // of every bench and CLI run guard it.)
  s->work_zero = true;
  GS_HIP(hipStreamBeginCapture(s->s_comp, hipStreamCaptureModeThreadLocal));
  int rc = 0;
  for (int i = 0; i < steps && rc == 0; ++i) rc = enqueue_step_any(s, true);
  hipError_t e = hipStreamEndCapture(s->s_comp, &g);
  s->k = k0;
  s->full[0] = f0;
  s->full[1] = f1;
  if (rc) return rc;
  GS_HIP(e);
  GS_HIP(hipGraphInstantiate(steps > 2 ? &s->graph_long : &s->graph, g, nullptr, nullptr, 0));
  GS_HIP(hipGraphDestroy(g));
  return 0;
}

// Multi-rank steps whose cross-stream points all go through comp_record / comp_wait /
// comm_do: the sym schedule.
bool plan_ok(const gs_stepper* s) {
  return xcomm(s) && use_sym(s) && s->cfg.use_graph == 1;
}

// Record one ping-pong period (two steps, from an even step whose buffer needs its gather)
// as a plan: compute segments captured on s_comp, the collectives kept as eager host ops.
int build_plan(gs_stepper* s) {
  const int64_t k0 = s->k;
  const bool f0 = s->full[0], f1 = s->full[1];
  drop_graphs(s);
  s->plan_fsync = fsync(s);
  s->work_zero = true;  // (as build_graph: the counter is 0 between steps)
  s->rec_step = 0;
  if (seg_open(s)) return -1;
  s->rec = true;
  int rc = enqueue_step_any(s, true);
  s->rec_step = 1;
  if (rc == 0) rc = enqueue_step_any(s, true);
  s->rec = false;
  s->rec_step = 0;
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

// A flag-sync plan: the period's comm ops (eager, in order; their spans recorded per step),
// then its one compute graph (timed as a whole: one event set of two steps; the compute
// stream's stalls come from the wait kernels' device counters).
int run_plan_fsync(gs_stepper* s) {
  gs_stepper::PhaseEv* pe[2] = {nullptr, nullptr};
  if (s->timed) {
    for (auto& p : pe)
      if (!(p = phase_begin(s))) break;
    if (pe[0] && pe[1]) {
      pe[0]->nsteps = 2;
      pe[1]->nsteps = 0;  // (comm spans of step 1 only)
    } else {
      // (the 256-set cap: a lone first set would never be recorded, so phase_stats must not
      // count it)
      if (pe[0]) --s->pev_used;
      pe[0] = pe[1] = nullptr;
    }
  }
  for (auto& op : s->plan) {
    if (op.kind != gs_stepper::PlanOp::kHost) continue;
    s->pe = pe[op.step & 1];
    const int rc = op.fn();
    s->pe = nullptr;
    if (rc) return -1;
  }
  if (pe[0]) GS_HIP(hipEventRecord(pe[0]->t0, s->s_comp));
  for (auto& op : s->plan) {
    if (op.kind == gs_stepper::PlanOp::kGraph) GS_HIP(hipGraphLaunch(op.g, s->s_comp));
    else if (op.kind != gs_stepper::PlanOp::kHost) {
      gs_set_error("run_plan: a flag-sync plan holds only graphs and comm ops");
      return -1;
    }
  }
  if (pe[0]) {
    GS_HIP(hipEventRecord(pe[0]->end, s->s_comp));
    s->pev_plan += 2;
  }
  return 0;
}

int run_plan(gs_stepper* s) {
  if (s->plan_fsync) return run_plan_fsync(s);
  // Phase timing (gs_stepper_set_timing): one event set per step of the period. Step 0 starts
  // before the first op, step 1 at its first op (a segment belongs to the step it began in);
  // the collectives' spans are recorded on s_comm by the host ops (GS_MARK with `pe` set).
  gs_stepper::PhaseEv* pe[2] = {nullptr, nullptr};
  if (s->timed) {
    for (auto& p : pe)
      if (!(p = phase_begin(s))) break;
    if (pe[0]) GS_HIP(hipEventRecord(pe[0]->t0, s->s_comp));
  }
  int at = 0;
  for (auto& op : s->plan) {
    if (op.step != at) {
      if (pe[at]) GS_HIP(hipEventRecord(pe[at]->end, s->s_comp));
      at = op.step;
      if (pe[at]) GS_HIP(hipEventRecord(pe[at]->t0, s->s_comp));
    }
    switch (op.kind) {
      case gs_stepper::PlanOp::kGraph: GS_HIP(hipGraphLaunch(op.g, s->s_comp)); break;
      case gs_stepper::PlanOp::kRecord: GS_HIP(hipEventRecord(op.ev, s->s_comp)); break;
      case gs_stepper::PlanOp::kWait:
        if (timed_wait(s, op.ev, op.mark, pe[at])) return -1;
        break;
      case gs_stepper::PlanOp::kHost: {
        s->pe = pe[at];
        const int rc = op.fn();
        s->pe = nullptr;
        if (rc) return -1;
        break;
      }
    }
  }
  if (pe[at]) GS_HIP(hipEventRecord(pe[at]->end, s->s_comp));
  if (pe[0] && pe[1]) s->pev_plan += 2;
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
    if (sync_failed(s)) return -1;
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
        abort_comm(s);
        s->have_comm = false;
      }
      // flag-sync waits still spinning fall through instead of holding the streams until
      // their own (longer) bound; the stepper stays failed
      if (s->sync_fail && s->sync_fail[0] == 0u) s->sync_fail[0] = 2u;
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

}  // namespace gs::rt
