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

}  // namespace gs::rt
