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
#include "gs_stepper.h"


namespace gs::rt {

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





// Bytes one rank receives per step: the all-gather's remote slices, and the node sums the
// other ranks send it (sym schedule).
size_t gather_bytes(const gs_stepper* s) {
  return (size_t)(s->L.n_pad - s->L.n_local) * row_bytes(s);
}
size_t exchange_bytes(const gs_stepper* s) {
  size_t nodes = 0;  // the other ranks' nodes this rank receives (live pairs only)
  for (int q = 0; q < s->cfg.nranks; ++q)
    if (q != s->cfg.rank && s->pair_live(q, s->cfg.rank)) nodes += (size_t)s->nn[q];
  return nodes * 3 * s->L.n_local * s->esz;
}


// Phase events of the step being enqueued (timed eager steps; at most 256 per phase_stats).
gs_stepper::PhaseEv* phase_begin(gs_stepper* s) {
  // (never reallocates: run_plan holds two of these pointers at once)
  if (s->pev.capacity() < 256) s->pev.reserve(256);
  if (s->pev_used >= (int)s->pev.size()) {
    if (s->pev.size() >= 256) return nullptr;
    gs_stepper::PhaseEv e{};
    for (hipEvent_t* p : {&e.t0, &e.end, &e.g0, &e.g1, &e.w0, &e.w1, &e.x0, &e.x1, &e.j0, &e.j1})
      if (hipEventCreate(p) != hipSuccess) return nullptr;
    s->pev.push_back(e);
  }
  gs_stepper::PhaseEv* p = &s->pev[s->pev_used++];
  p->g = p->w = p->x = p->j = false;
  p->nsteps = 1;
  return p;
}

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
  a.Px = s->sym_Px;
  a.Kr = s->sym_Kr;
  a.Np = s->sym_Np;
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
  gs::sym_cut_mask(a.cut2, &a.cut_k, &a.cut_c);
  a.band0 = 0;
  a.band_rows = a.rows;
  a.gate = nullptr;
  a.defer = s->defer;
  a.defer_max = s->gate_buf + 3;
  a.lf = s->sym_lf;
  a.defer_grid = 2 * s->cus;  // resident force workgroups: 2 per CU
  a.defer_index = 0;
  a.utrace = s->utrace;
  if (s->dyn_cap > 1) {
    a.work = s->gate_buf + 4;
    a.unit_cap = s->dyn_cap;
    a.first_wave = s->sym_first_wave;
    a.persist = s->cfg.nranks == 1 && !xcomm(s) && s->sym_persist ? 1 : 0;
  }
  a.trace_defer0 = (int32_t)s->utrace_main;
  a.audit = s->audit;
  a.clk = s->clk;
  return a;
}


int ensure_sym(gs_stepper* s) {
  if (s->L.mode != GS_MODE_SYM || s->sym_Pi) return 0;
  if (gs_sym_geometry(s->L.n_pad, &s->sym_NC, &s->sym_H, &s->sym_L, &s->sym_S_n, &s->sym_D))
    return -1;
  s->sym_Kr = gs_sym_split_segments(s->L.n_pad);
  s->sym_Np = gs_sym_split_parts(s->L.n_pad);
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
  s->live.assign((size_t)P * P, 1);
  for (int q = 0; q < P; ++q)
    for (int d = 0; d < P; ++d) {
      const int32_t v = gs_sym_pair_live(s->L.n_pad, P, q, d);
      if (v < 0) return -1;
      s->live[(size_t)q * P + d] = (char)v;
    }
  const size_t nl = (size_t)s->L.n_local, rows = nl / gs::kSymC;
  const size_t e = s->esz;
  // Rows per band: the partial slots of one band stay within the budget: half of the free
  // HBM at creation (an MI355X has 288 GB; at least 32 GiB), GRAVSIM_SYM_BAND_MB overrides
  // (tests use a tiny budget to force many bands). 1M bodies need 6.4 GB for all rows; 16M
  // on 8 ranks needs 109 GB per rank, one band on an otherwise empty MI355X.
  const size_t per_row =
      (size_t)(s->sym_S_n + s->sym_kx() + s->sym_H + s->sym_D) * 3 * gs::kSymC * e;
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
  if (s->sym_Kr > 0 &&
      dev_alloc(s, &s->sym_Px, band * s->sym_kx() * 3 * gs::kSymC * e, "sym_Px"))
    return -1;
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
  const int64_t ib = s->L.n_local / (gs::kForceBlock * s->L.ipl);
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
//   0: wait for the gather, then one launch of every unit.
// (Two launches split at the gather, diagonal units or all rank-local units first, paid a
// launch boundary - a unit is ~0.6 ms of work at 1M - to hide a ~0.1 ms gather and lost to 0:
// 21.4-21.6 and 22.4-22.6 against 21.0-21.2 ms, profiles/r1_sym_overlap_ab.txt; deleted.)
// With `exchange` the node reduce is pipelined with the RCCL node-sum exchange (two stages,
// sym_reduce_exchange), which runs beside the rest of the node reduce and the row reduce;
// the compute stream joins it before finalize.
// One rank (no exchange, no virtual shards), one band, up to 256K bodies: the tree over the
// row blocks, the row reduce and finalize run as one sym_tail_kernel (same bits). Interleaved A/B
// (profiles/r2_fused_tail_ab.jsonl): 65K 0.707 vs 0.708 ms, 256K 10.51 vs 10.57 ms, but 1M
// 166.8 vs 166.1 ms, where the fused kernel's fewer threads for the j-side sums lose.
// gs_stepper_set_tuning forces the three-kernel / fused tail at any size (bitwise tests).
// Every sym force launch goes through here: it tells the launcher whether the dynamic unit
// counter is known to be 0 (re-armed by the fused tail kernel enqueued after the previous
// launch on this stream), then marks it dirty until the next fused tail.
hipError_t force_sym_launch(gs_stepper* s, gs::SymArgs a, hipStream_t st) {
  a.work_zero = s->work_zero ? 1 : 0;
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

// `gated`: the units-6 launch (a.gate: the gather's gate flag, which its remote units test);
// `gflag`: the gate flag the compute stream's wait on the gather polls under flag sync.
int sym_force(gs_stepper* s, gs::SymArgs a, bool overlap_gather, bool exchange = false,
              bool gated = false, const unsigned* gflag = nullptr) {
  for (int b0 = 0; b0 < a.rows; b0 += s->sym_band) {
    a.band0 = b0;
    a.band_rows = s->sym_band < a.rows - b0 ? s->sym_band : a.rows - b0;
    a.units = 0;
    const bool one_band = a.band_rows == a.rows;
    if (overlap_gather && b0 == 0 && one_band && gated) {
      // 3: one launch with the local units first; remote units run in it once the gather is
      // published, or are deferred to a second launch queued behind the gather.
      a.units = 6;
      GS_HIP(force_sym_launch(s, a, s->s_comp));
      // (The units-7 launch polling the gate itself instead of a wait kernel in front of it
      // deadlocked two ranks sharing one GPU: its workgroups, at the force kernel's register
      // allocation, filled the GPU while the peer rank's launches needed it.)
      if (comp_wait_comm(s, s->ev_gathered, kMarkGather, -1, gflag)) return -1;
      a.units = 7;
      GS_HIP(force_sym_launch(s, a, s->s_comp));
      a.units = 0;
    } else {
      if (overlap_gather && b0 == 0) {
        if (comp_wait_comm(s, s->ev_gathered, kMarkGather, -1, gflag)) return -1;
      }
      GS_HIP(force_sym_launch(s, a, s->s_comp));
    }
    if (fused_tail(s)) continue;  // reductions + integrate in sym_tail_kernel (one band)
    const bool last = b0 + a.band_rows >= a.rows;
    // The row reduce (Pi, Pd -> Ti) runs after the block / node reduce (Pj) on the same
    // stream: forking it onto a second stream measured slower, the two streaming sums contend
    // (reduce phase at 1M 1533-1592 us per step against 1342-1381 in sequence;
    // profiles/r3_reduce_fork_split_ab.txt).
    if (a.Bbuf) GS_HIP(gs::launch_sym_block_reduce(a, s->s_comp));  // the band's leaves
    // (The row reduce on a second stream beside the node stages and the exchange measured
    // worse at rank 7 of 8, 1M: chain 650 against 257 us, step 22.1-22.2 against 21.4-21.5 ms,
    // profiles/r5_nt_loads_ab.txt; it stays in sequence.)
    bool exchanged = false, row_done = false;
    if (last) {
      if (exchange) {
        // node reduce pipelined with the sends (its last launch carries the row reduce)
        if (sym_reduce_exchange(s, a, &exchanged, &row_done)) return -1;
      } else if (!a.Bbuf && one_band) {
        // one launch for the node reduce and the row reduce (launch_sym_node_row)
        GS_HIP(gs::launch_sym_node_row(a, s->s_comp));
        row_done = true;
      } else {
        GS_HIP(gs::launch_sym_node_reduce(a, s->s_comp));
      }
    }
    if (!row_done) GS_HIP(gs::launch_sym_row_reduce(a, s->s_comp));
    if (exchanged) {
      if (comp_wait_comm(s, s->ev_sym, kMarkExchange, kSyncExch)) return -1;
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
  // Flag sync: every gather of this buffer is published by its gate flag, which finalize
  // re-arms for the gather two steps on (a.gate; the force kernel tests it in units 6 only).
  const bool fs = fsync(s) && !gathered_externally;
  if (gated || fs) {
    a.gate = s->sym_ring ? s->ring_gate + 8 * cur : s->gate_buf + cur;
    a.gate_n = s->sym_ring ? 8 : 1;
  }
  if (part & 1) {
    if (need_gather) {
      if (gathered_externally) s->full[cur] = true;
      else if (gather(s, cur, gated)) return -1;
    }
    if (sym_force(s, a, need_gather, xcomm(s), gated, fs ? s->gate_buf + cur : nullptr))
      return -1;
    if (timed) GS_HIP(hipEventRecord(s->ev_local, s->s_comp));
  }
  if (part & 2) {
    if (fused_tail(s)) {
      GS_HIP(gs::launch_sym_tail(a, s->s_comp, s->tail_split_on()));
    } else {
      GS_HIP(gs::launch_sym_finalize(a, s->s_comp));
    }
    // both re-armed the dynamic unit counter of this step's force launch: the next step's
    // launch needs no memset (one launch fewer per step)
    s->work_zero = true;
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

int enqueue_step_any(gs_stepper* s, bool capturing, bool gathered_externally) {
  return s->esz == 4 ? enqueue_step<float>(s, capturing, gathered_externally)
                     : enqueue_step<double>(s, capturing, gathered_externally);
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
  if (sync_failed(s)) return -1;  // (a state a wait gave up on is not returned)
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
      if (sym_force(s, sa, false, xcomm(s))) return -1;
      if (fused_tail(s)) {
        GS_HIP(gs::launch_sym_tail(sa, s->s_comp, s->tail_split_on()));
      } else {
        GS_HIP(gs::launch_sym_finalize(sa, s->s_comp));
      }
      s->work_zero = true;  // (both re-arm the unit counter)
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


}  // namespace gs::rt

using namespace gs::rt;

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
  // Environment knobs (read once, here): the per-rank emulation (GRAVSIM_EMULATE_RANK, its
  // modeled collectives GRAVSIM_EMU_COMM="GB/s[,latency us[,workgroups]]"), the multi-rank
  // overlap mode (GRAVSIM_SYM_OVERLAP), fault injection (GRAVSIM_FAULT_SKIP_UNITS). Band
  // budget, tracing and the 1-rank communicator are read where they act.
  s->emulate = getenv("GRAVSIM_EMULATE_RANK") != nullptr && cfg->nranks > 1;
  // Multi-rank sym steps default to the gated local-first launch (3): remote units start as
  // soon as the gather lands, nothing waits on it (see sym_force).
  s->sym_overlap = cfg->nranks > 1 ? 3 : 0;
  if (const char* ov = getenv("GRAVSIM_SYM_OVERLAP")) s->sym_overlap = atoi(ov);
  s->emu_links = getenv("GRAVSIM_EMU_LINKS") != nullptr && atoi(getenv("GRAVSIM_EMU_LINKS")) != 0;
  if (const char* v = getenv("GRAVSIM_EMU_COMM")) {
    double us = s->emu_lat_us;
    int wgs = s->emu_wgs;
    const int got = sscanf(v, "%lf,%lf,%d", &s->emu_gbps, &us, &wgs);
    if (got >= 2) s->emu_lat_us = us;
    if (got >= 3) s->emu_wgs = wgs;
  }
  if (s->esz == 8) s->dyn_cap = 4;  // fp64: 512K 101.9-102.0 ms at 4 vs 102.0-102.5 at 2
  if (const char* v = getenv("GRAVSIM_FAULT_SKIP_UNITS")) s->fault_skip = (unsigned)atoi(v);
  if (const char* v = getenv("GRAVSIM_TAIL_SPLIT")) s->tail_split = atoi(v);
  // Long one-rank graphs only where a launch of graph_steps steps stays far inside the host's
  // progress bound (one progress event per launch; >= 60 s): 32 steps up to 256K bodies, 8 up
  // to 2M (fp64 2M on one GPU: ~1.5 s per step). At 1M and above the launch gap is noise.
  // 32 against 8 steps: 16K -0.8 %, 65K -0.15 %, 256K even (profiles/r6_graph_steps_32_ab.jsonl).
  s->graph_steps = s->L.n_pad <= (int64_t{1} << 18) ? 32 : s->L.n_pad <= (int64_t{1} << 21) ? 8 : 2;
  if (const char* v = getenv("GRAVSIM_GRAPH_STEPS")) s->graph_steps = atoi(v) & ~1;
  // GRAVSIM_SYNC=events: the multi-rank step orders its streams by hipEvents (and replays a
  // segmented plan) instead of device counters (flag sync, one graph per period)
  if (const char* v = getenv("GRAVSIM_SYNC")) s->sync_events = strcmp(v, "events") == 0;
  // Under rocprofv3 --pmc (it exports ROCPROF_COUNTER_COLLECTION) every dispatch is
  // serialized, so a wait kernel would wait for a signal queued behind it until the step
  // timeout: counter collection runs with event ordering (GRAVSIM_SYNC=flags overrides).
  if (getenv("ROCPROF_COUNTER_COLLECTION") &&
      !(getenv("GRAVSIM_SYNC") && strcmp(getenv("GRAVSIM_SYNC"), "flags") == 0))
    s->sync_events = true;
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
    s->sym_first_wave = (occ > 0 ? occ : 2) * s->cus;  // (gs_stepper_set_tuning: tests)
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
  for (hipEvent_t& e : s->ev_stage) FAIL_CLEAN(hipEventCreateWithFlags(&e, hipEventDisableTiming));
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
  if (cfg->nranks > 1 || getenv("GRAVSIM_FORCE_COMM")) {
    // flag-sync counters of the multi-rank step (signals / waits per point) and the waits'
    // stall statistics
    ALLOC_CLEAN(&s->sync_buf, 2 * kSyncCount * sizeof(unsigned), "sync");
    FAIL_CLEAN(hipMemsetAsync(s->sync_buf, 0, 2 * kSyncCount * sizeof(unsigned), s->s_comp));
    // [0..8] stall statistics, [9] the wait kernels' give-up bound (write_sync_limit)
    ALLOC_CLEAN(&s->sync_stats, 10 * sizeof(unsigned long long), "sync_stats");
    FAIL_CLEAN(hipMemsetAsync(s->sync_stats, 0, 10 * sizeof(unsigned long long), s->s_comp));
    FAIL_CLEAN(hipStreamSynchronize(s->s_comp));
    if (write_sync_limit(s)) {
      gs_stepper_destroy(s);
      return -1;
    }
    void* hf = nullptr;
    FAIL_CLEAN(hipHostMalloc(&hf, 64, hipHostMallocMapped | hipHostMallocCoherent));
    s->sync_fail = static_cast<volatile unsigned*>(hf);
    s->sync_fail[0] = 0u;
    FAIL_CLEAN(hipHostGetDevicePointer(reinterpret_cast<void**>(&s->sync_fail_dev), hf, 0));
  }
  if (s->L.mode == GS_MODE_SYM) {
    // the work audit's unit counter (its cost is within noise: profiles/r3_abaudit*)
    ALLOC_CLEAN(&s->audit, sizeof(unsigned long long), "audit");
    FAIL_CLEAN(hipMemsetAsync(s->audit, 0, sizeof(unsigned long long), s->s_comp));
    ALLOC_CLEAN(&s->clk, 4 * sizeof(unsigned long long), "clock");
    FAIL_CLEAN(hipMemsetAsync(s->clk, 0, 4 * sizeof(unsigned long long), s->s_comp));
  }
  if (s->L.mode == GS_MODE_SYM) {
    // Deferred-unit list of the gated launch (one band's units) and the local-first order.
    const int rows = (int)(s->L.n_local / gs::kSymC);
    const size_t units = (size_t)rows * (s->sym_S_n + s->sym_D + s->sym_kx()) + 1;
    ALLOC_CLEAN(&s->defer, units * sizeof(unsigned), "defer");
    FAIL_CLEAN(hipMemsetAsync(s->defer, 0, units * sizeof(unsigned), s->s_comp));
    // unit -> row, segment (bit 31: remote), local units first (layout.cpp).
    const long fill = 4L * s->cus;  // two dispatch waves of 2 workgroups per CU
    std::vector<int32_t> lf(units - 1);
    s->sym_ring = cfg->strategy == GS_STRATEGY_RING && cfg->nranks > 1;
    const int64_t got =
        s->sym_ring ? gs_sym_unit_map_ring(s->L.n_pad, cfg->rank, cfg->nranks, fill, lf.data(),
                                           (int64_t)lf.size())
                    : gs_sym_unit_map_parts(s->L.n_pad, cfg->rank, cfg->nranks, fill, s->sym_Kr,
                                            s->sym_Np, lf.data(), (int64_t)lf.size());
    lf.resize(got > 0 ? (size_t)got : 0);  // 0: geometry too large for the entry fields
    if (!lf.empty()) {
      ALLOC_CLEAN(&s->sym_lf, lf.size() * sizeof(int32_t), "unit_map");
      FAIL_CLEAN(hipMemcpy(s->sym_lf, lf.data(), lf.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice));
    }
  }
  if (s->L.mode == GS_MODE_SYM && getenv("GRAVSIM_UNIT_TRACE")) {
    // One entry per unit of a band-wide launch plus as many deferred ones (units 7).
    s->utrace_main = (int64_t)s->sym_band * (s->sym_S_n + s->sym_D + s->sym_kx());
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
  // (a communicator aborted by a watchdog, a timeout or an async error is not destroyed)
  if (s->have_comm && s->comm_live.exchange(nullptr)) (void)ncclCommDestroy(s->comm);
  for (const auto& m : s->mem) (void)hipFree(m.p);
  s->mem.clear();
  if (s->sync_fail) (void)hipHostFree(const_cast<unsigned*>(s->sync_fail));
  for (hipEvent_t e : {s->ev_ready, s->ev_gathered, s->ev_t0, s->ev_local, s->ev_end,
                       s->ev_remote, s->ev_fork, s->ev_rem2, s->ev_sym, s->ev_stage[0],
                       s->ev_stage[1]})
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
  // (timed steps replay the graph too: a one-rank period is timed as a whole, so the phase
  // pass measures the schedule the timed loop ran; captured multi-rank steps stay eager)
  const bool graph_ok = seg || (s->cfg.use_graph >= (xcomm(s) ? 2 : 1) &&
                                !(xcomm(s) && (s->graph_failed || s->timed)));
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
      }
      // one-rank graphs: graph_steps steps per launch while that many are left
      const int gsteps = !seg && !xcomm(s) && s->graph_steps > 2 && left >= s->graph_steps
                             ? s->graph_steps : 2;
      if (!seg) {
        hipGraphExec_t& gx = gsteps > 2 ? s->graph_long : s->graph;
        if (!gx) {
          // both one-rank graphs at the first replay (the warm-up), so a timed loop never
          // pays a capture
          const bool both = !xcomm(s) && s->graph_steps > 2;
          if ((!s->graph && build_graph(s, 2)) ||
              (both && !s->graph_long && build_graph(s, s->graph_steps))) {
            if (!xcomm(s)) return -1;
            s->graph_failed = true;  // eager from here on (the error text is kept)
            continue;
          }
        }
        gs_stepper::PhaseEv* pe = s->timed ? phase_begin(s) : nullptr;
        if (pe) {
          pe->nsteps = gsteps;
          GS_HIP(hipEventRecord(pe->t0, s->s_comp));
        }
        GS_HIP(hipGraphLaunch(gx, s->s_comp));
        if (pe) {
          GS_HIP(hipEventRecord(pe->end, s->s_comp));
          s->pev_plan += gsteps;
        }
      }
      s->k += gsteps;
      // After one period: X[1] was gathered in the second step, X[0] holds only the own slice.
      s->full[0] = !xcomm(s);
      s->full[1] = true;
      left -= gsteps;
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
  s->pev_plan = 0;
  // (the wait kernels' stall counters restart with the timed steps. Both streams drain
  // first: the comm stream's waits add to stats[6..8] and nothing orders them against a
  // memset on the compute stream, so a comm-side timeout could be erased or an old stall
  // survive into the timed window. A timeout already counted fails here.)
  if (s->sync_stats) {
    // (a bounded wait for every stream: a hung collective fails here instead of blocking)
    if (wait_until(s, s->prog_rec, s->step_timeout_s)) return -1;
    GS_HIP(hipMemsetAsync(s->sync_stats, 0, 9 * sizeof(unsigned long long), s->s_comp));
    GS_HIP(hipStreamSynchronize(s->s_comp));
  }
  return 0;
}

int gs_stepper_set_overlap(gs_stepper* s, int32_t mode) {
  if (mode != 0 && mode != 3) { gs_set_error("set_overlap: mode must be 0 or 3"); return -1; }
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

int gs_stepper_set_tuning(gs_stepper* s, int32_t first_wave, int32_t fused_tail) {
  if (first_wave > 0) s->sym_first_wave = first_wave;
  if (fused_tail >= 0) s->fuse_tail = fused_tail ? 1 : 0;
  s->work_zero = false;
  drop_graphs(s);
  return 0;
}

int gs_stepper_set_persist(gs_stepper* s, int32_t on) {
  s->sym_persist = on != 0;
  s->work_zero = false;
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
int32_t gs_stepper_get_dyn_cap(gs_stepper* s) { return s->dyn_cap; }

int32_t gs_stepper_mem_entry(gs_stepper* s, int32_t i, const char** tag, uint64_t* bytes) {
  if (!s) return -1;
  if (i >= 0 && i < (int32_t)s->mem.size()) {
    if (tag) *tag = s->mem[i].tag;
    if (bytes) *bytes = s->mem[i].bytes;
  }
  return (int32_t)s->mem.size();
}

int gs_stepper_graph_steps(gs_stepper* s) {
  return s->graph_steps > 2 && s->cfg.nranks == 1 ? s->graph_steps : 2;
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
  // (a split segment counts as its Np parts, whichever way it ran)
  if (units_per_step) *units_per_step = rows * (uint64_t)(s->sym_S_n + s->sym_D + s->sym_kx());
  if (units_done) {
    GS_HIP(hipStreamSynchronize(s->s_comp));
    unsigned long long h = 0;
    GS_HIP(hipMemcpy(&h, s->audit, sizeof(h), hipMemcpyDeviceToHost));
    *units_done = h;
  }
  return 0;
}

int gs_stepper_clock(gs_stepper* s, double* out4) {
  for (int i = 0; i < 4; ++i) out4[i] = 0.0;
  if (!s->clk) return 0;  // one-sided schedules: no clock record
  GS_HIP(hipSetDevice(s->cfg.device));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_rem));
  unsigned long long h[3] = {0, 0, 0};
  GS_HIP(hipMemcpy(h, s->clk, sizeof(h), hipMemcpyDeviceToHost));
  GS_HIP(hipMemsetAsync(s->clk, 0, 4 * sizeof(unsigned long long), s->s_comp));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  out4[0] = h[1] ? (double)h[0] / (double)h[1] * s->clk_khz * 1e-6 : 0.0;  // GHz
  out4[1] = (double)h[0];
  out4[2] = (double)h[1] / (s->clk_khz * 1e3);  // workgroup-seconds
  out4[3] = (double)h[2];
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
  // the device-side bound follows (a word the wait kernels read, graphs included: ADVICE r5)
  return write_sync_limit(s);
}

int gs_stepper_sync(gs_stepper* s) {
  GS_HIP(hipStreamSynchronize(s->s_comm));
  GS_HIP(hipStreamSynchronize(s->s_rem));
  GS_HIP(hipStreamSynchronize(s->s_rem2));
  GS_HIP(hipStreamSynchronize(s->s_comp));
  s->prog_done = s->prog_rec;
  return sync_failed(s) ? -1 : 0;
}

// Bounded wait for every stream, polling RCCL async errors. The deadline bounds PROGRESS: it
// restarts whenever one more enqueued step (or graph period) completes, so a long healthy
// run never trips it while a hang (a dead peer, a stuck collective) or an RCCL error aborts
// the communicator and returns -1 instead of blocking forever (the reference's
// MPI_ERRORS_ARE_FATAL / silent CUDA errors: SURVEY.md §5).
int gs_stepper_wait(gs_stepper* s, double timeout_s) {
  return wait_until(s, s->prog_rec, timeout_s);
}

// Phase timing of the steps enqueued since gs_stepper_set_timing(s, 1) / the previous call
// (at most 256 event sets), averaged per step. out[0] steps, [1] total ms, [2] all-gather ms
// and [3] node-sum exchange ms (spans on the comm stream), [4] exposed gather ms and [5]
// exposed exchange ms (compute-stream stalls on them: exposed comm = [4] + [5]), [6] the
// most force units one step deferred past the gather (overlap 3), [7] how many of the steps
// were replayed (one-rank step graph, or the multi-rank segmented plan) instead of eager.
int gs_stepper_phase_stats(gs_stepper* s, double* out8) {
  for (int i = 0; i < 8; ++i) out8[i] = 0.0;
  for (hipStream_t st : {s->s_comm, s->s_rem, s->s_rem2, s->s_comp})
    GS_HIP(hipStreamSynchronize(st));
  s->prog_done = s->prog_rec;
  const int n_ev = s->pev_used;
  int n = 0;  // steps (a graph period's event set spans two; its partner set, none)
  for (int i = 0; i < n_ev; ++i) {
    const gs_stepper::PhaseEv& p = s->pev[i];
    n += p.nsteps;
    float v = 0.f;
    if (p.nsteps > 0) {
      GS_HIP(hipEventElapsedTime(&v, p.t0, p.end));
      out8[1] += v;
    }
    if (p.g) { GS_HIP(hipEventElapsedTime(&v, p.g0, p.g1)); out8[2] += v; }
    if (p.x) { GS_HIP(hipEventElapsedTime(&v, p.x0, p.x1)); out8[3] += v; }
    if (p.w) { GS_HIP(hipEventElapsedTime(&v, p.w0, p.w1)); out8[4] += v; }
    if (p.j) { GS_HIP(hipEventElapsedTime(&v, p.j0, p.j1)); out8[5] += v; }
  }
  if (s->sync_stats) {
    // flag sync: the compute stream's stalls are the wait kernels' own (device counters of
    // s_memrealtime ticks), not host-recorded event pairs
    unsigned long long st[9];
    GS_HIP(hipMemcpy(st, s->sync_stats, sizeof(st), hipMemcpyDeviceToHost));
    if (st[1] || st[4]) {
      out8[4] = st[0] / s->clk_khz;
      out8[5] = st[3] / s->clk_khz;
    }
    if (st[2] || st[5] || st[8]) {
      gs_set_error("flag sync: a wait kernel gave up after the step timeout");
      return -1;
    }
    GS_HIP(hipMemsetAsync(s->sync_stats, 0, sizeof(st), s->s_comp));
  }
  if (n > 0)
    for (int i = 1; i < 6; ++i) out8[i] /= n;
  out8[0] = n;
  unsigned d[2] = {0, 0};
  GS_HIP(hipMemcpy(d, s->gate_buf + 2, sizeof(d), hipMemcpyDeviceToHost));
  out8[6] = d[1];
  out8[7] = s->pev_plan;  // of them replayed (graph or segmented plan; the rest eager)
  s->pev_plan = 0;
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

int32_t gs_stepper_period_start(gs_stepper* s) {
  return (s->k & 1) == 0 && (xcomm(s) ? !s->full[0] : true) ? 1 : 0;
}

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


}  // extern "C"

