// Internal kernel-launch interface between nbody_kernels.hip and the Stepper runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace gs {

// Kernel arguments (passed by value). Arrays hold 4 components per body: X/X_next/partial
// are (x, y, z, mu) / (ax, ay, az, sum mu/r); vel is (vx, vy, vz, 0); acc_out is
// (ax, ay, az, phi). i-indexed arrays other than X/X_next are rank-local (li = gi - i_begin).
template <typename T>
struct KArgs {
  const T* X;        // [n_pad * 4] gathered positions for this step
  T* X_next;         // [n_pad * 4] next-step positions (own slice written)
  T* vel;            // [n_local * 4]
  T* partial;        // [n_chunks * n_local * 4] per-chunk partial sums
  T* acc_out;        // optional [n_local * 4]: emit accelerations instead of integrating
  int64_t i_begin;   // global index of this rank's first body
  int64_t n_local;   // padded bodies per rank
  int64_t n_real;    // real global body count
  int64_t chunk;     // canonical j-chunk length
  int32_t n_chunks;  // chunks holding real bodies
  int32_t c_begin, c_end;      // split kernel: chunk range ...
  int32_t skip_begin, skip_end;  // ... minus this sub-range (the rank's own chunks)
  int32_t phi;       // accumulate the potential sum too (implies the exact cutoff)
  int32_t exact;     // hard cutoff select (else the fast core-softened path)
  T dt, cut2, eps2;  // eps2: softening^2, or the fast path's core^2 when larger
};

// Chunks a split launch covers: [c_begin, c_end) minus [skip_begin, skip_end).
template <typename T>
inline int split_span(const KArgs<T>& a) {
  const int sb = a.skip_begin < a.c_begin ? a.c_begin : (a.skip_begin > a.c_end ? a.c_end : a.skip_begin);
  const int se = a.skip_end < sb ? sb : (a.skip_end > a.c_end ? a.c_end : a.skip_end);
  return (a.c_end - a.c_begin) - (se - sb);
}

// ---- Newton-3 symmetric schedule (fp32/fp64, fast cutoff; nbody_sym.hip) -------------
// Canonical decomposition, a function of the padded body count only (so every rank count
// P from 1 to 8 produces the same bits): chunks of kSymC = 2048 bodies, NC = n_pad / 2048 of
// them, B row blocks of RB = NC / B rows (gs_common.h sym_blocks: B <= 256). Chunk A pairs
// with the next h(A) chunks cyclically (h = NC/2 - 1, plus the antipodal chunk A + NC/2 for
// half of the rows, alternating by parity: every unordered chunk pair exactly once, equal
// work per block of rows) and with itself (one-sided). Row A's shell is cut into segments of
// L quanta (128 bodies; see gs_sym_geometry), its diagonal chunk into D parts; one workgroup
// per unit writes an i-side partial (Pi[row][segment] or Pd[row][part]) and, for every shell
// tile it visits, the j-side partial of its 2048 i-bodies into Pj[row][d-1]. Rows are
// processed in bands of whole blocks (all of a rank's rows unless the partial buffers would
// exceed the band budget); the row reduce forms Ti = sum_q Pd[q] + sum_s Pi[s] per band. The
// j-side sums reach a body as S = a binary tree over the B blocks (leaves row-ascending); a
// rank owns whole blocks (mpi.c's remainder rule) and reduces the dyadic nodes covering its
// range (from Pj with one band, from per-block leaves in Bbuf with several). Final:
// a = Ti + S, then the KD integrate. Every sum runs in the same order for any band size and
// any P from 1 to 8.
constexpr int kSymC = 2048;

struct SymArgs {
  // Arrays are float (fp32 run) or double (fp64 run); the launchers pick the instantiation.
  const void* X;       // [n_pad * 4] gathered positions (x, y, z, mu)
  void* Pi;            // [rows][S][3][kSymC] i-side partials (segment = L quanta of 128)
  void* Pj;            // [rows][H][3][kSymC] j-side partials, H = NC / 2
  void* Pd;            // [rows][D][3][kSymC] diagonal-chunk partials
  // Split segments (the launch tail): the last Kr shell segments of every row are summed as
  // Np parts of their tiles (gs_sym_split_parts: 4 when a segment has >= 4 quanta, else 2),
  // part 0 in Pi and part p > 0 in Px[rows][Kr][Np - 1][3][kSymC]; the row reduce adds
  // (((part 0 + part 1) + part 2) + ...) for them. A designated segment runs whole (all parts,
  // one workgroup) or as Np part units (entries at the end of the units 0 / units 6 orders, so
  // the launch's last units are 1 / Np as long); either way the same Np sums, so the same
  // bits. A step then runs rows x (S + D + (Np - 1) Kr) units.
  void* Px;
  int32_t Kr, Np;
  void* Ti;            // [3][n_local] per-body i-side total: sum_q Pd[q] + sum_s Pi[s]
  void* Sbuf;          // [dest rank q][own node k < nn][3][n_local(q)] node sums by destination
  const void* Rbuf;    // [node j, all ranks' nodes in global order][3][n_local] received
                       // (the own nodes' slots are not used: finalize reads them from Sbuf)
  int64_t x_lo, x_count;  // node reduce: bodies x_lo .. x_lo + x_count - 1 (cyclic mod n_pad;
                          // x_count 0: every real body), so the sums of some destination
                          // ranks can be sent while the next ones' are reduced
  void* Bbuf;          // multi-band only: [own block][3][real bodies] per-block leaf sums
  void* X_next;        // [n_pad * 4]
  void* vel;           // [n_local * 4]
  void* acc_out;       // optional [n_local * 4]: emit accelerations instead of integrating
  int64_t n_real, n_local, i_begin;
  int32_t NC, a0, rows, S, L, H, P, real_chunks;
  int32_t D;           // parts of the diagonal chunk (L < 16 quanta: 16 / L)
  int32_t B, RB;       // row blocks and rows per block
  int32_t rank, nn;    // this rank and the dyadic nodes it reduces and sends (maximal ones)
  int32_t blk_lo[9];   // rank q owns blocks [blk_lo[q], blk_lo[q + 1]), q < P
  int32_t band0, band_rows;  // rows [band0, band0 + band_rows) of this rank (rank-relative)
                             // are in the Pi/Pj/Pd buffers (row index - band0)
  int32_t fp64;        // element type of every array above
  int32_t exact;       // reference hard cutoff (select at cut2) instead of the fast core
  int32_t units;       // which units a force launch covers: 0 all (shell segments row by row,
                       // then the diagonal parts, then the split segments as part units:
                       // short units fill the launch's last wave), 6 all, rank-local units
                       // first, remote units gated on `gate`, 7 the units the units-6 launch
                       // deferred (after the gather)
  double dt, eps2, cut2;
  // fp32 exact cutoff as a clamp mask (gs_sym_tile.h cutoff_mask_r2): {-K, K cut2} with K a
  // power of two scaling (float)cut2 to ~2^40 (sym_cut_mask); both 0 when cut2 is 0.
  float cut_k, cut_c;
  // Gather gate (units 6/7): set on the comm stream right after the all-gather; a remote unit
  // that finds it still closed appends itself to defer[1..] (count defer[0]) and exits, and
  // the units-7 launch behind the gather event runs them. Finalize clears gate and count.
  // defer_max: the largest deferred count seen (diagnostics).
  unsigned* gate;        // gate[stage]: all-gather: gate[0]; ring: gate[k] after stage k
  int32_t gate_n;        // flags finalize re-arms: 1 (all-gather) or 8 (ring stages)
  unsigned* defer;
  unsigned* defer_max;
  const int32_t* lf;    // units 6 order: unit -> row, segment (bit 31: remote unit)
  int32_t defer_grid;   // units 7: workgroups walking the deferred list
  int32_t defer_index;  // (device-side) the deferred entry a units-7 workgroup is running
  // Unit timeline probe (GRAVSIM_UNIT_TRACE, diagnostics only; nullptr otherwise): per force
  // workgroup 4 words {start, end (s_memrealtime, 100 MHz), HW_ID | XCC_ID << 32,
  // row << 32 | segment}, at [blockIdx.x] (units 0/6) or [trace_defer0 + k] (units 7).
  unsigned long long* utrace;
  int32_t trace_defer0;
  // Dynamic unit fetch (units 0 / 6; nullptr: unit = blockIdx.x). Workgroups take unit
  // indices from work[0] in order, the first `first_wave` workgroups one unit each, the others
  // up to `unit_cap`, so XCDs that run faster take more units. The launcher zeroes work[0]
  // on the stream before every such launch. n_units: set by the launcher.
  unsigned* work;
  int32_t n_units, unit_cap, first_wave;
  // Persistent workgroups (one rank, no collective beside the launch): the grid is the
  // resident slots only and every workgroup takes units until the queue is empty, so no
  // workgroup exits early and no replacement has to be dispatched mid-launch.
  int32_t persist;
  // work[0] is already 0 on this stream (the fused tail kernel that ran after the previous
  // dynamic launch re-armed it): the launcher skips its memset.
  int32_t work_zero;
  // Work audit: +1 per force unit that ran to completion (or was empty), so a step's count
  // must be rows x (S + D + (Np - 1) Kr) whatever the launch split, deferral or fetch order (a
  // split segment run whole counts its Np parts).
  unsigned long long* audit;
  // Flag sync (comm_model.hip sync_signal_kernel): a counter the node reduce launch raises at
  // its start, for the exchange stage whose sums the launch before it produced (that launch has
  // completed and released its writes at the kernel boundary). Saves the one-lane signal
  // kernel between two stages. nullptr: none.
  unsigned* sig;
  // Engine-clock record of the force launches (nullptr: off): wave 0 of every workgroup reads
  // s_memtime (shader clock) and s_memrealtime (100 MHz) when it starts and when it leaves,
  // and adds the two differences and a count to clk[0..2] (one relaxed atomic each). The
  // duration-weighted clock the launch ran at is clk[0] / clk[1] x 100 MHz, and clk[0] is the
  // workgroup-cycles it took: a cost in cycles, independent of the box's DVFS state
  // (bench.py engine_clock_ghz / cycles_per_pair_eval). Diagnostic only: no output value
  // depends on it.
  unsigned long long* clk;
};

hipError_t launch_force_sym(const SymArgs& a, hipStream_t s);
// SymArgs::cut_k / cut_c for a cutoff^2 (as the fp32 tile sees it: (float)cut2).
inline void sym_cut_mask(double cut2, float* k, float* c) {
  const float c2 = (float)cut2;
  if (!(c2 > 0.f)) {
    *k = *c = 0.f;
    return;
  }
  int e = 0;
  (void)frexpf(c2, &e);  // c2 = f 2^e, f in [0.5, 1)
  int s = 40 - e;
  if (s > 126) s = 126;
  if (s < -126) s = -126;
  const float K = ldexpf(1.f, s);
  *k = -K;
  *c = K * c2;  // exact (a power-of-two scaling inside the normal range)
}
// Modeled collective (per-rank emulation) and the gather gate (comm_model.hip).
hipError_t launch_comm_model(const void* src, void* dst, size_t bytes, uint64_t ticks, int wgs,
                             hipStream_t s);
hipError_t launch_gate_set(unsigned* gate, hipStream_t s);
// Device-side stream ordering (comm_model.hip): signal = one release add to a counter (after
// zeroing the level flag `clear`, if given); wait =
// one wave polling `flag` until it passes seen[0] (a counter; seen nullptr: a level flag),
// adding its stall to stats[0] (s_memrealtime ticks) and 1 to stats[1]; gives up after
// *limit_ticks (a device word) or once the sticky host-mapped word *fail is set, counting it
// in stats[2], setting *fail and leaving seen[0] as it was.
hipError_t launch_sync_signal(unsigned* count, unsigned* clear, hipStream_t s);
hipError_t launch_sync_wait(const unsigned* flag, unsigned* seen, unsigned long long* stats,
                            const unsigned long long* limit_ticks, unsigned* fail,
                            hipStream_t s);
hipError_t launch_sym_block_reduce(const SymArgs& a, hipStream_t s);  // band leaves -> Bbuf
hipError_t launch_sym_node_reduce(const SymArgs& a, hipStream_t s);   // own nodes -> Sbuf
hipError_t launch_sym_row_reduce(const SymArgs& a, hipStream_t s);    // the band's rows -> Ti
// The own node sums (a.x_lo / x_count) and the row reduce as one launch (same bits).
hipError_t launch_sym_node_row(const SymArgs& a, hipStream_t s);
hipError_t launch_sym_finalize(const SymArgs& a, hipStream_t s);
// One rank, one band: group reduce + row reduce + finalize in one kernel, same bits.
// split: the two halves of Ti in separate waves (small N), else in one thread (same bits).
hipError_t launch_sym_tail(const SymArgs& a, hipStream_t s, bool split);
int sym_occupancy(int fp64);

template <typename T>
hipError_t launch_force_split(const KArgs<T>& a, int kernel, int ipl, int groups, hipStream_t s);
template <typename T>
hipError_t launch_force_fused(const KArgs<T>& a, int kernel, int ipl, hipStream_t s);
// Resident workgroups per CU of the split kernel (fm: 0 fast, 1 exact, 2 exact+phi).
template <typename T>
int split_occupancy(int kernel, int ipl, int fm);
// Experimental MFMA-assisted fp32 split kernel (nbody_mfma.hip); no potential sum.
hipError_t launch_force_mfma(const KArgs<float>& a, int groups, hipStream_t s);
int mfma_occupancy(int fm);
template <typename T>
hipError_t launch_reduce_integrate(const KArgs<T>& a, hipStream_t s);
template <typename T>
hipError_t launch_init_ics(int ic, uint64_t seed, int64_t n, int64_t n_pad, int64_t i_begin,
                           int64_t n_local, double G, T* X4, T* vel4, double* mass,
                           hipStream_t s);
template <typename T>
hipError_t launch_count_nonfinite(const T* X4, int64_t i0, int64_t nl, const T* vel4,
                                  unsigned long long* out, hipStream_t s);

}  // namespace gs
