// Step-schedule helper kernels of the multi-rank Stepper (csrc/hip/stepper.hip).
//
// * comm_model_kernel: a stand-in for one RCCL collective in the per-rank timing emulation
//   (GRAVSIM_EMULATE_RANK). It moves the collective's exact byte count through HBM and holds
//   its workgroups until the modeled transfer time (latency + bytes / rate) has passed on the
//   wall clock, so the emulated step pays what an xGMI collective costs: its duration on the
//   comm stream and the CUs its kernel occupies (RCCL runs its channels as workgroups). The
//   reference times its whole loop, MPI_Allgatherv included (mpi.c:189,227-247); round-1
//   emulations treated the exchange as free.
// * gate_set_kernel: publishes "the all-gather into X[cur] is complete" to the force launch
//   that may already be running (overlap 3, the multi-rank default, nbody_sym.hip): one
//   system-scope release store after the collective on the comm stream. Force units only
//   test it (no spinning), so the collective never competes with waiting workgroups for CUs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_kernels.h"

namespace gs {
namespace {

__global__ __launch_bounds__(256) void comm_model_kernel(const uint4* __restrict__ src,
                                                         uint4* __restrict__ dst, int64_t n16,
                                                         uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
    dst[i] = src[i];
  if (threadIdx.x == 0)
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
  __syncthreads();
}

// System-scope release to pair with the force units' system-scope acquire (nbody_sym.hip
// gate_open_or_defer): the gathered rows come from peer GPUs. The kernel writes nothing
// before the flag (the collective's writes precede it by the stream order), and the explicit
// vmcnt wait keeps the flag behind the L2 write-back whatever the compiler decides.
__global__ void gate_set_kernel(unsigned* gate) {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(gate, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- device-side stream ordering (flag sync: the multi-rank sym step as ONE graph) --------
// A cross-stream ordering point of the multi-rank step (the comm stream waiting for the node
// sums of an exchange stage, the compute stream waiting for the exchange...) was a hipEvent
// record / wait pair; inside a segmented plan every such point cut the step graph, and each
// cut cost 15-25 us of GPU idle time (profiles/r4s2_rank8_timeline.txt: 5 cuts per step at
// 1M / 8). Here a point is a device counter instead: the producing stream runs a one-lane
// signal kernel behind the producing work (stream order: that work has completed and its
// writes were released at its kernel boundary), the consuming stream a one-workgroup wait
// kernel in front of the consuming work, which polls the counter until it has passed the
// number of signals the consumer has already taken (`seen`, a word only this consumer's
// wait kernels touch, in stream order). Every signal is matched by exactly one wait, in FIFO
// order per counter, so graph replays and eager steps interleave freely. The wait kernel is
// one wave with a handful of registers: it never holds the CUs an RCCL kernel or the force
// launch needs (round 2's in-kernel spin held them and deadlocked), and the kernel after it
// starts with the dispatch's acquire. A level flag (the gather gate, re-armed by finalize)
// works the same way without `seen`. Each wait adds its stall (s_memrealtime ticks) to
// stats[0] and one to stats[1]: the exposed comm of the replayed step, which a single graph
// cannot bracket with host events.
// Give-up: the spin ends after *limit ticks (a device word, so a graph captured
// before the host changed its step timeout still uses the new bound; set above the host's
// own progress bound, so the host abort normally wins) or as soon as the sticky failure word
// `fail` (host-mapped memory) is nonzero: set by an earlier wait that gave up, or by the host
// when it aborts the communicator. A wait that gives up does NOT advance `seen` (the signal
// it missed must not satisfy a later wait), counts the timeout in stats[2] and sets `fail`,
// so every later wait on either stream falls through at once and the host's sync / wait /
// state read reports the failure instead of returning a step computed from an unfinished
// gather or exchange.
// `clear` (optional): a level flag this point re-arms first (the gather gate of the buffer
// the signalled gather fills: the gate's wait on the compute stream must not see a gate left
// set by an earlier gather of that buffer, e.g. a state read's, once init has reset the step).
__global__ void sync_signal_kernel(unsigned* count, unsigned* clear) {
  if (threadIdx.x == 0) {
    if (clear) __hip_atomic_store(clear, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void sync_wait_kernel(const unsigned* flag, unsigned* seen,
                                 unsigned long long* stats, const unsigned long long* limit_p,
                                 unsigned* fail) {
  if (threadIdx.x != 0) return;
  const unsigned want = seen ? seen[0] + 1u : 1u;  // a level flag: any nonzero value
  const uint64_t limit = __hip_atomic_load(limit_p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  bool ok = true;
  for (unsigned it = 0;; ++it) {
    const unsigned v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (seen ? (int)(v - want) >= 0 : v != 0u) break;
    // (the host-mapped failure word: one system-scope read every 256 polls, ~100 us)
    if ((it & 255u) == 0u &&
        __hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(8);
    t = __builtin_amdgcn_s_memrealtime();
    if (t - t0 > limit) {
      ok = false;
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (ok && seen) seen[0] = want;
  if (!ok) __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (stats) {
    __hip_atomic_fetch_add(stats, (unsigned long long)(t - t0), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(stats + 1, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!ok) __hip_atomic_fetch_add(stats + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

hipError_t launch_sync_signal(unsigned* count, unsigned* clear, hipStream_t s) {
  hipLaunchKernelGGL(sync_signal_kernel, dim3(1), dim3(64), 0, s, count, clear);
  return hipGetLastError();
}

hipError_t launch_sync_wait(const unsigned* flag, unsigned* seen, unsigned long long* stats,
                            const unsigned long long* limit_ticks, unsigned* fail, hipStream_t s) {
  hipLaunchKernelGGL(sync_wait_kernel, dim3(1), dim3(64), 0, s, flag, seen, stats, limit_ticks,
                     fail);
  return hipGetLastError();
}

hipError_t launch_comm_model(const void* src, void* dst, size_t bytes, uint64_t ticks, int wgs,
                             hipStream_t s) {
  if (wgs < 1) wgs = 1;
  hipLaunchKernelGGL(comm_model_kernel, dim3(wgs), dim3(256), 0, s,
                     static_cast<const uint4*>(src), static_cast<uint4*>(dst),
                     (int64_t)(bytes / sizeof(uint4)), ticks);
  return hipGetLastError();
}

hipError_t launch_gate_set(unsigned* gate, hipStream_t s) {
  hipLaunchKernelGGL(gate_set_kernel, dim3(1), dim3(64), 0, s, gate);
  return hipGetLastError();
}

}  // namespace gs
