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

}  // namespace

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
