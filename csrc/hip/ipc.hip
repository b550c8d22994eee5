// Cross-process device-memory and event sharing on one node (HIP IPC), the mechanism RCCL's
// intra-node P2P transport builds on: a rank exports a handle to its buffer, a peer process
// maps it and reads/writes it directly. The reference's intra-node transport is whatever
// MPI_Allgatherv picks (mpi.c:227-236); here RCCL over xGMI moves the positions, and these
// entry points let tests/test_ipc_gpu.py check, on a one-GPU box, that the IPC path itself
// works under the launcher's environment (HSA_ENABLE_IPC_MODE_LEGACY=0: this driver only
// supports dmabuf IPC) before an 8-GPU node depends on it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "gravsim.h"

void gs_set_error(const char* msg);

namespace {
int fail(const char* what, hipError_t e) {
  char b[256];
  snprintf(b, sizeof(b), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
  gs_set_error(b);
  return -1;
}
#define GS_IPC(call)                          \
  do {                                        \
    const hipError_t e_ = (call);             \
    if (e_ != hipSuccess) return fail(#call, e_); \
  } while (0)
}  // namespace

extern "C" {

int gs_dev_alloc(int32_t device, uint64_t bytes, void** out) {
  GS_IPC(hipSetDevice(device));
  GS_IPC(hipMalloc(out, bytes));
  return 0;
}

int gs_dev_free(void* p) {
  GS_IPC(hipFree(p));
  return 0;
}

int gs_dev_copy(void* dst, const void* src, uint64_t bytes, int32_t to_device) {
  GS_IPC(hipMemcpy(dst, src, bytes, to_device ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost));
  return 0;
}

int gs_ipc_mem_handle(void* p, void* out64) {
  hipIpcMemHandle_t h;
  GS_IPC(hipIpcGetMemHandle(&h, p));
  memcpy(out64, &h, sizeof(h));
  return 0;
}

int gs_ipc_mem_open(int32_t device, const void* h64, void** out) {
  hipIpcMemHandle_t h;
  memcpy(&h, h64, sizeof(h));
  GS_IPC(hipSetDevice(device));
  GS_IPC(hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess));
  return 0;
}

int gs_ipc_mem_close(void* p) {
  GS_IPC(hipIpcCloseMemHandle(p));
  return 0;
}

// Interprocess event: created by the exporter, opened by the peer, which records it after
// its writes; the exporter waits for it on its own stream (RCCL's P2P flags do the same job
// inside its kernels; this checks the runtime path).
int gs_ipc_event_create(int32_t device, void** ev, void* out64) {
  GS_IPC(hipSetDevice(device));
  hipEvent_t e;
  GS_IPC(hipEventCreateWithFlags(&e, hipEventInterprocess | hipEventDisableTiming));
  hipIpcEventHandle_t h;
  GS_IPC(hipIpcGetEventHandle(&h, e));
  memcpy(out64, &h, sizeof(h));
  *ev = e;
  return 0;
}

int gs_ipc_event_open(int32_t device, const void* h64, void** ev) {
  hipIpcEventHandle_t h;
  memcpy(&h, h64, sizeof(h));
  GS_IPC(hipSetDevice(device));
  hipEvent_t e;
  GS_IPC(hipIpcOpenEventHandle(&e, h));
  *ev = e;
  return 0;
}

int gs_event_record_sync(void* ev) {
  GS_IPC(hipEventRecord(static_cast<hipEvent_t>(ev), nullptr));
  GS_IPC(hipEventSynchronize(static_cast<hipEvent_t>(ev)));
  return 0;
}

int gs_event_wait_sync(void* ev) {
  GS_IPC(hipStreamWaitEvent(nullptr, static_cast<hipEvent_t>(ev), 0));
  GS_IPC(hipStreamSynchronize(nullptr));
  return 0;
}

int gs_event_destroy(void* ev) {
  GS_IPC(hipEventDestroy(static_cast<hipEvent_t>(ev)));
  return 0;
}

}  // extern "C"
