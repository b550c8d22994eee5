// Probe: can a hipGraph carry an *external* event record node that another stream waits on
// while the rest of the graph is still running? (HIP: hipEventRecordWithFlags(...,
// hipEventRecordExternal) during stream capture.) If yes, the segmented multi-rank plan
// (stepper_plan.hip) could keep its event records inside graph segments instead of cutting a
// segment at every record.
//
// Per iteration: graph on s1 = [A: counter += 1, stamp] -> record E (external) -> [B: spin
// ~spin_us, stamp]; then, issued after the graph launch, s2 waits E and runs C (reads the
// counter, stamps). Checks: C saw this iteration's increment (the wait did not refer to an older
// record), and C started before B ended (the wait released at the record, not at the graph's
// end). Output: one JSON line per iteration and a verdict line.
//
// Result on MI355X / ROCm 7: "correct and early" here, with the host running ahead too (async
// pass). Inside the stepper's plan, however (records after memset / kernel nodes, several
// events per segment), HIP logged "hipEventRecord add external event node failed" and the next
// launch returned hipErrorInvalidValue, so the plan still cuts a segment at every record
// (docs/DESIGN.md §11). In the stepper the first external record of a plan (ev_stage[0], right
// after the node-reduce kernel node, one dependency) returns hipErrorInvalidValue. The last
// block checks the obvious suspects (the same event recorded twice in one capture or in a
// second live graph, after a memset node, after an eager record on the same stream, while that
// record is still pending and waited on, a 2-D grid kernel node, a priority stream, a timing
// event): all succeed here, so the stepper's failing pattern is none of them.
// Build: hipcc -O2 --offload-arch=gfx950 graph_event_probe.hip.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

__global__ void kern_a(unsigned* counter, unsigned long long* stamp) {
  if (threadIdx.x == 0) {
    counter[0] += 1u;
    stamp[0] = __builtin_amdgcn_s_memrealtime();
    __threadfence_system();
  }
}

// Spins for `ticks` of the 100 MHz realtime clock (one workgroup: the GPU stays free for C).
__global__ void kern_b(unsigned long long ticks, unsigned long long* stamp) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    stamp[1] = __builtin_amdgcn_s_memrealtime();
  }
}

__global__ void kern_c(const unsigned* counter, unsigned* seen, unsigned long long* stamp, int it) {
  if (threadIdx.x == 0) {
    stamp[2 + it] = __builtin_amdgcn_s_memrealtime();
    seen[it] = counter[0];
  }
}

// Also built as a shared library (-DGS_PROBE_LIB -shared): scripts/graph_event_probe_torch.py
// loads it into a process that imported torch first, so the probe runs on the HIP runtime the
// stepper itself runs on there (torch bundles its own libamdhip64.so.7, and the stepper's
// DT_NEEDED soname resolves to that already-loaded copy), not on /opt/rocm's.
extern "C" int gs_graph_event_probe(int iters, int spin_us) {
  const unsigned long long spin_ticks = 100ull * (unsigned long long)spin_us;
  {
    int rt = 0, drv = 0;
    (void)hipRuntimeGetVersion(&rt);
    (void)hipDriverGetVersion(&drv);
    printf("{\"hip_runtime_version\": %d, \"hip_driver_version\": %d}\n", rt, drv);
    fflush(stdout);
  }
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e;
  CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  unsigned *counter, *seen;
  unsigned long long *stamp_a, *stamp_c;
  CHECK(hipMalloc(&counter, sizeof(unsigned)));
  CHECK(hipMalloc(&seen, 64 * sizeof(unsigned)));
  CHECK(hipMalloc(&stamp_a, 2 * 64 * sizeof(unsigned long long)));
  CHECK(hipMalloc(&stamp_c, 80 * sizeof(unsigned long long)));
  CHECK(hipMemset(counter, 0, sizeof(unsigned)));
  CHECK(hipMemset(seen, 0, 64 * sizeof(unsigned)));
  CHECK(hipDeviceSynchronize());

  hipGraph_t g;
  hipGraphExec_t x;
  CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
  hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
  CHECK(hipEventRecordWithFlags(e, s1, hipEventRecordExternal));
  {
    // does the capture-time record leave a sticky error behind for hipGetLastError?
    const hipError_t le = hipGetLastError();
    printf("{\"last_error_after_external_record\": \"%s\"}\n", hipGetErrorName(le));
  }
  hipLaunchKernelGGL(kern_b, dim3(1), dim3(64), 0, s1, spin_ticks, stamp_a);
  CHECK(hipStreamEndCapture(s1, &g));
  CHECK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));

  // async pass first: every launch, wait and C issued back to back, one sync at the end (the
  // way the plan runs ahead of the GPU): each C must still see its own iteration's increment
  const int n_async = iters < 32 ? iters : 32;
  for (int it = 0; it < n_async; ++it) {
    CHECK(hipGraphLaunch(x, s1));
    CHECK(hipStreamWaitEvent(s2, e, 0));
    hipLaunchKernelGGL(kern_c, dim3(1), dim3(64), 0, s2, counter, seen, stamp_c, it);
  }
  CHECK(hipDeviceSynchronize());
  int bad_async = 0;
  {
    unsigned v[32];
    CHECK(hipMemcpy(v, seen, n_async * sizeof(unsigned), hipMemcpyDeviceToHost));
    for (int it = 0; it < n_async; ++it) bad_async += v[it] != (unsigned)(it + 1);
    printf("{\"async_iters\": %d, \"async_wrong\": %d, \"first\": %u, \"last\": %u}\n",
           n_async, bad_async, v[0], v[n_async - 1]);
  }
  CHECK(hipMemset(counter, 0, sizeof(unsigned)));
  CHECK(hipMemset(seen, 0, 64 * sizeof(unsigned)));
  CHECK(hipDeviceSynchronize());

  int bad_value = bad_async, waited_for_end = 0;
  for (int it = 0; it < iters && it < 64; ++it) {
    CHECK(hipGraphLaunch(x, s1));
    CHECK(hipStreamWaitEvent(s2, e, 0));
    hipLaunchKernelGGL(kern_c, dim3(1), dim3(64), 0, s2, counter, seen, stamp_c, it);
    CHECK(hipStreamSynchronize(s2));
    CHECK(hipStreamSynchronize(s1));
    unsigned v = 0;
    unsigned long long sa[2], sc = 0;
    CHECK(hipMemcpy(&v, seen + it, sizeof(v), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(sa, stamp_a, sizeof(sa), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&sc, stamp_c + 2 + it, sizeof(sc), hipMemcpyDeviceToHost));
    const bool ok_value = v == (unsigned)(it + 1);
    const bool before_end = sc < sa[1];
    bad_value += !ok_value;
    waited_for_end += !before_end;
    printf("{\"iter\": %d, \"seen\": %u, \"expect\": %d, \"c_after_a_us\": %.1f, "
           "\"b_end_after_c_us\": %.1f}\n",
           it, v, it + 1, (double)((long long)(sc - sa[0])) / 100.0,
           (double)((long long)(sa[1] - sc)) / 100.0);
  }
  printf("{\"verdict\": \"%s\", \"stale_waits\": %d, \"waits_released_at_graph_end\": %d}\n",
         bad_value ? "stale" : waited_for_end ? "correct but serial" : "correct and early",
         bad_value, waited_for_end);
  // Two external records of the SAME event: a second node in one capture, and a second graph.
  {
    hipGraph_t g2;
    (void)hipGetLastError();
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
    hipError_t r1 = hipEventRecordWithFlags(e, s1, hipEventRecordExternal);
    hipError_t l1 = hipGetLastError();
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
    hipError_t r2 = hipEventRecordWithFlags(e, s1, hipEventRecordExternal);
    hipError_t l2 = hipGetLastError();
    CHECK(hipStreamEndCapture(s1, &g2));
    printf("{\"same_event_twice_in_one_capture\": [\"%s\", \"%s\", \"%s\", \"%s\"]}\n",
           hipGetErrorName(r1), hipGetErrorName(l1), hipGetErrorName(r2), hipGetErrorName(l2));
    (void)hipGraphDestroy(g2);
    // the first graph g (with its record of e) is still alive: record e in a new capture
    hipGraph_t g3;
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
    hipError_t r3 = hipEventRecordWithFlags(e, s1, hipEventRecordExternal);
    hipError_t l3 = hipGetLastError();
    CHECK(hipStreamEndCapture(s1, &g3));
    printf("{\"same_event_in_a_second_graph\": [\"%s\", \"%s\"]}\n", hipGetErrorName(r3),
           hipGetErrorName(l3));
    (void)hipGraphDestroy(g3);
    // a record right after a memset node, and with the event also recorded eagerly before
    hipEvent_t e2;
    CHECK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CHECK(hipEventRecord(e2, s2));
    hipGraph_t g4;
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    CHECK(hipMemsetAsync(counter, 0, 4, s1));
    hipError_t r4 = hipEventRecordWithFlags(e2, s1, hipEventRecordExternal);
    hipError_t l4 = hipGetLastError();
    CHECK(hipStreamEndCapture(s1, &g4));
    printf("{\"after_memset_node_eagerly_recorded_event\": [\"%s\", \"%s\"]}\n",
           hipGetErrorName(r4), hipGetErrorName(l4));
    (void)hipGraphDestroy(g4);
    // an event recorded eagerly on the capturing stream itself and waited on by s2 first
    hipEvent_t e3;
    CHECK(hipEventCreateWithFlags(&e3, hipEventDisableTiming));
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
    CHECK(hipEventRecord(e3, s1));
    CHECK(hipStreamWaitEvent(s2, e3, 0));
    CHECK(hipDeviceSynchronize());
    hipGraph_t g5;
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
    hipError_t r5 = hipEventRecordWithFlags(e3, s1, hipEventRecordExternal);
    hipError_t l5 = hipGetLastError();
    CHECK(hipStreamEndCapture(s1, &g5));
    printf("{\"after_eager_record_on_same_stream\": [\"%s\", \"%s\"]}\n", hipGetErrorName(r5),
           hipGetErrorName(l5));
    (void)hipGraphDestroy(g5);
    // a 2-D grid kernel node before the record
    hipGraph_t g6;
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kern_a, dim3(4, 3), dim3(256), 0, s1, counter, stamp_a);
    hipError_t r6 = hipEventRecordWithFlags(e2, s1, hipEventRecordExternal);
    hipError_t l6 = hipGetLastError();
    CHECK(hipStreamEndCapture(s1, &g6));
    printf("{\"after_2d_grid_kernel\": [\"%s\", \"%s\"]}\n", hipGetErrorName(r6),
           hipGetErrorName(l6));
    (void)hipGraphDestroy(g6);
    // non-blocking stream created with a priority (as the stepper's compute stream)
    hipStream_t sp;
    int lo = 0, hi = 0;
    CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CHECK(hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, hi));
    hipGraph_t g7;
    CHECK(hipStreamBeginCapture(sp, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, sp, counter, stamp_a);
    hipError_t r7 = hipEventRecordWithFlags(e2, sp, hipEventRecordExternal);
    hipError_t l7 = hipGetLastError();
    CHECK(hipStreamEndCapture(sp, &g7));
    printf("{\"priority_stream\": [\"%s\", \"%s\"]}\n", hipGetErrorName(r7), hipGetErrorName(l7));
    (void)hipGraphDestroy(g7);
    // the event's eager record is still pending (behind a 20 ms spin on s1) and s2 waits on it
    hipEvent_t e4;
    CHECK(hipEventCreateWithFlags(&e4, hipEventDisableTiming));
    hipLaunchKernelGGL(kern_b, dim3(1), dim3(64), 0, s1, 2000000ull, stamp_a);
    CHECK(hipEventRecord(e4, s1));
    CHECK(hipStreamWaitEvent(s2, e4, 0));
    hipGraph_t g8;
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
    hipError_t r8 = hipEventRecordWithFlags(e4, s1, hipEventRecordExternal);
    hipError_t l8 = hipGetLastError();
    CHECK(hipStreamEndCapture(s1, &g8));
    printf("{\"while_eager_record_pending\": [\"%s\", \"%s\"]}\n", hipGetErrorName(r8),
           hipGetErrorName(l8));
    (void)hipGraphDestroy(g8);
    CHECK(hipDeviceSynchronize());
    // event created with default flags (timing enabled)
    hipEvent_t e5;
    CHECK(hipEventCreate(&e5));
    hipGraph_t g9;
    CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(kern_a, dim3(1), dim3(64), 0, s1, counter, stamp_a);
    hipError_t r9 = hipEventRecordWithFlags(e5, s1, hipEventRecordExternal);
    hipError_t l9 = hipGetLastError();
    CHECK(hipStreamEndCapture(s1, &g9));
    printf("{\"timing_event\": [\"%s\", \"%s\"]}\n", hipGetErrorName(r9), hipGetErrorName(l9));
    (void)hipGraphDestroy(g9);
  }
  CHECK(hipGraphExecDestroy(x));
  CHECK(hipGraphDestroy(g));
  fflush(stdout);
  return bad_value ? 2 : 0;
}

#ifndef GS_PROBE_LIB
int main(int argc, char** argv) {
  return gs_graph_event_probe(argc > 1 ? atoi(argv[1]) : 6, argc > 2 ? atoi(argv[2]) : 20000);
}
#endif
