// Cross-stream ordering for the step's three streams (main, weight-gradient side stream, skip
// branch; dorknet_amd/_hip.py).  torch's Stream.wait_stream / Event record with the runtime's
// default event, whose record carries a system-scope release: a marker on the main stream that cost
// ~7 us of idle time before the next kernel at each of the step's ~24 hand-overs
// (profiles/r06aa_step_timeline.txt).  These events are created without the system-scope fence
// (hipEventDisableSystemFence) and without timing: every consumer of the hand-over is a kernel on the
// same device, whose visibility the device-scope release at kernel completion already provides.
#include "dk_common.h"

using dk::DK_ERR_ARGS;

DK_API int dk_sync_event_create(void** event) {
  if (!event) return DK_ERR_ARGS;
  hipEvent_t e = nullptr;
  const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence);
  *event = r == hipSuccess ? reinterpret_cast<void*>(e) : nullptr;
  return r == hipSuccess ? 0 : (int)r;
}

DK_API int dk_sync_event_destroy(void* event) {
  return event ? (int)hipEventDestroy(reinterpret_cast<hipEvent_t>(event)) : 0;
}

// Work enqueued on `waiter` from now on starts after everything enqueued on `src` so far (`event`:
// one of dk_sync_event_create's, free to be recorded again once this call has returned).
DK_API int dk_stream_wait_stream(void* waiter, void* src, void* event) {
  if (!event) return DK_ERR_ARGS;
  hipEvent_t e = reinterpret_cast<hipEvent_t>(event);
  hipError_t r = hipEventRecord(e, reinterpret_cast<hipStream_t>(src));
  if (r != hipSuccess) return (int)r;
  r = hipStreamWaitEvent(reinterpret_cast<hipStream_t>(waiter), e, 0);
  return r == hipSuccess ? 0 : (int)r;
}

DK_API int dk_sync_event_record(void* event, void* stream) {
  if (!event) return DK_ERR_ARGS;
  const hipError_t r = hipEventRecord(reinterpret_cast<hipEvent_t>(event), reinterpret_cast<hipStream_t>(stream));
  return r == hipSuccess ? 0 : (int)r;
}

DK_API int dk_stream_wait_event(void* stream, void* event) {
  if (!event) return DK_ERR_ARGS;
  const hipError_t r = hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<hipEvent_t>(event), 0);
  return r == hipSuccess ? 0 : (int)r;
}
