// hip_status.h — a launch's own status under HIP's per-thread last error (not part of the public ABI).
//
// HIP keeps the last error per host thread with CUDA's semantics: hipGetLastError() returns the last
// FAILURE of any earlier call on the thread (successful calls do not reset it), so the
// hipGetLastError() that reports a hipLaunchKernelGGL can also carry an older call's failure. Round 3
// cleared that slot unconditionally before every launch, which would also have swallowed such an
// older error. Now:
//   * every HIP call the library makes is checked where it is made; a failure it reports goes through
//     decds_hip_error and one it tolerates (teardown, a device allocation past the budget that makes
//     it spill) through hip_tolerate — both consume the thread's error slot, so no failure of the
//     library's own calls stays pending;
//   * hip_launch_begin, right before a launch, peeks at the slot: an error still pending there was
//     left by a HIP call outside the library on this thread (the caller's, torch's) — it is consumed
//     and returned, and decds_hip_error reports it as "left pending ... by an earlier HIP call on this
//     thread, outside the library (not this launch's)" instead of blaming the launch.
#pragma once
#include <hip/hip_runtime.h>

namespace decds {
void hip_tolerate(hipError_t e, const char *what);
hipError_t hip_launch_begin(const char *kernel);
}  // namespace decds
