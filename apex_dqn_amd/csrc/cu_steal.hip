// CU-stealing proxy for the data-parallel step (VERDICT r2 "next round" #2).
//
// With data parallelism RCCL's collective kernels run beside the learner's kernels and
// hold some CUs for their duration.  A persistent kernel that splits its images
// statically over 256 workgroups then waits for the workgroups that could not start:
// their whole share runs after the others finish.  This kernel stands in for RCCL on one
// GPU: K workgroups, each holding one CU (a dynamic LDS request no second 160-KB
// workgroup fits beside), spinning on the 100-MHz real-time counter for a fixed time.
// scripts/bench_cu_steal.py launches it on a second stream and times learner steps
// under it.  Every wave leaves the loop when the deadline passes (no flag from the host).
#include "apex_common.h"

__global__ void __launch_bounds__(64) spin_hold_kernel(uint64_t ticks, int* started) {
  extern __shared__ uint8_t hold[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    hold[0] = 1;                                   // the LDS request must stay live
    atomicAdd(started, 1);
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

// K workgroups holding `lds_bytes` of LDS each for `usec` microseconds on `st`
APEX_EXPORT int apex_spin_hold(int k, int usec, int lds_bytes, int* started, hipStream_t st) {
  if (k <= 0) return 0;
  if (usec <= 0 || lds_bytes < 0 || lds_bytes > 160 * 1024 || started == nullptr) return (int)hipErrorInvalidValue;
  if (lds_bytes > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(spin_hold_kernel),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (e != hipSuccess) return (int)e;
  }
  spin_hold_kernel<<<k, 64, lds_bytes, st>>>((uint64_t)usec * 100u, started);
  return (int)hipGetLastError();
}
