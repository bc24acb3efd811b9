// False-dependency probe for HIP streams that share a hardware queue (GPU_MAX_HW_QUEUES).
//
// A pipeline stage posts RCCL receives ahead of its compute; RCCL's receive kernel spins until the
// peer's data lands.  If the stream of that receive shares a hardware queue with the compute
// stream, kernels enqueued later on the compute stream may wait behind the spinning receive.
// This probe measures exactly that on one GPU: `spin_wait` (stream X) spins on a flag with a
// wall-clock bound, `set_flag` (stream Y, launched after) sets it.  If Y runs behind X, the wait
// times out.  Every wave exits (bounded spin), so the grid always drains.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void spin_wait(const int* flag, int* out, uint64_t max_ticks) {
  const uint64_t t0 = wall_clock64();
  int seen = 0;
  while (true) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) { seen = 1; break; }
    if (wall_clock64() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x == 0) out[0] = seen ? 1 : 2;
}

__global__ void set_flag(int* flag) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" int probe_pair(const int* flag_w, int* flag_s, int* out, uint64_t max_ticks,
                          hipStream_t wait_stream, hipStream_t set_stream) {
  // flag_w == flag_s (same slot); two names keep const-correctness explicit
  hipLaunchKernelGGL(spin_wait, dim3(1), dim3(64), 0, wait_stream, flag_w, out, max_ticks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(set_flag, dim3(1), dim3(64), 0, set_stream, flag_s);
  return (int)hipGetLastError();
}
