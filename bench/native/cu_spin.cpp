// CU-occupancy probe for bench/cu_steal.py: `blocks` one-wave workgroups that stay resident until
// the 100 MHz chip clock passes start + ticks (bounded: every wave exits by its own clock read),
// standing in for the workgroups a concurrent collective (RCCL channel blocks) keeps on the CUs.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC bench/native/cu_spin.cpp -o bench/native/bin/libcu_spin.so
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(64) void cu_spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

extern "C" int llmt_cu_spin(int blocks, unsigned long long ticks, void* stream) {
  if (blocks <= 0) return 0;
  if (ticks > 300000000ull) ticks = 300000000ull;  // at most 3 s
  hipLaunchKernelGGL(cu_spin_kernel, dim3(blocks), dim3(64), 0, (hipStream_t)stream, ticks);
  return (int)hipGetLastError();
}
