// CU hog (test tooling, not product): K workgroups that each hold a CU's worth of LDS and
// spin for a fixed wall time, launched on a side stream beside a training step -- what the
// RCCL all-reduce kernels of a data-parallel step do to the persistent one-workgroup-per-CU
// kernels (stem, big-box conv, ConvTranspose stream) while a gradient bucket is in flight.
// Built by tests/kexp/Makefile (libcuhog.so), driven by tests/kexp/cu_hog.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
__global__ void __launch_bounds__(64) hog_kernel(unsigned long long ticks, int* sink) {
  // 24 KiB of LDS: with it no 150+ KiB persistent workgroup fits beside this one
  __shared__ int pad[6144];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  int v = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    v += pad[(threadIdx.x + v) & 63];
  }
  if (v == 0x7fffffff) sink[threadIdx.x] = v;  // keeps the loop (never true: pad is never written)
}
}  // namespace

// K workgroups spinning for us microseconds on stream s
extern "C" int cu_hog(int k, double us, int* sink, hipStream_t s) {
  if (k <= 0) return 0;
  hipLaunchKernelGGL(hog_kernel, dim3(k), dim3(64), 0, s, (unsigned long long)(us * 100.0), sink);
  return (int)hipGetLastError();
}
