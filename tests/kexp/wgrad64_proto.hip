// Register-feasibility prototype (test tooling, not product): a 64 co x 64 ci weight-gradient
// workgroup tile on four 512-VGPR waves (one per SIMD), wave w = (co half w >> 1, ci half
// w & 1) owning all 27 taps = 27 accumulators of 32x32 (432 registers).  Per 16-voxel k-step:
// one A fragment (dy, the wave's co half) read once and fed to 27 MFMAs, one B fragment
// (x halo row of the tap) per MFMA, read one tap ahead.  Compiled only (hipcc -S) to see
// whether the allocation fits without scratch; DESIGN.md §7 has the plan it belongs to.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "conv_common.h"

namespace {
__global__ void __launch_bounds__(256, 1) wgrad64_proto_kernel(const char* __restrict__ src, float* out, int nstep) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = wave >> 1, cit = wave & 1;
  f32x16_t acc[27];
#pragma unroll
  for (int t = 0; t < 27; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  // the box's tiles are already in LDS (the prototype measures registers, not staging)
  for (int i = tid; i < 16384; i += 256) reinterpret_cast<uint32_t*>(lds)[i] = reinterpret_cast<const uint32_t*>(src)[i];
  __syncthreads();
  const char* ab = lds + ct * 64 + (lane & 15) * 8 + (lane >> 4) * 512;
  const char* bb = lds + 32768 + cit * 64 + (lane & 15) * 8 + (lane >> 4) * 1024;
  auto cat = [](s16x4_t lo, s16x4_t hi) __attribute__((always_inline)) {
    return (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  for (int s = 0; s < nstep; ++s) {
    const s16x8_t a = cat(tr_read(ab, s * 2048), tr_read(ab, s * 2048 + 256));
    s16x8_t b[2];
    b[0] = cat(tr_read(bb, s * 128), tr_read(bb, s * 128 + 4096));
    static_for<27>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t + 1 < 27) {
        constexpr int kd = (t + 1) / 9, kh = ((t + 1) / 3) % 3, kw = (t + 1) % 3;
        constexpr int off = ((kd * 10 + kh) * 10 + kw) * 128;
        b[(t + 1) & 1] = cat(tr_read(bb, s * 128 + off), tr_read(bb, s * 128 + off + 4096));
      }
      acc[t] = mfma(a, b[t & 1], acc[t]);
    });
  }
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 27; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) sum += acc[t][e];
  out[blockIdx.x * 256 + tid] = sum;
}
}  // namespace

extern "C" int wgrad64_proto(const void* src, float* out, int nstep, hipStream_t s) {
  hipLaunchKernelGGL(wgrad64_proto_kernel, dim3(256), dim3(256), 65536 + 32768, s, (const char*)src, out, nstep);
  return (int)hipGetLastError();
}
