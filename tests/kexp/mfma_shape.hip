// MFMA shape probe (test tooling, not product): the big-box conv's inner-loop structure on
// every CU (8 waves, two per SIMD, 128 accumulator registers per wave, A fragments from LDS,
// B fragments from L1/L2-resident weights, random bf16 data) with the 32x32x16 MFMA (the
// product: 8 M-tiles x 1 N-tile per wave, 8 A reads + 1 B load per 8 MFMAs) against the
// 16x16x32 MFMA (8 M-tiles x 4 N-tiles, 8 A reads + 4 B loads per 32 MFMAs: the same FLOPs per
// step, half the A bytes per FLOP).  Time and clock per launch: tests/kexp/mfma_shape.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

__device__ __forceinline__ f32x16_t mfma32(s16x8_t a, s16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}
__device__ __forceinline__ f32x4_t mfma16(s16x8_t a, s16x8_t b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}

constexpr int kLds = 64 * 1024;

// SHAPE 32: per step 8 x (ds_read_b128, 32x32x16) with one B; SHAPE 16: per step 8 ds_read_b128,
// 4 B, 32 x 16x32x32.  steps: SHAPE 32 runs 2x the steps of SHAPE 16 (equal FLOPs).
template <int SHAPE>
__global__ void __launch_bounds__(512, 1) mfma_shape_kernel(const s16x8_t* src, const s16x8_t* wts, float* out,
                                                            int steps) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < kLds / 16; i += 512) reinterpret_cast<s16x8_t*>(lds)[i] = src[(blockIdx.x * 97 + i) & 16383];
  __syncthreads();
  const char* abase = lds + lane * 16 + wave * 1024;
  // weights: 27 taps x 8 fragments of 1 KiB, the wave's N-tile(s) (L1 / L2 resident)
  const s16x8_t* wb = wts + (wave >> 2) * 64 + lane;
  if constexpr (SHAPE == 32) {
    f32x16_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    s16x8_t b = wb[0];
    for (int s = 0; s < steps; ++s) {
      const int t = s % 27;
      const s16x8_t bn = wb[(t + 1) * 512];
      const char* ab = abase + (s & 7) * 1024;
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const s16x8_t a = *reinterpret_cast<const s16x8_t*>(ab + mt * 4096);
        acc[mt] = mfma32(a, b, acc[mt]);
      }
      b = bn;
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) sum += acc[i][e];
    out[blockIdx.x * 512 + tid] = sum;
  } else {
    f32x4_t acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    s16x8_t b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = wb[j * 128];
    for (int s = 0; s < steps; ++s) {
      const int t = s % 27;
      s16x8_t bn[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bn[j] = wb[(t + 1) * 512 + j * 128];
      const char* ab = abase + (s & 7) * 1024;
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const s16x8_t a = *reinterpret_cast<const s16x8_t*>(ab + mt * 4096);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[mt][j] = mfma16(a, b[j], acc[mt][j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = bn[j];
    }
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) sum += acc[i][j][e];
    out[blockIdx.x * 512 + tid] = sum;
  }
}

extern "C" int mfma_shape(int shape, const void* src, const void* wts, void* out, int steps, int grid, hipStream_t s) {
  auto k = shape == 32 ? mfma_shape_kernel<32> : mfma_shape_kernel<16>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, kLds);
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), kLds, s, (const s16x8_t*)src, (const s16x8_t*)wts, (float*)out, steps);
  return (int)hipGetLastError();
}
