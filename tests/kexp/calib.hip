// HBM calibration kernels (test tooling, not product): what this chip sustains for the
// access shapes the stem kernels use.  Built by tests/kexp/Makefile into libcalib.so and
// driven by tests/kexp/calib.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(4))) uint32_t u32x4_t;

// 16-B per lane streaming store, grid-stride (the "float4 write" shape)
__global__ void __launch_bounds__(256) write16_kernel(u32x4_t* y, long n16) {
  const u32x4_t v = {threadIdx.x, 1u, 2u, 3u};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) y[i] = v;
}

// the stem's store shape: one dword per lane; lanes 0-31 write 128 contiguous bytes of one
// voxel row, lanes 32-63 another 128 B one W-row (wstride bytes) away; persistent WGs of
// 8 waves, each wave writing 32 instructions per 512-voxel box.
__global__ void __launch_bounds__(512) write_stemshape_kernel(char* y, int nbox, uint32_t ybytes, int wstride) {
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(y, 0, ybytes, 0x00020000);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t voff = (lane & 31) * 4 + (lane >> 5) * wstride;
  for (int b = blockIdx.x; b < nbox; b += gridDim.x) {
    // 512 voxels x 128 B = 64 KiB per box: 8 waves x 32 instr x 256 B
    const uint32_t base = (uint32_t)b * 65536u + wave * 8192u;
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      const uint32_t so = __builtin_amdgcn_readfirstlane(base + (e >> 1) * 512 + (e & 1) * 128);
      __builtin_amdgcn_raw_buffer_store_b32(lane + e, yr, voff, so, 0);
    }
  }
}

// read-only: 16 B per lane, reduce to one word per thread
__global__ void __launch_bounds__(256) read16_kernel(const u32x4_t* x, long n16, uint32_t* out) {
  uint32_t s = 0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) {
    const u32x4_t v = x[i];
    s ^= v.x + v.y + v.z + v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

__global__ void __launch_bounds__(256) copy16_kernel(const u32x4_t* x, u32x4_t* y, long n16) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += (long)gridDim.x * 256) y[i] = x[i];
}

extern "C" {
int calib_write16(void* y, long bytes, int grid, hipStream_t s) {
  hipLaunchKernelGGL(write16_kernel, dim3(grid), dim3(256), 0, s, (u32x4_t*)y, bytes / 16);
  return (int)hipGetLastError();
}
int calib_write_stemshape(void* y, long bytes, int grid, int wstride, hipStream_t s) {
  hipLaunchKernelGGL(write_stemshape_kernel, dim3(grid), dim3(512), 0, s, (char*)y, (int)(bytes / 65536),
                     (uint32_t)bytes, wstride);
  return (int)hipGetLastError();
}
int calib_read16(const void* x, long bytes, int grid, void* out, hipStream_t s) {
  hipLaunchKernelGGL(read16_kernel, dim3(grid), dim3(256), 0, s, (const u32x4_t*)x, bytes / 16, (uint32_t*)out);
  return (int)hipGetLastError();
}
int calib_copy16(const void* x, void* y, long bytes, int grid, hipStream_t s) {
  hipLaunchKernelGGL(copy16_kernel, dim3(grid), dim3(256), 0, s, (const u32x4_t*)x, (u32x4_t*)y, bytes / 16);
  return (int)hipGetLastError();
}
}
