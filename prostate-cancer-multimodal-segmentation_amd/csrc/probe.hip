// Shader-clock probe (bench.py's `sclk_mhz`): one tiny launch that stamps the shader cycle
// counter (s_memtime) and the 100 MHz real-time counter (s_memrealtime) on each XCD.  Two
// probes bracketing a stretch of work give the average clock the XCDs held over it:
// f = d(memtime) / d(memrealtime) x 100 MHz.  The shader cycle counters of different CUs
// carry different offsets (tests/tools/clock_check.py), so stamps are matched by the CU
// that wrote them (XCC id + the CU / SH / SE fields of HW_ID), never by block index.  Not part
// of any training path; nothing reads these records but the host.
#include "common.h"
#include "../../include/pcms_hip.h"

namespace {

__global__ void __launch_bounds__(64) clock_probe_kernel(unsigned long long* out) {
  if (threadIdx.x != 0) return;
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  const unsigned long long r = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  unsigned long long* o = out + 3 * blockIdx.x;
  o[0] = t;
  o[1] = r;
  o[2] = xcc | (((hw >> 8) & 0xffu) << 8);  // XCC id | (CU, SH, SE ids of HW_ID) << 8
}

// in-kernel reference for the probe (tests/tools/clock_check.py): every wave spins `cycles`
// shader cycles and its lane 0 records its own (memtime, memrealtime) at start and end
__global__ void __launch_bounds__(64) clock_spin_kernel(unsigned long long* out, long long cycles) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while ((long long)(t - t0) < cycles) {
    __builtin_amdgcn_s_sleep(8);
    t = __builtin_amdgcn_s_memtime();
  }
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if (threadIdx.x == 0) {
    unsigned long long* o = out + 5 * blockIdx.x;
    o[0] = t0;
    o[1] = r0;
    o[2] = t;
    o[3] = r1;
    o[4] = xcc | (((hw >> 8) & 0xffu) << 8);
  }
}

}  // namespace

extern "C" {

int pcms_clock_probe(void* out, int nblocks, hipStream_t s) {
  if (nblocks <= 0 || nblocks > 4096) return -1;
  hipLaunchKernelGGL(clock_probe_kernel, dim3(nblocks), dim3(64), 0, s, (unsigned long long*)out);
  PCMS_CHECK_LAUNCH();
}

int pcms_clock_spin(void* out, int nblocks, long cycles, hipStream_t s) {
  if (nblocks <= 0 || nblocks > 4096 || cycles < 0 || cycles > (1L << 34)) return -1;
  hipLaunchKernelGGL(clock_spin_kernel, dim3(nblocks), dim3(64), 0, s, (unsigned long long*)out,
                     (long long)cycles);
  PCMS_CHECK_LAUNCH();
}

}  // extern "C"
