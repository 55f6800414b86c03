// LDS-DMA staging probe (test tooling, not product): the level-0 weight gradient's staging
// stream alone -- per 4x8x8 box a dy tile (256 rows x 128 B, 64-channel rows) and an x halo
// (6x10x10 rows x 64 B, one 32-channel half of 64-channel rows) -- with no MFMAs, to find
// what sets its rate.  Workgroup lg stages boxes [64 (lg / 2), 64 (lg / 2) + 64) (ci half
// lg & 1), as the product's 256-workgroup plan does.  Variants (flags):
//   1  depth 2: the box after next is issued before waiting for the next (3 buffers)
//   2  register loads (global 16-B loads + ds_write_b128) instead of LDS-DMA
//   4  L2-resident source: every box re-reads box 0 of its workgroup's sample
//   8  x halo as whole 128-B rows (both ci halves; halo 77 KB)
//   16 dy tile only
//   32 x halo only
//   64 + a compute phase per box while the next box streams in: 16 steps x 8 MFMAs per wave
//      (the product's per-box MFMA count) on register operands
//   128 the same phase's LDS reads only (12 ds_read_b64_tr_b16 per step)
//   192 MFMAs fed by those reads (the product's compute_fixed shape)
//   256 no staging at all (the compute phase alone)
//   512 the next box's pieces issued one per compute step (interleaved with the MFMAs)
//   1024 MFMA operands all zero (lower power: tells clock effects from pipeline conflicts)
//   2048 wave specialisation: the two waves of SIMD 3 issue every piece and run no MFMAs
//   4096 16 waves (1024 threads) share the pieces and the MFMAs (half the MFMAs per wave)
//   8192 channel-blocked x: the halo read from a [N][C/32][D][H][W][32] layout (the same
//        bytes; a halo W-row of 10 voxels is one contiguous 640-B run = 5 whole lines,
//        instead of 10 half lines of 128-B voxel rows)
// Built by tests/kexp/Makefile (libdmaprobe.so), driven by tests/kexp/dma_probe.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "conv_common.h"

namespace {
constexpr int kT = 512;
constexpr int kNB = 64;                     // boxes per workgroup
constexpr int kDyP = 256 * 8;               // 16-B pieces of the dy tile
constexpr int kHalo = 6 * 10 * 10;
constexpr int kBuf = 256 * 128 + kHalo * 128;  // room for the 128-B-row halo variant
// (every in-flight box lands in the same LDS region: nothing reads it, only the traffic counts)

// per workgroup: shader-clock counter (s_memtime) and the 100 MHz real-time counter at the
// kernel's start and end, read by workgroup thread 0 -> the clock the CU ran at
__device__ unsigned long long g_clk[4096 * 4];

template <int F>
__global__ void __launch_bounds__((F & 4096) ? 1024 : 512, 1) probe_kernel(const uint16_t* x, const uint16_t* dy, int D, int H, int W,
                                                      uint32_t xbytes, uint32_t dybytes, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr bool kDepth2 = F & 1, kReg = F & 2, kL2 = F & 4, kWide = F & 8, kDyOnly = F & 16, kXOnly = F & 32;
  constexpr int kT = (F & 4096) ? 1024 : 512;
  constexpr bool kMfma = F & 64, kLdsRd = F & 128, kNoStage = F & 256, kInter = F & 512, kZero = F & 1024, kSpec = F & 2048;
  constexpr bool kBlocked = F & 8192;
  constexpr bool kHalfRd = F & 16384;  // LDS-fed: 3 fragments (6 tr reads) per 8 MFMAs instead of 6 (12)
  constexpr int XROWB = kWide ? 128 : 64;
  constexpr int XP = kHalo * XROWB / 16;
  constexpr int NP = (kXOnly ? 0 : kDyP) + (kDyOnly ? 0 : XP);
  constexpr int PER = (NP + kT - 1) / kT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int lg = blockIdx.x;
  unsigned long long clk0 = 0, rt0 = 0;
  if (tid == 0) {
    clk0 = __builtin_amdgcn_s_memtime();
    rt0 = __builtin_amdgcn_s_memrealtime();
  }
  const int half = lg & 1, split = lg >> 1;
  const int nbw = W / 8, nbh = H / 8, nbd = D / 4;
  const i32x4_t xr = buffer_desc(x, xbytes), dr = buffer_desc(dy, dybytes);
  const auto xr2 = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)xbytes, 0x00020000);
  const auto dr2 = __builtin_amdgcn_make_buffer_rsrc((void*)dy, (short)0, (int)dybytes, 0x00020000);
  const uint32_t l0 = lds_addr(lds);
  u32x4_t v[PER];
  u32x4_t accum = {0u, 0u, 0u, 0u};
  auto stage = [&](int b, int buf, int only = -1) {
    if (kNoStage) return;
    if (kL2) b = split * kNB;
    int q = b;
    const int bwi = q % nbw; q /= nbw;
    const int bhi = q % nbh; q /= nbh;
    const int bdi = q % nbd;
    const int n = q / nbd;
    const int d0 = bdi * 4, h0 = bhi * 8, w0 = bwi * 8;
    (void)buf;
    const uint32_t lb = l0;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (kSpec && (wv & 3) != 3) return;
    constexpr int NI = kSpec ? (NP + 127) / 128 : PER;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int pc0 = kSpec ? __builtin_amdgcn_readfirstlane((wv >> 2) * 64 + i * 128)
                            : __builtin_amdgcn_readfirstlane((tid & ~63) + i * kT);
      if (pc0 >= NP) break;
      if (only >= 0 && i != only) continue;
      const int pc = pc0 + lane;
      uint32_t voff = kOOB;
      const bool isdy = !kXOnly && pc0 < kDyP;
      if (isdy) {
        const int r = pc >> 3, qq = pc & 7;
        const int rd = r >> 6, rh = (r >> 3) & 7, rw = r & 7;
        voff = (uint32_t)(((((n * D + d0 + rd) * H + h0 + rh) * W + w0 + rw) * 64 + qq * 8) * 2);
      } else {
        const int hp = pc - (kXOnly ? 0 : kDyP);
        const int hv = hp / (XROWB / 16), qq = hp % (XROWB / 16);
        const int hw_ = hv % 10, t_ = hv / 10, hh_ = t_ % 10, hd_ = t_ / 10;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        if (hv < kHalo && gd >= 0 && gd < D && gh >= 0 && gh < H && gw >= 0 && gw < W) {
          if constexpr (kBlocked)
            voff = (uint32_t)((((((n * 2 + half) * D + gd) * H + gh) * W + gw) * 32 + qq * 8) * 2);
          else
            voff = (uint32_t)(((((n * D + gd) * H + gh) * W + gw) * 64 + (kWide ? 0 : half * 32) + qq * 8) * 2);
        }
      }
      if constexpr (kReg) {
        v[i] = (isdy ? __builtin_amdgcn_raw_buffer_load_b128(dr2, voff, 0, 0) : __builtin_amdgcn_raw_buffer_load_b128(xr2, voff, 0, 0));
      } else {
        if (isdy) dma16(dr, lb + pc0 * 16, voff, 0);
        else dma16(xr, lb + pc0 * 16, voff, 0);
      }
    }
  };
  auto commit = [&]() {
    if constexpr (kReg && !kNoStage) {
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int pc0 = (tid & ~63) + i * kT;
        if (pc0 < NP) *reinterpret_cast<u32x4_t*>(lds + pc0 * 16 + lane * 16) = v[i];
      }
    }
  };
  f32x16_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
  s16x8_t fr[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    fr[j] = kZero ? (s16x8_t){0, 0, 0, 0, 0, 0, 0, 0} : (s16x8_t){(short)lane, (short)j, 1, 2, 3, 4, 5, 6};
    asm volatile("" : "+v"(fr[j]));
  }
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const char* rb = lds + lane * 8 + wave * 1024;
  auto compute = [&](int nb) __attribute__((always_inline)) {
    if constexpr (!kMfma && !kLdsRd) return;
    if (kSpec && (wave & 3) == 3) return;
#pragma unroll
    for (int st = 0; st < (kT == 1024 ? 8 : 16); ++st) {
      if constexpr (kInter) if (st < PER && nb >= 0) stage(nb, 0, st);
      if constexpr (kInter) __builtin_amdgcn_sched_barrier(0);
      s16x8_t f[6];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        if constexpr (kLdsRd && kHalfRd) {
          if (j < 3) {
            const s16x4_t lo = tr_read(rb, st * 2048 + j * 128), hi = tr_read(rb, st * 2048 + j * 128 + 512);
            f[j] = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          } else {
            f[j] = f[j - 3];
          }
        } else if constexpr (kLdsRd) {
          const s16x4_t lo = tr_read(rb, st * 2048 + j * 128), hi = tr_read(rb, st * 2048 + j * 128 + 512);
          f[j] = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else {
          f[j] = fr[j];
        }
      }
      if constexpr (kMfma) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = mfma(f[j & 1], f[2 + (j & 3)], acc[j]);
        if (kInter) __builtin_amdgcn_sched_barrier(0);
        if (st == (kT == 1024 ? 7 : 15))
#pragma unroll
          for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(acc[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 6; ++j) accum[j & 3] ^= (uint32_t)(uint16_t)f[j][j];
      }
    }
  };
  const int b0 = split * kNB;
  stage(b0, 0);
  commit();
  if (kDepth2) stage(b0 + 1, 1);
  for (int k = 0; k < kNB; ++k) {
    if (kDepth2) {
      if (k + 2 < kNB) stage(b0 + k + 2, k + 2);
      if (k + 2 < kNB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      else if (k + 1 < kNB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (!kInter && k + 1 < kNB) stage(b0 + k + 1, k + 1);
      compute(k + 1 < kNB ? b0 + k + 1 : -1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (kReg) __builtin_amdgcn_s_barrier();  // every wave is done reading before the commit
      commit();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    accum += *reinterpret_cast<const u32x4_t*>(lds + tid * 16);
  }
  float t = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) t += acc[j][j];
  if (accum[0] == 0x12345678u || t == 1234.5f) sink[tid] = (float)accum[1] + t;
  if (tid == 0 && blockIdx.x < 4096) {
    const unsigned long long clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    g_clk[4 * blockIdx.x] = clk0;
    g_clk[4 * blockIdx.x + 1] = clk1;
    g_clk[4 * blockIdx.x + 2] = rt0;
    g_clk[4 * blockIdx.x + 3] = rt1;
  }
}
}  // namespace

extern "C" int probe_lds_bytes() { return kBuf; }
// the last launch's clock records of its first n workgroups (4 values each) into host memory
extern "C" int probe_clocks(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_clk), sizeof(unsigned long long) * 4 * n, 0, hipMemcpyDeviceToHost);
}

extern "C" int probe_run(int flags, const void* x, const void* dy, int N, int D, int H, int W, float* sink,
                         hipStream_t s) {
  const long nvox = (long)N * D * H * W;
  const uint32_t xb = (uint32_t)(nvox * 128), db = (uint32_t)(nvox * 128);
  const int nbox = N * (D / 4) * (H / 8) * (W / 8);
  const dim3 grid(2 * nbox / kNB);
  const int lds = kBuf;
#define PROBE(F)                                                                                               \
  case F:                                                                                                      \
    (void)hipFuncSetAttribute((const void*)probe_kernel<F>, hipFuncAttributeMaxDynamicSharedMemorySize, lds); \
    hipLaunchKernelGGL(probe_kernel<F>, grid, dim3((F & 4096) ? 1024 : 512), lds, s, (const uint16_t*)x, (const uint16_t*)dy, D, H, W, xb, db, sink); \
    break;
  switch (flags) {
    PROBE(0) PROBE(1) PROBE(2) PROBE(3) PROBE(4) PROBE(5) PROBE(8) PROBE(9) PROBE(16) PROBE(17) PROBE(32) PROBE(33)
    PROBE(20) PROBE(36) PROBE(64) PROBE(128) PROBE(192) PROBE(320) PROBE(384) PROBE(448) PROBE(576) PROBE(704) PROBE(66) PROBE(194) PROBE(1088) PROBE(1344) PROBE(1600) PROBE(2048) PROBE(2112) PROBE(2240) PROBE(2368) PROBE(2496) PROBE(4096) PROBE(4160) PROBE(4416) PROBE(4544) PROBE(4288)
    PROBE(8192) PROBE(8193) PROBE(8224) PROBE(8228) PROBE(8256) PROBE(8384) PROBE(16832) PROBE(16576)
    default: return -1;
  }
#undef PROBE
  return (int)hipGetLastError();
}
