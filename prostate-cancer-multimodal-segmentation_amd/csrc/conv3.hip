// 3x3x3 / stride 1 / pad 1 convolution for the U-Net DoubleConv blocks, NDHWC, gfx950.
//
// Replaces nn.Conv3d(k=3, padding=1) of models/unet3d.py:29,35 (forward, and the two
// autograd backward products of aten::convolution_backward).
//
//   conv3_fwd   implicit GEMM  Y[v, co] = sum_{tap, ci} X[v + tap, ci] * W[co, ci, tap]
//               M = voxels (a spatial box of <= 512 voxels per workgroup), N = 64 output
//               channels per workgroup, K = 27 * Cin walked as (ci-chunk, tap).  The
//               chunk's (box + halo) input tile is staged once in LDS and re-read for all
//               27 taps through an LDS row offset; weights stream from L2 into registers.
//               Epilogue: + bias, store, per-workgroup BatchNorm partial sums (sum, sumsq).
//               Also serves dgrad (dX = conv(dY, W flipped + transposed)), with
//               `accumulate` and a two-pointer output for the concat split of Up3D.
//   conv3_wgrad dW[tap, co, ci] += sum_v dY[v, co] * X[v + tap, ci]   (K = voxels)
//               Both MFMA operands need the voxel index contiguous: they are read from
//               natural NDHWC LDS tiles with ds_read_b64_tr_b16 (hardware transpose).
//
// bf16 path: v_mfma_f32_32x32x16_bf16; fp32 path (parity build): v_mfma_f32_32x32x2_f32.
#include "common.h"
#include "pcms_hip.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

// PCMS_ABL: ablation switches for the stem kernels, set only by the test-tooling build
// (tests/kexp/Makefile) to time their parts separately; 0 in the product build.
#ifndef PCMS_ABL
#define PCMS_ABL 0
#endif

namespace {

constexpr int kThreads = 256;
constexpr int kRowBytes = 64;      // one halo row = one LDS row of the current ci-chunk
constexpr int kHaloMax = 1152;     // halo voxels per workgroup (72 KiB LDS, 2 WG / CU)

__device__ __attribute__((aligned(16))) uint32_t g_zero16[4];  // zero page for LDS-DMA padding
constexpr uint32_t kOOB = 0x80000000u;  // buffer voffset past num_records: reads zeros

template <typename T> struct Traits;
template <> struct Traits<bf16_t> {
  static constexpr int CK = 32;    // channels per chunk (64 B rows)
  static constexpr int KS = 2;     // MFMA k-steps per chunk and tap (K = 16 each)
  static constexpr int VEC = 8;    // elements per 16-byte piece
  typedef s16x8_t Frag;
};
template <> struct Traits<float> {
  static constexpr int CK = 16;
  static constexpr int KS = 8;     // K = 2 each
  static constexpr int VEC = 4;
  typedef float Frag;
};

__device__ __forceinline__ f32x16_t mfma(s16x8_t a, s16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x16_t mfma(float a, float b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// 16-byte slot swizzle inside a 64-byte halo row (spreads ds_read_b128 lane groups).
__device__ __forceinline__ int swz(int row) { return (row >> 2) & 3; }

// MFMA row -> box voxel permutation inside a 32-row M-tile.  ds_read_b128 serves a wave in
// the lane groups G0 = {0-3, 12-15, 20-27} and G1 = {4-11, 16-19, 28-31} (and +32).  With
// 16-voxel w-runs (box width 16) G0 reads 16 consecutive halo rows of one h-row and G1 16 of
// the next, so with swz() every group covers all 64 banks exactly once, for every tap.
__device__ __forceinline__ int perm32(int r) {
  if (r < 4) return r;
  if (r < 12) return 16 + (r - 4);
  if (r < 16) return 4 + (r - 12);
  if (r < 20) return 24 + (r - 16);
  if (r < 28) return 8 + (r - 20);
  return 28 + (r - 28);
}

// A fragment from the halo tile. ks = k-step inside the chunk, h = lane >> 5.
__device__ __forceinline__ s16x8_t lds_a(const char* lds, int row, int ks, int h, bf16_t*) {
  int slot = (ks * 2 + h) ^ swz(row);
  return *reinterpret_cast<const s16x8_t*>(lds + row * kRowBytes + slot * 16);
}
__device__ __forceinline__ float lds_a(const char* lds, int row, int ks, int h, float*) {
  int c = ks * 2 + h;  // channel in chunk (0..15)
  int slot = (c >> 2) ^ swz(row);
  return *reinterpret_cast<const float*>(lds + row * kRowBytes + slot * 16 + (c & 3) * 4);
}
// B fragment (weights) straight from global: packed [chunk][27][Cout][CK].
__device__ __forceinline__ s16x8_t gl_b(const bf16_t* wrow, int ks, int h) {
  return *reinterpret_cast<const s16x8_t*>(wrow + ks * 16 + h * 8);
}
__device__ __forceinline__ float gl_b(const float* wrow, int ks, int h) { return wrow[ks * 2 + h]; }

struct Conv3Params {
  const void* x0; const void* x1; int c0; int c1;
  const void* w; const float* bias;
  void* y0; void* y1; int cy0;
  float* yacc; float* stats;
  int accumulate;
  int N, D, H, W, Cin, Cout;
  int nchunk, chunks_per_split;
  int lbd, lbh, lbw, nbd, nbh, nbw;
};

// LBD/LBH/LBW >= 0: compile-time box geometry (the hot (4, 8, 16) box: halo decode and tap
// offsets become constant arithmetic); -1: runtime geometry from p.
template <typename T, int MINW, int LBD, int LBH, int LBW>
__global__ void __launch_bounds__(kThreads, MINW) conv3_fwd_kernel(Conv3Params p) {
  const int lbd_ = LBW >= 0 ? LBD : p.lbd, lbh_ = LBW >= 0 ? LBH : p.lbh, lbw_ = LBW >= 0 ? LBW : p.lbw;
  typedef Traits<T> Tr;
  typedef typename Tr::Frag Frag;
  __shared__ __attribute__((aligned(16))) char lds[kHaloMax * kRowBytes];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r_lane = lane & 31, hsel = lane >> 5;
  int mb = blockIdx.x;
  const int bwi = mb % p.nbw; mb /= p.nbw;
  const int bhi = mb % p.nbh; mb /= p.nbh;
  const int bdi = mb % p.nbd;
  const int n = mb / p.nbd;
  const int co_base = blockIdx.y * 64;
  const int cbeg = blockIdx.z * p.chunks_per_split;
  const int cend = min(p.nchunk, cbeg + p.chunks_per_split);
  const int bd = 1 << lbd_, bh = 1 << lbh_, bw = 1 << lbw_;
  const int boxvol = bd * bh * bw;
  const int d0 = bdi * bd, h0 = bhi * bh, w0 = bwi * bw;
  const int HH = bh + 2, HW = bw + 2;
  const int HV = (bd + 2) * HH * HW;

  const bool w16 = lbw_ == 4;
  const int prow = w16 ? perm32(r_lane) : r_lane;
  int hb[4];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    int r = wave * 128 + mt * 32 + prow;
    if (r >= boxvol) r = 0;
    int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
    hb[mt] = (rd * HH + rh) * HW + rw;
  }
  const bool wave_active = wave * 128 < boxvol;

  // fp32 build: three-level summation (one MFMA chain per tap = 16 products, per-chunk sum,
  // master) keeps the error at the level of a blocked CPU conv; bf16 build: one chain.
  constexpr bool kF32 = sizeof(T) == 4;
  f32x16_t acc[4][2], cacc[4][2], macc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) { acc[i][j][e] = 0.f; cacc[i][j][e] = 0.f; macc[i][j][e] = 0.f; }

  const T* x0 = (const T*)p.x0;
  const T* x1 = (const T*)p.x1;
  const T* wp = (const T*)p.w;
  const long plane = (long)p.H * p.W;

  for (int chunk = cbeg; chunk < cend; ++chunk) {
    __syncthreads();
    // ---- stage the halo tile of this chunk by LDS-DMA: piece p (16 B) -> LDS [16p, 16p+16).
    // The LDS image is lane-linear, so the slot swizzle is applied to the SOURCE address
    // (physical slot qp of row hv holds logical slot qp ^ swz(hv)); out-of-range pieces
    // read the zero page.  All pieces are in flight at once (no register staging).
    for (int base = wave * 64; base < HV * 4; base += kThreads) {
      const int pc = base + lane;
      const int hv = pc >> 2;
      const int ql = (pc & 3) ^ swz(hv);
      const void* src = g_zero16;
      if (pc < HV * 4) {
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        const int c = chunk * Tr::CK + ql * Tr::VEC;
        if (gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && c < p.Cin) {
          const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
          src = (c < p.c0) ? (const void*)(x0 + vox * p.c0 + c) : (const void*)(x1 + vox * p.c1 + (c - p.c0));
        }
      }
      __builtin_amdgcn_global_load_lds(src, (LDS_AS void*)(lds + base * 16), 16, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (!wave_active) continue;

    const T* wchunk = wp + (long)chunk * 27 * p.Cout * Tr::CK;
    // B fragments rotate through 3 register sets: the loads of tap t+2 are issued while
    // tap t computes (kw unrolled, so every set index is a compile-time constant).
    Frag bset[3][2][Tr::KS];
    auto load_b = [&](Frag (&dst)[2][Tr::KS], int tap) {
      const T* wt = wchunk + ((long)tap * p.Cout + co_base + r_lane) * Tr::CK;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int ks = 0; ks < Tr::KS; ++ks) dst[nt][ks] = gl_b(wt + nt * 32 * Tr::CK, ks, hsel);
    };
    load_b(bset[0], 0);
    load_b(bset[1], 1);
    for (int kdh = 0; kdh < 9; ++kdh) {
      const int kd = kdh / 3, kh = kdh % 3;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kdh * 3 + kw;
        if (tap + 2 < 27) load_b(bset[(kw + 2) % 3], tap + 2);
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this tap's MFMAs
        const int off = (kd * HH + kh) * HW + kw;
        if constexpr (kF32) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        }
#pragma unroll
        for (int ks = 0; ks < Tr::KS; ++ks) {
#pragma unroll
          for (int mt = 0; mt < 4; ++mt) {
            Frag a = lds_a(lds, hb[mt] + off, ks, hsel, (T*)nullptr);
#pragma unroll
            for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(a, bset[kw][nt][ks], acc[mt][nt]);
          }
        }
        if constexpr (kF32) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) cacc[i][j] += acc[i][j];
        }
      }
    }
    if constexpr (kF32) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          macc[i][j] += cacc[i][j];
#pragma unroll
          for (int e = 0; e < 16; ++e) cacc[i][j][e] = 0.f;
        }
    }
  }
  if constexpr (kF32) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = macc[i][j];
  }

  // ---- epilogue ----
  // BatchNorm partials per workgroup row: (sum, M2 = sum of squared deviations from the
  // row's own mean) + the row's voxel count.  Each wave first forms its own per-channel
  // mean (two passes over the accumulator registers), waves are merged with Chan's formula:
  // no E[x^2] - E[x]^2 cancellation (BN over few voxels / large |mean| / std).
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  float bias_l[2] = {0.f, 0.f};
  if (p.bias) {
    bias_l[0] = p.bias[co_base + r_lane];
    bias_l[1] = p.bias[co_base + 32 + r_lane];
  }
  const bool want_stats = p.stats && !p.yacc;
  const bool interior = d0 + bd <= p.D && h0 + bh <= p.H && w0 + bw <= p.W;
  uint64_t vmask = 0;  // bit mt * 16 + e: row valid
  if (wave_active) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * hsel;
        const int r = wave * 128 + mt * 32 + (w16 ? perm32(rr) : rr);
        bool valid = r < boxvol;
        if (valid && !interior) {
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          valid = d0 + rd < p.D && h0 + rh < p.H && w0 + rw < p.W;
        }
        if (valid) vmask |= 1ull << (mt * 16 + e);
      }
  }
  constexpr int kRedOff = 512 * 64 * 2;  // bf16 C tile [512][64] occupies the first 64 KiB
  if (!kF32 && !p.yacc && !p.accumulate) {
    // bf16 fast path: + bias, stats from the fp32 values, C tile -> LDS (box order), then
    // 16-byte coalesced stores (one box row = a contiguous w-run of voxels).
    __syncthreads();  // every wave is done reading the halo
    bf16_t* ct = reinterpret_cast<bf16_t*>(lds);
    if (wave_active) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rr = (e & 3) + 8 * (e >> 2) + 4 * hsel;
          const int r = wave * 128 + mt * 32 + (w16 ? perm32(rr) : rr);
          const bool valid = (vmask >> (mt * 16 + e)) & 1;
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const float v = acc[mt][nt][e] + bias_l[nt];
            ct[r * 64 + nt * 32 + r_lane] = f2bf(v);
            if (valid) s1[nt] += v;
          }
        }
      }
    }
    __syncthreads();
    for (int pc = tid; pc < boxvol * 8; pc += kThreads) {
      const int r = pc >> 3, q = pc & 7;
      const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
      const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
      if (!interior && (gd >= p.D || gh >= p.H || gw >= p.W)) continue;
      const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
      const int co = co_base + q * 8;
      T* dst = (co < p.cy0) ? (T*)p.y0 + vox * p.cy0 + co : (T*)p.y1 + vox * (p.Cout - p.cy0) + (co - p.cy0);
      *reinterpret_cast<u32x4_t*>(dst) = *reinterpret_cast<const u32x4_t*>(ct + r * 64 + q * 8);
    }
  } else if (wave_active) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        if (!((vmask >> (mt * 16 + e)) & 1)) continue;
        const int rr = (e & 3) + 8 * (e >> 2) + 4 * hsel;
        const int r = wave * 128 + mt * 32 + (w16 ? perm32(rr) : rr);
        const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
        const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
        const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int co = co_base + nt * 32 + r_lane;
          float v = acc[mt][nt][e];
          if (p.yacc) {
            atomicAdd(p.yacc + vox * p.Cout + co, v);
            continue;
          }
          v += bias_l[nt];
          T* dst = (co < p.cy0) ? (T*)p.y0 + vox * p.cy0 + co
                                : (T*)p.y1 + vox * (p.Cout - p.cy0) + (co - p.cy0);
          if (p.accumulate) v += Elem<T>::ld(dst);  // (stats are refused with accumulate)
          Elem<T>::st(dst, v);
          s1[nt] += v;
        }
      }
    }
  }
  if (want_stats) {
    // wave-level mean per channel (rows of a channel live in lanes r_lane and r_lane + 32)
    const float nw = (float)(__popcll(vmask) + __shfl_xor(__popcll(vmask), 32, 64));
    float mw[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      s1[nt] += __shfl_xor(s1[nt], 32, 64);
      mw[nt] = nw > 0.f ? s1[nt] / nw : 0.f;
    }
    // squared deviations about the rounded wave mean, corrected by (sum d)^2 / n
    float sd[2] = {0.f, 0.f};
    if (wave_active) {
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          if (!((vmask >> (mt * 16 + e)) & 1)) continue;
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) {
            const float d = acc[mt][nt][e] + bias_l[nt] - mw[nt];
            s2[nt] += d * d;
            sd[nt] += d;
          }
        }
    }
    __syncthreads();  // halo / C tile no longer read: reuse LDS for the cross-wave reduction
    float* red = reinterpret_cast<float*>(lds + (kF32 ? 0 : kRedOff));
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      s2[nt] += __shfl_xor(s2[nt], 32, 64);
      sd[nt] += __shfl_xor(sd[nt], 32, 64);
      if (nw > 0.f) s2[nt] -= sd[nt] * sd[nt] / nw;
      if (hsel == 0) {
        float* rp = red + (wave * 64 + nt * 32 + r_lane) * 3;
        rp[0] = s1[nt];
        rp[1] = s2[nt];
        rp[2] = nw;
      }
    }
    __syncthreads();
    if (tid < 64) {
      float S = 0.f, Nn = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        S += red[(w * 64 + tid) * 3 + 0];
        Nn += red[(w * 64 + tid) * 3 + 2];
      }
      const float m = Nn > 0.f ? S / Nn : 0.f;
      float M2 = 0.f, sdd = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const float c = red[(w * 64 + tid) * 3 + 2];
        if (c > 0.f) {
          const float d = red[(w * 64 + tid) * 3 + 0] / c - m;
          M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
          sdd += c * d;
        }
      }
      if (Nn > 0.f) M2 -= sdd * sdd / Nn;
      float* st = p.stats + ((long)blockIdx.x * p.Cout + co_base + tid) * 2;
      st[0] = S;
      st[1] = M2;
      if (tid == 0 && blockIdx.y == 0) p.stats[(long)gridDim.x * p.Cout * 2 + blockIdx.x] = Nn;
    }
  }
}

// ------------------------------------------------------------------------------------
// weight-gradient kernel
// ------------------------------------------------------------------------------------
constexpr int kWThreads = 512;          // 8 waves: wave = (co-tile, tap-group)
constexpr int kWHaloMax = 720;          // halo rows (box <= 256 voxels)

template <typename T> struct WTraits;
template <> struct WTraits<bf16_t> {
  static constexpr int BV = 256;        // voxels per staged box
  static constexpr int KV = 16;         // voxels per MFMA
  static constexpr int NBUF = 2;
  static constexpr int DYROW = 128;     // 64 co x 2 B
  static constexpr int XROW = 64;       // 32 ci x 2 B
  static constexpr int VEC = 8;
  typedef s16x8_t Frag;
};
template <> struct WTraits<float> {
  static constexpr int BV = 128;
  static constexpr int KV = 2;
  static constexpr int NBUF = 1;
  static constexpr int DYROW = 256;     // 64 co x 4 B
  static constexpr int XROW = 128;      // 32 ci x 4 B
  static constexpr int VEC = 4;
  typedef float Frag;
};

struct WgradParams {
  const void* x0; const void* x1; int c0; int c1;
  const void* dy;
  float* dwt;            // fp32 workspace: one [27][Cout][Cin] partial row per split
  int N, D, H, W, Cin, Cout;
  int lbd, lbh, lbw, nbd, nbh, nbw;
  int nbox, boxes_per_split;
  int nco, nci;          // 64-channel output blocks, 32-channel input blocks
  int dma;               // bf16: stage by buffer LDS-DMA (byte sizes below < 2^31)
  uint32_t x0bytes, x1bytes, dybytes;
  float* dw;             // direct (one split, bf16): dw [Cout][cw][27] += through an LDS transpose
  int cw, direct;
};

// dy tile: 128-B (bf16) rows, 64-B halves swizzled by row bit 1 (conflict-free tr reads).
__device__ __forceinline__ int dy_off_bf16(int v, int co) {  // co in 0..63 (element)
  int half = (co >> 5) ^ ((v >> 1) & 1);
  return v * 128 + half * 64 + (co & 31) * 2;
}

__device__ __forceinline__ s16x4_t tr_read(const char* lds, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4_t*)(lds + byte_off));
}

template <typename T, int LBD, int LBH, int LBW>
__global__ void __launch_bounds__(kWThreads, 1) conv3_wgrad_kernel(WgradParams p) {
  const int lbd_ = LBW >= 0 ? LBD : p.lbd, lbh_ = LBW >= 0 ? LBH : p.lbh, lbw_ = LBW >= 0 ? LBW : p.lbw;
  typedef WTraits<T> Tr;
  typedef typename Tr::Frag Frag;
  constexpr int DYBYTES = Tr::BV * Tr::DYROW;
  constexpr int XBYTES = kWHaloMax * Tr::XROW;
  constexpr int BUFBYTES = DYBYTES + XBYTES;
  extern __shared__ __attribute__((aligned(16))) char wlds[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hsel = lane >> 5;
  const int cot = wave & 1;           // co tile (32 rows of the 64-wide dy tile)
  const int tg = wave >> 1;           // taps tg, tg+4, ...
  const int ntap = (tg == 3) ? 6 : 7;
  // bf16 layout: wave w owns taps w, w + 8, w + 16 (, w + 24) for BOTH co tiles, so each B
  // (x) fragment feeds 2 MFMAs: 1.5 LDS reads per MFMA instead of 2.3 (8 accumulators)
  constexpr bool kW2 = sizeof(T) == 2 && !(PCMS_ABL & 16384);
  const int ntap2 = wave < 3 ? 4 : 3;
  // 1-D grid, logical id XCD-aware (dispatch is round-robin over 8 XCDs: consecutive logical
  // ids land on one XCD at about the same time), tile (co block, ci block) fastest: the
  // workgroups of one split that share its dy boxes (and its halos) share an L2
  const int G = gridDim.x, ntile = p.nco * p.nci;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int tile = lg % ntile, split = lg / ntile;
  const int co_base = (tile % p.nco) * 64;
  const int ci_base = (tile / p.nco) * 32;
  const int bd = 1 << lbd_, bh = 1 << lbh_, bw = 1 << lbw_;
  const int HH = bh + 2, HW = bw + 2;
  const int HV = (bd + 2) * HH * HW;
  const int boxvol = bd * bh * bw;
  const long plane = (long)p.H * p.W;
  const T* x0 = (const T*)p.x0;
  const T* x1 = (const T*)p.x1;
  const T* dy = (const T*)p.dy;

  const int b_beg = split * p.boxes_per_split;
  const int b_end = min(p.nbox, b_beg + p.boxes_per_split);

  f32x16_t acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;

  // register staging: pieces of 16 B
  constexpr int DYP = Tr::BV * Tr::DYROW / 16;
  const int XP = HV * Tr::XROW / 16;
  constexpr int MAXP = Tr::NBUF == 2 ? (DYP + kWHaloMax * Tr::XROW / 16 + kWThreads - 1) / kWThreads : 1;
  u32x4_t stg[MAXP];

  auto box_origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int bwi = b % p.nbw; b /= p.nbw;
    int bhi = b % p.nbh; b /= p.nbh;
    int bdi = b % p.nbd;
    n = b / p.nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  auto stage_load = [&](int b) {
    int n, d0, h0, w0;
    box_origin(b, n, d0, h0, w0);
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      // one unconditional 16-B load per piece (invalid pieces read the zero page): a
      // conditional load merged with a zero default makes the compiler drain vmcnt before
      // the merge, serialising the prefetch with the compute it should overlap
      const int pc = tid + i * kWThreads;
      const void* src = g_zero16;
      if (pc < DYP) {
        const int r = pc / (Tr::DYROW / 16), q = pc % (Tr::DYROW / 16);
        if (r < boxvol) {
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
          if (gd < p.D && gh < p.H && gw < p.W) {
            const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
            src = dy + vox * p.Cout + co_base + q * Tr::VEC;
          }
        }
      } else if (pc < DYP + XP) {
        const int hp = pc - DYP;
        const int hv = hp / (Tr::XROW / 16), q = hp % (Tr::XROW / 16);
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        const int c = ci_base + q * Tr::VEC;
        if (gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && c < p.Cin) {
          const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
          src = (c < p.c0) ? (const void*)(x0 + vox * p.c0 + c) : (const void*)(x1 + vox * p.c1 + (c - p.c0));
        }
      }
      stg[i] = *reinterpret_cast<const u32x4_t*>(src);
    }
  };
  auto stage_store = [&](char* buf) {
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int pc = tid + i * kWThreads;
      if (pc < DYP) {
        const int r = pc / (Tr::DYROW / 16), q = pc % (Tr::DYROW / 16);
        int off;
        if (sizeof(T) == 2) off = dy_off_bf16(r, q * 8);
        else off = r * Tr::DYROW + q * 16;
        *reinterpret_cast<u32x4_t*>(buf + off) = stg[i];
      } else if (pc < DYP + XP) {
        const int hp = pc - DYP;
        *reinterpret_cast<u32x4_t*>(buf + DYBYTES + hp * 16) = stg[i];
      }
    }
  };

  // fp32 build: stage without a register array (one 16-B piece in flight per thread)
  auto stage_direct = [&](char* buf, int b) {
    int n, d0, h0, w0;
    box_origin(b, n, d0, h0, w0);
    for (int pc = tid; pc < DYP + XP; pc += kWThreads) {
      u32x4_t v = {0u, 0u, 0u, 0u};
      int off;
      if (pc < DYP) {
        const int r = pc / (Tr::DYROW / 16), q = pc % (Tr::DYROW / 16);
        off = r * Tr::DYROW + q * 16;
        if (r < boxvol) {
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
          if (gd < p.D && gh < p.H && gw < p.W) {
            const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
            v = *reinterpret_cast<const u32x4_t*>(dy + vox * p.Cout + co_base + q * Tr::VEC);
          }
        }
      } else {
        const int hp = pc - DYP;
        off = DYBYTES + hp * 16;
        const int hv = hp / (Tr::XROW / 16), q = hp % (Tr::XROW / 16);
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        const int c = ci_base + q * Tr::VEC;
        if (gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && c < p.Cin) {
          const long vox = ((long)n * p.D + gd) * plane + (long)gh * p.W + gw;
          const T* src = (c < p.c0) ? x0 + vox * p.c0 + c : x1 + vox * p.c1 + (c - p.c0);
          v = *reinterpret_cast<const u32x4_t*>(src);
        }
      }
      *reinterpret_cast<u32x4_t*>(buf + off) = v;
    }
  };

  // per-lane voxel-row helpers for the k index (voxel inside the box)
  auto halo_row = [&](int r) {
    const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
    return (rd * HH + rh) * HW + rw;
  };

  auto compute = [&](const char* buf) {
    const char* xb = buf + DYBYTES;
#pragma unroll 2
    for (int k0 = 0; k0 < boxvol; k0 += Tr::KV) {
      Frag a;
      Frag bf[7];
      if constexpr (kW2) {
        const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
        const int v_a = k0 + 8 * hsel + qq;
        s16x8_t a2[2];
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const int co = ct * 32 + g * 16 + pp * 4;
          s16x4_t lo = tr_read(buf, dy_off_bf16(v_a, co));
          s16x4_t hi = tr_read(buf, dy_off_bf16(v_a + 4, co));
          a2[ct] = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
        const int hr0 = LBW >= 4 ? halo_row(k0) + 8 * hsel + qq : halo_row(v_a);
        const int hr1 = LBW >= 4 ? hr0 + 4 : halo_row(v_a + 4);
        const int ci = g * 16 + pp * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j < ntap2) {
            const int tap = wave + 8 * j;
            const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
            const int off = (kd * HH + kh) * HW + kw;
            s16x4_t l2 = tr_read(xb, (hr0 + off) * Tr::XROW + ci * 2);
            s16x4_t h2 = tr_read(xb, (hr1 + off) * Tr::XROW + ci * 2);
            const s16x8_t b = (s16x8_t){l2[0], l2[1], l2[2], l2[3], h2[0], h2[1], h2[2], h2[3]};
            acc[j] = mfma(a2[0], b, acc[j]);
            acc[4 + j] = mfma(a2[1], b, acc[4 + j]);
          }
        }
        continue;
      } else if constexpr (sizeof(T) == 2) {
        // lane 4q+p of each 16-lane group: row q, cols 4p..4p+3 of a 4x16 block
        const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
        const int v_a = k0 + 8 * hsel + qq;          // rows for elements 0..3; +4 for 4..7
        const int co = cot * 32 + g * 16 + pp * 4;
        s16x4_t lo = tr_read(buf, dy_off_bf16(v_a, co));
        s16x4_t hi = tr_read(buf, dy_off_bf16(v_a + 4, co));
        a = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        // with a compile-time box of width >= 16 the lane's rows share (rd, rh) with k0
        const int hr0 = LBW >= 4 ? halo_row(k0) + 8 * hsel + qq : halo_row(v_a);
        const int hr1 = LBW >= 4 ? hr0 + 4 : halo_row(v_a + 4);
        const int ci = g * 16 + pp * 4;
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          if (j < ntap) {
            const int tap = tg + 4 * j;
            const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
            const int off = (kd * HH + kh) * HW + kw;
            s16x4_t l2 = tr_read(xb, (hr0 + off) * Tr::XROW + ci * 2);
            s16x4_t h2 = tr_read(xb, (hr1 + off) * Tr::XROW + ci * 2);
            bf[j] = (s16x8_t){l2[0], l2[1], l2[2], l2[3], h2[0], h2[1], h2[2], h2[3]};
          }
        }
      } else {
        const int v = k0 + hsel;
        a = *reinterpret_cast<const float*>(buf + v * Tr::DYROW + (cot * 32 + (lane & 31)) * 4);
        const int hr = halo_row(v);
#pragma unroll
        for (int j = 0; j < 7; ++j) {
          if (j < ntap) {
            const int tap = tg + 4 * j;
            const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
            const int off = (kd * HH + kh) * HW + kw;
            bf[j] = *reinterpret_cast<const float*>(xb + (hr + off) * Tr::XROW + (lane & 31) * 4);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 7; ++j)
        if (j < ntap) acc[j] = mfma(a, bf[j], acc[j]);
    }
  };

  // bf16 hot path: both tiles arrive by buffer LDS-DMA (no register staging); the next box
  // streams in while this one computes.  The dy tile keeps dy_off_bf16's half swap (applied
  // to the source address); each wave instruction is all-dy or all-halo (2048 dy pieces);
  // out-of-range pieces read zeros.
  auto stage_dma = [&](char* buf, int b) {
    int n, d0, h0, w0;
    box_origin(b, n, d0, h0, w0);
    const uint32_t lb0 = lds_addr(buf);
    const bool first = ci_base < p.c0;  // a 32-channel block lies in one source
    const i32x4_t xr = buffer_desc(first ? p.x0 : p.x1, first ? p.x0bytes : p.x1bytes);
    const i32x4_t dr = buffer_desc(p.dy, p.dybytes);
    const int xs = first ? p.c0 : p.c1, xc = first ? ci_base : ci_base - p.c0;
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int pc0 = (tid & ~63) + i * kWThreads;  // wave-uniform first piece
      if (pc0 >= DYP + XP) break;
      const int pc = pc0 + lane;
      uint32_t voff = kOOB;
      if (pc0 < DYP) {
        const int r = pc >> 3, q = pc & 7;
        const int ql = q ^ (((r >> 1) & 1) << 2);
        if (r < boxvol) {
          const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
          const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
          if (gd < p.D && gh < p.H && gw < p.W)
            voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * p.Cout + co_base + ql * 8) * 2);
        }
        dma16(dr, __builtin_amdgcn_readfirstlane(lb0 + pc0 * 16), voff, 0);
      } else {
        const int hp = pc - DYP;
        const int hv = hp >> 2, q = hp & 3;
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        if (hp < XP && gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W && xc + q * 8 < xs)
          voff = (uint32_t)(((((n * p.D + gd) * p.H + gh) * p.W + gw) * xs + xc + q * 8) * 2);
        dma16(xr, __builtin_amdgcn_readfirstlane(lb0 + DYBYTES + (pc0 - DYP) * 16), voff, 0);
      }
    }
  };

  if (b_beg < b_end && p.dma) {
    if constexpr (Tr::NBUF == 2) {
      stage_dma(wlds, b_beg);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int b = b_beg; b < b_end; ++b) {
        const int cur = (b - b_beg) & 1;
        if (b + 1 < b_end) stage_dma(wlds + (cur ^ 1) * BUFBYTES, b + 1);
        compute(wlds + cur * BUFBYTES);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
    }
  } else if (b_beg < b_end) {
    if constexpr (Tr::NBUF == 2) {
      stage_load(b_beg);
      stage_store(wlds);
      __syncthreads();
      for (int b = b_beg; b < b_end; ++b) {
        const int cur = (b - b_beg) & 1;
        if (b + 1 < b_end && !(PCMS_ABL & 4096)) stage_load(b + 1);
        if (!(PCMS_ABL & 8192)) compute(wlds + cur * BUFBYTES);
        if (b + 1 < b_end && !(PCMS_ABL & 4096)) stage_store(wlds + (cur ^ 1) * BUFBYTES);
        __syncthreads();
      }
    } else {
      // fp32 build: per-box MFMA chains summed into a master accumulator (two-level sum)
      f32x16_t macc[7];
#pragma unroll
      for (int t = 0; t < 7; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) macc[t][e] = 0.f;
      for (int b = b_beg; b < b_end; ++b) {
        __syncthreads();
        stage_direct(wlds, b);
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 7; ++t)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
        compute(wlds);
#pragma unroll
        for (int t = 0; t < 7; ++t) macc[t] += acc[t];
      }
#pragma unroll
      for (int t = 0; t < 7; ++t) acc[t] = macc[t];
    }
  }

  // flush: C[row = co][col = ci] of tap -> this split's partial row dwt[split][tap][co][ci]
  // with plain stores (two 128-B row segments per instruction); the splits are summed in a
  // fixed order by wgrad_group_sum_kernel / wgrad_reduce_kernel.  (fp32 atomics from every
  // split into one [27][Cout][Cin] image serialised on the contended addresses: 2-4x the
  // kernel's own time at level 0.)
  float* prow = p.dwt + (long)split * 27 * p.Cout * p.Cin;
  if constexpr (kW2) {
    if (p.direct) {
      // one split: no partial rows to reduce.  Per 32-row co half, the workgroup's
      // [32 co][32 ci][27 taps] tile is transposed through LDS (the staging buffers are free)
      // and added to the contiguous [ci][27] runs of the torch-layout dw.
      float* tile = reinterpret_cast<float*>(wlds);
      const int nci = min(32, p.cw - ci_base);
      for (int ct = 0; ct < 2; ++ct) {
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j >= ntap2) continue;
          const int tap = wave + 8 * j;
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int col = (e & 3) + 8 * (e >> 2) + 4 * hsel;
            tile[(col * 32 + (lane & 31)) * 27 + tap] = acc[ct * 4 + j][e];
          }
        }
        __syncthreads();
        for (int i = tid; i < 32 * 32 * 27; i += kWThreads) {
          const int col = i / 864, r = i % 864;  // r = ci * 27 + tap
          const int co = co_base + ct * 32 + col;
          if (co < p.Cout && r < nci * 27) p.dw[((long)co * p.cw + ci_base) * 27 + r] += tile[i];
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= ntap2) continue;
      const int tap = wave + 8 * j;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int co = co_base + ct * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
          const int ci = ci_base + (lane & 31);
          if (co < p.Cout && ci < p.Cin) prow[((long)tap * p.Cout + co) * p.Cin + ci] = acc[ct * 4 + j][e];
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    if (j >= ntap) continue;
    const int tap = tg + 4 * j;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int co = co_base + cot * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
      const int ci = ci_base + (lane & 31);
      if (co < p.Cout && ci < p.Cin) prow[((long)tap * p.Cout + co) * p.Cin + ci] = acc[j][e];
    }
  }
}

// Weight-gradient split reduction (deterministic, fixed order).  part: S rows of
// E = 27 * Cout * Cin floats ([split][tap][co][ci], Cin = stored channels).
// Stage 1 (S > 16): rows r*16 .. r*16+15 summed in place into row r*16.
__global__ void __launch_bounds__(256) wgrad_group_sum_kernel(float* part, int S, long E) {
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= E) return;
  const int r0 = blockIdx.y * 16, r1 = min(S, r0 + 16);
  float* src = part + (long)r0 * E + e;
  float sum = 0.f;
  for (int r = r0; r < r1; ++r, src += E) sum += *src;
  part[(long)r0 * E + e] = sum;
}
// Stage 2: dw [Cout][Cw][27] (torch OIDHW, the weight's own input-channel count Cw <= Cin;
// stem: 5 of 8) += sum of R rows spaced `stride` rows apart.  Block = (co, 32 channels): the
// [27][32] tiles are read as 128-B rows, transposed through LDS, added to the contiguous
// 32 x 27 run of dw.
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* part, int R, int stride, float* dw,
                                                           int Cout, int Cin, int Cw) {
  __shared__ float tile[27][33];
  const int co = blockIdx.x, ci0 = blockIdx.y * 32;
  const long rstep = (long)stride * 27 * Cout * Cin;
  for (int e = threadIdx.x; e < 27 * 32; e += 256) {
    const int t = e >> 5, c = e & 31, ci = ci0 + c;
    float sum = 0.f;
    if (ci < Cw) {
      const float* src = part + ((long)t * Cout + co) * Cin + ci;
      for (int r = 0; r < R; ++r, src += rstep) sum += *src;
    }
    tile[t][c] = sum;
  }
  __syncthreads();
  float* dst = dw + ((long)co * Cw + ci0) * 27;
  const int n = min(32, Cw - ci0) * 27;
  for (int e = threadIdx.x; e < n; e += 256) dst[e] += tile[e % 27][e / 27];
}

// master fp32 W[Cout][Cin][27] -> packed T [chunk][27][J][CK]
//   fwd  (flip=0): J = Cout, k-index = ci
//   dgrad(flip=1): J = Cin,  k-index = co, tap mirrored (26 - t)
// One block per (chunk, 8 consecutive j): the 8 x CK x 27 source block is read with unit
// stride into LDS and written back with unit stride in the packed order.
template <typename T, int CK>
__global__ void __launch_bounds__(256) pack_conv3_kernel(const float* w, T* out, int Cout, int Cin, int flip) {
  __shared__ float tile[8][CK][27];
  const int J = flip ? Cin : Cout;
  const int Kdim = flip ? Cout : Cin;
  const int chunk = blockIdx.y;
  const int j0 = blockIdx.x * 8;
  constexpr int E = 8 * CK * 27;
  for (int e = threadIdx.x; e < E; e += 256) {
    int jj, k, t;
    if (!flip) { t = e % 27; k = (e / 27) % CK; jj = e / (27 * CK); }      // w[j][chunk*CK + k][t]
    else { t = e % 27; jj = (e / 27) % 8; k = e / (27 * 8); }             // w[chunk*CK + k][j][t]
    const int kk = chunk * CK + k, j = j0 + jj;
    float v = 0.f;
    if (kk < Kdim && j < J) v = flip ? w[((long)kk * Cin + j) * 27 + t] : w[((long)j * Cin + kk) * 27 + t];
    tile[jj][k][t] = v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < E; e += 256) {
    const int k = e % CK, jj = (e / CK) % 8, t = e / (CK * 8);
    if (j0 + jj >= J) continue;
    const float v = flip ? tile[jj][k][26 - t] : tile[jj][k][t];
    out[(((long)chunk * 27 + t) * J + j0 + jj) * CK + k] = Elem<T>::cvt(v);
  }
}

// bf16 fast path (Kdim % 32 == 0, J % 8 == 0: every layer but the stem): the same block, read
// as 16-B vectors (the block's source is 8 contiguous 864-float runs (fwd) or 32 contiguous
// 216-float runs (dgrad)) and written as 16-B vectors of 8 packed k.
__global__ void __launch_bounds__(256) pack_conv3_bf16_kernel(const float* w, bf16_t* out, int Cout, int Cin,
                                                              int flip) {
  __shared__ float tile[8][32][27];
  const int J = flip ? Cin : Cout;
  const int chunk = blockIdx.y;
  const int j0 = blockIdx.x * 8;
  for (int e = threadIdx.x; e < 1728; e += 256) {
    int base, run, q;
    if (!flip) {  // w[j0 + jj][chunk*32 .. +32][27]: run jj of 864 floats
      run = e / 216; q = e % 216;
      base = ((j0 + run) * Cin + chunk * 32) * 27;
    } else {      // w[chunk*32 + k][j0 .. j0+8][27]: run k of 216 floats
      run = e / 54; q = e % 54;
      base = ((chunk * 32 + run) * Cin + j0) * 27;
    }
    const f32x4_t v = *reinterpret_cast<const f32x4_t*>(w + base + 4 * q);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = 4 * q + i;
      if (!flip) tile[run][idx / 27][idx % 27] = v[i];
      else tile[idx / 27][run][idx % 27] = v[i];
    }
  }
  __syncthreads();
  for (int g = threadIdx.x; g < 864; g += 256) {
    const int t = g >> 5, jj = (g >> 2) & 7, k8 = (g & 3) * 8;
    const int ts = flip ? 26 - t : t;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = pack_bf16x2(tile[jj][k8 + 2 * i][ts], tile[jj][k8 + 2 * i + 1][ts]);
    *reinterpret_cast<u32x4_t*>(out + (((long)chunk * 27 + t) * J + j0 + jj) * 32 + k8) = o;
  }
}

struct Box { int lbd, lbh, lbw; };

int ilog2(int v) { int l = 0; while ((1 << l) < v) ++l; return l; }

// Pick a power-of-two box (<= maxvol voxels, halo <= maxhalo rows) minimising padded
// volume (then maximising box size) for a D x H x W grid.
Box choose_box(int D, int H, int W, int maxvol, int maxhalo, int minw, int minvol) {
  Box best{3, 3, 3};  // (8,8,8): always valid (vol 512, halo 1000) -- overwritten below
  double best_cost = 1e30;
  for (int a = 0; a <= 4; ++a)
    for (int b = 0; b <= 5; ++b)
      for (int c = 0; c <= 6; ++c) {
        const int bd = 1 << a, bh = 1 << b, bw = 1 << c;
        if (bd * bh * bw > maxvol || bd * bh * bw < minvol) continue;
        if ((bd + 2) * (bh + 2) * (bw + 2) > maxhalo) continue;
        if (bw < minw && bw < W) continue;
        const double padded = (double)cdiv(D, bd) * bd * cdiv(H, bh) * bh * cdiv(W, bw) * bw;
        const double halo = (double)cdiv(D, bd) * cdiv(H, bh) * cdiv(W, bw) * (bd + 2) * (bh + 2) * (bw + 2);
        const double cost = padded + 0.15 * halo;
        if (cost < best_cost - 1e-9) { best_cost = cost; best = Box{a, b, c}; }
      }
  return best;
}

// Forward/dgrad box: 512 voxels; width 16 whenever the grid is that wide (perm32 layout).
Box fwd_box(int D, int H, int W) {
  if (W >= 16) {
    Box best{0, 0, 4};
    double bc = 1e30;
    for (int a = 0; a <= 5; ++a) {
      const int b = 5 - a;  // bd * bh = 32
      const int bd = 1 << a, bh = 1 << b;
      if ((bd + 2) * (bh + 2) * 18 > kHaloMax) continue;
      const double cost = (double)cdiv(D, bd) * bd * cdiv(H, bh) * bh +
                          0.15 * cdiv(D, bd) * cdiv(H, bh) * (bd + 2) * (bh + 2) * 18 / 16.0;
      if (cost < bc - 1e-9 || (cost < bc + 1e-9 && a == 2)) { bc = cost; best = Box{a, b, 4}; }
    }
    return best;
  }
  return choose_box(D, H, W, 512, kHaloMax, 4, 32);
}

// ------------------------------------------------------------------------------------
// Stem conv (inc.conv.0: n_modalities -> 64, input stored with 8 channels), bf16.
// The generic kernel would spend 4x its MFMA work on zero channels (K = 27 x 32); here the
// K dimension packs two taps per MFMA k-step: k = (tap 2s + h, channel c), h = lane >> 5,
// so K = 14 x 16 = 224 (135 real).  HBM-bound: 16 B in + 128 B out per voxel.
// ------------------------------------------------------------------------------------
constexpr int kStemSteps = 14;                    // 28 taps (27 + 1 zero) / 2
constexpr int kStemWBytes = kStemSteps * 64 * 16 * 2;  // packed weights [14][64][16] bf16

// master W[64][cin_w][27] fp32 -> [14][64][16] bf16, k = h * 8 + c <-> (tap 2s + h, c);
// the 64 output columns are ordered (nt, j) -> channel 2 j + nt so that a lane's two MFMA
// tiles hold an adjacent channel pair (one packed bf16x2 LDS write per row)
__global__ void stem_pack_kernel(const float* w, bf16_t* out, int cin_w) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kStemSteps * 64 * 16) return;
  const int k = i & 15, col = (i >> 4) & 63, s = i >> 10;
  const int co = 2 * (col & 31) + (col >> 5);  // MFMA column (nt, j) <-> channel 2 j + nt
  const int tap = 2 * s + (k >> 3), c = k & 7;
  float v = 0.f;
  if (tap < 27 && c < cin_w) v = w[((long)co * cin_w + c) * 27 + tap];
  out[i] = f2bf(v);
}

__device__ __forceinline__ int tap_off(int tap, int HH, int HW) {
  if (tap >= 27) return 0;  // zero-weight pad tap: any in-halo row
  const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
  return (kd * HH + kh) * HW + kw;
}

// Both bf16 packs of one conv from ONE read of the fp32 weight (Cin % 32 == Cout % 32 == 0).
// Block (co j0 .. j0+32, ci c*32 .. +32): the 32 contiguous 864-float runs w[co][c*32..][27]
// are converted to bf16 once into LDS (same rounding as pack_bf16x2), then both packs are
// written as whole 64-B rows:
//   fwd   [ci/32][t][co][ci%32] = w[co][ci][t]
//   dgrad [co/32][t][ci][co%32] = w[co][ci][26 - t]
__global__ void __launch_bounds__(256) pack_conv3_bf16_both_kernel(const float* w, bf16_t* fwd, bf16_t* dgr,
                                                                   int Cout, int Cin) {
  __shared__ __attribute__((aligned(16))) uint16_t tb[32 * 864];
  const int chunk = blockIdx.y;
  const int j0 = blockIdx.x * 32;
  // all 27 loads of a thread in flight at once (the tile is 32 x 216 = 27 x 256 f32x4)
  f32x4_t v[27];
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const int e = threadIdx.x + i * 256, run = e / 216, q = e % 216;
    v[i] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(w + ((long)(j0 + run) * Cin + chunk * 32) * 27) + q);
  }
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const int e = threadIdx.x + i * 256, run = e / 216, q = e % 216;
    uint2 o;
    o.x = pack_bf16x2(v[i][0], v[i][1]);
    o.y = pack_bf16x2(v[i][2], v[i][3]);
    *reinterpret_cast<uint2*>(tb + run * 864 + 4 * q) = o;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < 27 * 128; g += 256) {
    const int t = g >> 7, co = (g >> 2) & 31, k8 = (g & 3) * 8;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (uint32_t)tb[co * 864 + (k8 + 2 * i) * 27 + t] | ((uint32_t)tb[co * 864 + (k8 + 2 * i + 1) * 27 + t] << 16);
    *reinterpret_cast<u32x4_t*>(fwd + (((long)chunk * 27 + t) * Cout + j0 + co) * 32 + k8) = o;
  }
  for (int g = threadIdx.x; g < 27 * 128; g += 256) {
    const int t = g >> 7, ci = (g >> 2) & 31, k8 = (g & 3) * 8, ts = 26 - t;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (uint32_t)tb[(k8 + 2 * i) * 864 + ci * 27 + ts] | ((uint32_t)tb[(k8 + 2 * i + 1) * 864 + ci * 27 + ts] << 16);
    *reinterpret_cast<u32x4_t*>(dgr + (((long)(j0 >> 5) * 27 + t) * Cin + chunk * 32 + ci) * 32 + k8) = o;
  }
}

// Persistent stem forward: one 8-wave workgroup per CU walks boxes b = blockIdx.x,
// b += gridDim.x.  LDS: weights (loaded once) | halo x2 (LDS-DMA, next box prefetched while
// the current one computes) | bf16 C tile (16-B coalesced stores).  Every thread issues
// exactly kStemStores stores per box (invalid ones go to a sink), so the next halo's DMA,
// issued before them, is retired by s_waitcnt vmcnt(kStemStores).
constexpr int kStemThreads = 512;
constexpr int kStemHaloBytes = kHaloMax * 16;                 // 18 KiB
constexpr int kStemCtOff = 2 * kStemHaloBytes;                 // C tile offset
constexpr int kStemLds = kStemCtOff + 512 * 64 * 2 + 6144;     // + stats reduction [8][64][3]
constexpr int kStemStores = 512 * 8 / kStemThreads;            // 16-B stores per thread per box
__device__ __attribute__((aligned(16))) uint32_t g_sink[4 * 512];

template <int LBD, int LBH, int LBW>
__global__ void __launch_bounds__(kStemThreads, 1) stem_fwd_kernel(Conv3Params p, int nbox) {
  const int lbd_ = LBW >= 0 ? LBD : p.lbd, lbh_ = LBW >= 0 ? LBH : p.lbh, lbw_ = LBW >= 0 ? LBW : p.lbw;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  bf16_t* ct = reinterpret_cast<bf16_t*>(lds + kStemCtOff);
  float* red = reinterpret_cast<float*>(lds + kStemCtOff + 512 * 64 * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r_lane = lane & 31, hsel = lane >> 5;
  const int bd = 1 << lbd_, bh = 1 << lbh_, bw = 1 << lbw_;
  const int boxvol = bd * bh * bw;
  const int HH = bh + 2, HW = bw + 2;
  const int HV = (bd + 2) * HH * HW;
  const long plane = (long)p.H * p.W;
  const bf16_t* x0 = (const bf16_t*)p.x0;
  const bool w16 = lbw_ == 4;
  const int prow = w16 ? perm32(r_lane) : r_lane;
  int hb[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    int r = wave * 64 + mt * 32 + prow;
    if (r >= boxvol) r = 0;
    const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
    hb[mt] = (rd * HH + rh) * HW + rw;
  }
  const bool wave_active = wave * 64 < boxvol;
  float bias_l[2] = {0.f, 0.f};
  if (p.bias) { bias_l[0] = p.bias[2 * r_lane]; bias_l[1] = p.bias[2 * r_lane + 1]; }

  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int bwi = b % p.nbw; b /= p.nbw;
    int bhi = b % p.nbh; b /= p.nbh;
    int bdi = b % p.nbd;
    n = b / p.nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  auto stage_halo = [&](int b, char* hl) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    for (int base = wave * 64; base < HV; base += kStemThreads) {
      const int hv = base + lane;
      const void* src = g_zero16;
      if (hv < HV) {
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        if (gd >= 0 && gd < p.D && gh >= 0 && gh < p.H && gw >= 0 && gw < p.W)
          src = x0 + (((long)n * p.D + gd) * plane + (long)gh * p.W + gw) * 8;
      }
      __builtin_amdgcn_global_load_lds(src, (LDS_AS void*)(hl + base * 16), 16, 0, 0);
    }
  };
  // prologue: the B fragments of all 14 k-steps stay in registers for the whole kernel
  // (28 x 16 B per lane, loaded once); first halo
  s16x8_t wb[kStemSteps][2];
  {
    const bf16_t* wg = (const bf16_t*)p.w;
#pragma unroll
    for (int st = 0; st < kStemSteps; ++st) {
      wb[st][0] = *reinterpret_cast<const s16x8_t*>(wg + (st * 64 + r_lane) * 16 + hsel * 8);
      wb[st][1] = *reinterpret_cast<const s16x8_t*>(wg + (st * 64 + 32 + r_lane) * 16 + hsel * 8);
    }
  }
  int b = blockIdx.x;
  if (b < nbox) stage_halo(b, lds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; b < nbox; b += gridDim.x, ++it) {
    char* hl = lds + (it & 1) * kStemHaloBytes;
    const int bn = b + gridDim.x;
    if (bn < nbox) stage_halo(bn, lds + ((it + 1) & 1) * kStemHaloBytes);
    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = bias_l[j];  // bias folded into the accumulator
    if (wave_active) {
      // lane half hsel reads tap 2 st + hsel: constant base offset + hsel * constant delta.
      // A fragments are prefetched one k-step ahead; sched_barrier keeps the compiler from
      // hoisting every step's LDS reads (register pressure: the weights live in VGPRs).
      // (hs16 is opaque so the 28 per-step lane addresses are formed in the loop, not
      // hoisted out of it into spilled registers)
      int hs16 = hsel * 16;
      asm volatile("" : "+v"(hs16));
      auto load_a = [&](int st, s16x8_t (&a)[2]) {
        const int o0 = tap_off(2 * st, HH, HW), o1 = tap_off(2 * st + 1, HH, HW);
        const int off16 = o0 * 16 + hs16 * (o1 - o0);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) a[mt] = *reinterpret_cast<const s16x8_t*>(hl + hb[mt] * 16 + off16);
      };
      s16x8_t abuf[2][2];
      load_a(0, abuf[0]);
#pragma unroll
      for (int st = 0; st < kStemSteps; ++st) {
        if (st + 1 < kStemSteps) load_a(st + 1, abuf[(st + 1) & 1]);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          acc[mt][0] = mfma(abuf[st & 1][mt], wb[st][0], acc[mt][0]);
          acc[mt][1] = mfma(abuf[st & 1][mt], wb[st][1], acc[mt][1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const bool interior = d0 + bd <= p.D && h0 + bh <= p.H && w0 + bw <= p.W;
    // Epilogue: C tile -> LDS as packed bf16 channel pairs; BatchNorm partials single-pass,
    // shifted by the wave's row-0 value K of each channel: per wave S1 = sum d + n K,
    // M2 = sum d^2 - (sum d)^2 / n (d = v - K), waves merged with Chan's formula below.
    float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, K[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) K[nt] = __shfl(acc[0][nt][0], r_lane, 64);
    float nw = 0.f;
    __syncthreads();  // previous box's C-tile reads (stores) are done in every wave
    if (wave_active) {
      // row of (mt, e) = perm32((e & 3) + 8 (e >> 2) + 4 hsel) as constant + (+-16 hsel); the
      // opaque hp keeps the per-row indices from being hoisted out of the box loop (they
      // would pin ~100 VGPRs)
      int hp = hsel * 16;
      asm volatile("" : "+v"(hp));
      auto row_of = [&](int mt, int e) {
        const int g = e >> 2;
        const int base = wave * 64 + mt * 32 + (e & 3);
        if (w16) return base + (g == 0 ? hp : g == 1 ? 20 - hp : g == 2 ? 24 - hp : 12 + hp);
        return base + 8 * g + (hp >> 2);
      };
      if (interior && boxvol == 512) {  // every row valid: no per-row tests
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int r = row_of(mt, e);
            const float v0 = acc[mt][0][e], v1 = acc[mt][1][e];
            *reinterpret_cast<uint32_t*>(ct + r * 64 + 2 * r_lane) = pack_bf16x2(v0, v1);
            const float e0 = v0 - K[0], e1 = v1 - K[1];
            s1[0] += e0; s2[0] += e0 * e0;
            s1[1] += e1; s2[1] += e1 * e1;
          }
        nw = 64.f;
      } else {
        int cnt = 0;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int r = row_of(mt, e);
            const float v0 = acc[mt][0][e], v1 = acc[mt][1][e];
            *reinterpret_cast<uint32_t*>(ct + r * 64 + 2 * r_lane) = pack_bf16x2(v0, v1);
            const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
            const bool valid = r < boxvol && d0 + rd < p.D && h0 + rh < p.H && w0 + rw < p.W;
            const float e0 = valid ? v0 - K[0] : 0.f, e1 = valid ? v1 - K[1] : 0.f;
            s1[0] += e0; s2[0] += e0 * e0;
            s1[1] += e1; s2[1] += e1 * e1;
            cnt += valid ? 1 : 0;
          }
        nw = (float)(cnt + __shfl_xor(cnt, 32, 64));
      }
    }
    if (p.stats) {
      const float inv = nw > 0.f ? 1.f / nw : 0.f;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        s1[nt] += __shfl_xor(s1[nt], 32, 64);
        s2[nt] += __shfl_xor(s2[nt], 32, 64);
        if (hsel == 0) {
          float* rp = red + (wave * 64 + 2 * r_lane + nt) * 3;
          rp[0] = s1[nt] + nw * K[nt];
          rp[1] = s2[nt] - s1[nt] * s1[nt] * inv;
          rp[2] = nw;
        }
      }
    }
    __syncthreads();
    if (p.stats && tid < 64) {
      float S = 0.f, Nn = 0.f;
#pragma unroll
      for (int w = 0; w < kStemThreads / 64; ++w) { S += red[(w * 64 + tid) * 3]; Nn += red[(w * 64 + tid) * 3 + 2]; }
      const float m = Nn > 0.f ? S / Nn : 0.f;
      float M2 = 0.f, sdd = 0.f;
#pragma unroll
      for (int w = 0; w < kStemThreads / 64; ++w) {
        const float c = red[(w * 64 + tid) * 3 + 2];
        if (c > 0.f) {
          const float d = red[(w * 64 + tid) * 3] / c - m;
          M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
          sdd += c * d;
        }
      }
      if (Nn > 0.f) M2 -= sdd * sdd / Nn;
      float* stp = p.stats + ((long)b * 64 + tid) * 2;
      stp[0] = S;
      stp[1] = M2;
      if (tid == 0) p.stats[(long)nbox * 64 * 2 + b] = Nn;
    }
#pragma unroll 2
    for (int i = 0; i < kStemStores; ++i) {
      const int pc = tid + i * kStemThreads;
      const int r = pc >> 3, q = pc & 7;
      const int rd = r >> (lbh_ + lbw_), rh = (r >> lbw_) & (bh - 1), rw = r & (bw - 1);
      const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
      u32x4_t* dst = reinterpret_cast<u32x4_t*>(g_sink) + (tid & 511);
      if (r < boxvol && (interior || (gd < p.D && gh < p.H && gw < p.W)))
        dst = reinterpret_cast<u32x4_t*>((bf16_t*)p.y0 + (((long)n * p.D + gd) * plane + (long)gh * p.W + gw) * 64 + q * 8);
      *dst = *reinterpret_cast<const u32x4_t*>(ct + r * 64 + q * 8);
    }
    // the next halo's LDS-DMA (issued before the stores) has landed; make it visible
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kStemStores) : "memory");
    __syncthreads();
  }
}

// Persistent stem forward, direct-store variant for 16-wide 512-voxel boxes (bd x bh = 32).
// No C tile: the weight columns are ordered so that lane r_lane of a wave holds channels
// (2 r_lane, 2 r_lane + 1) of each of its rows, so the 32 lanes of a half-wave write one
// voxel's 64 channels (128 contiguous bytes) with ONE buffer_store_dword, addressed by a
// per-lane voffset (2 variants), a wave-uniform soffset and an immediate offset: no VALU
// address math, no LDS round trip, one barrier per box.  The halo arrives by buffer LDS-DMA
// (out-of-range voffset = zero padding); weights stay in VGPRs; BatchNorm partials are
// accumulated over all boxes of the workgroup (shifted sums) and written as ONE stats row
// per workgroup (rows >= gridDim.x are zeroed: count 0).
// THR = 512: one 8-wave workgroup per CU, 512-voxel boxes; THR = 256: two independent
// 4-wave workgroups per CU with 256-voxel boxes (each workgroup's barrier-synchronised
// compute and store phases drift against the other's).
constexpr int kSDHaloRows = kHaloMax;                         // 1152 rows (18 x 64)
constexpr int kSDHaloBytes = kSDHaloRows * 16;
constexpr int kSDLds = 2 * kSDHaloBytes + 8 * 64 * 3 * 4;     // halo x2 + stats reduction
constexpr int kSDThr = (PCMS_ABL & 8192) ? 256 : 512;  // product variant (256: same time, 101 vs 102 us)

// PIPE: software-pipelined stores.  Tile mt = 0 of a box is computed first and its 16
// stores are issued between the MFMAs of tile mt = 1; tile 1's stores go out between the
// MFMAs of the NEXT box's tile 0 (the last one after the loop).  Stores and BN sums thus run
// inside the MFMA gaps of the same wave instead of after all its MFMAs.
template <int LBD, int LBH, int THR, bool PIPE = false>
__global__ void __launch_bounds__(THR, (PIPE && THR == 256) ? 1 : 512 / THR) stem_fwd_direct_kernel(Conv3Params p, int nbox, int mrows,
                                                                         uint32_t xbytes, uint32_t ybytes) {
  constexpr int kSDThreads = THR, NWV = THR / 64;
  static_assert((1 << (LBD + LBH + 4)) == NWV * 64, "box = 64 voxels per wave");
  constexpr int bd = 1 << LBD, bh = 1 << LBH, bw = 16;
  constexpr int HH = bh + 2, HW = bw + 2, HV = (bd + 2) * HH * HW;
  constexpr int NP = (HV + kSDThreads - 1) / kSDThreads;  // halo pieces per thread
  static_assert(HV <= kSDHaloRows, "halo fits");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* red = reinterpret_cast<float*>(lds + 2 * kSDHaloBytes);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR math)
  const int r_lane = lane & 31, hsel = lane >> 5;
  const int D = p.D, H = p.H, W = p.W;
  const auto xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x0, 0, xbytes, 0x00020000);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(p.y0, 0, ybytes, 0x00020000);

  // weights: B fragments of all 14 k-steps in registers
  s16x8_t wb[kStemSteps][2];
  {
    const bf16_t* wg = (const bf16_t*)p.w;
#pragma unroll
    for (int st = 0; st < kStemSteps; ++st) {
      wb[st][0] = *reinterpret_cast<const s16x8_t*>(wg + (st * 64 + r_lane) * 16 + hsel * 8);
      wb[st][1] = *reinterpret_cast<const s16x8_t*>(wg + (st * 64 + 32 + r_lane) * 16 + hsel * 8);
    }
  }
  float bias_l[2] = {0.f, 0.f};
  if (p.bias) { bias_l[0] = p.bias[2 * r_lane]; bias_l[1] = p.bias[2 * r_lane + 1]; }
  // halo rows of the two 32-row MFMA tiles (perm32 layout)
  int hb16[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int r = wave * 64 + mt * 32 + perm32(r_lane);
    const int rd = r >> (LBH + 4), rh = (r >> 4) & (bh - 1), rw = r & 15;
    hb16[mt] = ((rd * HH + rh) * HW + rw) * 16;
  }
  // halo pieces of this thread: relative source offset (bytes) and packed coordinates
  int prel[NP], pco[NP];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int hv = tid + i * kSDThreads;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    prel[i] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    pco[i] = hv < HV ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  // store voffsets: rows x = perm32((e & 3) + 8 g + 4 hsel) have x & 15 = 4 g + (e & 3) and
  // x >> 4 = (g in {1, 2}) ^ hsel
  const uint32_t vb0 = r_lane * 4, vb1 = r_lane * 4 + (uint32_t)W * 128;
  const uint32_t vA = hsel ? vb1 : vb0;  // g = 0, 3
  const uint32_t vB = hsel ? vb0 : vb1;  // g = 1, 2

  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    const int nbw = p.nbw, nbh = p.nbh, nbd = p.nbd;
    int q = b;
    const int bwi = q % nbw; q /= nbw;
    const int bhi = q % nbh; q /= nbh;
    const int bdi = q % nbd;
    n = q / nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  auto stage = [&](int b, int buf) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int base16 = ((((n * D + d0) * H + h0) * W) + w0) * 16;
    const bool inner = d0 >= 1 && d0 + bd < D && h0 >= 1 && h0 + bh < H && w0 >= 1 && w0 + bw < W;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (wave * 64 + i * kSDThreads >= HV) break;  // whole wave past the halo (uniform)
      uint32_t voff = (uint32_t)(base16 + prel[i]);
      const int c = pco[i];
      if (c < 0) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (LDS_AS void*)(lds + buf * kSDHaloBytes + (wave * 64 + i * kSDThreads) * 16),
                                           16, voff, 0, 0, 0);
    }
  };

  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, K[2] = {0.f, 0.f};
  float cnt = 0.f;
  bool first = true;
  int b = blockIdx.x;
  if (b < nbox) stage(b, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (PIPE) {
    // one pending tile: values, store soffset, validity inputs
    struct Tile {
      f32x16_t v[2];
      uint32_t so;
      int rd, rh, d0, h0, w0;
      bool full;
    };
    auto tile_meta = [&](Tile& t, int bb, int mt) {
      int n, d0, h0, w0;
      origin(bb, n, d0, h0, w0);
      const int R0 = wave * 4 + mt * 2;
      t.rd = R0 >> LBH; t.rh = R0 & (bh - 1);
      t.d0 = d0; t.h0 = h0; t.w0 = w0;
      t.full = d0 + bd <= D && h0 + bh <= H && w0 + bw <= W;
      const int bv = ((n * D + d0) * H + h0) * W + w0;
      t.so = __builtin_amdgcn_readfirstlane((uint32_t)(bv + (t.rd * H + t.rh) * W) * 128u);
    };
    // element e of tile t: one buffer store + BN shifted sums
    auto store_e = [&](const Tile& t, int e) {
      const int g = e >> 2, rw = 4 * g + (e & 3);
      const bool gB = (g == 1 || g == 2);
      const float v0 = t.v[0][e], v1 = t.v[1][e];
      uint32_t voff = gB ? vB : vA;
      float e0 = v0 - K[0], e1 = v1 - K[1];
      if (!t.full) {
        const int xh = (gB ? 1 : 0) ^ hsel;
        const bool valid = (t.d0 + t.rd < D) & (t.h0 + t.rh + xh < H) & (t.w0 + rw < W);
        voff = valid ? voff : kOOB;
        e0 = valid ? e0 : 0.f;
        e1 = valid ? e1 : 0.f;
        cnt += valid ? 1.f : 0.f;
      }
      __builtin_amdgcn_raw_buffer_store_b32(pack_bf16x2(v0, v1), yr, voff, t.so + rw * 128, 0);
      s1[0] += e0; s2[0] += e0 * e0;
      s1[1] += e1; s2[1] += e1 * e1;
    };
    auto count_full = [&](const Tile& t) { if (t.full) cnt += 16.f; };
    Tile pend, cur;
    bool have_pend = false;
    int hs16 = hsel * 16;
    asm volatile("" : "+v"(hs16));
    for (int it = 0; b < nbox; b += gridDim.x, ++it) {
      __syncthreads();
      const int bn = b + gridDim.x;
      if (bn < nbox) stage(bn, (it + 1) & 1);
      const char* hl = lds + (it & 1) * kSDHaloBytes;
      // one 32-row tile: 14 k-steps x 2 MFMAs; `st_` = the tile whose stores fill the gaps
      auto run_tile = [&](auto with_st, int mt, Tile& out, const Tile& st_) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) out.v[j][e] = bias_l[j];
        auto load_a = [&](int st) {
          const int o0 = tap_off(2 * st, HH, HW), o1 = tap_off(2 * st + 1, HH, HW);
          return *reinterpret_cast<const s16x8_t*>(hl + hb16[mt] + o0 * 16 + hs16 * (o1 - o0));
        };
        s16x8_t abuf[2];
        abuf[0] = load_a(0);
#pragma unroll
        for (int st = 0; st < kStemSteps; ++st) {
          if (st + 1 < kStemSteps) abuf[(st + 1) & 1] = load_a(st + 1);
          out.v[0] = mfma(abuf[st & 1], wb[st][0], out.v[0]);
          out.v[1] = mfma(abuf[st & 1], wb[st][1], out.v[1]);
          if constexpr (decltype(with_st)::value) {  // 16 stores over 14 steps: two extra on the first two
            store_e(st_, st);
            if (st < 2) store_e(st_, 14 + st);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      if (have_pend) {
        run_tile(std::true_type{}, 0, cur, pend);
        count_full(pend);
      } else {
        run_tile(std::false_type{}, 0, cur, pend);
      }
      tile_meta(cur, b, 0);
      if (first) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) K[nt] = __shfl(cur.v[nt][0], r_lane, 64);
        first = false;
      }
      run_tile(std::true_type{}, 1, pend, cur);
      count_full(cur);
      tile_meta(pend, b, 1);
      have_pend = true;
      // the next halo's DMA was issued before this box's stores (16 on the first box, 32 after)
      if (it == 0) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    }
    if (have_pend) {
#pragma unroll
      for (int e = 0; e < 16; ++e) store_e(pend, e);
      count_full(pend);
    }
  } else
  for (int it = 0; b < nbox; b += gridDim.x, ++it) {
    // halo(b) has landed for this wave (vmcnt above / at the loop end); barrier: for all
    // waves, and every wave is done reading the buffer the next DMA overwrites
    __syncthreads();
    const int bn = b + gridDim.x;
    if (bn < nbox && !(PCMS_ABL & 4)) stage(bn, (it + 1) & 1);
    const char* hl = lds + (it & 1) * kSDHaloBytes;
    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = bias_l[j];
    if (!(PCMS_ABL & 1)) {
      int hs16 = hsel * 16;
      asm volatile("" : "+v"(hs16));
      auto load_a = [&](int st, s16x8_t (&a)[2]) {
        const int o0 = tap_off(2 * st, HH, HW), o1 = tap_off(2 * st + 1, HH, HW);
        const int off16 = o0 * 16 + hs16 * (o1 - o0);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) a[mt] = *reinterpret_cast<const s16x8_t*>(hl + hb16[mt] + off16);
      };
      s16x8_t abuf[2][2];
      load_a(0, abuf[0]);
#pragma unroll
      for (int st = 0; st < kStemSteps; ++st) {
        if (st + 1 < kStemSteps) load_a(st + 1, abuf[(st + 1) & 1]);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          acc[mt][0] = mfma(abuf[st & 1][mt], wb[st][0], acc[mt][0]);
          acc[mt][1] = mfma(abuf[st & 1][mt], wb[st][1], acc[mt][1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // ---- epilogue: direct stores + shifted BN sums ----
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const bool full = d0 + bd <= D && h0 + bh <= H && w0 + bw <= W;
    if (first) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) K[nt] = __shfl(acc[0][nt][0], r_lane, 64);
      first = false;
    }
    const int bv = ((n * D + d0) * H + h0) * W + w0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int R0 = wave * 4 + mt * 2;          // even (rd, rh) linear index of the tile
      const int rd0 = R0 >> LBH, rh0 = R0 & (bh - 1);
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(bv + (rd0 * H + rh0) * W) * 128u);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int g = e >> 2, rw = 4 * g + (e & 3);
        const bool gB = (g == 1 || g == 2);
        const float v0 = acc[mt][0][e], v1 = acc[mt][1][e];
        uint32_t voff = gB ? vB : vA;
        float e0 = v0 - K[0], e1 = v1 - K[1];
        if (!full) {  // uniform branch: boundary boxes only
          const int xh = (gB ? 1 : 0) ^ hsel;
          const bool valid = (d0 + rd0 < D) & (h0 + rh0 + xh < H) & (w0 + rw < W);
          voff = valid ? voff : kOOB;
          e0 = valid ? e0 : 0.f;
          e1 = valid ? e1 : 0.f;
          cnt += valid ? 1.f : 0.f;
        }
        if (!(PCMS_ABL & 2)) __builtin_amdgcn_raw_buffer_store_b32(pack_bf16x2(v0, v1), yr, voff, so + rw * 128, 0);
        s1[0] += e0; s2[0] += e0 * e0;
        s1[1] += e1; s2[1] += e1 * e1;
      }
    }
    if (full) cnt += 32.f;
    // the next halo's DMA was issued before this box's 32 stores
    asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  }
  if (!p.stats) return;
  // per wave (lanes r_lane and r_lane + 32 share channels and K): S = sum d + n K,
  // M2 = sum d^2 - (sum d)^2 / n; then Chan across the 8 waves
  const float nw = cnt + __shfl_xor(cnt, 32, 64);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s1[nt] += __shfl_xor(s1[nt], 32, 64);
    s2[nt] += __shfl_xor(s2[nt], 32, 64);
    if (hsel == 0) {
      float* rp = red + (wave * 64 + 2 * r_lane + nt) * 3;
      rp[0] = s1[nt] + nw * K[nt];
      rp[1] = nw > 0.f ? s2[nt] - s1[nt] * s1[nt] / nw : 0.f;
      rp[2] = nw;
    }
  }
  __syncthreads();
  if (tid < 64) {
    float S = 0.f, Nn = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) { S += red[(w * 64 + tid) * 3]; Nn += red[(w * 64 + tid) * 3 + 2]; }
    const float m = Nn > 0.f ? S / Nn : 0.f;
    float M2 = 0.f, sdd = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      const float c = red[(w * 64 + tid) * 3 + 2];
      if (c > 0.f) {
        const float d = red[(w * 64 + tid) * 3] / c - m;
        M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
        sdd += c * d;
      }
    }
    if (Nn > 0.f) M2 -= sdd * sdd / Nn;
    float* st = p.stats + ((long)blockIdx.x * 64 + tid) * 2;
    st[0] = S;
    st[1] = M2;
    float* cnts = p.stats + (long)mrows * 128;  // row counts after the [mrows][64][2] block
    if (tid == 0) cnts[blockIdx.x] = Nn;
    // zero this workgroup's share of the rows past gridDim.x
    for (int r = blockIdx.x + gridDim.x; r < mrows; r += gridDim.x) {
      p.stats[((long)r * 64 + tid) * 2] = 0.f;
      p.stats[((long)r * 64 + tid) * 2 + 1] = 0.f;
      if (tid == 0) cnts[r] = 0.f;
    }
  }
}

// Wave-independent persistent stem forward: the hot case D % 2 == H % 2 == 0, W % 16 == 0.
// Every wave owns a private stream of 2x2x16-voxel boxes (64 voxels = two 32-row MFMA
// tiles) with its own 3-slot LDS ring of halos (4x4x18 rows, buffer LDS-DMA, prefetch
// distance 2): no barrier inside the box loop, so the two waves sharing a SIMD drift apart
// and one's MFMAs cover the other's epilogue.  MFMA row r of tile mt is voxel
// (rd, rh, rw) = (mt, r >> 4, 2 (r & 3) + ((r >> 2) & 1) + 8 ((r >> 3) & 1)), so an
// accumulator register of the 32x32 layout holds two ADJACENT voxels (lane halves) and each
// buffer_store_dword writes 256 contiguous bytes with a per-lane constant voffset, a
// per-(mt, row pair) soffset and an immediate offset.  Weights stay in VGPRs; BatchNorm
// partials (shifted sums) are merged over the workgroup once at the end: ONE stats row per
// workgroup (pcms_stem_fwd_rows).  Box order is XCD-aware (8 consecutive logical
// workgroups' neighbouring boxes share one L2).
constexpr int kSWvThreads = 512;
constexpr int kSWvHalo = 4 * 4 * 18;                           // 288 halo rows
constexpr int kSWvPieces = 5;                                  // DMA instructions per box (320 rows)
constexpr int kSWvSlot = kSWvPieces * 64 * 16;                 // 5 KiB per ring slot
constexpr int kSWvLds = 8 * 3 * kSWvSlot + 8 * 64 * 3 * 4;     // 120 KiB rings + stats merge

__global__ void __launch_bounds__(kSWvThreads, 1) stem_fwd_wave_kernel(const bf16_t* x, const bf16_t* wpack,
                                                                      const float* bias, bf16_t* y, float* stats,
                                                                      int N, int D, int H, int W,
                                                                      uint32_t xbytes, uint32_t ybytes) {
  constexpr int HH = 4, HW = 18;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  float* red = reinterpret_cast<float*>(lds + 8 * 3 * kSWvSlot);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r_lane = lane & 31, hsel = lane >> 5;
  const i32x4_t xr = buffer_desc(x, xbytes);
  const auto yr = __builtin_amdgcn_make_buffer_rsrc(y, 0, ybytes, 0x00020000);
  const int nbw = W >> 4, nbh = H >> 1, nbd = D >> 1;
  const int nwb = N * nbd * nbh * nbw;
  // logical workgroup: consecutive logical ids on one XCD (dispatch is round-robin over 8)
  const int G = gridDim.x;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int stride = G * 8;

  s16x8_t wb[kStemSteps][2];
#pragma unroll
  for (int st = 0; st < kStemSteps; ++st) {
    wb[st][0] = *reinterpret_cast<const s16x8_t*>(wpack + (st * 64 + r_lane) * 16 + hsel * 8);
    wb[st][1] = *reinterpret_cast<const s16x8_t*>(wpack + (st * 64 + 32 + r_lane) * 16 + hsel * 8);
  }
  const float bias0 = bias ? bias[2 * r_lane] : 0.f, bias1 = bias ? bias[2 * r_lane + 1] : 0.f;
  // A rows: halo row of this lane's voxel in tile mt
  int hb16[2];
  {
    const int q = r_lane & 15;
    const int rw = 2 * (q & 3) + ((q >> 2) & 1) + 8 * ((q >> 3) & 1);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) hb16[mt] = ((mt * HH + (r_lane >> 4)) * HW + rw) * 16;
  }
  // halo pieces: row hv = 64 j + lane of the 4x4x18 halo; source offset relative to the box
  // origin voxel, packed halo coordinates (-1: past the halo)
  int prel[kSWvPieces], pco[kSWvPieces];
#pragma unroll
  for (int j = 0; j < kSWvPieces; ++j) {
    const int hv = j * 64 + lane;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    prel[j] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    pco[j] = hv < kSWvHalo ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  const uint32_t ring = lds_addr(lds) + wave * 3 * kSWvSlot;
  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int q = b;
    const int bwi = q % nbw; q /= nbw;
    const int bhi = q % nbh; q /= nbh;
    const int bdi = q % nbd;
    n = q / nbd;
    d0 = bdi * 2; h0 = bhi * 2; w0 = bwi * 16;
  };
  // exactly kSWvPieces DMA instructions per call (b >= nwb: all out of range -> zeros), so
  // the vmcnt arithmetic below is the same for every iteration
  auto stage = [&](int b, int slot) {
    const uint32_t lb = __builtin_amdgcn_readfirstlane(ring + slot * kSWvSlot);
    if (b >= nwb) {
#pragma unroll
      for (int j = 0; j < kSWvPieces; ++j) dma16(xr, lb + j * 1024, kOOB, 0);
      return;
    }
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int base16 = (((n * D + d0) * H + h0) * W + w0) * 16;
    const bool inner = d0 >= 1 && d0 + 2 < D && h0 >= 1 && h0 + 2 < H && w0 >= 1 && w0 + 16 < W;
#pragma unroll
    for (int j = 0; j < kSWvPieces; ++j) {
      uint32_t voff = (uint32_t)(base16 + prel[j]);
      const int c = pco[j];
      if (c < 0) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      dma16(xr, lb + j * 1024, voff, 0);
    }
  };

  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f}, K[2] = {0.f, 0.f};
  float cnt = 0.f;
  const uint32_t vlane = r_lane * 4 + hsel * 128;  // store voffset: channel pair + odd voxel
  int b = lg * 8 + wave;
  stage(b, 0);
  stage(b + stride, 1);
  for (int it = 0; b < nwb; b += stride, ++it) {
    // this box's halo has landed (issued after it: DMA of the next box + the stores of the
    // previous two; capped at the 6-bit counter)
    if (it == 0) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if (it == 1) asm volatile("s_waitcnt vmcnt(37)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    stage(b + 2 * stride, (it + 2) % 3);
    const char* hl = lds + wave * 3 * kSWvSlot + (it % 3) * kSWvSlot;
    f32x16_t acc[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) { acc[mt][0][e] = bias0; acc[mt][1][e] = bias1; }
    if (!(PCMS_ABL & 1)) {
      int hs16 = hsel * 16;
      asm volatile("" : "+v"(hs16));
      auto load_a = [&](int st, s16x8_t (&a)[2]) {
        const int o0 = tap_off(2 * st, HH, HW), o1 = tap_off(2 * st + 1, HH, HW);
        const int off16 = o0 * 16 + hs16 * (o1 - o0);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) a[mt] = *reinterpret_cast<const s16x8_t*>(hl + hb16[mt] + off16);
      };
      s16x8_t abuf[2][2];
      load_a(0, abuf[0]);
#pragma unroll
      for (int st = 0; st < kStemSteps; ++st) {
        if (st + 1 < kStemSteps) load_a(st + 1, abuf[(st + 1) & 1]);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          acc[mt][0] = mfma(abuf[st & 1][mt], wb[st][0], acc[mt][0]);
          acc[mt][1] = mfma(abuf[st & 1][mt], wb[st][1], acc[mt][1]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (it == 0) {
      K[0] = __shfl(acc[0][0][0], r_lane, 64);
      K[1] = __shfl(acc[0][1][0], r_lane, 64);
    }
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int bv = ((n * D + d0) * H + h0) * W + w0;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int gh = 0; gh < 2; ++gh) {
        const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(bv + (mt * H + gh) * W) * 128u);
#pragma unroll
        for (int gl = 0; gl < 2; ++gl)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int e = (2 * gh + gl) * 4 + i;  // g = e >> 2: gh = g >> 1, gl = g & 1
            const float v0 = acc[mt][0][e], v1 = acc[mt][1][e];
            if (!(PCMS_ABL & 2))
              __builtin_amdgcn_raw_buffer_store_b32(pack_bf16x2(v0, v1), yr, vlane + (2 * i + 8 * gl) * 128, so, 0);
            const float e0 = v0 - K[0], e1 = v1 - K[1];
            s1[0] += e0; s2[0] = fmaf(e0, e0, s2[0]);
            s1[1] += e1; s2[1] = fmaf(e1, e1, s2[1]);
          }
      }
    cnt += 32.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!stats) return;
  // per wave: S = sum d + n K, M2 = sum d^2 - (sum d)^2 / n; Chan merge over the 8 waves
  const float nw = 2.f * cnt;
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s1[nt] += __shfl_xor(s1[nt], 32, 64);
    s2[nt] += __shfl_xor(s2[nt], 32, 64);
    if (hsel == 0) {
      float* rp = red + (wave * 64 + 2 * r_lane + nt) * 3;
      rp[0] = s1[nt] + nw * K[nt];
      rp[1] = nw > 0.f ? s2[nt] - s1[nt] * s1[nt] / nw : 0.f;
      rp[2] = nw;
    }
  }
  __syncthreads();
  if (tid < 64) {
    float S = 0.f, Nn = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) { S += red[(w * 64 + tid) * 3]; Nn += red[(w * 64 + tid) * 3 + 2]; }
    const float m = Nn > 0.f ? S / Nn : 0.f;
    float M2 = 0.f, sdd = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const float c = red[(w * 64 + tid) * 3 + 2];
      if (c > 0.f) {
        const float d = red[(w * 64 + tid) * 3] / c - m;
        M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
        sdd += c * d;
      }
    }
    if (Nn > 0.f) M2 -= sdd * sdd / Nn;
    float* st = stats + ((long)blockIdx.x * 64 + tid) * 2;
    st[0] = S;
    st[1] = M2;
    if (tid == 0) stats[(long)gridDim.x * 128 + blockIdx.x] = Nn;
  }
}

// Stem weight gradient.  dW[co][c][t] = sum_v dy[v][co] * x[v + t][c], c < cin_w <= 8.
// Output columns j = (t, c) = 8 t + c, 224 of them in 7 tiles of 32 (= 4 taps x 8 channels).
// Wave w: both co tiles (64 co), column tiles {w, w + 4} (w < 3) or {3}.  Voxel boxes of
// 256 are double-buffered through LDS (register-staged prefetch); one atomic flush per WG.
constexpr int kSBV = 256;
constexpr int kSHalo = 648;                         // (4+2)(4+2)(16+2) for the 4x4x16 box
constexpr int kSBuf = kSBV * 128 + kSHalo * 16;     // dy tile (128 B rows) + halo (16 B rows)

template <int LBD, int LBH, int LBW>
__global__ void __launch_bounds__(256, 1) stem_wgrad_kernel(const bf16_t* x, const bf16_t* dy, float* dw,
                                                            int N, int D, int H, int W, int cin_w,
                                                            int lbd_r, int lbh_r, int lbw_r, int nbd, int nbh, int nbw,
                                                            int nbox, int boxes_per_split) {
  const int lbd = LBW >= 0 ? LBD : lbd_r, lbh = LBW >= 0 ? LBH : lbh_r, lbw = LBW >= 0 ? LBW : lbw_r;
  extern __shared__ __attribute__((aligned(16))) char slds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hsel = lane >> 5;
  const int bd = 1 << lbd, bh = 1 << lbh, bw = 1 << lbw;
  const int HH = bh + 2, HW = bw + 2;
  const int HV = (bd + 2) * HH * HW;
  const int boxvol = bd * bh * bw;
  const long plane = (long)H * W;
  const int nj = (wave < 3) ? 2 : 1;
  const int jt0 = wave, jt1 = wave + 4;
  const int b_beg = blockIdx.x * boxes_per_split;
  const int b_end = min(nbox, b_beg + boxes_per_split);
  f32x16_t acc[2][2];  // [co tile][column tile slot]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  constexpr int DYP = kSBV * 8;                      // 16-B pieces of the dy tile
  constexpr int MAXP = (DYP + kSHalo + 255) / 256;  // per thread
  u32x4_t stg[MAXP];
  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int bwi = b % nbw; b /= nbw;
    int bhi = b % nbh; b /= nbh;
    int bdi = b % nbd;
    n = b / nbd;
    d0 = bdi * bd; h0 = bhi * bh; w0 = bwi * bw;
  };
  auto stage_load = [&](int b) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int pc = tid + i * 256;
      u32x4_t v = {0u, 0u, 0u, 0u};
      if (pc < DYP) {
        const int r = pc >> 3, q = pc & 7;
        if (r < boxvol) {
          const int rd = r >> (lbh + lbw), rh = (r >> lbw) & (bh - 1), rw = r & (bw - 1);
          const int gd = d0 + rd, gh = h0 + rh, gw = w0 + rw;
          if (gd < D && gh < H && gw < W)
            v = *reinterpret_cast<const u32x4_t*>(dy + (((long)n * D + gd) * plane + (long)gh * W + gw) * 64 + q * 8);
        }
      } else if (pc < DYP + HV) {
        const int hv = pc - DYP;
        const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
        const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
        if (gd >= 0 && gd < D && gh >= 0 && gh < H && gw >= 0 && gw < W)
          v = *reinterpret_cast<const u32x4_t*>(x + (((long)n * D + gd) * plane + (long)gh * W + gw) * 8);
      }
      stg[i] = v;
    }
  };
  auto stage_store = [&](char* buf) {
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const int pc = tid + i * 256;
      if (pc < DYP) {
        const int r = pc >> 3, q = pc & 7;
        *reinterpret_cast<u32x4_t*>(buf + dy_off_bf16(r, q * 8)) = stg[i];
      } else if (pc < DYP + HV) {
        *reinterpret_cast<u32x4_t*>(buf + kSBV * 128 + (pc - DYP) * 16) = stg[i];
      }
    }
  };
  auto halo_row = [&](int r) {
    const int rd = r >> (lbh + lbw), rh = (r >> lbw) & (bh - 1), rw = r & (bw - 1);
    return (rd * HH + rh) * HW + rw;
  };
  // per-lane column -> (tap, channel half) for the transposed B reads: in a 16-lane group
  // lane 4q+p supplies row q and columns 4p..4p+3 of its 16-column block
  const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  auto compute = [&](const char* buf) {
    const char* xb = buf + kSBV * 128;
#pragma unroll 4
    for (int k0 = 0; k0 < boxvol; k0 += 16) {
      const int v_a = k0 + 8 * hsel + qq;
      s16x8_t a[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const int co = ct * 32 + g * 16 + pp * 4;
        s16x4_t lo = tr_read(buf, dy_off_bf16(v_a, co)), hi = tr_read(buf, dy_off_bf16(v_a + 4, co));
        a[ct] = (s16x8_t){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      // with a compile-time box of width >= 16 the lane's rows share (rd, rh) with k0
        const int hr0 = LBW >= 4 ? halo_row(k0) + 8 * hsel + qq : halo_row(v_a);
        const int hr1 = LBW >= 4 ? hr0 + 4 : halo_row(v_a + 4);
#pragma unroll
      for (int js = 0; js < 2; ++js) {
        if (js >= nj) break;
        const int jt = js ? jt1 : jt0;
        // column block of this lane group: 16 columns = taps 4 jt + 2 g, +1; lane: tap + (pp >> 1), ch 4 (pp & 1)
        const int tap = 4 * jt + 2 * g + (pp >> 1);
        const int off = tap_off(tap, HH, HW);
        const int cb = (pp & 1) * 8;  // byte offset of channels 4..7
        s16x4_t lo = tr_read(xb, (hr0 + off) * 16 + cb), hi = tr_read(xb, (hr1 + off) * 16 + cb);
        s16x8_t bfr = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct][js] = mfma(a[ct], bfr, acc[ct][js]);
      }
    }
  };
  if (b_beg < b_end) {
    stage_load(b_beg);
    stage_store(slds);
    __syncthreads();
    for (int b = b_beg; b < b_end; ++b) {
      const int cur = (b - b_beg) & 1;
      if (b + 1 < b_end) stage_load(b + 1);
      compute(slds + cur * kSBuf);
      if (b + 1 < b_end) stage_store(slds + (cur ^ 1) * kSBuf);
      __syncthreads();
    }
  }
  // flush: C tile -> LDS [co][t][c] (fp32), then coalesced atomics into dw[co][c][t]
  __syncthreads();
  float* red = reinterpret_cast<float*>(slds);  // 64 x 28 x 8 floats = 56 KiB
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int js = 0; js < 2; ++js) {
      if (js >= nj) continue;
      const int jt = js ? jt1 : jt0;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int co = ct * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
        const int j = jt * 32 + (lane & 31);  // column = 8 t + c
        red[co * 224 + j] = acc[ct][js][e];
      }
    }
  __syncthreads();
  const int total = 64 * cin_w * 27;
  for (int i = tid; i < total; i += 256) {
    const int t = i % 27, c = (i / 27) % cin_w, co = i / (27 * cin_w);
    atomicAdd(dw + i, red[co * 224 + t * 8 + c]);
  }
}

// Streaming stem weight gradient (the HBM-bound hot case: D % 4 == H % 4 == W % 16 == 0).
// dW[co][c][t] = sum_v dy[v][co] x[v + t][c]: GEMM with M = 64 co, N = 224 (tap, channel)
// columns, K = voxels.  Persistent: one 4-wave workgroup per CU walks 4x4x16 voxel boxes
// b = blockIdx.x + k gridDim.x.  Each box's dy tile (256 voxels x 128 B) and x halo
// (6x6x18 rows x 16 B) arrive by buffer LDS-DMA (inline asm, see dma16) into a 3-slot ring:
// two boxes in flight while one computes, counted vmcnt + raw s_barrier, every source
// offset a per-thread constant + the box base.  Wave w owns k-steps w, w + 4, w + 8, w + 12
// of every box and ALL 14 output tiles (2 co x 7 column tiles, accumulators in AGPRs), so
// each A / B fragment is read from LDS exactly once per box (ds_read_b64_tr_b16 transposes
// both operands) and the next k-step's fragments are read during this one's 14 MFMAs.
// Flush: one fp32 partial row [64][cin_w][27] per workgroup (plain stores), summed into dw
// by stem_wgrad_reduce_kernel (deterministic, no atomics).
constexpr int kSWT = 256;                                  // 4 waves, one per SIMD
// BD = box depth (boxes BD x 4 x 16), NS = ring slots (NS - 1 boxes in flight).  The load
// pipeline is latency-bound (bytes in flight per CU), so the product ring uses 2-deep boxes
// in 6 slots (115 KB in flight) rather than 4-deep boxes in 3 slots (86 KB).
template <int BD> struct SWGeom {
  static constexpr int BV = BD * 64;                            // voxels per box
  static constexpr int HV = (BD + 2) * 6 * 18;                  // halo rows (16 B)
  static constexpr int HRows = (HV + 63) / 64 * 64;             // rows written
  static constexpr int Buf = BV * 128 + HRows * 16;             // bytes per ring slot
  static constexpr int DYP = BV * 8 / kSWT;                     // dy DMA pieces per thread
  static constexpr int XI = (HRows / 64 + 3) / 4;               // halo DMA rounds per wave
};
constexpr int kSWBD = (PCMS_ABL & 4096) ? 2 : 4;  // 2-deep x 6 slots measured slower
constexpr int kSWNS = kSWBD == 4 ? 3 : 6;
constexpr int kSWLds = kSWNS * SWGeom<kSWBD>::Buf;
static_assert(kSWLds >= 64 * 224 * 4, "flush tile fits in the ring");
static_assert(kSWLds <= 160 * 1024, "ring fits in LDS");

template <int BD, int NS>
__global__ void __launch_bounds__(kSWT, 1) stem_wgrad_stream_kernel(const bf16_t* x, const bf16_t* dy, float* part,
                                                                    int N, int D, int H, int W, int cin_w,
                                                                    uint32_t xbytes, uint32_t dybytes) {
  typedef SWGeom<BD> Gm;
  constexpr int BH = 4, BW = 16, HH = BH + 2, HW = BW + 2;
  constexpr int kSWBV = Gm::BV, kSWHV = Gm::HV, kSWBuf = Gm::Buf;
  extern __shared__ __attribute__((aligned(16))) char swl[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hsel = lane >> 5;
  const int nbw = W / BW, nbh = H / BH, nbd = D / BD;
  const int nbox = N * nbd * nbh * nbw;
  const i32x4_t xr = buffer_desc(x, xbytes);
  const i32x4_t dr = buffer_desc(dy, dybytes);

  // per-thread DMA source offsets relative to the box origin (constant over boxes)
  uint32_t dyrel[Gm::DYP];
#pragma unroll
  for (int i = 0; i < Gm::DYP; ++i) {
    const int pc = tid + i * kSWT;
    const int r = pc >> 3, q = pc & 7;
    const int ql = q ^ (((r >> 1) & 1) << 2);  // dy_off_bf16: 64-B halves swapped on odd row pairs
    const int rd = r >> 6, rh = (r >> 4) & 3, rw = r & 15;
    dyrel[i] = (uint32_t)(((rd * H + rh) * W + rw) * 128 + ql * 16);
  }
  // halo pieces of this wave: rows wave*64 + lane + 256 i < HRows (XI or XI - 1 of them)
  const int nxp = (Gm::HRows / 64 - wave + 3) / 4;
  int xrel[Gm::XI], xco[Gm::XI];
#pragma unroll
  for (int i = 0; i < Gm::XI; ++i) {
    const int hv = wave * 64 + lane + i * kSWT;
    const int hw_ = hv % HW, t_ = hv / HW, hh_ = t_ % HH, hd_ = t_ / HH;
    xrel[i] = (((hd_ - 1) * H + (hh_ - 1)) * W + (hw_ - 1)) * 16;
    xco[i] = hv < kSWHV ? (hd_ | (hh_ << 8) | (hw_ << 16)) : -1;
  }
  auto origin = [&](int b, int& n, int& d0, int& h0, int& w0) {
    int q = b;
    const int bwi = q % nbw; q /= nbw;
    const int bhi = q % nbh; q /= nbh;
    const int bdi = q % nbd;
    n = q / nbd;
    d0 = bdi * BD; h0 = bhi * BH; w0 = bwi * BW;
  };
  auto stage = [&](int b, int slot) {
    int n, d0, h0, w0;
    origin(b, n, d0, h0, w0);
    const int vb = ((n * D + d0) * H + h0) * W + w0;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_addr(swl) + slot * kSWBuf + wave * 64 * 16);
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)vb * 128u);
#pragma unroll
    for (int i = 0; i < Gm::DYP; ++i) dma16(dr, lb + i * kSWT * 16, dyrel[i], so);
    const bool inner = d0 >= 1 && d0 + BD < D && h0 >= 1 && h0 + BH < H && w0 >= 1 && w0 + BW < W;
#pragma unroll
    for (int i = 0; i < Gm::XI; ++i) {
      if (i >= nxp) break;
      uint32_t voff = (uint32_t)(vb * 16 + xrel[i]);
      const int c = xco[i];
      if (c < 0) {
        voff = kOOB;
      } else if (!inner) {
        const int gd = d0 + (c & 255) - 1, gh = h0 + ((c >> 8) & 255) - 1, gw = w0 + (c >> 16) - 1;
        if ((unsigned)gd >= (unsigned)D || (unsigned)gh >= (unsigned)H || (unsigned)gw >= (unsigned)W) voff = kOOB;
      }
      dma16(xr, lb + kSWBV * 128 + i * kSWT * 16, voff, 0);
    }
  };

  const int g = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  f32x16_t acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // lane offsets of the tr reads, with the wave's k-step offset folded in (k-step s = wave +
  // 4 i is box row (rd = i, rh = wave): dy rows at s * 2048, halo rows at (i HH + wave) HW)
  const int aoff0 = dy_off_bf16(8 * hsel + qq, g * 16 + pp * 4) + wave * 2048;
  const int aoff1 = dy_off_bf16(8 * hsel + qq, 32 + g * 16 + pp * 4) + wave * 2048;
  int boff[7];  // column tile j: taps 4 j + 2 g + (pp >> 1), channels 4 (pp & 1) .. + 3
#pragma unroll
  for (int j = 0; j < 7; ++j)
    boff[j] = kSWBV * 128 + (8 * hsel + qq + tap_off(4 * j + 2 * g + (pp >> 1), HH, HW) + wave * HW) * 16 + (pp & 1) * 8;
  auto compute = [&](const char* buf) {
    uint32_t pa0 = lds_addr(buf) + aoff0, pa1 = lds_addr(buf) + aoff1, pb[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) pb[j] = lds_addr(buf) + boff[j];
    asm volatile("" : "+v"(pa0), "+v"(pa1), "+v"(pb[0]), "+v"(pb[1]), "+v"(pb[2]), "+v"(pb[3]), "+v"(pb[4]),
                 "+v"(pb[5]), "+v"(pb[6]));
    auto tr = [](uint32_t p, int off) {
      return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4_t*)(uintptr_t)(p + off));
    };
    auto cat = [](s16x4_t lo, s16x4_t hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); };
    auto load = [&](int i, s16x8_t (&a)[2], s16x8_t (&bq)[7]) {
      const int dyb = i * 4 * 2048;
      const int hrb = i * HH * HW * 16;
      a[0] = cat(tr(pa0, dyb), tr(pa0, dyb + 512));
      a[1] = cat(tr(pa1, dyb), tr(pa1, dyb + 512));
#pragma unroll
      for (int j = 0; j < 7; ++j) bq[j] = cat(tr(pb[j], hrb), tr(pb[j], hrb + 64));
    };
    s16x8_t a[2][2], bq[2][7];
    load(0, a[0], bq[0]);
#pragma unroll
    for (int i = 0; i < BD; ++i) {
      if (i + 1 < BD) load(i + 1, a[(i + 1) & 1], bq[(i + 1) & 1]);
#pragma unroll
      for (int j = 0; j < 7; ++j)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) acc[ct][j] = mfma(a[i & 1][ct], bq[i & 1][j], acc[ct][j]);
    }
  };

  const int G = gridDim.x;
  int b = blockIdx.x;
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (b + k * G < nbox) stage(b + k * G, k);
  for (int it = 0; b < nbox; b += G, ++it) {
    // retire box b's DMA (the NS - 2 boxes after it may stay in flight), then barrier:
    // every wave's share of box b has landed and every wave is done reading the slot
    // refilled below
    if (b + (NS - 2) * G < nbox) {
      if (nxp == Gm::XI) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (Gm::DYP + Gm::XI)) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 2) * (Gm::DYP + Gm::XI - 1)) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int b2 = b + (NS - 1) * G;
    if (b2 < nbox) stage(b2, (it + NS - 1) % NS);
    compute(swl + (it % NS) * kSWBuf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // flush: the 4 waves' partial tiles summed in LDS [co][224 cols] (fixed order)
  float* red = reinterpret_cast<float*>(swl);
  for (int pass = 0; pass < 4; ++pass) {
    if (wave == pass) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int j = 0; j < 7; ++j)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int co = ct * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
            float* dst = red + co * 224 + j * 32 + (lane & 31);
            if (pass == 0) *dst = acc[ct][j][e];
            else *dst += acc[ct][j][e];
          }
    }
    __syncthreads();
  }
  const int total = 64 * cin_w * 27;
  float* prow = part + (long)blockIdx.x * total;
  for (int i = tid; i < total; i += kSWT) {
    const int t = i % 27, c = (i / 27) % cin_w, co = i / (27 * cin_w);
    prow[i] = red[co * 224 + t * 8 + c];
  }
}

// dw[o] += sum over the workgroup partial rows (fixed order).  Block = 32 outputs x 8 row
// groups: 32 independent 128-B row segments in flight per thread group, LDS combine.
__global__ void __launch_bounds__(256) stem_wgrad_reduce_kernel(const float* part, int rows, int total, float* dw) {
  __shared__ float red[8][32];
  const int ol = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int o = blockIdx.x * 32 + ol;
  float s = 0.f;
  if (o < total) {
#pragma unroll 8
    for (int r = rg; r < rows; r += 8) s += part[(long)r * total + o];
  }
  red[rg][ol] = s;
  __syncthreads();
  if (rg == 0 && o < total) {
    float t = 0.f;
#pragma unroll
    for (int g2 = 0; g2 < 8; ++g2) t += red[g2][ol];
    dw[o] += t;
  }
}

// ------------------------------------------------------------------------------------
// Big-box forward / dgrad (bf16; the level-0/1 hot case: D % 8 == H % 8 == 0, W % 16 == 0,
// input channels in 16-channel chunks).  One 4-wave workgroup per CU computes an
// 8 x 8 x 16 = 1024-voxel box x 64 output channels.  Wave w owns voxel rows
// [256 w, 256 w + 256) = 8 M-tiles, so every B fragment (weights, L2-resident) feeds 8 MFMAs,
// half the weight traffic per MFMA of conv3_fwd_kernel.  The 10 x 10 x 18 halo of a chunk
// (32-B rows; the two 16-B halves swapped on odd row octets, so 16 consecutive rows hit 16
// distinct bank groups) is double-buffered: the next chunk's halo streams in by buffer
// LDS-DMA, one piece per thread and tap over the first 15 taps of the current chunk, and A
// fragments of tap t + 1 are read while tap t's 16 MFMAs run.  Output columns are channel
// pairs (column j of N-tile nt = channel 2 j + nt): each accumulator register pair stores as
// one packed bf16x2, a store instruction writes two 128-B voxel rows.  BatchNorm partials:
// one stats row per box (sum, M2 about the row mean; counts after the [rows][Cout][2] block).
// ------------------------------------------------------------------------------------
constexpr int kBgThreads = 256;
constexpr int kBgHH = 10, kBgHW = 18;
// BD = box depth: 8 (1024 voxels, 8 M-tiles per wave, one workgroup per CU) or 4 (512
// voxels, 4 M-tiles per wave, two workgroups per CU that cover each other's prologue,
// chunk barriers and store tail)
template <int BD> struct BgGeom {
  static constexpr int MT = BD;                                           // M-tiles per wave
  static constexpr int Halo = (BD + 2) * kBgHH * kBgHW;                   // rows x 32 B
  static constexpr int Pieces = (2 * Halo + kBgThreads - 1) / kBgThreads; // DMA pieces / thread
  static constexpr int Buf = Pieces * kBgThreads * 16;                    // (tail pad)
  static constexpr int Lds = 2 * Buf + 4 * 64 * 3 * 4;                    // + stats merge
  static constexpr int PerCU = BD == 8 ? 1 : 2;
  static constexpr int Dist = BD == 8 ? 8 : 2;  // B prefetch distance (taps); (Dist + 1) | 27
  static_assert(27 % (Dist + 1) == 0, "B ring index must continue across chunks");
};
constexpr int kBgBD = (PCMS_ABL & 1024) ? 4 : 8;  // product box depth (depth 4 measured slower)

// hidden 16-B global load (the compiler's waitcnt pass does not count it): retired by
// vm_wait2<N>, which also orders the register's readers after the wait
__device__ __forceinline__ void gload16(s16x8_t& dst, const void* ptr) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst) : "v"(ptr) : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait2(s16x8_t& a, s16x8_t& b) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F> __device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
// vector-memory ops issued after B(t)'s second load by the time tap t waits for it: every
// tap s issues B(s + D) x 2 then piece(s) (s < 15, chunk-relative, every chunk alike)
template <int P> constexpr int bg_piece(int s) { return ((s % 27) + 27) % 27 < P ? 1 : 0; }
template <int P, int Dist> constexpr int bg_wait(int t) {
  int n = bg_piece<P>(t - Dist);
  for (int s = t - Dist + 1; s <= t; ++s) n += 2 + bg_piece<P>(s);
  return n;
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }


template <int BD>
__global__ void __launch_bounds__(kBgThreads, BgGeom<BD>::PerCU) conv3_fwd_big_kernel(Conv3Params p, uint32_t x0bytes,
                                                                                     uint32_t x1bytes) {
  typedef BgGeom<BD> Gm;
  constexpr int MT = Gm::MT;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r_lane = lane & 31, hsel = lane >> 5;
  const int Cout = p.Cout, ncob = Cout >> 6;
  // logical workgroup id: consecutive ids on one XCD (dispatch is round-robin over 8), output
  // channel block fastest, so the workgroups sharing a halo (and neighbouring boxes) share L2
  const int G = gridDim.x;
  const int lg = (G & 7) == 0 ? (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int cob = lg % ncob, box = lg / ncob, nbox = G / ncob;
  int q = box;
  const int bwi = q % p.nbw; q /= p.nbw;
  const int bhi = q % p.nbh; q /= p.nbh;
  const int bdi = q % p.nbd;
  const int n = q / p.nbd;
  const int d0 = bdi * BD, h0 = bhi * 8, w0 = bwi * 16;
  const int co_base = cob * 64;

  // this thread's halo pieces: (voxel << 1 | logical 16-B half), -1 = zero (padding, tail)
  int pv[Gm::Pieces];
#pragma unroll
  for (int j = 0; j < Gm::Pieces; ++j) {
    const int pc = tid + j * kBgThreads;
    const int hv = pc >> 1;
    int e = -1;
    if (hv < Gm::Halo) {
      const int hw_ = hv % kBgHW, t_ = hv / kBgHW, hh_ = t_ % kBgHH, hd_ = t_ / kBgHH;
      const int gd = d0 + hd_ - 1, gh = h0 + hh_ - 1, gw = w0 + hw_ - 1;
      if ((unsigned)gd < (unsigned)p.D && (unsigned)gh < (unsigned)p.H && (unsigned)gw < (unsigned)p.W)
        e = ((((n * p.D + gd) * p.H + gh) * p.W + gw) << 1) | ((pc & 1) ^ ((hw_ >> 3) & 1));
    }
    pv[j] = e;
  }
  const i32x4_t xr0 = buffer_desc(p.x0, x0bytes);
  const i32x4_t xr1 = buffer_desc(p.x1 ? p.x1 : p.x0, x1bytes);
  const uint32_t lds0 = lds_addr(lds);
  // live = false (past the last chunk): the piece is still issued (the vmcnt arithmetic is
  // the same for every chunk) but reads out of range = zeros into the idle buffer
  auto stage_piece = [&](int chunk, int buf, int j, bool live) {
    const int c = chunk * 16;
    const bool first = c < p.c0;  // workgroup-uniform: the chunk lies in x0 or in x1
    const uint32_t stride = first ? p.c0 : p.c1;
    const uint32_t cofs = first ? c : c - p.c0;
    const int e = pv[j];
    const uint32_t voff = (e < 0 || !live) ? kOOB
                                           : ((uint32_t)(e >> 1) * stride + cofs + (uint32_t)(e & 1) * 8u) * 2u;
    const uint32_t lb = __builtin_amdgcn_readfirstlane(lds0 + buf * Gm::Buf + (wave * 64 + j * kBgThreads) * 16);
    dma16(first ? xr0 : xr1, lb, voff, 0);
  };

  // A fragment byte offsets in a halo buffer: MFMA row r = 256 wave + 32 mt + perm32(lane)
  // is box voxel (2 wave + mt / 4, 2 (mt % 4) + prow / 16, prow % 16).  The half swizzle
  // depends on the halo w coordinate only, so for each kw the (kd, kh) part of a tap is a
  // constant row offset (kd * 10 + kh) * 18 * 32 bytes folded into the ds_read immediate.
  const int prow = perm32(r_lane);
  int hb32[MT], swk[3];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int rd = (BD / 4) * wave + (mt >> 2), rh = 2 * (mt & 3) + (prow >> 4);
    hb32[mt] = ((rd * kBgHH + rh) * kBgHW + (prow & 15)) * 32;
  }
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) swk[kw] = kw * 32 + ((hsel ^ ((((prow & 15) + kw) >> 3) & 1)) << 4);
  // B fragment: packed [Cin/32][27][Cout][32]; 16-channel chunk c = half (c & 1) of c >> 1
  // B fragments (weights, packed [Cin/32][27][Cout][32]; 16-channel chunk c = half c & 1 of
  // 32-chunk c >> 1) come through hidden loads Dist taps ahead: vector-memory returns are
  // in order, so a wait on B(t) also retires every halo piece issued before it; the pieces
  // get >= Dist taps to arrive from HBM before anything waits on them.
  const bf16_t* wp = (const bf16_t*)p.w;
  const int nchunk = p.Cin >> 4;
  auto load_b = [&](s16x8_t (&dst)[2], int chunk, int tap) {
    chunk = min(chunk, nchunk - 1);  // past the last chunk: a harmless reload (fixed counts)
    const bf16_t* wt = wp + ((long)((chunk >> 1) * 27 + tap) * Cout + co_base + 2 * r_lane) * 32 + (chunk & 1) * 16 +
                       hsel * 8;
    gload16(dst[0], wt);
    gload16(dst[1], wt + 32);
  };

  f32x16_t acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

#pragma unroll
  for (int j = 0; j < Gm::Pieces; ++j) stage_piece(0, 0, j, true);
  s16x8_t bset[Gm::Dist + 1][2];
#pragma unroll
  for (int t = 0; t < Gm::Dist; ++t) load_b(bset[t], 0, t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int chunk = 0; chunk < nchunk; ++chunk) {
    const int buf = chunk & 1;
    const bool more = chunk + 1 < nchunk;
    const char* hl = lds + buf * Gm::Buf;
    auto read_a = [&](s16x8_t (&dst)[MT], int tap) {
      const int kd = tap / 9, kh = (tap / 3) % 3, kw = tap % 3;
      const char* base = hl + swk[kw] + (kd * kBgHH + kh) * kBgHW * 32;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) dst[mt] = *reinterpret_cast<const s16x8_t*>(base + hb32[mt]);
    };
    s16x8_t a[2][MT];
    read_a(a[0], 0);
    // per tap: B(tap + D) (the set index runs on across chunks: (D + 1) | 27), one halo piece
    // of the next chunk (taps < 15), A of tap + 1; wait for B(tap); this tap's 16 MFMAs
    static_for<27>([&](auto tc) {
      constexpr int tap = decltype(tc)::value;
      constexpr int tn = tap + Gm::Dist;
      if constexpr (!(PCMS_ABL & 64)) {
        if constexpr (tn < 27) load_b(bset[tn % (Gm::Dist + 1)], chunk, tn);
        else load_b(bset[tn % (Gm::Dist + 1)], chunk + 1, tn - 27);
      }
      if constexpr (tap < Gm::Pieces && !(PCMS_ABL & 32)) stage_piece(chunk + 1, buf ^ 1, tap, more);
      constexpr int cur = tap & 1;
      if constexpr (tap + 1 < 27) {
        if constexpr (!(PCMS_ABL & 256)) read_a(a[cur ^ 1], tap + 1);
        else if constexpr (tap == 0) read_a(a[1], 1);
      }
      s16x8_t(&b)[2] = bset[tap % (Gm::Dist + 1)];
      if constexpr (!(PCMS_ABL & 128)) vm_wait2<bg_wait<Gm::Pieces, Gm::Dist>(tap)>(b[0], b[1]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(a[cur][mt], b[nt], acc[mt][nt]);
    });
    // the next chunk's halo has landed (the newest piece is followed by the B loads of the
    // remaining taps) and every wave is done with buf; after the last chunk retire everything
    if (more) vm_wait<2 * (27 - Gm::Pieces)>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: + bias, packed channel-pair stores (two-pointer output split at cy0)
  const int cpair = co_base + 2 * r_lane;
  float bias0 = 0.f, bias1 = 0.f;
  if (p.bias) {
    bias0 = p.bias[cpair];
    bias1 = p.bias[cpair + 1];
  }
  const bool to0 = co_base < p.cy0;
  bf16_t* yb = to0 ? (bf16_t*)p.y0 : (bf16_t*)p.y1;
  const long ys = to0 ? p.cy0 : Cout - p.cy0;
  const int yc = to0 ? cpair : cpair - p.cy0;
  const long plane = (long)p.H * p.W;
  const long vbase = (((long)n * p.D + d0) * p.H + h0) * p.W + w0;
  float s1[2] = {0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int pr = perm32((e & 3) + 8 * (e >> 2) + 4 * hsel);
    const long vrow = vbase + (long)(pr >> 4) * p.W + (pr & 15);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int rd = (BD / 4) * wave + (mt >> 2), rh = 2 * (mt & 3);
      const long vox = vrow + (long)rd * plane + (long)rh * p.W;
      const float v0 = acc[mt][0][e] + bias0, v1 = acc[mt][1][e] + bias1;
      if (!(PCMS_ABL & 512)) *reinterpret_cast<uint32_t*>(yb + vox * ys + yc) = pack_bf16x2(v0, v1);
      s1[0] += v0;
      s1[1] += v1;
    }
  }
  if (!p.stats) return;
  // BatchNorm partials: per-wave mean, squared deviations about it (corrected by
  // (sum d)^2 / n), Chan merge over the 4 waves
  constexpr float nw = 32.f * MT;
  float mw[2], s2[2] = {0.f, 0.f}, sd[2] = {0.f, 0.f};
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s1[nt] += __shfl_xor(s1[nt], 32, 64);
    mw[nt] = s1[nt] / nw;
  }
  const float sh[2] = {bias0 - mw[0], bias1 - mw[1]};  // d = acc + bias - mean
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int e = 0; e < 16; ++e)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const float d = acc[mt][nt][e] + sh[nt];
        s2[nt] = fmaf(d, d, s2[nt]);
        sd[nt] += d;
      }
  float* red = reinterpret_cast<float*>(lds + 2 * Gm::Buf);
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) {
    s2[nt] += __shfl_xor(s2[nt], 32, 64);
    sd[nt] += __shfl_xor(sd[nt], 32, 64);
    s2[nt] -= sd[nt] * sd[nt] / nw;
    if (hsel == 0) {
      float* rp = red + (wave * 64 + 2 * r_lane + nt) * 3;
      rp[0] = s1[nt];
      rp[1] = s2[nt];
      rp[2] = nw;
    }
  }
  __syncthreads();
  if (tid < 64) {
    float S = 0.f, Nn = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      S += red[(w * 64 + tid) * 3];
      Nn += red[(w * 64 + tid) * 3 + 2];
    }
    const float m = S / Nn;
    float M2 = 0.f, sdd = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float c = red[(w * 64 + tid) * 3 + 2];
      const float d = red[(w * 64 + tid) * 3] / c - m;
      M2 += red[(w * 64 + tid) * 3 + 1] + c * d * d;
      sdd += c * d;
    }
    M2 -= sdd * sdd / Nn;
    float* st = p.stats + ((long)box * Cout + co_base + tid) * 2;
    st[0] = S;
    st[1] = M2;
    if (tid == 0 && cob == 0) p.stats[(long)nbox * Cout * 2 + box] = Nn;
  }
}

}  // namespace

// big-box forward: bf16, whole 8x8x16 boxes, 16-channel chunks of both sources, enough boxes
// to give every CU one (pcms_conv3_big_min_boxes), every byte offset inside a 32-bit voffset
static int g_big_min_boxes = 256;
static bool big_fwd_ok(int dtype, int N, int D, int H, int W, int c0, int c1) {
  if (dtype != PCMS_BF16 || D % kBgBD || H % 8 || W % 16 || c0 % 16 || c1 % 16 || c0 < 16) return false;
  const long nvox = (long)N * D * H * W;
  if ((long)N * (D / kBgBD) * (H / 8) * (W / 16) < g_big_min_boxes) return false;
  return nvox < (1L << 30) && nvox * std::max(c0, c1) * 2 < (long)kOOB;
}

extern "C" {

// Returns the m-block count (workgroups along M) of the general fwd kernel for a grid
// (an upper bound on every fwd path's BatchNorm row count; sizes the split decision).
int pcms_conv3_mblocks(int N, int D, int H, int W) {
  Box b = fwd_box(D, H, W);
  return N * cdiv(D, 1 << b.lbd) * cdiv(H, 1 << b.lbh) * cdiv(W, 1 << b.lbw);
}

// BatchNorm partial rows an unsplit pcms_conv3_fwd with these sources writes
int pcms_conv3_fwd_rows(int dtype, int N, int D, int H, int W, int c0, int c1) {
  if (big_fwd_ok(dtype, N, D, H, W, c0, c1)) return N * (D / kBgBD) * (H / 8) * (W / 16);
  return pcms_conv3_mblocks(N, D, H, W);
}

// Minimum box count for the big-box forward (tests lower it to reach small grids);
// v <= 0 only queries.  Returns the previous value.
int pcms_conv3_big_min_boxes(int v) {
  const int old = g_big_min_boxes;
  if (v > 0) g_big_min_boxes = v;
  return old;
}

int pcms_conv3_chunk(int dtype) { return dtype == PCMS_BF16 ? Traits<bf16_t>::CK : Traits<float>::CK; }

// forward and dgrad packs together (one weight read); other shapes / dtypes: the two packs
int pcms_conv3_pack2(int dtype, const float* w, void* fwd, void* dgrad, int Cout, int Cin, hipStream_t s) {
  if (dtype == PCMS_BF16 && Cin % 32 == 0 && Cout % 32 == 0) {
    hipLaunchKernelGGL(pack_conv3_bf16_both_kernel, dim3(Cout / 32, Cin / 32), dim3(256), 0, s, w, (bf16_t*)fwd,
                       (bf16_t*)dgrad, Cout, Cin);
    PCMS_CHECK_LAUNCH();
  }
  const int rc = pcms_conv3_pack(dtype, w, fwd, Cout, Cin, 0, s);
  return rc ? rc : pcms_conv3_pack(dtype, w, dgrad, Cout, Cin, 1, s);
}

int pcms_conv3_pack(int dtype, const float* w, void* out, int Cout, int Cin, int flip, hipStream_t s) {
  const int CK = pcms_conv3_chunk(dtype);
  const int J = flip ? Cin : Cout;
  const int Kdim = flip ? Cout : Cin;
  dim3 grid(cdiv(J, 8), cdiv(Kdim, CK));
  if (dtype == PCMS_BF16 && Kdim % 32 == 0 && J % 8 == 0)
    hipLaunchKernelGGL(pack_conv3_bf16_kernel, grid, dim3(256), 0, s, w, (bf16_t*)out, Cout, Cin, flip);
  else if (dtype == PCMS_BF16)
    hipLaunchKernelGGL((pack_conv3_kernel<bf16_t, 32>), grid, dim3(256), 0, s, w, (bf16_t*)out, Cout, Cin, flip);
  else
    hipLaunchKernelGGL((pack_conv3_kernel<float, 16>), grid, dim3(256), 0, s, w, (float*)out, Cout, Cin, flip);
  PCMS_CHECK_LAUNCH();
}

// Forward (or dgrad) 3x3x3 conv. See Conv3Params.  splits > 1: fp32 atomic accumulate
// into yacc (caller zeroes it; bias/stats/conversion then done by pcms_conv3_split_epilogue).
int pcms_conv3_fwd(int dtype, const void* x0, int c0, const void* x1, int c1,
                   const void* wpack, const float* bias, void* y0, void* y1, int cy0,
                   float* yacc, float* stats, int accumulate,
                   int N, int D, int H, int W, int Cout, int splits, hipStream_t s) {
  const int Cin = c0 + c1;
  const int CK = pcms_conv3_chunk(dtype);
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (Cout % 64 != 0 || c0 % VEC != 0 || c1 % VEC != 0 || (c1 > 0 && x1 == nullptr)) return -1;
  if (stats && accumulate) return -6;  // BN statistics describe a fresh output only
  if (y1 == nullptr) cy0 = Cout;
  if (cy0 % 64 != 0 && cy0 != Cout) return -2;
  Box b = fwd_box(D, H, W);
  Conv3Params p;
  p.x0 = x0; p.x1 = x1; p.c0 = c0; p.c1 = c1;
  p.w = wpack; p.bias = bias; p.y0 = y0; p.y1 = y1; p.cy0 = cy0;
  p.yacc = splits > 1 ? yacc : nullptr;
  p.stats = stats; p.accumulate = accumulate;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
  p.nchunk = cdiv(Cin, CK);
  if (splits < 1) splits = 1;
  if (splits > p.nchunk) splits = p.nchunk;
  p.chunks_per_split = cdiv(p.nchunk, splits);
  splits = cdiv(p.nchunk, p.chunks_per_split);
  if (splits > 1 && yacc == nullptr) return -3;
  p.lbd = b.lbd; p.lbh = b.lbh; p.lbw = b.lbw;
  p.nbd = cdiv(D, 1 << b.lbd); p.nbh = cdiv(H, 1 << b.lbh); p.nbw = cdiv(W, 1 << b.lbw);
  if (splits > 1) p.yacc = yacc;
  if (splits == 1 && !accumulate && big_fwd_ok(dtype, N, D, H, W, c0, c1)) {
    p.nbd = D / kBgBD; p.nbh = H / 8; p.nbw = W / 16;
    const int nbox = N * p.nbd * p.nbh * p.nbw;
    const long nvox = (long)N * D * H * W;
    constexpr int lds = BgGeom<kBgBD>::Lds;
    (void)hipFuncSetAttribute((const void*)conv3_fwd_big_kernel<kBgBD>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(conv3_fwd_big_kernel<kBgBD>, dim3(nbox * (Cout / 64)), dim3(kBgThreads), lds, s, p,
                       (uint32_t)(nvox * c0 * 2), (uint32_t)(nvox * c1 * 2));
    PCMS_CHECK_LAUNCH();
  }
  dim3 grid(N * p.nbd * p.nbh * p.nbw, Cout / 64, splits);
  const bool hot = b.lbd == 2 && b.lbh == 3 && b.lbw == 4;
  if (dtype == PCMS_BF16) {
    if (hot) hipLaunchKernelGGL((conv3_fwd_kernel<bf16_t, 2, 2, 3, 4>), grid, dim3(kThreads), 0, s, p);
    else hipLaunchKernelGGL((conv3_fwd_kernel<bf16_t, 2, -1, -1, -1>), grid, dim3(kThreads), 0, s, p);
  } else {
    hipLaunchKernelGGL((conv3_fwd_kernel<float, 1, -1, -1, -1>), grid, dim3(kThreads), 0, s, p);
  }
  PCMS_CHECK_LAUNCH();
}


// ---- stem (inc.conv.0), bf16: dedicated HBM-bound kernels ----
int pcms_stem_pack(const float* w, void* out, int cin_w, hipStream_t s) {
  if (cin_w > 8) return -1;
  hipLaunchKernelGGL(stem_pack_kernel, dim3(cdiv(kStemSteps * 64 * 16, 256)), dim3(256), 0, s, w, (bf16_t*)out, cin_w);
  PCMS_CHECK_LAUNCH();
}
int pcms_stem_pack_elems(void) { return kStemSteps * 64 * 16; }

static int device_cus();
// the wave-independent stem forward measured slower than the direct kernel (110 vs 97 us at
// config 2): kept for tuning behind an ablation switch
static bool stem_fwd_wave_shape(int N, int D, int H, int W) {
  return (PCMS_ABL & 2048) && D % 2 == 0 && H % 2 == 0 && W % 16 == 0 && (long)N * D * H * W * 128 < (long)kOOB;
}
static int stem_fwd_wave_grid(int N, int D, int H, int W) {
  const long nwb = (long)N * (D / 2) * (H / 2) * (W / 16);
  return (int)std::max(1L, std::min((long)device_cus(), (nwb + 7) / 8));
}

// BatchNorm statistics rows pcms_stem_fwd writes
int pcms_stem_fwd_rows(int N, int D, int H, int W) {
  if (stem_fwd_wave_shape(N, D, H, W)) return stem_fwd_wave_grid(N, D, H, W);
  return pcms_conv3_mblocks(N, D, H, W);
}

// x: (N, D, H, W, 8) bf16; y: (N, D, H, W, 64) bf16; stats rows = pcms_stem_fwd_rows
int pcms_stem_fwd(const void* x, const void* wpack, const float* bias, void* y, float* stats,
                  int N, int D, int H, int W, hipStream_t s) {
  Box b = fwd_box(D, H, W);
  Conv3Params p;
  p.x0 = x; p.x1 = nullptr; p.c0 = 8; p.c1 = 0;
  p.w = wpack; p.bias = bias; p.y0 = y; p.y1 = nullptr; p.cy0 = 64;
  p.yacc = nullptr; p.stats = stats; p.accumulate = 0;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = 8; p.Cout = 64;
  p.nchunk = 1; p.chunks_per_split = 1;
  p.lbd = b.lbd; p.lbh = b.lbh; p.lbw = b.lbw;
  p.nbd = cdiv(D, 1 << b.lbd); p.nbh = cdiv(H, 1 << b.lbh); p.nbw = cdiv(W, 1 << b.lbw);
  const int nbox = N * p.nbd * p.nbh * p.nbw;
  if ((1 << (b.lbd + b.lbh + b.lbw)) > 512) return -5;
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const long xbytes = (long)N * D * H * W * 16, ybytes = (long)N * D * H * W * 128;
  if (stem_fwd_wave_shape(N, D, H, W)) {
    const int grid = stem_fwd_wave_grid(N, D, H, W);
    (void)hipFuncSetAttribute((const void*)stem_fwd_wave_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kSWvLds);
    hipLaunchKernelGGL(stem_fwd_wave_kernel, dim3(grid), dim3(kSWvThreads), kSWvLds, s, (const bf16_t*)x,
                       (const bf16_t*)wpack, bias, (bf16_t*)y, stats, N, D, H, W, (uint32_t)xbytes, (uint32_t)ybytes);
    PCMS_CHECK_LAUNCH();
  }
  const bool direct = b.lbw == 4 && b.lbd + b.lbh == 5 && (b.lbd == 2 || b.lbd == 3) && ybytes < (long)kOOB;
  if (direct) {
    const int grid = std::min(nbox, ncu);
    // store-pipelined variant unless PCMS_STEM_FWD_PIPE=0 (A/B switch for the measurements)
    // 0: plain stores after the MFMAs; 1: store-pipelined, 8 waves; 2: store-pipelined,
    // one 4-wave workgroup per CU (512 registers per wave)
    static const int pipe = [] { const char* e = getenv("PCMS_STEM_FWD_PIPE"); return e ? atoi(e) : 0; }();
    auto kern = b.lbd == 2 ? (pipe == 1 ? stem_fwd_direct_kernel<2, 3, 512, true> : stem_fwd_direct_kernel<2, 3, 512>)
                           : (pipe == 1 ? stem_fwd_direct_kernel<3, 2, 512, true> : stem_fwd_direct_kernel<3, 2, 512>);
    int g2 = grid;
    int thr = kSDThr;
    if (pipe == 2) {  // 4x4x16 boxes, one 4-wave workgroup per CU
      p.lbd = 2; p.lbh = 2;
      p.nbd = cdiv(D, 4); p.nbh = cdiv(H, 4);
      g2 = std::min(std::min(p.N * p.nbd * p.nbh * p.nbw, ncu), nbox);
      kern = stem_fwd_direct_kernel<2, 2, 256, true>;
      thr = 256;
    } else if (kSDThr == 256) {  // 4x4x16 boxes, two workgroups per CU; rows stay <= the caller's
      p.lbd = 2; p.lbh = 2;
      p.nbd = cdiv(D, 4); p.nbh = cdiv(H, 4);
      g2 = std::min(std::min(p.N * p.nbd * p.nbh * p.nbw, 2 * ncu), nbox);
      kern = stem_fwd_direct_kernel<2, 2, 256>;
    }
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kSDLds);
    hipLaunchKernelGGL(kern, dim3(g2), dim3(thr), kSDLds, s, p, thr == 256 ? p.N * p.nbd * p.nbh * p.nbw : nbox,
                       nbox, (uint32_t)xbytes,
                       (uint32_t)ybytes);
    PCMS_CHECK_LAUNCH();
  }
  if (b.lbd == 2 && b.lbh == 3 && b.lbw == 4) {
    (void)hipFuncSetAttribute((const void*)stem_fwd_kernel<2, 3, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, kStemLds);
    hipLaunchKernelGGL((stem_fwd_kernel<2, 3, 4>), dim3(std::min(nbox, ncu)), dim3(kStemThreads), kStemLds, s, p, nbox);
  } else {
    (void)hipFuncSetAttribute((const void*)stem_fwd_kernel<-1, -1, -1>, hipFuncAttributeMaxDynamicSharedMemorySize, kStemLds);
    hipLaunchKernelGGL((stem_fwd_kernel<-1, -1, -1>), dim3(std::min(nbox, ncu)), dim3(kStemThreads), kStemLds, s, p, nbox);
  }
  PCMS_CHECK_LAUNCH();
}

static int device_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ncu;
}

static bool stem_wgrad_streams(int N, int D, int H, int W) {
  return D % kSWBD == 0 && H % 4 == 0 && W % 16 == 0 && (long)N * D * H * W * 128 < (1L << 31);
}

// fp32 workspace floats pcms_stem_wgrad needs (0: none)
int pcms_stem_wgrad_ws_floats(int N, int D, int H, int W, int cin_w) {
  if (!stem_wgrad_streams(N, D, H, W)) return 0;
  const int nbox = N * (D / kSWBD) * (H / 4) * (W / 16);
  return std::min(nbox, device_cus()) * 64 * cin_w * 27;
}

// dw [64][cin_w][27] fp32 += stem weight gradient (x: 8-channel bf16 input, dy: 64 ch);
// ws: pcms_stem_wgrad_ws_floats(...) floats
int pcms_stem_wgrad(const void* x, const void* dy, float* dw, float* ws, int cin_w, int N, int D, int H, int W,
                    int target_wgs, hipStream_t s) {
  if (cin_w > 8 || cin_w < 1) return -1;
  if (stem_wgrad_streams(N, D, H, W)) {
    if (ws == nullptr) return -2;
    const int nbox = N * (D / kSWBD) * (H / 4) * (W / 16);
    const int grid = std::min(nbox, device_cus());
    const long xbytes = (long)N * D * H * W * 16, dybytes = (long)N * D * H * W * 128;
    auto kern = stem_wgrad_stream_kernel<kSWBD, kSWNS>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kSWLds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kSWT), kSWLds, s, (const bf16_t*)x,
                       (const bf16_t*)dy, ws, N, D, H, W, cin_w, (uint32_t)xbytes, (uint32_t)dybytes);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    const int total = 64 * cin_w * 27;
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(cdiv(total, 32)), dim3(256), 0, s, (const float*)ws, grid,
                       total, dw);
    PCMS_CHECK_LAUNCH();
  }
  Box b = choose_box(D, H, W, kSBV, kSHalo, 4, 16);
  const int nbd = cdiv(D, 1 << b.lbd), nbh = cdiv(H, 1 << b.lbh), nbw = cdiv(W, 1 << b.lbw);
  const int nbox = N * nbd * nbh * nbw;
  if (target_wgs <= 0) target_wgs = 256;
  int splits = std::max(1, std::min(nbox, target_wgs));
  const int bps = cdiv(nbox, splits);
  splits = cdiv(nbox, bps);
  const size_t lds = 2 * (size_t)kSBuf;
  auto kern = (b.lbd == 2 && b.lbh == 2 && b.lbw == 4) ? stem_wgrad_kernel<2, 2, 4> : stem_wgrad_kernel<-1, -1, -1>;
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, dim3(splits), dim3(256), lds, s, (const bf16_t*)x, (const bf16_t*)dy, dw,
                     N, D, H, W, cin_w, b.lbd, b.lbh, b.lbw, nbd, nbh, nbw, nbox, bps);
  PCMS_CHECK_LAUNCH();
}

// Weight-gradient launch plan: box geometry, boxes per split, split count (shared by the
// launch and its workspace query)
struct WgradPlan { Box b; int nbd, nbh, nbw, nbox, bps, splits; };
static WgradPlan wgrad_plan(int dtype, int N, int D, int H, int W, int Cin, int Cout, int target_wgs) {
  WgradPlan q;
  const int bv = dtype == PCMS_BF16 ? WTraits<bf16_t>::BV : WTraits<float>::BV;
  q.b = choose_box(D, H, W, bv, kWHaloMax, 4, 16);
  q.nbd = cdiv(D, 1 << q.b.lbd); q.nbh = cdiv(H, 1 << q.b.lbh); q.nbw = cdiv(W, 1 << q.b.lbw);
  q.nbox = N * q.nbd * q.nbh * q.nbw;
  const int tiles = (Cout / 64) * cdiv(Cin, 32);
  if (target_wgs <= 0) target_wgs = 512;
  const int splits = std::max(1, std::min(q.nbox, cdiv(target_wgs, tiles)));
  q.bps = cdiv(q.nbox, splits);
  q.splits = cdiv(q.nbox, q.bps);
  return q;
}

// fp32 workspace floats pcms_conv3_wgrad needs: one [27][Cout][c0+c1] partial row per split
int pcms_conv3_wgrad_ws_floats(int dtype, int N, int D, int H, int W, int c0, int c1, int Cout, int target_wgs) {
  const int Cin = c0 + c1;
  return wgrad_plan(dtype, N, D, H, W, Cin, Cout, target_wgs).splits * 27 * Cout * Cin;
}

// Weight gradient: dw (torch layout [Cout][cin_w][27], fp32) += sum_v dy (x) x, where
// cin_w <= c0 + c1 is the weight's input-channel count (the stored input may be padded).
// dwt: pcms_conv3_wgrad_ws_floats(...) fp32 workspace (per-split partial rows, summed in a
// fixed order: the result is deterministic).
int pcms_conv3_wgrad(int dtype, const void* x0, int c0, const void* x1, int c1, const void* dy,
                     float* dw, float* dwt, int N, int D, int H, int W, int Cout, int cin_w, int target_wgs,
                     hipStream_t s) {
  const int Cin = c0 + c1;
  if (cin_w <= 0 || cin_w > Cin) return -4;
  const int VEC = dtype == PCMS_BF16 ? 8 : 4;
  if (Cout % 64 != 0 || c0 % VEC != 0 || c1 % VEC != 0) return -1;
  const WgradPlan q = wgrad_plan(dtype, N, D, H, W, Cin, Cout, target_wgs);
  WgradParams p;
  p.x0 = x0; p.x1 = x1; p.c0 = c0; p.c1 = c1; p.dy = dy; p.dwt = dwt;
  p.N = N; p.D = D; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
  p.lbd = q.b.lbd; p.lbh = q.b.lbh; p.lbw = q.b.lbw;
  p.nbd = q.nbd; p.nbh = q.nbh; p.nbw = q.nbw;
  p.nbox = q.nbox;
  p.boxes_per_split = q.bps;
  const long nvox = (long)N * D * H * W;
  p.dma = dtype == PCMS_BF16 && (c1 == 0 || c0 % 32 == 0) && nvox * std::max(Cout, std::max(c0, c1)) * 2 < (long)kOOB;
  p.x0bytes = (uint32_t)(nvox * c0 * 2);
  p.x1bytes = (uint32_t)(nvox * c1 * 2);
  p.dybytes = (uint32_t)(nvox * Cout * 2);
  const int splits = q.splits;
  p.nco = Cout / 64;
  p.nci = cdiv(Cin, 32);
  p.dw = dw;
  p.cw = cin_w;
  p.direct = splits == 1 && dtype == PCMS_BF16 && !(PCMS_ABL & 16384);
  dim3 grid(splits * p.nco * p.nci);
  size_t lds;
  if (dtype == PCMS_BF16) {
    lds = (size_t)WTraits<bf16_t>::NBUF * (WTraits<bf16_t>::BV * WTraits<bf16_t>::DYROW + kWHaloMax * WTraits<bf16_t>::XROW);
    auto kern = conv3_wgrad_kernel<bf16_t, -1, -1, -1>;
    if (q.b.lbd == 2 && q.b.lbh == 2 && q.b.lbw == 4) kern = conv3_wgrad_kernel<bf16_t, 2, 2, 4>;
    else if (q.b.lbd == 1 && q.b.lbh == 3 && q.b.lbw == 4) kern = conv3_wgrad_kernel<bf16_t, 1, 3, 4>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, dim3(kWThreads), lds, s, p);
  } else {
    lds = (size_t)WTraits<float>::NBUF * (WTraits<float>::BV * WTraits<float>::DYROW + kWHaloMax * WTraits<float>::XROW);
    (void)hipFuncSetAttribute((const void*)conv3_wgrad_kernel<float, -1, -1, -1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((conv3_wgrad_kernel<float, -1, -1, -1>), grid, dim3(kWThreads), lds, s, p);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (p.direct) return 0;  // the kernel added into dw itself
  const long E = 27L * Cout * Cin;
  int R = splits, stride = 1;
  if (splits > 16) {
    hipLaunchKernelGGL(wgrad_group_sum_kernel, dim3((unsigned)cdiv(E, 256), cdiv(splits, 16)), dim3(256), 0, s, dwt,
                       splits, E);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    R = cdiv(splits, 16);
    stride = 16;
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(Cout, cdiv(cin_w, 32)), dim3(256), 0, s, (const float*)dwt, R, stride,
                     dw, Cout, Cin, cin_w);
  PCMS_CHECK_LAUNCH();
}

}  // extern "C"
