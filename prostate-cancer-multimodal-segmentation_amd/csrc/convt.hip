// ConvTranspose3d(k=2, s=2) of Up3D (models/unet3d.py:120), NDHWC, gfx950.
//
// Every output voxel receives exactly one input voxel through one of the 8 taps, so the
// three products are plain GEMMs with a scattered/gathered voxel index:
//   fwd   out[child(v,t), co] = b[co] + sum_ci x[v, ci] * W[ci, co, t]
//         M = input voxels, N = 8*Cout (t-major), K = Cin        (K-contiguous operands)
//   dgrad dx[v, ci] = sum_{t, co} dout[child(v,t), co] * W[ci, co, t]
//         M = input voxels, N = Cin, K = 8*Cout                  (K-contiguous operands)
//   wgrad dW[ci, t, co] += sum_v x[v, ci] * dout[child(v,t), co]
//         K = voxels: LDS tiles read with ds_read_b64_tr_b16 (bf16) like conv3_wgrad.
// child(v, t) = (n, 2d+i+pz, 2h+j+py, 2w+k+px) on the skip-sized grid: the symmetric
// F.pad of models/unet3d.py:143-151 is folded into the offsets (pz, py, px).
#include "common.h"
#include "pcms_hip.h"
#include <algorithm>

namespace {

__device__ __forceinline__ f32x16_t mfma(s16x8_t a, s16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x16_t mfma(float a, float b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <typename T> struct GT;
template <> struct GT<bf16_t> { static constexpr int KS = 16; typedef s16x8_t Frag; };
template <> struct GT<float> { static constexpr int KS = 2; typedef float Frag; };

__device__ __forceinline__ s16x8_t ldfrag(const bf16_t* p, int h) { return *reinterpret_cast<const s16x8_t*>(p + 8 * h); }
__device__ __forceinline__ float ldfrag(const float* p, int h) { return p[h]; }

struct UpGeom {
  int N, Din, Hin, Win;     // input grid
  int Do, Ho, Wo;           // output (skip-sized) grid
  int pz, py, px;           // pad-lo offsets
};

// child voxel of input voxel m through tap t = (i, j, k) = (t >> 2, (t >> 1) & 1, t & 1).
// 32-bit index math (the host checks M < 2^31): 64-bit division is a long software sequence.
__device__ __forceinline__ long child_base(const UpGeom& g, long m) {
  const uint32_t mm = (uint32_t)m;
  const uint32_t w = mm % (uint32_t)g.Win; uint32_t r = mm / (uint32_t)g.Win;
  const uint32_t h = r % (uint32_t)g.Hin; r /= (uint32_t)g.Hin;
  const uint32_t d = r % (uint32_t)g.Din; const uint32_t n = r / (uint32_t)g.Din;
  return (((long)n * g.Do + 2 * d + g.pz) * g.Ho + 2 * h + g.py) * g.Wo + 2 * w + g.px;
}
__device__ __forceinline__ long tap_delta(const UpGeom& g, int t) {
  return ((long)(t >> 2) * g.Ho + ((t >> 1) & 1)) * g.Wo + (t & 1);
}
__device__ __forceinline__ long child_vox(const UpGeom& g, long m, int t) { return child_base(g, m) + tap_delta(g, t); }

// wave tile 32 (M) x 64 (N); workgroup 4 waves stacked along M -> 128 x 64.
template <typename T>
__global__ void __launch_bounds__(256) convt_fwd_kernel(const T* x, const T* wt, const float* bias, T* out,
                                                        UpGeom g, int Cin, int Cout) {
  typedef typename GT<T>::Frag Frag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  const long m0 = (long)blockIdx.x * 128 + wave * 32;
  const int q0 = blockIdx.y * 64;
  if (m0 >= M) return;
  const long ma = std::min<long>(m0 + r, M - 1);
  const T* arow = x + ma * Cin;
  // MFMA column r of N-tile j is output column q0 + 2 r + j: a lane holds a channel pair, so
  // the bf16 build stores packed bf16x2 (two 128-B row segments per store instruction)
  const T* b0 = wt + (long)(q0 + 2 * r) * Cin;
  const T* b1 = b0 + Cin;
  f32x16_t acc0, acc1;
  for (int e = 0; e < 16; ++e) { acc0[e] = 0.f; acc1[e] = 0.f; }
  for (int k = 0; k < Cin; k += GT<T>::KS) {
    Frag a = ldfrag(arow + k, h);
    acc0 = mfma(a, ldfrag(b0 + k, h), acc0);
    acc1 = mfma(a, ldfrag(b1 + k, h), acc1);
  }
  const int q = q0 + 2 * r;             // Cout % 64 == 0: the pair shares one tap
  const int t = q / Cout, co = q % Cout;
  const float bias0 = bias[co], bias1 = bias[co + 1];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const long m = m0 + (e & 3) + 8 * (e >> 2) + 4 * h;
    if (m >= M) continue;
    T* dst = out + child_vox(g, m, t) * Cout + co;
    if constexpr (sizeof(T) == 2) {
      *reinterpret_cast<uint32_t*>(dst) = pack_bf16x2(acc0[e] + bias0, acc1[e] + bias1);
    } else {
      Elem<T>::st(dst, acc0[e] + bias0);
      Elem<T>::st(dst + 1, acc1[e] + bias1);
    }
  }
}

// dx[m, ci] = sum_{t,co} dout[child(m,t), co] * Wd[ci][t][co]
template <typename T>
__global__ void __launch_bounds__(256) convt_dgrad_kernel(const T* dout, const T* wd, T* dx, UpGeom g,
                                                          int Cin, int Cout) {
  typedef typename GT<T>::Frag Frag;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  const long m0 = (long)blockIdx.x * 128 + wave * 32;
  const int q0 = blockIdx.y * 64;
  if (m0 >= M) return;
  const long ma = std::min<long>(m0 + r, M - 1);
  const int K = 8 * Cout;
  const T* b0 = wd + (long)(q0 + r) * K;
  const T* b1 = wd + (long)(q0 + 32 + r) * K;
  f32x16_t acc0, acc1, s0, s1;
  for (int e = 0; e < 16; ++e) { acc0[e] = 0.f; acc1[e] = 0.f; s0[e] = 0.f; s1[e] = 0.f; }
  for (int t = 0; t < 8; ++t) {
    const T* arow = dout + child_vox(g, ma, t) * Cout;
    for (int k = 0; k < Cout; k += GT<T>::KS) {
      Frag a = ldfrag(arow + k, h);
      acc0 = mfma(a, ldfrag(b0 + t * Cout + k, h), acc0);
      acc1 = mfma(a, ldfrag(b1 + t * Cout + k, h), acc1);
    }
    if constexpr (sizeof(T) == 4) {  // fp32 build: one chain per tap, summed (two-level)
      s0 += acc0; s1 += acc1;
      for (int e = 0; e < 16; ++e) { acc0[e] = 0.f; acc1[e] = 0.f; }
    }
  }
  if constexpr (sizeof(T) == 4) { acc0 = s0; acc1 = s1; }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const long m = m0 + (e & 3) + 8 * (e >> 2) + 4 * h;
    if (m >= M) continue;
    Elem<T>::st(dx + m * Cin + q0 + r, acc0[e]);
    Elem<T>::st(dx + m * Cin + q0 + 32 + r, acc1[e]);
  }
}

// bf16 forward at Cout = 64, Cin = 128 (Up3D up4, the level-0 upsample: 67 MB in, 268 MB
// out -- a store stream).  PERSISTENT: one 8-wave workgroup per CU walks 64-voxel tiles
// slot, slot + nslot, ...; wave t computes tap t (its 64 x 128 weights held in registers
// for the whole launch: no weight traffic), so a tile's A rows (64 x 256 B, LDS, 16-B slots
// XOR row & 15) are read from HBM exactly once and feed all 8 taps.  The next tile's rows are
// register-prefetched while this one computes and stores; LDS is double-buffered with one raw
// barrier per tile (no vmcnt(0): the output stores stay in flight across tiles).  Output:
// each lane a channel pair (packed bf16x2), 32 lanes = one whole 128-B child row,
// non-temporal.
constexpr int kSTM = 64;                           // voxels per tile
constexpr int kSTRow = 256;                        // 128 ci x 2 B
__global__ void __launch_bounds__(512, 1) convt_fwd_stream_kernel(const bf16_t* x, const bf16_t* wpk,
                                                                  const float* bias, bf16_t* out, UpGeom g,
                                                                  int ntile) {
  constexpr int Cin = 128, Cout = 64;
  __shared__ __attribute__((aligned(16))) char lds[2 * kSTM * kSTRow];
  const int tid = threadIdx.x, lane = tid & 63, t = tid >> 6, r = lane & 31, h = lane >> 5;
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  // this wave's weights: B fragment (ks, nt) = row (t, co = 2 r + nt), K = 16 ks + 8 h
  s16x8_t b[8][2];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
      b[ks][nt] = *reinterpret_cast<const s16x8_t*>(wpk + ((long)t * Cout + 2 * r + nt) * Cin + ks * 16 + 8 * h);
  // opaque: the compiler would otherwise re-load the weights inside the tile loop (cheap
  // rematerialisation) and wait for them with vmcnt(0) -- draining the output stores
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) asm volatile("" : "+v"(b[ks][nt]));
  const float b0 = bias[2 * r], b1 = bias[2 * r + 1];
  const long dt = tap_delta(g, t) * Cout + 2 * r;
  // staging: piece pc = tid + 512 j (j < 2) = row pc >> 4, slot pc & 15
  u32x4_t stg[2];
  auto load = [&](int tile) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = tid + 512 * j, row = pc >> 4, sl = pc & 15;
      const long m = std::min<long>((long)tile * kSTM + row, M - 1);  // clamped tail rows: never stored
      stg[j] = *reinterpret_cast<const u32x4_t*>(x + m * Cin + sl * 8);
    }
  };
  auto put = [&](char* buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = tid + 512 * j, row = pc >> 4, sl = pc & 15;
      *reinterpret_cast<u32x4_t*>(buf + row * kSTRow + ((sl ^ (row & 15)) << 4)) = stg[j];
    }
  };
  int tile = blockIdx.x;
  if (tile >= ntile) return;
  load(tile);
  put(lds);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int it = 0; tile < ntile; ++it, tile += gridDim.x) {
    const char* buf = lds + (it & 1) * kSTM * kSTRow;
    const int next = tile + gridDim.x;
    if (next < ntile) load(next);
    f32x16_t acc[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[mt][nt][e] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const int row = mt * 32 + r;
        const s16x8_t a = *reinterpret_cast<const s16x8_t*>(buf + row * kSTRow + (((ks * 2 + h) ^ (row & 15)) << 4));
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[mt][nt] = mfma(a, b[ks][nt], acc[mt][nt]);
      }
    // a lane's rows come in runs of 4 consecutive voxels starting at a multiple of 4 (Win % 4
    // == 0: a run never leaves its w-row), whose children are 2 voxels apart: one child_base
    // per run.  All 32 values are packed before the first store: rewriting a register that an
    // in-flight store still reads costs a vmcnt(0) per store (measured: 158 us with per-store
    // packing; one wait per tile left: 70.5 us; alternating two register sets by tile: 73 us).
    uint32_t pk[2][16];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int e = 0; e < 16; ++e) pk[mt][e] = pack_bf16x2(acc[mt][0][e] + b0, acc[mt][1][e] + b1);
    const long mbase = (long)tile * kSTM + 4 * h;
    if ((long)(tile + 1) * kSTM <= M) {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int grp = 0; grp < 4; ++grp) {
          uint32_t* base = reinterpret_cast<uint32_t*>(out + child_base(g, mbase + mt * 32 + 8 * grp) * Cout + dt);
#pragma unroll
          for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(pk[mt][grp * 4 + i], base + i * Cout);
        }
    } else {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const long m = mbase + mt * 32 + (e & 3) + 8 * (e >> 2);
          if (m < M) __builtin_nontemporal_store(pk[mt][e], reinterpret_cast<uint32_t*>(out + child_base(g, m) * Cout + dt));
        }
    }
    if (next < ntile) put(lds + ((it + 1) & 1) * kSTM * kSTRow);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
}

// fp32 build (bf16x6, see conv_common.h): K steps of 8 channels; the A row (8 fp32) split
// into h, m, l in registers, the weights pre-split in their pack (per 8 K-elements the three
// B fragments [h|h] [m|h] [l|m], 48 bf16); three MFMAs per step and N-tile.
__device__ __forceinline__ void afrag_x6(const float* p, int h, s16x8_t& a1, s16x8_t& a2) {
  const f32x4_t u = *reinterpret_cast<const f32x4_t*>(p), v = *reinterpret_cast<const f32x4_t*>(p + 4);
  const float f[8] = {u[0], u[1], u[2], u[3], v[0], v[1], v[2], v[3]};
  u32x4_t hh, mm, ll;
  split3x8(f, hh, mm, ll);
  a1 = __builtin_bit_cast(s16x8_t, h ? mm : hh);  // [h | m]
  a2 = __builtin_bit_cast(s16x8_t, h ? ll : hh);  // [h | l]
}
__device__ __forceinline__ f32x16_t mfma_x6(s16x8_t a1, s16x8_t a2, const bf16_t* b, int h, f32x16_t c) {
  c = mfma(a1, *reinterpret_cast<const s16x8_t*>(b + 8 * h), c);
  c = mfma(a2, *reinterpret_cast<const s16x8_t*>(b + 16 + 8 * h), c);
  return mfma(a1, *reinterpret_cast<const s16x8_t*>(b + 32 + 8 * h), c);
}

// forward, fp32 build: out[child(m, t)][co] = b[co] + sum_ci x[m][ci] W[ci][co][t]
// (pack rows q = t Cout + co, Cin / 8 groups of 48 bf16).  Each wave owns MT 32-row M-tiles,
// so every B fragment (L2) feeds MT x 3 MFMAs: at MT = 1 the weight fragments were 3/4 of the
// ~8.6 GB a level-0 launch pulled from L2.  The K loop order per accumulator is unchanged.
template <int MT>
__global__ void __launch_bounds__(256, 2) convt_fwd_x6_kernel(const float* x, const bf16_t* wt, const float* bias,
                                                           float* out, UpGeom g, int Cin, int Cout) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  const long m0 = (long)blockIdx.x * (128 * MT) + wave * (32 * MT);
  const int q0 = blockIdx.y * 64;
  if (m0 >= M) return;
  const float* arow[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) arow[i] = x + std::min<long>(m0 + 32 * i + r, M - 1) * Cin;
  const bf16_t* bp[2];
  bp[0] = wt + (long)(q0 + 2 * r) * Cin * 6;
  bp[1] = bp[0] + (long)Cin * 6;
  f32x16_t acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) { acc[i][0][e] = 0.f; acc[i][1][e] = 0.f; }
  for (int k = 0; k < Cin; k += 8) {
    s16x8_t bb[2][3];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 3; ++j) bb[n][j] = *reinterpret_cast<const s16x8_t*>(bp[n] + k * 6 + 16 * j + 8 * h);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      s16x8_t a1, a2;
      afrag_x6(arow[i] + k, h, a1, a2);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        acc[i][n] = mfma(a1, bb[n][0], acc[i][n]);
        acc[i][n] = mfma(a2, bb[n][1], acc[i][n]);
        acc[i][n] = mfma(a1, bb[n][2], acc[i][n]);
      }
    }
  }
  const int q = q0 + 2 * r;
  const int t = q / Cout, co = q % Cout;
  const float bias0 = bias[co], bias1 = bias[co + 1];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const long m = m0 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (m >= M) continue;
      float* dst = out + child_vox(g, m, t) * Cout + co;
      dst[0] = acc[i][0][e] + bias0;
      dst[1] = acc[i][1][e] + bias1;
    }
}

// dgrad, fp32 build: dx[m][ci] = sum_{t, co} dout[child(m, t)][co] Wd[ci][t][co]
// (pack rows ci, 8 Cout / 8 groups of 48 bf16); MT 32-row M-tiles per wave as the forward.
// ws != nullptr: blockIdx.z takes K groups [z G / Z, (z + 1) G / Z) of the G = Cout / 8 per tap
// x 8 taps and stores its fp32 partial sums to ws[z][m][ci] (summed in z order afterwards)
template <int MT>
__global__ void __launch_bounds__(256, 2) convt_dgrad_x6_kernel(const float* dout, const bf16_t* wd, float* dx,
                                                             UpGeom g, int Cin, int Cout, float* ws) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  const long m0 = (long)blockIdx.x * (128 * MT) + wave * (32 * MT);
  const int q0 = blockIdx.y * 64;
  if (m0 >= M) return;
  long ma[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) ma[i] = std::min<long>(m0 + 32 * i + r, M - 1);
  const long K = 8L * Cout;
  const bf16_t* bp[2];
  bp[0] = wd + (long)(q0 + r) * K * 6;
  bp[1] = wd + (long)(q0 + 32 + r) * K * 6;
  f32x16_t acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) { acc[i][0][e] = 0.f; acc[i][1][e] = 0.f; }
  const int G = Cout / 8 * 8, Z = gridDim.z;
  const int g0 = (int)((long)blockIdx.z * G / Z), g1 = (int)((long)(blockIdx.z + 1) * G / Z);
  for (int gi = g0; gi < g1; ++gi) {
    const int t = gi / (Cout / 8), k = (gi % (Cout / 8)) * 8;
    s16x8_t bb[2][3];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 3; ++j)
        bb[n][j] = *reinterpret_cast<const s16x8_t*>(bp[n] + ((long)t * Cout + k) * 6 + 16 * j + 8 * h);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      s16x8_t a1, a2;
      afrag_x6(dout + child_vox(g, ma[i], t) * Cout + k, h, a1, a2);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        acc[i][n] = mfma(a1, bb[n][0], acc[i][n]);
        acc[i][n] = mfma(a2, bb[n][1], acc[i][n]);
        acc[i][n] = mfma(a1, bb[n][2], acc[i][n]);
      }
    }
  }
  float* dst = ws ? ws + (long)blockIdx.z * M * Cin : dx;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const long m = m0 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (m >= M) continue;
      dst[m * Cin + q0 + r] = acc[i][0][e];
      dst[m * Cin + q0 + 32 + r] = acc[i][1][e];
    }
}

// bf16 forward and dgrad, LDS-staged (the hot path).  The direct kernels above read each A
// row 32 B per lane pair and instruction (the 32x32 A layout): ~25 % of each 128-B line per
// request, ~1/5 of the HBM roofline.  Here a 512-thread workgroup owns 256 input voxels x 128
// GEMM columns; per stage (a 64-channel chunk of K) it stages the 256 A rows (full 128-B
// rows, 8 lanes per row) and the 128 x 64 weight tile into LDS (16-B slots XOR-swizzled by
// row & 7), register-prefetching the next stage while 8 waves (32 voxels x 128 columns, 4
// N-tiles) run their MFMAs.  Columns are channel pairs (packed bf16x2 stores).  One 48-KiB
// stage buffer and <= 128 VGPRs: two workgroups per CU hide each other's staging and
// epilogue (vs a double buffer at one workgroup per CU: level-0 forward 164 -> 125 us,
// convT dgrad 0.238 -> 0.222 ms/step).
//   FWD:   A = x[m][Cin],                 K = Cin,      columns q = (t, co), out[child(m,t)][co] + b
//   dgrad: A = dout[child(m, t)][Cout],   K = 8 Cout,   columns = ci,        dx[m][ci]
constexpr int kCDM = 256, kCDN = 128;
constexpr int kCDStage = kCDM * 128 + kCDN * 128;                 // 48 KiB per stage
constexpr int kCDPieces = kCDStage / 16 / 512;                    // 6 per thread

__device__ __forceinline__ int cd_slot(int row, int slot) { return row * 128 + ((slot ^ (row & 7)) << 4); }

// NT: non-temporal streams for tensors far larger than the Infinity Cache (forward: the
// output stores; dgrad: the dout loads)
// SPLIT (dgrad with few workgroups): blockIdx.z takes an equal share of the K stages and
// writes fp32 partials ws[z][m][ci], summed in z order by convt_dgrad_reduce.
template <bool FWD, bool NT = false, bool SPLIT = false>
__global__ void __launch_bounds__(512, 2) convt_lds_kernel(const bf16_t* a_src, const bf16_t* wpk, const float* bias,
                                                           bf16_t* out, UpGeom g, int Cin, int Cout, float* ws) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r_lane = lane & 31, hsel = lane >> 5;
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  // forward on a 1-D grid: the column blocks of one voxel tile run back to back on one XCD
  // (workgroups are dealt to the 8 XCDs round-robin), so its A rows are re-read from that L2
  int bx = blockIdx.x, by = blockIdx.y;
  if (FWD && gridDim.y == 1) {
    const int ny = 8 * Cout / kCDN, b = blockIdx.x;
    if ((gridDim.x / ny) % 8 == 0) {
      by = (b >> 3) % ny;
      bx = (b >> 3) / ny * 8 + (b & 7);
    } else {
      by = b % ny;
      bx = b / ny;
    }
  }
  const long m0 = (long)bx * kCDM;
  const int q0 = by * kCDN;
  const int K = FWD ? Cin : 8 * Cout, Ka = FWD ? Cin : Cout;  // K, A row pitch
  const int nst = K / 64 / (SPLIT ? (int)gridDim.z : 1), st0 = SPLIT ? (int)blockIdx.z * nst : 0;
  // staging pieces of this thread: j < 4: A rows (256 x 8 slots), j >= 4: weight rows (128 x 8)
  long arow[4];  // FWD: input voxel; dgrad: its tap-0 child voxel
  int aslot[4], aoff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pc = tid + j * 512, row = pc >> 3, sl = pc & 7;
    const long m = std::min<long>(m0 + row, M - 1);  // clamped tail rows are computed, never stored
    arow[j] = FWD ? m : child_base(g, m);
    aslot[j] = sl;
    aoff[j] = cd_slot(row, sl);
  }
  int brow[2], bslot[2], boff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pc = tid + j * 512, row = pc >> 3, sl = pc & 7;
    // LDS weight row = MFMA column (nt, cl): GEMM column q0 + 64 (nt / 2) + 2 cl + nt % 2
    const int nt = row >> 5, cl = row & 31;
    brow[j] = q0 + 64 * (nt >> 1) + 2 * cl + (nt & 1);
    bslot[j] = sl;
    boff[j] = kCDM * 128 + cd_slot(row, sl);
  }
  u32x4_t stg[kCDPieces];
  auto load = [&](int st) {
    if constexpr (FWD) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        stg[j] = *reinterpret_cast<const u32x4_t*>(a_src + arow[j] * Ka + st * 64 + aslot[j] * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        stg[4 + j] = *reinterpret_cast<const u32x4_t*>(wpk + (long)brow[j] * K + st * 64 + bslot[j] * 8);
    } else {
      const int t = st % 8, kc = st / 8;
      const long dt = tap_delta(g, t);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u32x4_t* src = reinterpret_cast<const u32x4_t*>(a_src + (arow[j] + dt) * Ka + kc * 64 + aslot[j] * 8);
        if constexpr (NT) stg[j] = __builtin_nontemporal_load(src);
        else stg[j] = *src;
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
        stg[4 + j] = *reinterpret_cast<const u32x4_t*>(wpk + (long)brow[j] * K + t * Cout + kc * 64 + bslot[j] * 8);
    }
  };
  auto store = [&](char* buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) *reinterpret_cast<u32x4_t*>(buf + aoff[j]) = stg[j];
#pragma unroll
    for (int j = 0; j < 2; ++j) *reinterpret_cast<u32x4_t*>(buf + boff[j]) = stg[4 + j];
  };
  f32x16_t acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  const int arw = wave * 32 + r_lane;
  load(st0);
  store(lds);
  __syncthreads();
  for (int st = st0; st < st0 + nst; ++st) {
    const char* buf = lds;
    if (st + 1 < st0 + nst) load(st + 1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const s16x8_t a = *reinterpret_cast<const s16x8_t*>(buf + cd_slot(arw, ks * 2 + hsel));
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const s16x8_t b = *reinterpret_cast<const s16x8_t*>(buf + kCDM * 128 + cd_slot(nt * 32 + r_lane, ks * 2 + hsel));
        acc[nt] = mfma(a, b, acc[nt]);
      }
    }
    if (st + 1 < st0 + nst) {
      __syncthreads();
      store(lds);
    }
    __syncthreads();
  }
  if constexpr (FWD && SPLIT) {
    // fp32 partials ws[z][m][q] (q = GEMM column = tap x Cout + co), summed in z order with
    // the bias by convt_fwd_reduce
    const long Q = 8L * Cout;
    float* part = ws + (long)blockIdx.z * M * Q + q0 + 2 * r_lane;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const long m = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
      if (m >= M) continue;
      *reinterpret_cast<f32x2_t*>(part + m * Q) = f32x2_t{acc[0][e], acc[1][e]};
      *reinterpret_cast<f32x2_t*>(part + m * Q + 64) = f32x2_t{acc[2][e], acc[3][e]};
    }
  } else if constexpr (FWD) {
    long dq[2];
    int cq[2];
    float b0[2], b1[2];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const int q = q0 + 64 * pr + 2 * r_lane;  // Cout even: the pair shares one tap
      dq[pr] = tap_delta(g, q / Cout) * Cout;
      cq[pr] = q % Cout;
      b0[pr] = bias[cq[pr]];
      b1[pr] = bias[cq[pr] + 1];
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const long m = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
      if (m >= M) continue;
      bf16_t* crow = out + child_base(g, m) * Cout;
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const uint32_t v = pack_bf16x2(acc[2 * pr][e] + b0[pr], acc[2 * pr + 1][e] + b1[pr]);
        uint32_t* dst = reinterpret_cast<uint32_t*>(crow + dq[pr] + cq[pr]);
        if constexpr (NT) __builtin_nontemporal_store(v, dst);
        else *dst = v;
      }
    }
  } else if constexpr (SPLIT) {
    float* part = ws + (long)blockIdx.z * M * Cin + q0 + 2 * r_lane;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const long m = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
      if (m >= M) continue;
      *reinterpret_cast<f32x2_t*>(part + m * Cin) = f32x2_t{acc[0][e], acc[1][e]};
      *reinterpret_cast<f32x2_t*>(part + m * Cin + 64) = f32x2_t{acc[2][e], acc[3][e]};
    }
  } else {
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const long m = m0 + wave * 32 + (e & 3) + 8 * (e >> 2) + 4 * hsel;
      if (m >= M) continue;
      bf16_t* row = out + m * Cin + q0 + 2 * r_lane;
      *reinterpret_cast<uint32_t*>(row) = pack_bf16x2(acc[0][e], acc[1][e]);
      *reinterpret_cast<uint32_t*>(row + 64) = pack_bf16x2(acc[2][e], acc[3][e]);
    }
  }
}

// dx[m][ci] = T(sum over z = 0..S-1 of ws[z][m][ci]), z in order; 4 elements per thread
template <typename T>
__global__ void __launch_bounds__(256) convt_dgrad_reduce(const float* ws, int S, long E, T* dx) {
  const long i = (blockIdx.x * 256L + threadIdx.x) * 4;
  if (i >= E) return;
  f32x4_t v[16];
  f32x4_t a = *reinterpret_cast<const f32x4_t*>(ws + i);
  for (int z0 = 1; z0 < S; z0 += 16) {
    const int nz = std::min(16, S - z0);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < nz) v[j] = *reinterpret_cast<const f32x4_t*>(ws + (z0 + j) * E + i);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (j < nz) a += v[j];
  }
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<f32x4_t*>(dx + i) = a;
  } else {
    uint32_t* d = reinterpret_cast<uint32_t*>(dx + i);
    d[0] = pack_bf16x2(a[0], a[1]);
    d[1] = pack_bf16x2(a[2], a[3]);
  }
}

// forward K splits: out[child(m, t)][co] = bf16(sum over z = 0..S-1 of ws[z][m][t Cout + co] +
// bias[co]), z in order; 4 columns (one tap, Cout % 4 == 0) per thread
__global__ void __launch_bounds__(256) convt_fwd_reduce(const float* ws, int S, long M, int Cout,
                                                        const float* bias, bf16_t* out, UpGeom g) {
  const long Q = 8L * Cout, E = M * Q;
  const long i = (blockIdx.x * 256L + threadIdx.x) * 4;
  if (i >= E) return;
  f32x4_t a = *reinterpret_cast<const f32x4_t*>(ws + i);
  for (int z = 1; z < S; ++z) a += *reinterpret_cast<const f32x4_t*>(ws + (long)z * E + i);
  const long m = i / Q;
  const int q = (int)(i % Q), t = q / Cout, co = q % Cout;
  uint2 o;
  o.x = pack_bf16x2(a[0] + bias[co], a[1] + bias[co + 1]);
  o.y = pack_bf16x2(a[2] + bias[co + 2], a[3] + bias[co + 3]);
  *reinterpret_cast<uint2*>(out + child_vox(g, m, t) * Cout + co) = o;
}

// ---- weight gradient: C[p = ci][q = (t, co)] over K = input voxels ----
constexpr int kVB = 64;  // voxels per staged block

__device__ __forceinline__ int half_swz(int v, int c) {  // 128-B rows (64 bf16), c element
  return v * 128 + (((c >> 5) ^ ((v >> 1) & 1)) * 64) + (c & 31) * 2;
}
__device__ __forceinline__ s16x4_t tr_read(const char* lds, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4_t*)(lds + off));
}

// Workgroup tile: 64 ci x (8 taps x 64 co) over a voxel split.  A block of VB input voxels
// stages x [VB][64 ci] once and the 8 taps' dout child rows [8][VB][64 co], so the x tile
// feeds all 8 taps: 8 waves = (ci half, co half, tap half), 4 tap tiles each (16 MFMAs per
// 64 voxels between barriers).  All of a thread's 16-B pieces of a block are loaded into
// registers before any is written to LDS (the loads overlap instead of each waiting alone).
template <typename T> struct CW { static constexpr int VB = sizeof(T) == 2 ? 64 : 32; };

template <typename T>
__global__ void __launch_bounds__(512, 1) convt_wgrad_kernel(const T* x, const T* dout, float* ws, UpGeom g,
                                                          int Cin, int Cout, int vox_per_split) {
  constexpr int VB = CW<T>::VB;
  constexpr int ROW = 64 * (int)sizeof(T);
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int PPR = 64 / VEC;                  // 16-B pieces per row
  constexpr int NP = 9 * VB * PPR;               // pieces per block: x + 8 taps
  constexpr int PT = NP / 512;                   // per thread
  static_assert(NP % 512 == 0, "whole pieces per thread");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* P = lds;                                 // x tile [VB][64]
  char* Q = lds + VB * ROW;                      // dout tiles [8][VB][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int wp = wave & 1, wq = (wave >> 1) & 1, t0 = (wave >> 2) * 4;  // ci half, co half, taps t0..t0+3
  const int p0 = blockIdx.z * 64;     // ci tile
  const int co0 = blockIdx.y * 64;    // co tile
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  const long vbeg = (long)blockIdx.x * vox_per_split;
  const long vend = std::min<long>(M, vbeg + vox_per_split);
  f32x16_t acc[4], macc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) { acc[t][e] = 0.f; macc[t][e] = 0.f; }
  for (long vb = vbeg; vb < vend; vb += VB) {
    if constexpr (sizeof(T) == 4) {  // fp32 build: per-block chains summed (two-level)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        macc[t] += acc[t];
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
      }
    }
    u32x4_t stg[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int pc = tid + i * 512;
      const int which = pc / (VB * PPR), rem = pc % (VB * PPR);   // 0: x, 1 + t: dout tap t
      const int v = rem / PPR, q = rem % PPR;
      const long m = std::min<long>(vb + v, vend - 1);             // clamped (zeroed below)
      const T* src = which == 0 ? x + m * Cin + p0 + q * VEC : dout + child_vox(g, m, which - 1) * Cout + co0 + q * VEC;
      stg[i] = *reinterpret_cast<const u32x4_t*>(src);
      if (vb + v >= vend) stg[i] = (u32x4_t){0u, 0u, 0u, 0u};
    }
    __syncthreads();  // every wave is done with the previous block's tiles
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int pc = tid + i * 512;
      const int which = pc / (VB * PPR), rem = pc % (VB * PPR);
      const int v = rem / PPR, q = rem % PPR;
      const int off = sizeof(T) == 2 ? half_swz(v, q * VEC) : v * ROW + q * 16;
      *reinterpret_cast<u32x4_t*>((which == 0 ? P : Q + (which - 1) * VB * ROW) + off) = stg[i];
    }
    __syncthreads();
    if constexpr (sizeof(T) == 2) {
      const int gg = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
      const int ca = wp * 32 + gg * 16 + pp * 4, cb = wq * 32 + gg * 16 + pp * 4;
#pragma unroll
      for (int k0 = 0; k0 < VB; k0 += 16) {
        const int v = k0 + 8 * h + qq;
        s16x4_t a0 = tr_read(P, half_swz(v, ca)), a1 = tr_read(P, half_swz(v + 4, ca));
        s16x8_t a = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const char* Qt = Q + (t0 + t) * VB * ROW;
          s16x4_t b0 = tr_read(Qt, half_swz(v, cb)), b1 = tr_read(Qt, half_swz(v + 4, cb));
          s16x8_t b = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
          acc[t] = mfma(a, b, acc[t]);
        }
      }
    } else {
      for (int k0 = 0; k0 < VB; k0 += 2) {
        const int v = k0 + h;
        float a = *reinterpret_cast<const float*>(P + v * ROW + (wp * 32 + (lane & 31)) * 4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          float b = *reinterpret_cast<const float*>(Q + (t0 + t) * VB * ROW + v * ROW + (wq * 32 + (lane & 31)) * 4);
          acc[t] = mfma(a, b, acc[t]);
        }
      }
    }
  }
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] += macc[t];
  }
  // C[row = ci][col = co] per tap -> this split's partial row ws[split][Cin][8][Cout] (plain
  // stores; fp32 atomics from every split into one image serialise on contended addresses)
  float* prow = ws + (long)blockIdx.x * 8 * Cin * Cout;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ci = p0 + wp * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      const int co = co0 + wq * 32 + (lane & 31);
      prow[((long)ci * 8 + t0 + t) * Cout + co] = acc[t][e];
    }
}

// bf16, Cin % 128 == 0: the same product with all 128 input channels of a tile in one
// workgroup, so each dout child row is staged once per 128 ci instead of once per 64 (at
// level 0, Cin = 128: dout -- 268 MB -- read once, not twice).  x tile [VB][128] as two
// [VB][64] halves; 8 waves = (ci quarter cq, co half), each all 8 taps (8 accumulators):
// per 16 voxels one x fragment and 8 dout fragments feed 8 MFMAs.
// NT: non-temporal loads (dout far larger than the Infinity Cache)
// BIAS (bpart != nullptr; ci tile 0's workgroups): the bias gradient sum_v dout[v][co] from the
// same read of dout -- a thread's dout pieces are always channels 8 (tid % 8) .. of its co
// tile (the piece index steps by 512, a multiple of 8), summed in registers in piece order and
// then over the 64 threads of each channel group in thread order: one [Cout] partial row per
// voxel split (the ConvT bias-gradient pass over dout -- 268 MB at level 0 -- is gone)
// TT (taps per workgroup, 8 / 4 / 2): the deep levels' grids -- a few thousand input voxels,
// 16-64 (ci, co) tiles -- fill the chip with voxel splits whose fp32 partial rows (67 MB per
// launch at the engine's 512-workgroup target) cost more than the MFMAs; splitting the 8 taps
// over G = 8 / TT workgroups instead cuts the splits (and the partial rows) by G, at G x the x
// staging.  blockIdx.z = ci tile x G + tap group.  DIRECT (one split): dw += the tile itself
// (torch layout [Cin][Cout][8], each element owned by one workgroup), no partial rows.
// Bias (ci tile 0): one [Cout] row per (split, tap group).
#ifndef CTW_PF
#define CTW_PF 1
#endif
#ifndef CTW_OMAP
#define CTW_OMAP 0
#endif
template <bool NT, int TT, bool DIRECT>
__global__ void __launch_bounds__(512, (TT <= 4 && !CTW_PF) ? 2 : 1) convt_wgrad128_kernel(const bf16_t* x, const bf16_t* dout,
                                                                             float* ws, UpGeom g, int Cin, int Cout,
                                                                             int vox_per_split, float* bpart) {
  constexpr int VB = 64, ROW = 128, PPR = 8, G = 8 / TT;
  constexpr int XP = VB * 2 * PPR;               // x pieces (two 64-ci halves)
  constexpr int NP = XP + TT * VB * PPR;         // + TT taps
  constexpr int PT = NP / 512;                   // 2 + TT per thread
  static_assert(NP % 512 == 0, "whole pieces per thread");
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* P = lds;                                 // x tiles [2][VB][64]
  char* Q = lds + 2 * VB * ROW;                  // dout tiles [TT][VB][64]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int cq = wave & 3, wq = wave >> 2;       // ci quarter, co half
  const int tg = blockIdx.z % G, tb = tg * TT;   // tap group, its first tap
  const int p0 = (blockIdx.z / G) * 128;         // ci tile
  const int co0 = blockIdx.y * 64;               // co tile
  const long M = (long)g.N * g.Din * g.Hin * g.Win;
  const long vbeg = (long)blockIdx.x * vox_per_split;
  const long vend = std::min<long>(M, vbeg + vox_per_split);
  f32x16_t acc[TT];
#pragma unroll
  for (int t = 0; t < TT; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
  const int gg = (lane >> 4) & 1, qq = (lane & 15) >> 2, pp = lane & 3;
  const int ca = (cq & 1) * 32 + gg * 16 + pp * 4, cb = wq * 32 + gg * 16 + pp * 4;
  const char* Pq = P + (cq >> 1) * VB * ROW;
  const bool bias = bpart != nullptr && blockIdx.z < G;
  float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // CTW_PF: the next block's pieces are loaded into registers right after this block's are
  // written to LDS, so their latency runs under this block's MFMAs (without it each block's
  // loads -> LDS -> MFMAs run in series)
  u32x4_t stg[PT];
  // dout piece r (0 .. TT VB PPR) -> (tap t of the group, block voxel v, 16-B piece q).
  // CTW_OMAP 0: tap-major (a wave-instruction reads 8 child rows 256 B apart: every other
  // voxel of an output row).  1: the two k taps of each (i, j) interleaved in output-voxel
  // order, so a wave-instruction reads 1 KiB of contiguous output rows (child (2w + k))
  auto dout_piece = [&](int r, int& t, int& v, int& q) {
    q = r % PPR;
    if constexpr (CTW_OMAP && TT >= 2) {
      const int pair = r / (2 * VB * PPR), ow = (r % (2 * VB * PPR)) / PPR;
      t = 2 * pair + (ow & 1);
      v = ow >> 1;
    } else {
      t = r / (VB * PPR);
      v = (r % (VB * PPR)) / PPR;
    }
  };
  auto load_block = [&](long vb) {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int pc = tid + i * 512;
      const bf16_t* src;
      int v;
      if (pc < XP) {                             // x: (half, voxel, piece)
        const int hf = pc / (VB * PPR), rem = pc % (VB * PPR);
        v = rem / PPR;
        const long m = std::min<long>(vb + v, vend - 1);
        src = x + m * Cin + p0 + hf * 64 + (rem % PPR) * 8;
      } else {                                   // dout tap tb + t
        int t, q;
        dout_piece(pc - XP, t, v, q);
        const long m = std::min<long>(vb + v, vend - 1);
        src = dout + child_vox(g, m, tb + t) * Cout + co0 + q * 8;
      }
      stg[i] = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src))
                  : *reinterpret_cast<const u32x4_t*>(src);
      if (vb + v >= vend) stg[i] = (u32x4_t){0u, 0u, 0u, 0u};
    }
  };
#if CTW_PF
  if (vbeg < vend) load_block(vbeg);
#endif
  for (long vb = vbeg; vb < vend; vb += VB) {
#if !CTW_PF
    load_block(vb);
#endif
    if (bias) {
#pragma unroll
      for (int i = XP / 512; i < PT; ++i)  // the dout pieces (pc >= XP)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          bs[2 * k] += __uint_as_float(stg[i][k] << 16);
          bs[2 * k + 1] += __uint_as_float(stg[i][k] & 0xffff0000u);
        }
    }
    __syncthreads();  // every wave is done with the previous block's tiles
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int pc = tid + i * 512;
      int tile = pc / (VB * PPR), rem = pc % (VB * PPR);  // tiles 0-1: x halves, 2..: taps
      int v = rem / PPR, q = rem % PPR;
      if (pc >= XP) {
        int t;
        dout_piece(pc - XP, t, v, q);
        tile = 2 + t;
      }
      *reinterpret_cast<u32x4_t*>(lds + tile * VB * ROW + half_swz(v, q * 8)) = stg[i];
    }
    __syncthreads();
#if CTW_PF
    if (vb + VB < vend) load_block(vb + VB);
#endif
#pragma unroll
    for (int k0 = 0; k0 < VB; k0 += 16) {
      const int v = k0 + 8 * h + qq;
      s16x4_t a0 = tr_read(Pq, half_swz(v, ca)), a1 = tr_read(Pq, half_swz(v + 4, ca));
      s16x8_t a = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
      for (int t = 0; t < TT; ++t) {
        const char* Qt = Q + t * VB * ROW;
        s16x4_t b0 = tr_read(Qt, half_swz(v, cb)), b1 = tr_read(Qt, half_swz(v + 4, cb));
        s16x8_t b = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        acc[t] = mfma(a, b, acc[t]);
      }
    }
  }
  const int co = co0 + wq * 32 + (lane & 31);
  if constexpr (DIRECT) {
    // dw[ci][co][tb .. tb + TT) += acc: TT contiguous floats per (ci, co), one owner
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int ci = p0 + cq * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
      float* d = ws + ((long)ci * Cout + co) * 8 + tb;
#pragma unroll
      for (int t0 = 0; t0 < TT; t0 += (TT < 4 ? TT : 4)) {
        if constexpr (TT == 2) {
          float2 o = *reinterpret_cast<float2*>(d + t0);
          o.x += acc[t0][e]; o.y += acc[t0 + 1][e];
          *reinterpret_cast<float2*>(d + t0) = o;
        } else {
          f32x4_t o = *reinterpret_cast<f32x4_t*>(d + t0);
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] += acc[t0 + k][e];
          *reinterpret_cast<f32x4_t*>(d + t0) = o;
        }
      }
    }
  } else {
    // C[row = ci][col = co] per tap -> this split's partial row ws[split][Cin][8][Cout]
    float* prow = ws + (long)blockIdx.x * 8 * Cin * Cout;
#pragma unroll
    for (int t = 0; t < TT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int ci = p0 + cq * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        prow[((long)ci * 8 + tb + t) * Cout + co] = acc[t][e];
      }
  }
  if (bias) {
    __syncthreads();  // every wave is done reading the tiles
    float* red = reinterpret_cast<float*>(lds);  // [512][8]
#pragma unroll
    for (int j = 0; j < 8; ++j) red[tid * 8 + j] = bs[j];
    __syncthreads();
    if (tid < 64) {  // channel co0 + tid = group tid / 8, element tid % 8
      const int q = tid >> 3, j = tid & 7;
      float sum = 0.f;
      for (int t = q; t < 512; t += 8) sum += red[t * 8 + j];
      bpart[((long)blockIdx.x * G + tg) * Cout + co0 + tid] = sum;
    }
  }
}

// db[c] += sum of the R bias partial rows [R][C] in row order (8 columns x 32 row lanes per
// block, the 32 lane sums added in lane order)
__global__ void __launch_bounds__(256) convt_bias_reduce(const float* part, int R, int C, float* db) {
  __shared__ float red[32][9];
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int c = blockIdx.x * 8 + cl;
  float s = 0.f;
  if (c < C)
    for (int r = rl; r < R; r += 32) s += part[(long)r * C + c];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < C) {
    float t = 0.f;
    for (int k = 0; k < 32; ++k) t += red[k][cl];
    db[c] += t;
  }
}

// split reduction, fixed order.  Stage 1 (S > 16): rows r*16 .. r*16+15 summed in place into
// row r*16 (E floats per row).
__global__ void __launch_bounds__(256) convt_group_sum(float* ws, int S, long E) {
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= E) return;
  const int r0 = blockIdx.y * 16, r1 = min(S, r0 + 16);
  ws[(long)r0 * E + e] = sum_rows16(ws + (long)r0 * E + e, E, r1 - r0);
}
// Stage 2: dw [Cin][Cout][8] (torch ConvTranspose3d layout, +=) = sum of R rows of
// [Cin][8][Cout] spaced `stride` rows apart.  Block = (ci, 32 co): [8][32] tiles read as
// 128-B rows, transposed through LDS, added to the contiguous 32 x 8 run of dw.
__global__ void __launch_bounds__(256) convt_wgrad_reduce(const float* ws, int R, int stride, float* dw, int Cin,
                                                          int Cout) {
  __shared__ float tile[8][33];
  const int ci = blockIdx.x, co0 = blockIdx.y * 32;
  const long rstep = (long)stride * 8 * Cin * Cout;
  const int e = threadIdx.x, t = e >> 5, c = e & 31;
  tile[t][c] = sum_rows16(ws + ((long)ci * 8 + t) * Cout + co0 + c, rstep, R);
  __syncthreads();
  dw[((long)ci * Cout + co0) * 8 + e] += tile[e & 7][e >> 3];
}

// One launch for the split reduction and the bias rows, bit-identical to convt_group_sum +
// convt_wgrad_reduce and convt_bias_reduce: blocks [0, Cin Cout / 32) sum one (ci, 32 co) tile's
// S partial rows -- groups of 16 rows in row order per thread (all 16 loads in flight), the
// group sums in group order -- and add them to dw through the same LDS transpose; the blocks
// past those (bpart != nullptr) add the RB bias rows to db with convt_bias_reduce's order (8
// rows' loads in flight per trip instead of one).
#ifndef PCMS_CONVT_RED_FUSED
#define PCMS_CONVT_RED_FUSED 1
#endif
static int g_convt_red_fused = PCMS_CONVT_RED_FUSED;  // 0: the separate launches (A/B, bit-identity test)
__global__ void __launch_bounds__(256) convt_reduce_fused_kernel(const float* ws, int S, float* dw, int Cin, int Cout,
                                                                 const float* bpart, int RB, float* db) {
  __shared__ float tile[8][33];
  __shared__ float red[32][9];
  const int nw = Cin * (Cout / 32);
  if ((int)blockIdx.x < nw) {
    const int ci = blockIdx.x / (Cout / 32), co0 = (blockIdx.x % (Cout / 32)) * 32;
    const long E = 8L * Cin * Cout;
    const int e = threadIdx.x, t = e >> 5, c = e & 31;
    const float* src = ws + ((long)ci * 8 + t) * Cout + co0 + c;
    float total = 0.f;
    for (int r0 = 0; r0 < S; r0 += 16) {
      const int n = min(16, S - r0);
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r < n) v[r] = src[(long)(r0 + r) * E];
      float gsum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (r < n) gsum += v[r];
      total += gsum;
    }
    tile[t][c] = total;
    __syncthreads();
    dw[((long)ci * Cout + co0) * 8 + e] += tile[e & 7][e >> 3];
    return;
  }
  const int cl = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int cc = (blockIdx.x - nw) * 8 + cl;
  float sb = 0.f;
  if (cc < Cout) {
    int r = rl;
    for (; r + 7 * 32 < RB; r += 8 * 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = bpart[(long)(r + 32 * u) * Cout + cc];
#pragma unroll
      for (int u = 0; u < 8; ++u) sb += v[u];
    }
    for (; r < RB; r += 32) sb += bpart[(long)r * Cout + cc];
  }
  red[rl][cl] = sb;
  __syncthreads();
  if (rl == 0 && cc < Cout) {
    float tt = 0.f;
    for (int k = 0; k < 32; ++k) tt += red[k][cl];
    db[cc] += tt;
  }
}

// master W[Cin][Cout][8] fp32 ->  fwd pack [8][Cout][Cin]  /  dgrad pack [Cin][8][Cout]
// (x6: element i = (row, k) of that order becomes the three B fragments of its 8-group:
// [row][k / 8][48] bf16, see afrag_x6)
template <typename T>
__global__ void convt_pack_kernel(const float* w, T* out, int Cin, int Cout, int dgrad) {
  const long total = (long)Cin * Cout * 8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    int t, co, ci;
    if (!dgrad) { ci = i % Cin; long r = i / Cin; co = r % Cout; t = r / Cout; }
    else { co = i % Cout; long r = i / Cout; t = r % 8; ci = r / 8; }
    const float v = w[((long)ci * Cout + co) * 8 + t];
    if constexpr (std::is_same<T, x6_t>::value) {
      bf16_t* o = reinterpret_cast<bf16_t*>(out) + (i >> 3) * 48;
      const int j = (int)(i & 7);
      const bf16_t hh = f2bf(v);
      const float rr = v - bf2f(hh);
      const bf16_t mm = f2bf(rr), ll = f2bf(rr - bf2f(mm));
      o[j] = hh; o[8 + j] = hh; o[16 + j] = mm; o[24 + j] = hh; o[32 + j] = ll; o[40 + j] = mm;
    } else {
      out[i] = Elem<T>::cvt(v);
    }
  }
}

// Adam + both bf16 ConvTranspose3d packs in one pass (cf. adam_pack_conv3_kernel).  Table
// entry [off, Cin, Cout, fwd pack, dgrad pack, first tile, -, -] (int64); one block per
// (32 ci x 32 co) tile: the 32 contiguous 256-float runs w[ci][co0..co0+32][8] are updated,
// converted to bf16 into LDS, and written as
//   fwd   [t][co][ci]   (64-B runs of 32 ci)
//   dgrad [ci][t][co]   (64-B runs of 32 co)
__global__ void __launch_bounds__(256) adam_pack_convt_kernel(float* P, float* Gr, float* Mo, float* Vo,
                                                              const long long* tab, int ntab, AdamCoef c,
                                                              const float* gmul) {
  __shared__ __attribute__((aligned(16))) uint16_t tb[32 * 256];  // [ci][co][t]
  int ei = 0;
  while (ei + 1 < ntab && tab[8 * (ei + 1) + 5] <= (long long)blockIdx.x) ++ei;
  const long long* e = tab + 8 * ei;
  const long off = (long)e[0];
  const int Cin = (int)e[1], Cout = (int)e[2];
  bf16_t* fwd = reinterpret_cast<bf16_t*>(e[3]);
  bf16_t* dgr = reinterpret_cast<bf16_t*>(e[4]);
  const int local = blockIdx.x - (int)e[5];
  const int co0 = (local % (Cout / 32)) * 32, ci0 = (local / (Cout / 32)) * 32;
  const float s = gmul ? c.gscale * gmul[0] : c.gscale;
  for (int i = 0; i < 8; ++i) {
    const int q4 = threadIdx.x + i * 256, run = q4 >> 6, q = q4 & 63;
    const long idx = off + ((long)(ci0 + run) * Cout + co0) * 8 + 4 * q;
    f32x4_t pv = *reinterpret_cast<const f32x4_t*>(P + idx), gv = *reinterpret_cast<const f32x4_t*>(Gr + idx);
    f32x4_t mv = *reinterpret_cast<const f32x4_t*>(Mo + idx), vv = *reinterpret_cast<const f32x4_t*>(Vo + idx);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float pk = pv[k], gk = gv[k], mk = mv[k], vk = vv[k];
      adam_update(pk, gk, mk, vk, c, s);
      pv[k] = pk; gv[k] = gk; mv[k] = mk; vv[k] = vk;
    }
    *reinterpret_cast<f32x4_t*>(P + idx) = pv;
    *reinterpret_cast<f32x4_t*>(Mo + idx) = mv;
    *reinterpret_cast<f32x4_t*>(Vo + idx) = vv;
    if (s != 1.f) *reinterpret_cast<f32x4_t*>(Gr + idx) = gv;
    uint2 o;
    o.x = pack_bf16x2(pv[0], pv[1]);
    o.y = pack_bf16x2(pv[2], pv[3]);
    *reinterpret_cast<uint2*>(tb + run * 256 + 4 * q) = o;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 8 * 32 * 4; k += 256) {  // fwd: (t, co, 8-ci group)
    const int grp = k & 3, co = (k >> 2) & 31, t = k >> 7;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (uint32_t)tb[(grp * 8 + 2 * i) * 256 + co * 8 + t] |
             ((uint32_t)tb[(grp * 8 + 2 * i + 1) * 256 + co * 8 + t] << 16);
    *reinterpret_cast<u32x4_t*>(fwd + ((long)t * Cout + co0 + co) * Cin + ci0 + grp * 8) = o;
  }
  for (int k = threadIdx.x; k < 32 * 8 * 4; k += 256) {  // dgrad: (ci, t, 8-co group)
    const int grp = k & 3, t = (k >> 2) & 7, ci = k >> 5;
    u32x4_t o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      o[i] = (uint32_t)tb[ci * 256 + (grp * 8 + 2 * i) * 8 + t] |
             ((uint32_t)tb[ci * 256 + (grp * 8 + 2 * i + 1) * 8 + t] << 16);
    *reinterpret_cast<u32x4_t*>(dgr + ((long)(ci0 + ci) * 8 + t) * Cout + co0 + grp * 8) = o;
  }
}

// fp32 build: Adam + both bf16x6 ConvTranspose3d packs (convt_pack_kernel<x6_t> layouts:
// fwd [t][co][ci / 8][48], dgrad [ci][t][co / 8][48]).  One block per (32 ci x 32 co) tile,
// the updated fp32 tile [ci][co][t] kept in LDS (32 KiB).
__global__ void __launch_bounds__(256) adam_pack_convt_x6_kernel(float* P, float* Gr, float* Mo, float* Vo,
                                                                 const long long* tab, int ntab, AdamCoef c,
                                                                 const float* gmul) {
  __shared__ float tf[32][257];  // [ci][co * 8 + t], rows padded by one float
  int ei = 0;
  while (ei + 1 < ntab && tab[8 * (ei + 1) + 5] <= (long long)blockIdx.x) ++ei;
  const long long* e = tab + 8 * ei;
  const long off = (long)e[0];
  const int Cin = (int)e[1], Cout = (int)e[2];
  bf16_t* fwd = reinterpret_cast<bf16_t*>(e[3]);
  bf16_t* dgr = reinterpret_cast<bf16_t*>(e[4]);
  const int local = blockIdx.x - (int)e[5];
  const int co0 = (local % (Cout / 32)) * 32, ci0 = (local / (Cout / 32)) * 32;
  const float s = gmul ? c.gscale * gmul[0] : c.gscale;
  for (int i = 0; i < 8; ++i) {
    const int q4 = threadIdx.x + i * 256, run = q4 >> 6, q = q4 & 63;
    const long idx = off + ((long)(ci0 + run) * Cout + co0) * 8 + 4 * q;
    f32x4_t pv = *reinterpret_cast<const f32x4_t*>(P + idx), gv = *reinterpret_cast<const f32x4_t*>(Gr + idx);
    f32x4_t mv = *reinterpret_cast<const f32x4_t*>(Mo + idx), vv = *reinterpret_cast<const f32x4_t*>(Vo + idx);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float pk = pv[k], gk = gv[k], mk = mv[k], vk = vv[k];
      adam_update(pk, gk, mk, vk, c, s);
      pv[k] = pk; gv[k] = gk; mv[k] = mk; vv[k] = vk;
      tf[run][4 * q + k] = pk;
    }
    *reinterpret_cast<f32x4_t*>(P + idx) = pv;
    *reinterpret_cast<f32x4_t*>(Mo + idx) = mv;
    *reinterpret_cast<f32x4_t*>(Vo + idx) = vv;
    if (s != 1.f) *reinterpret_cast<f32x4_t*>(Gr + idx) = gv;
  }
  __syncthreads();
  auto put = [](bf16_t* row, const float (&f)[8]) {
    u32x4_t h, m, l;
    split3x8(f, h, m, l);
    u32x4_t* o = reinterpret_cast<u32x4_t*>(row);
    o[0] = h; o[1] = h; o[2] = m; o[3] = h; o[4] = l; o[5] = m;
  };
  for (int k = threadIdx.x; k < 8 * 32 * 4; k += 256) {  // fwd rows (t, co, 8-ci group)
    const int grp = k & 3, co = (k >> 2) & 31, t = k >> 7;
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = tf[grp * 8 + i][co * 8 + t];
    put(fwd + (((long)t * Cout + co0 + co) * Cin + ci0 + grp * 8) * 6, f);
  }
  for (int k = threadIdx.x; k < 32 * 8 * 4; k += 256) {  // dgrad rows (ci, t, 8-co group)
    const int grp = k & 3, t = (k >> 2) & 7, ci = k >> 5;
    float f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = tf[ci][(grp * 8 + i) * 8 + t];
    put(dgr + (((long)(ci0 + ci) * 8 + t) * Cout + co0 + grp * 8) * 6, f);
  }
}

static int g_convt_stream = 1;  // the persistent forward at Cin 128 / Cout 64 (A/B switch)

inline int device_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ncu;
}

UpGeom make_geom(int N, int Din, int Hin, int Win, int Do, int Ho, int Wo) {
  UpGeom g;
  g.N = N; g.Din = Din; g.Hin = Hin; g.Win = Win; g.Do = Do; g.Ho = Ho; g.Wo = Wo;
  g.pz = (Do - 2 * Din) / 2; g.py = (Ho - 2 * Hin) / 2; g.px = (Wo - 2 * Win) / 2;
  return g;
}

}  // namespace

extern "C" {

// Adam over the ConvTranspose3d weights of a table (Cin % 32 == Cout % 32 == 0), writing both
// bf16 packs (pcms_convt_pack layouts).
int pcms_adam_pack_convt(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                         float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                         const float* gmul, hipStream_t s) {
  if (ntab <= 0 || ntiles <= 0) return 0;
  const AdamCoef c{step_size, b1, b2, eps, wd, bc2_sqrt, gscale};
  hipLaunchKernelGGL(adam_pack_convt_kernel, dim3(ntiles), dim3(256), 0, s, p, g, m, v, table, ntab, c, gmul);
  PCMS_CHECK_LAUNCH();
}

// the same for the fp32 build: both bf16x6 packs (pcms_convt_pack dtype 0 layouts)
int pcms_adam_pack_convt_x6(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                            float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                            const float* gmul, hipStream_t s) {
  if (ntab <= 0 || ntiles <= 0) return 0;
  const AdamCoef c{step_size, b1, b2, eps, wd, bc2_sqrt, gscale};
  hipLaunchKernelGGL(adam_pack_convt_x6_kernel, dim3(ntiles), dim3(256), 0, s, p, g, m, v, table, ntab, c, gmul);
  PCMS_CHECK_LAUNCH();
}

int pcms_convt_pack(int dtype, const float* w, void* out, int Cin, int Cout, int dgrad, hipStream_t s) {
  const long total = (long)Cin * Cout * 8;
  const int grid = (int)std::min<long>(4096, (total + 255) / 256);
  if (dtype == PCMS_BF16)
    hipLaunchKernelGGL(convt_pack_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, w, (bf16_t*)out, Cin, Cout, dgrad);
  else
    hipLaunchKernelGGL(convt_pack_kernel<x6_t>, dim3(grid), dim3(256), 0, s, w, (x6_t*)out, Cin, Cout, dgrad);
  PCMS_CHECK_LAUNCH();
}

// the persistent bf16 forward for Cin 128 / Cout 64 on (v = 1) / off (0); v < 0 queries
int pcms_convt_fwd_stream(int v) {
  const int old = g_convt_stream;
  if (v >= 0) g_convt_stream = v;
  return old;
}

// elements (activation dtype) of one ConvTranspose3d pack: bf16 8 Cin Cout; fp32 build
// (bf16x6) 48 bf16 per 8 weights = 3x the fp32 count
int pcms_convt_pack_elems(int dtype, int Cin, int Cout) {
  return dtype == PCMS_BF16 ? 8 * Cin * Cout : 3 * 8 * Cin * Cout;
}

// out: skip-sized (N, Do, Ho, Wo, Cout). If the grid is larger than 2x the input the pad
// ring is zero-filled here (F.pad semantics).
// fp32 build: 4 M-tiles per wave where that still leaves a workgroup per CU (level-0 forward
// 1072 -> 657 us, dgrad 1172 -> 744 us, level-1 dgrad 515 -> 363 us; 2 M-tiles, or a
// 2-workgroups-per-CU threshold, measured slower)
constexpr int kX6MT = 4;
static bool x6_mt4(long M, long colblocks) { return cdiv(M, 128 * kX6MT) * colblocks >= device_cus(); }

// K splits of the bf16 LDS forward: doubled while the grid is under 256 workgroups (level 4:
// 64 workgroups x 16 stages -> 256 x 4), each a power of two dividing the Cin / 64 stages
static int convt_fwd_splits(long M, int Cin, int Cout) {
  if (Cin % 64 || (8 * Cout) % kCDN) return 1;
  const long wgs = cdiv(M, kCDM) * (8 * Cout / kCDN);
  const int nst = Cin / 64;
  int S = 1;
  while (wgs * S < 256 && S < 16 && nst % (2 * S) == 0) S *= 2;
  return S;
}

int pcms_convt_fwd_ws_floats(int N, int Din, int Hin, int Win, int Cin, int Cout) {
  const long M = (long)N * Din * Hin * Win, S = convt_fwd_splits(M, Cin, Cout);
  const long f = S > 1 ? S * M * 8 * Cout : 0;
  return f >= (1L << 31) ? -7 : (int)f;
}

int pcms_convt_fwd(int dtype, const void* x, const void* wpack, const float* bias, void* out,
                   int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s) {
  return pcms_convt_fwd_ws(dtype, x, wpack, bias, out, nullptr, N, Din, Hin, Win, Cin, Cout, Do, Ho, Wo, s);
}

int pcms_convt_fwd_ws(int dtype, const void* x, const void* wpack, const float* bias, void* out, float* ws,
                      int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s) {
  if (Cin % 16 || Cout % 64) return -1;
  UpGeom g = make_geom(N, Din, Hin, Win, Do, Ho, Wo);
  if ((long)N * Do * Ho * Wo >= (1L << 31)) return -7;  // 32-bit voxel index math
  const size_t es = dtype == PCMS_BF16 ? 2 : 4;
  if (Do != 2 * Din || Ho != 2 * Hin || Wo != 2 * Win) {
    hipError_t e = hipMemsetAsync(out, 0, es * N * (size_t)Do * Ho * Wo * Cout, s);
    if (e != hipSuccess) return (int)e;
  }
  const long M = (long)N * Din * Hin * Win;
  if (dtype == PCMS_BF16 && Cin == 128 && Cout == 64 && Win % 4 == 0 && g_convt_stream) {
    const int ntile = cdiv(M, kSTM);
    hipLaunchKernelGGL(convt_fwd_stream_kernel, dim3(std::min(ntile, device_cus())), dim3(512), 0, s,
                       (const bf16_t*)x, (const bf16_t*)wpack, bias, (bf16_t*)out, g, ntile);
    PCMS_CHECK_LAUNCH();
  }
  if (dtype == PCMS_BF16 && Cin % 64 == 0 && (8 * Cout) % kCDN == 0) {
    const int S = ws ? convt_fwd_splits(M, Cin, Cout) : 1;
    if (S > 1) {
      auto kern = convt_lds_kernel<true, false, true>;
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kCDStage);
      hipLaunchKernelGGL(kern, dim3(cdiv(M, kCDM), 8 * Cout / kCDN, S), dim3(512), kCDStage, s,
                         (const bf16_t*)x, (const bf16_t*)wpack, bias, (bf16_t*)out, g, Cin, Cout, ws);
      const long E = M * 8 * Cout;
      hipLaunchKernelGGL(convt_fwd_reduce, dim3((unsigned)cdiv(E / 4, 256)), dim3(256), 0, s, (const float*)ws, S, M,
                         Cout, bias, (bf16_t*)out, g);
      PCMS_CHECK_LAUNCH();
    }
    const bool nt = 2L * N * Do * Ho * Wo * Cout >= kNtBytes;
    auto kern = nt ? convt_lds_kernel<true, true> : convt_lds_kernel<true, false>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kCDStage);
    // 1-D grid, XCD-aware tile order (level-0 forward 125 -> 117 us vs the 2-D grid)
    hipLaunchKernelGGL(kern, dim3(cdiv(M, kCDM) * (8 * Cout / kCDN)), dim3(512), kCDStage, s,
                       (const bf16_t*)x, (const bf16_t*)wpack, bias, (bf16_t*)out, g, Cin, Cout, nullptr);
    PCMS_CHECK_LAUNCH();
  }
  dim3 grid(cdiv(M, 128), 8 * Cout / 64);
  if (dtype == PCMS_BF16) {
    hipLaunchKernelGGL(convt_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)wpack, bias, (bf16_t*)out, g, Cin, Cout);
  } else if (x6_mt4(M, 8 * Cout / 64)) {
    grid.x = cdiv(M, 128 * kX6MT);
    hipLaunchKernelGGL(convt_fwd_x6_kernel<kX6MT>, grid, dim3(256), 0, s, (const float*)x, (const bf16_t*)wpack, bias, (float*)out, g, Cin, Cout);
  } else {
    hipLaunchKernelGGL(convt_fwd_x6_kernel<1>, grid, dim3(256), 0, s, (const float*)x, (const bf16_t*)wpack, bias, (float*)out, g, Cin, Cout);
  }
  PCMS_CHECK_LAUNCH();
}

// K splits of the bf16 LDS dgrad: doubled while the grid is under 256 workgroups (level 4:
// 16 workgroups x 64 stages -> 256 x 4), each a power of two dividing the 8 Cout / 64 stages
static int convt_dgrad_splits(long M, int Cin, int Cout) {
  if (Cin % kCDN || Cout % 64) return 1;
  const long wgs = cdiv(M, kCDM) * (Cin / kCDN);
  const int nst = 8 * Cout / 64;
  int S = 1;
  while (wgs * S < 256 && S < 16 && nst % (2 * S) == 0) S *= 2;
  return S;
}

int pcms_convt_dgrad_ws_floats(int N, int Din, int Hin, int Win, int Cin, int Cout) {
  const long M = (long)N * Din * Hin * Win, S = convt_dgrad_splits(M, Cin, Cout);
  const long f = S > 1 ? S * M * Cin : 0;
  return f >= (1L << 31) ? -7 : (int)f;
}

int pcms_convt_dgrad(int dtype, const void* dout, const void* wpack_d, void* dx,
                     int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s) {
  return pcms_convt_dgrad_ws(dtype, dout, wpack_d, dx, nullptr, N, Din, Hin, Win, Cin, Cout, Do, Ho, Wo, s);
}

int pcms_convt_dgrad_ws(int dtype, const void* dout, const void* wpack_d, void* dx, float* ws,
                        int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s) {
  if (Cin % 64 || Cout % 16) return -1;
  UpGeom g = make_geom(N, Din, Hin, Win, Do, Ho, Wo);
  if ((long)N * Do * Ho * Wo >= (1L << 31)) return -7;  // 32-bit voxel index math
  const long M = (long)N * Din * Hin * Win;
  if (dtype == PCMS_BF16 && Cin % kCDN == 0 && Cout % 64 == 0) {
    const bool nt = 2L * N * Do * Ho * Wo * Cout >= kNtBytes;  // dout
    const int S = ws ? convt_dgrad_splits(M, Cin, Cout) : 1;
    if (S > 1) {
      auto kern = convt_lds_kernel<false, false, true>;
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kCDStage);
      hipLaunchKernelGGL(kern, dim3(cdiv(M, kCDM), Cin / kCDN, S), dim3(512), kCDStage, s,
                         (const bf16_t*)dout, (const bf16_t*)wpack_d, nullptr, (bf16_t*)dx, g, Cin, Cout, ws);
      const long E = M * Cin;
      hipLaunchKernelGGL(convt_dgrad_reduce<bf16_t>, dim3((unsigned)cdiv(E / 4, 256)), dim3(256), 0, s, (const float*)ws, S,
                         E, (bf16_t*)dx);
      PCMS_CHECK_LAUNCH();
    }
    auto kern = nt ? convt_lds_kernel<false, true> : convt_lds_kernel<false, false>;
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, kCDStage);
    hipLaunchKernelGGL(kern, dim3(cdiv(M, kCDM), Cin / kCDN), dim3(512), kCDStage, s,
                       (const bf16_t*)dout, (const bf16_t*)wpack_d, nullptr, (bf16_t*)dx, g, Cin, Cout, nullptr);
    PCMS_CHECK_LAUNCH();
  }
  dim3 grid(cdiv(M, 128), Cin / 64);
  if (dtype == PCMS_BF16) {
    hipLaunchKernelGGL(convt_dgrad_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)dout, (const bf16_t*)wpack_d, (bf16_t*)dx, g, Cin, Cout);
    PCMS_CHECK_LAUNCH();
  }
  // fp32 build: K split into the workspace's slabs where the grid is small (level 4: 16
  // workgroups -> 256)
  const int S = ws ? convt_dgrad_splits(M, Cin, Cout) : 1;
  grid.z = S;
  if (x6_mt4(M, Cin / 64 * S)) {
    grid.x = cdiv(M, 128 * kX6MT);
    hipLaunchKernelGGL(convt_dgrad_x6_kernel<kX6MT>, grid, dim3(256), 0, s, (const float*)dout, (const bf16_t*)wpack_d,
                       (float*)dx, g, Cin, Cout, S > 1 ? ws : nullptr);
  } else {
    hipLaunchKernelGGL(convt_dgrad_x6_kernel<1>, grid, dim3(256), 0, s, (const float*)dout, (const bf16_t*)wpack_d,
                       (float*)dx, g, Cin, Cout, S > 1 ? ws : nullptr);
  }
  if (S > 1) {
    const long E = M * Cin;
    hipLaunchKernelGGL(convt_dgrad_reduce<float>, dim3((unsigned)cdiv(E / 4, 256)), dim3(256), 0, s, (const float*)ws,
                       S, E, (float*)dx);
  }
  PCMS_CHECK_LAUNCH();
}

// (the 128-ci bf16 kernel keeps the 64-ci split count: half the workgroups, the same
// partial rows -- doubling the splits doubled the partial-row traffic: slower at levels 1-3)
// G = 8 / TT tap groups divide the splits by G (the bf16 128-ci kernel's TT, see
// convt_wgrad128_kernel)
static int convt_wgrad_splits(int N, int Din, int Hin, int Win, int Cin, int Cout, int target_wgs, int* vps,
                              int G = 1) {
  const long M = (long)N * Din * Hin * Win;
  const int tiles = (Cout / 64) * (Cin / 64) * G;
  if (target_wgs <= 0) target_wgs = 512;
  const long nvb = (M + kVB - 1) / kVB;
  int splits = (int)std::max<long>(1, std::min<long>(nvb, cdiv(target_wgs, tiles)));
  *vps = (int)(cdiv(nvb, splits) * kVB);
  return (int)((M + *vps - 1) / *vps);
}

static int g_convt_wg_tt = 0;  // taps per workgroup of the bf16 128-ci weight gradient (0: by shape)

// The bf16 128-ci weight gradient's plan: taps per workgroup TT and the voxel splits.  By shape
// (`tests/tools/convt_wgrad_sweep.py`, `profiles/r4_convt_wgrad_sweep*.txt`): TT = 2 for
// Cin >= 256 at twice the workgroup target (the grids land at ~512 workgroups), TT = 4 at
// Cin = 128 at the target itself (103-107 us on both boxes measured; at twice the target 93
// on one box but 124-127 on another, `r4_convt_wgrad_l1_boxes.txt`);
// a plan of <= 2 splits runs as ONE split that writes dw directly (level 4: 49 -> 30 us; the
// partial rows and their reduce launch cost more than the extra staging per workgroup).
// pcms_convt_wgrad_taps(TT) pins TT at the plain target instead.  Other dtypes / Cin: TT = 8.
static int convt_wgrad_plan(int dtype, int N, int Din, int Hin, int Win, int Cin, int Cout, int target_wgs,
                            int* tt, int* vps) {
  if (dtype != PCMS_BF16 || Cin % 128) {
    *tt = 8;
    return convt_wgrad_splits(N, Din, Hin, Win, Cin, Cout, target_wgs, vps);
  }
  if (g_convt_wg_tt) {
    *tt = g_convt_wg_tt;
    return convt_wgrad_splits(N, Din, Hin, Win, Cin, Cout, target_wgs, vps, 8 / *tt);
  }
  if (target_wgs <= 0) target_wgs = 512;
  *tt = Cin >= 256 ? 2 : 4;
  const int splits = convt_wgrad_splits(N, Din, Hin, Win, Cin, Cout, Cin >= 256 ? 2 * target_wgs : target_wgs, vps,
                                        8 / *tt);
  if (splits > 2) return splits;
  const long M = (long)N * Din * Hin * Win;
  *vps = (int)(cdiv(M, kVB) * kVB);
  return 1;
}

// fp32 workspace floats pcms_convt_wgrad needs: one [Cin][8][Cout] partial row per split (the
// one-tap-group split count: tap groups only ever lower it, whatever the dtype)
int pcms_convt_wgrad_ws_floats(int N, int Din, int Hin, int Win, int Cin, int Cout, int target_wgs) {
  int vps;
  return convt_wgrad_splits(N, Din, Hin, Win, Cin, Cout, target_wgs, &vps) * 8 * Cin * Cout;
}

// A/B switch: taps per workgroup of the bf16 128-ci weight gradient (8, 4, 2; 0 = by shape);
// returns the previous value.  Set before the workspace queries.
// the ConvTranspose weight gradient's split rows and bias rows summed by one launch (1) or by
// the group-sum / reduce / bias-reduce launches (0), bit-identical; v < 0 queries.  Returns the
// previous value.
int pcms_convt_reduce_fused(int v) {
  const int old = g_convt_red_fused;
  if (v >= 0) g_convt_red_fused = v;
  return old;
}

int pcms_convt_wgrad_taps(int tt) {
  const int old = g_convt_wg_tt;
  if (tt == 0 || tt == 2 || tt == 4 || tt == 8) g_convt_wg_tt = tt;
  return old;
}

extern "C++" {
template <int TT>
static void launch_wgrad128(bool nt, bool direct, dim3 grid, hipStream_t s, const bf16_t* x, const bf16_t* dout,
                            float* ws, UpGeom g, int Cin, int Cout, int vps, float* bpart) {
  const int lds = (2 + TT) * 64 * 128;
  auto kern = nt ? (direct ? convt_wgrad128_kernel<true, TT, true> : convt_wgrad128_kernel<true, TT, false>)
                 : (direct ? convt_wgrad128_kernel<false, TT, true> : convt_wgrad128_kernel<false, TT, false>);
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(kern, grid, dim3(512), lds, s, x, dout, ws, g, Cin, Cout, vps, bpart);
}
}  // extern "C++"

// dw (torch layout [Cin][Cout][2][2][2], fp32) += ...; ws: pcms_convt_wgrad_ws_floats(...)
// floats (per-split partial rows summed in a fixed order: deterministic)
static int convt_wgrad_any(int dtype, const void* x, const void* dout, float* dw, float* ws, float* bpart,
                           float* db, int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo,
                           int target_wgs, hipStream_t s) {
  if (Cin % 64 || Cout % 64) return -1;
  UpGeom g = make_geom(N, Din, Hin, Win, Do, Ho, Wo);
  if ((long)N * Do * Ho * Wo >= (1L << 31)) return -7;  // 32-bit voxel index math
  int vps;
  const bool ci128 = dtype == PCMS_BF16 && Cin % 128 == 0;
  int TT;
  const int splits = convt_wgrad_plan(dtype, N, Din, Hin, Win, Cin, Cout, target_wgs, &TT, &vps), G = 8 / TT;
  if (ci128) {
    dim3 grid(splits, Cout / 64, (Cin / 128) * G);
    const bool nt = 2L * N * Do * Ho * Wo * Cout >= kNtBytes;
    const bool direct = splits == 1;
    float* dst = direct ? dw : ws;
    if (TT == 8) launch_wgrad128<8>(nt, direct, grid, s, (const bf16_t*)x, (const bf16_t*)dout, dst, g, Cin, Cout, vps, bpart);
    else if (TT == 4) launch_wgrad128<4>(nt, direct, grid, s, (const bf16_t*)x, (const bf16_t*)dout, dst, g, Cin, Cout, vps, bpart);
    else launch_wgrad128<2>(nt, direct, grid, s, (const bf16_t*)x, (const bf16_t*)dout, dst, g, Cin, Cout, vps, bpart);
    if (direct || !g_convt_red_fused) {
      if (bpart != nullptr) {
        hipError_t eb = hipGetLastError();
        if (eb != hipSuccess) return (int)eb;
        hipLaunchKernelGGL(convt_bias_reduce, dim3(cdiv(Cout, 8)), dim3(256), 0, s, (const float*)bpart, splits * G,
                           Cout, db);
      }
      if (direct) PCMS_CHECK_LAUNCH();
    }
  }
  dim3 grid(splits, Cout / 64, Cin / 64);
  if (ci128) {
    // launched above
  } else if (dtype == PCMS_BF16) {
    constexpr int lds = 9 * CW<bf16_t>::VB * 128;
    (void)hipFuncSetAttribute((const void*)convt_wgrad_kernel<bf16_t>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(convt_wgrad_kernel<bf16_t>, grid, dim3(512), lds, s, (const bf16_t*)x, (const bf16_t*)dout, ws, g,
                       Cin, Cout, vps);
  } else {
    constexpr int lds = 9 * CW<float>::VB * 256;
    (void)hipFuncSetAttribute((const void*)convt_wgrad_kernel<float>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(convt_wgrad_kernel<float>, grid, dim3(512), lds, s, (const float*)x, (const float*)dout, ws, g,
                       Cin, Cout, vps);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const long E = 8L * Cin * Cout;
  if (g_convt_red_fused) {  // the split rows (and, bf16 128-ci path, the bias rows) in one launch
    const bool bias = ci128 && bpart != nullptr;
    const int nblk = Cin * (Cout / 32) + (bias ? cdiv(Cout, 8) : 0);
    hipLaunchKernelGGL(convt_reduce_fused_kernel, dim3(nblk), dim3(256), 0, s, (const float*)ws, splits, dw, Cin, Cout,
                       bias ? (const float*)bpart : nullptr, bias ? splits * G : 0, db);
    PCMS_CHECK_LAUNCH();
  }
  int R = splits, stride = 1;
  if (splits > 16) {
    hipLaunchKernelGGL(convt_group_sum, dim3((unsigned)cdiv(E, 256), cdiv(splits, 16)), dim3(256), 0, s, ws, splits, E);
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    R = cdiv(splits, 16);
    stride = 16;
  }
  hipLaunchKernelGGL(convt_wgrad_reduce, dim3(Cin, Cout / 32), dim3(256), 0, s, (const float*)ws, R, stride, dw, Cin,
                     Cout);
  PCMS_CHECK_LAUNCH();
}

int pcms_convt_wgrad(int dtype, const void* x, const void* dout, float* dw, float* ws,
                     int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo,
                     int target_wgs, hipStream_t s) {
  return convt_wgrad_any(dtype, x, dout, dw, ws, nullptr, nullptr, N, Din, Hin, Win, Cin, Cout, Do, Ho, Wo,
                         target_wgs, s);
}

// the bias-gradient workspace of pcms_convt_wgrad_bias: one [Cout] row per voxel split (fused
// path) or pcms_box_channel_sum's rows (the other paths), whichever is larger
int pcms_convt_wgrad_bias_ws_floats(int dtype, int N, int Din, int Hin, int Win, int Cin, int Cout, int target_wgs) {
  int vps;
  int TT;
  const int splits = convt_wgrad_plan(dtype, N, Din, Hin, Win, Cin, Cout, target_wgs, &TT, &vps);
  const int fused = splits * (8 / TT) * Cout;
  const int box = pcms_box_channel_sum_ws_floats(dtype, N, Cout, 2 * Din, 2 * Hin, 2 * Win);
  return std::max(fused, box);
}

// pcms_convt_wgrad + db[co] += the sum of dout over the ConvT output box (the bias gradient;
// F.pad's front offsets floor((Do - 2 Din) / 2), ...): from the weight gradient's own read of
// dout on the bf16 128-ci path, else pcms_box_channel_sum after it
int pcms_convt_wgrad_bias(int dtype, const void* x, const void* dout, float* dw, float* db, float* ws, float* bws,
                          int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo,
                          int target_wgs, hipStream_t s) {
  if (db == nullptr || bws == nullptr) return -2;
  if (dtype == PCMS_BF16 && Cin % 128 == 0 && Cout % 64 == 0)
    return convt_wgrad_any(dtype, x, dout, dw, ws, bws, db, N, Din, Hin, Win, Cin, Cout, Do, Ho, Wo, target_wgs, s);
  const int rc = convt_wgrad_any(dtype, x, dout, dw, ws, nullptr, nullptr, N, Din, Hin, Win, Cin, Cout, Do, Ho, Wo,
                                 target_wgs, s);
  if (rc) return rc;
  return pcms_box_channel_sum(dtype, dout, db, bws, N, Do, Ho, Wo, Cout, (Do - 2 * Din) / 2, (Ho - 2 * Hin) / 2,
                              (Wo - 2 * Win) / 2, 2 * Din, 2 * Hin, 2 * Win, s);
}

}  // extern "C"
