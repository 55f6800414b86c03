// Device helpers shared by the 3x3x3 convolution kernels (conv3.hip, stem.hip), gfx950.
#pragma once
#include "common.h"
#include <algorithm>
#include <utility>

namespace {

constexpr int kThreads = 256;
constexpr int kRowBytes = 64;      // one halo row = one LDS row of the current ci-chunk
constexpr int kHaloMax = 1152;     // halo voxels per workgroup (72 KiB LDS, 2 WG / CU)

__device__ __attribute__((aligned(16))) uint32_t g_zero16[4];  // zero page for LDS-DMA padding
constexpr uint32_t kOOB = 0x80000000u;  // buffer voffset past num_records: reads zeros

// fp32 data in HBM, split-bf16 arithmetic on the bf16 MFMA (the halo is split in LDS once per
// chunk, the weights in their pack):
//  x6_t (dtype PCMS_F32, the parity build): v = h + m + l, three bf16 parts (24 significant
//       bits: v to fp32 rounding); a product keeps the six terms down to 2^-16 of it (hh, hm,
//       mh, hl, lh, mm) in THREE MFMAs over 8 channels, by concatenating K halves:
//       [h|m].[h|h] + [h|l].[m|h] + [h|m].[l|m];
//  x3_t (dtype PCMS_F32X3): v = h + l (16 bits), hh + lh + hl in three MFMAs over 16
//       channels: twice the rate, ~10x the fp32 rounding error (measured: misses the
//       north-star 1e-3 logit bar by ~30 %; kept as an explicit faster mode).
// (the tags x3_t / x6_t live in common.h)

template <typename T> struct Traits;
template <> struct Traits<bf16_t> {
  static constexpr int CK = 32;    // channels per chunk (64 B rows)
  static constexpr int KS = 2;     // MFMA k-steps per chunk and tap (K = 16 each)
  static constexpr int VEC = 8;    // elements per 16-byte piece
  static constexpr int WK = 32;    // bf16 weights per pack row
  typedef s16x8_t Frag;
  typedef bf16_t Mem;              // activation element in HBM
};
template <> struct Traits<x3_t> {
  static constexpr int CK = 16;    // fp32 channels per chunk (64 B rows, split in place into
  static constexpr int KS = 2;     //   [hi 0-7 | hi 8-15 | lo 0-7 | lo 8-15]: "k-step" 0 = hi, 1 = lo)
  static constexpr int VEC = 4;
  static constexpr int WK = 32;    // pack row: 16 hi weights, then their 16 lo parts
  typedef s16x8_t Frag;
  typedef float Mem;
};
template <> struct Traits<x6_t> {
  static constexpr int CK = 8;     // fp32 channels per chunk (32 B of a 64-B row, split in
  static constexpr int KS = 3;     //   place into logical slots [h 0-7 | m 0-7 | l 0-7 | -])
  static constexpr int VEC = 4;
  static constexpr int WK = 48;    // pack row: the three B fragments [h|h] [m|h] [l|m]
  typedef s16x8_t Frag;
  typedef float Mem;
};

__device__ __forceinline__ f32x16_t mfma(s16x8_t a, s16x8_t b, f32x16_t c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}
// two floats -> {hi, lo}: their bf16 halves, each packed bf16x2 (element 0 in the low half)
__device__ __forceinline__ u32x2_t split2(float a, float b) {
  const uint32_t hi = pack_bf16x2(a, b);
  return (u32x2_t){hi, pack_bf16x2(a - __uint_as_float(hi << 16), b - __uint_as_float(hi & 0xffff0000u))};
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
__device__ __forceinline__ s16x8_t lds_a(const char* lds, int row, int ks, int h) {
  int slot = (ks * 2 + h) ^ swz(row);
  return *reinterpret_cast<const s16x8_t*>(lds + row * kRowBytes + slot * 16);
}
// the 16-B logical slot s of a halo row
__device__ __forceinline__ s16x8_t lds_slot(const char* lds, int row, int s) {
  return *reinterpret_cast<const s16x8_t*>(lds + row * kRowBytes + (s ^ swz(row)) * 16);
}
// B fragment (weights) straight from global: packed [chunk][27][Cout][WK] (fp32-data builds).
__device__ __forceinline__ s16x8_t gl_b(const bf16_t* wrow, int ks, int h) {
  return *reinterpret_cast<const s16x8_t*>(wrow + ks * 16 + h * 8);
}
// bf16 weight pack, fragment-major (round 5): element (chunk c = k / 32, tap t, row j, k % 32)
// of a J-row pack (J % 32 == 0) sits in the 1 KiB block (c, t, row tile j / 32, k-step
// ks = (k / 16) % 2) at lane (j % 32) + 32 ((k / 8) % 2), element k % 8 -- exactly the
// v_mfma_f32_32x32x16_bf16 B operand of that (32-row tile, k-step), so one B fragment is ONE
// contiguous 1 KiB wave load (8 whole 128-B lines) instead of 16-32 lines touched in part,
// and a row tile's two k-steps are adjacent (constant offsets from one address).
__device__ __forceinline__ long pack_bf16_off(int c, int t, int j, int k, int J) {
  return (((long)c * 27 + t) * (J >> 5) + (j >> 5)) * 1024 + (k >> 4 & 1) * 512 +
         ((j & 31) + (k >> 3 & 1) * 32) * 8 + (k & 7);
}

struct Conv3Params {
  const void* x0; const void* x1; int c0; int c1;
  const void* w; const float* bias;
  void* y0; void* y1; int cy0;
  float* yacc; float* stats;
  int accumulate;        // PCMS_CONV_ACCUMULATE: y += conv; PCMS_CONV_RELU: y = relu(conv + b)
  int N, D, H, W, Cin, Cout;
  int nchunk, chunks_per_split;
  long nvox;             // N * D * H * W (split-K slab stride, in voxels)
  int lbd, lbh, lbw, nbd, nbh, nbw;
  // conv3_fwd_big_kernel<true> (pcms_conv3_fwd_bnin): the input is relu(x * isc + ish) per
  // input channel, applied to the staged halo in LDS (the BatchNorm + ReLU of the layer below)
  const float* isc = nullptr; const float* ish = nullptr;
};

// dy tile: 128-B (bf16) rows, 64-B halves swizzled by row bit 1 (conflict-free tr reads).
__device__ __forceinline__ int dy_off_bf16(int v, int co) {  // co in 0..63 (element)
  int half = (co >> 5) ^ ((v >> 1) & 1);
  return v * 128 + half * 64 + (co & 31) * 2;
}

__device__ __forceinline__ s16x4_t tr_read(const char* lds, int byte_off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4_t*)(lds + byte_off));
}

// an opaque copy: values derived from it are recomputed where used instead of being hoisted
// out of a loop (and spilled: a spill reload is a vector-memory load whose wait would
// also drain the hidden B loads and halo DMA in flight)
__device__ __forceinline__ int opaque(int v) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// compile-time loop: f(integral_constant<int, i>) for i < N
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F> __device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
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

// Forward/dgrad box: `vol` (512 or 256) voxels; width 16 whenever the grid is that wide
// (perm32 layout).
Box fwd_box(int D, int H, int W, int vol = 512) {
  const int lv = vol >= 512 ? 5 : 4;  // log2(bd * bh) at width 16
  if (W >= 16) {
    Box best{0, 0, 4};
    double bc = 1e30;
    for (int a = 0; a <= lv; ++a) {
      const int b = lv - a;  // bd * bh = vol / 16
      const int bd = 1 << a, bh = 1 << b;
      if ((bd + 2) * (bh + 2) * 18 > kHaloMax) continue;
      const double cost = (double)cdiv(D, bd) * bd * cdiv(H, bh) * bh +
                          0.15 * cdiv(D, bd) * cdiv(H, bh) * (bd + 2) * (bh + 2) * 18 / 16.0;
      if (cost < bc - 1e-9 || (cost < bc + 1e-9 && a == 2)) { bc = cost; best = Box{a, b, 4}; }
    }
    return best;
  }
  return choose_box(D, H, W, vol >= 512 ? 512 : 256, kHaloMax, 4, 32);
}

// compute units of the current device (persistent-grid sizing)
inline int device_cus() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ncu;
}

}  // namespace
